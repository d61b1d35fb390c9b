"""Diagnostics: the batched-leaf SYRK (k_lb_syrk) and the big-front kernels on a dense-column K2 of a
chosen size, without the MPC setup: K2 = [diag(sig) A^T; A -delta I] with dense A (m x n), natural
order, factorised `reps` times with live kernel timing.  Prints per-kernel time and TF/s.
usage (GPU box): python tools/lb_syrk_bench.py [m n reps]   (MADIPM_LIB selects a variant build)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "madipm.jl_amd"))


def main():
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 16000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    import torch
    from madipm_amd.linear_solver import HIPLDLSolver
    N = n + m
    t0 = time.perf_counter()
    # lower CSC: x column j = diagonal + the m rows of A; y columns = diagonal only
    cp = np.zeros(N + 1, np.int64)
    cp[1:n + 1] = m + 1
    cp[n + 1:] = 1
    cp = np.cumsum(cp)
    rv = np.empty(cp[-1], np.int32)
    blk = np.concatenate([[0], np.arange(n, N, dtype=np.int32)])
    for j in range(n):
        blk[0] = j
        rv[cp[j]:cp[j + 1]] = blk
    rv[cp[n]:] = np.arange(n, N, dtype=np.int32)
    rng = np.random.default_rng(0)
    vals = rng.standard_normal(cp[-1])
    diag = cp[:-1]
    vals[diag[:n]] = 10.0 ** rng.uniform(-1, 1, n)
    vals[diag[n:]] = -1e-2
    t1 = time.perf_counter()
    ls = HIPLDLSolver(N, cp, rv, ordering=0)
    t2 = time.perf_counter()
    print(f"m={m} n={n} nnz={cp[-1]:.3e}  pattern {t1 - t0:.1f} s  analysis+upload {t2 - t1:.1f} s", flush=True)
    dv = torch.from_numpy(vals).cuda()
    assert ls.factorize(dv) == 0  # warm-up
    ls.set_kernel_timing()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    for _ in range(reps):
        rc = ls.factorize(dv)
        assert rc == 0, rc
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"factorisation {1e3 * (t4 - t3) / reps:.2f} ms (wall, incl. sync)")
    for k in ls.kernel_stats():
        if k["launches"] == 0:
            continue
        tf = k["flops"] / (k["time_ms"] * 1e-3) / 1e12 if k["time_ms"] > 0 else 0.0
        print(f"  {k['name']:16s} launches {k['launches']:6d}  {k['time_ms'] / reps:9.3f} ms/fact  {tf:7.2f} TF/s")


if __name__ == "__main__":
    main()
