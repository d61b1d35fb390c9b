"""CPU baseline of bench.py — BENCHMARK INFRASTRUCTURE, not product code.

Run as its own process (`python -m oracle.cpu_baseline ...`, spawned by bench.py's `cpu_baseline`
leg after the GPU timed region) so that MKL's threads share the process with nothing else: no torch
OpenMP pool, no HIP runtime threads, MKL's own Intel OpenMP layer (the in-process GNU layer was the
one torch's libgomp forced), idle threads sleeping at once (KMP_BLOCKTIME=0: spinning threads burn a
container's CPU quota and get the whole process throttled), the process pinned to `threads` CPUs of
its affinity set.

What is timed (SURVEY §8 d; scripts/benchmarks_cpu.jl:26-50 drives MadIPM with a multithreaded
supernodal LDL^T, HSL MA57, which cannot run here): the oracle's MPC loop (oracle/mpc.py, a
restatement of src/solver.jl) with MKL PARDISO (oracle/pardiso.py; symmetric indefinite, the GPU's
fill-reducing order) as its linear solver, on the same standard-form problem as the GPU, to
optimality, once per thread count of the sweep.  value = MPC iterations / the whole loop's time
(PARDISO factor + solve AND the numpy vector work, the reference's total_time scope) at the thread
count with the fastest loop; the PARDISO-only rate (what a native host driver around PARDISO would
reach) is reported beside it as pardiso_iters_per_s.  cores = the distinct physical cores the
measured thread count ran on (the process is pinned one thread per physical core first); threads =
that thread count.

Prints ONE JSON line.
"""
from __future__ import annotations

import os
import sys


def _topo(cpu: int) -> dict:
    """(package, core, SMT siblings) of a CPU from sysfs (None where not readable)."""
    base = f"/sys/devices/system/cpu/cpu{cpu}/topology/"
    out = {"cpu": cpu}
    for k, f in (("package", "physical_package_id"), ("core", "core_id"), ("siblings", "thread_siblings_list")):
        try:
            with open(base + f) as fh:
                v = fh.read().strip()
            out[k] = int(v) if k != "siblings" else v
        except OSError:
            out[k] = None
    return out


def _pin(threads: int) -> list:
    """Pin to `threads` CPUs of the affinity set, one per physical core first (an SMT sibling shares
    the core's FPUs and caches with the thread beside it: MKL's threads then compete for them)."""
    cpus = sorted(os.sched_getaffinity(0))
    topo = [_topo(c) for c in cpus]
    seen, first, rest = set(), [], []
    for t in topo:
        key = (t["package"], t["core"])
        if t["core"] is None or key not in seen:
            seen.add(key)
            first.append(t["cpu"])
        else:
            rest.append(t["cpu"])
    use = (first + rest)[:threads]
    os.sched_setaffinity(0, use)
    return use


def _loadavg():
    try:
        with open("/proc/loadavg") as f:
            return f.read().split()[:3]
    except OSError:
        return None


def _cgroup_quota():
    for p in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(p) as f:
                return f.read().strip()
        except OSError:
            pass
    return None


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="ex10")
    ap.add_argument("--perm", default="", help=".npy pivot order of the GPU analysis (default: PARDISO's METIS)")
    ap.add_argument("--threads", default="1,2,4,8,16")
    ap.add_argument("--max-threads", type=int, default=16)
    args = ap.parse_args()
    tmax = max(1, args.max_threads)
    counts = sorted({min(int(t), tmax) for t in args.threads.split(",") if int(t) > 0})
    # environment of MKL / OpenMP before anything loads them
    os.environ.setdefault("MKL_THREADING_LAYER", "INTEL")
    os.environ["KMP_BLOCKTIME"] = "0"
    os.environ["OMP_WAIT_POLICY"] = "PASSIVE"
    os.environ["MKL_DYNAMIC"] = "FALSE"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"     # numpy's own BLAS: the loop's vector work is serial
    naff = len(os.sched_getaffinity(0))
    cpus = _pin(tmax)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "madipm.jl_amd"))
    sys.path.insert(0, root)
    import json
    import time
    import numpy as np
    from bench import build_problem
    from oracle.mpc import OracleMPC, OracleOptions
    from oracle import pardiso

    qp, name = build_problem(args.config)
    perm = np.load(args.perm) if args.perm else None
    runs = []
    ref = None
    import resource
    load0 = _loadavg()
    for t in counts:
        got = pardiso.set_threads(t)
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        o = OracleMPC(qp, OracleOptions(regularization=("fixed", 1e-8, -1e-8), step_rule=("adaptive", 0.99),
                                        max_iter=300, tol=1e-8), record_trace=False)
        o.linear_solver = "pardiso"
        o.ldl_perm = perm
        t0 = time.perf_counter()
        st = o.solve()
        wall = time.perf_counter() - t0
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        F = o._pardiso
        fs = F.t_factor + F.t_solve
        runs.append({"threads": got, "iters": st.iter, "iters_per_s": st.iter / fs if fs > 0 else None,
                     "loop_s": st.total_time, "wall_s": wall, "pardiso_factor_s": F.t_factor,
                     "pardiso_solve_s": F.t_solve, "factorizations": F.nfactor, "solves": F.nsolve,
                     "pardiso_analysis_s": F.t_analysis, "nnzL_pardiso": F.nnzL,
                     "perturbed_pivots": F.nperturbed, "status": st.status, "objective": st.objective,
                     # process CPU time / wall: how many of the t threads actually ran (a cgroup quota,
                     # co-tenants or SMT siblings show up as a ratio well below t)
                     "cpu_s": cpu_s, "cpu_per_wall": cpu_s / wall if wall > 0 else None,
                     "involuntary_switches": ru1.ru_nivcsw - ru0.ru_nivcsw})
        if ref is None:
            ref = st
        F.free()
    for r in runs:
        r["loop_iters_per_s"] = r["iters"] / r["loop_s"] if r["loop_s"] > 0 else None
    best = max(runs, key=lambda r: r["loop_iters_per_s"] or 0.0)
    bestp = max(runs, key=lambda r: r["iters_per_s"] or 0.0)
    one = next((r for r in runs if r["threads"] == 1), None)
    top = max(runs, key=lambda r: r["threads"])
    used = cpus[:best["threads"]]
    cores = len({(t["package"], t["core"]) if t["core"] is not None else ("cpu", t["cpu"]) for t in map(_topo, used)})
    out = {"value": best["loop_iters_per_s"], "unit": "iters/s", "cores": cores, "threads": best["threads"],
           "kind": "port",
           "sample": (f"oracle/mpc.py MPC loop + MKL PARDISO (mtype -2, GPU's fill-reducing order) on the same "
                      f"standard-form problem ({name}), to optimality ({ref.iter} iterations) at "
                      f"{', '.join(str(r['threads']) for r in runs)} threads in a process of its own pinned to "
                      f"{len(cpus)} CPUs; value = iterations / whole-loop time (PARDISO + numpy vector work) "
                      f"at the fastest thread count ({best['threads']} threads on {cores} physical cores)"),
           "pardiso_iters_per_s": bestp["iters_per_s"], "pardiso_threads": bestp["threads"],
           "value_threads": top["loop_iters_per_s"], "threads_max": top["threads"],
           "value_1thread": one["loop_iters_per_s"] if one else None,
           "pardiso_iters_per_s_1thread": one["iters_per_s"] if one else None,
           "sweep": runs, "cpus": cpus, "cpu_topology": [_topo(c) for c in cpus],
           "affinity_cpus_before_pin": naff,
           "loadavg_before": load0, "loadavg_after": _loadavg(), "cgroup_cpu_quota": _cgroup_quota(),
           "env": {k: os.environ.get(k) for k in ("MKL_THREADING_LAYER", "KMP_BLOCKTIME", "OMP_WAIT_POLICY")},
           "ref_status": ref.status, "ref_objective": ref.objective, "ref_iter": ref.iter}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
