"""Construction time of MPCSolver on one config (run on the GPU box, MADIPM_SYMBOLIC_TIMING=1 for the
phases): python tools/ctor_time.py [config]"""
import sys
import time

sys.path[:0] = [".", "madipm.jl_amd"]
import torch  # noqa: E402

torch.cuda.set_device(0)
from madipm_amd import _lib  # noqa: E402

_lib.madipm_set_device(0)
import bench  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "dense_qp"
t = time.perf_counter()
qp, _ = bench.build_problem(cfg)
print("build", round(time.perf_counter() - t, 2), flush=True)
from madipm_amd import MPCSolver  # noqa: E402

t = time.perf_counter()
s = MPCSolver(qp, **bench.solver_opts(), **({"ordering": 0} if cfg.startswith("dense_qp") else {}))
print("ctor", round(time.perf_counter() - t, 2), flush=True)
t = time.perf_counter()
del s
print("del", round(time.perf_counter() - t, 2), flush=True)
