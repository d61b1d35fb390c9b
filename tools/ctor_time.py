"""Wall time of MPCSolver construction (bench.py's `analysis_s`) per bench config on the GPU box, with
each construction phase on stderr (MADIPM_SYMBOLIC_TIMING=1 python tools/ctor_time.py ex10 neos).
As in bench.py, torch's CUDA context exists before the first construction; every config is
constructed twice (the first construction of the process pays one-off runtime set-up)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "madipm.jl_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from madipm_amd import MPCSolver  # noqa: E402
from madipm_amd import _lib  # noqa: E402

torch.cuda.set_device(0)
_lib.check(_lib.madipm_set_device(0), "madipm_set_device")
torch.zeros(1, device="cuda")
for name in sys.argv[1:]:
    qp, _ = bench.build_problem(name)
    for rep in range(2):
        t = time.perf_counter()
        s = MPCSolver(qp, **bench.solver_opts())
        dt = time.perf_counter() - t
        print(f"{name} ctor {dt:.3f} s", flush=True)
        print(f"{name} ctor {dt:.3f} s", file=sys.stderr, flush=True)
        del s
