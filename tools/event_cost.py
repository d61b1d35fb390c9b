"""Cost of the bench's HIP events around the dominant kernel: ex10's MPC loop timed with the dominant
kind's events on (every launch) and off, alternating, in one process (python tools/event_cost.py)."""
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
cfg = sys.argv[1] if len(sys.argv) > 1 else "ex10"
qp, _ = bench.build_problem(cfg)
s = MPCSolver(qp, **bench.solver_opts())
s.set_kernel_timing()
s.set_max_iter(2)
s.solve()
warm = s.kernel_stats()
names = [k["name"] for k in warm]
dom = max(warm, key=lambda k: k["time_ms"])["name"]
for rep in range(4):
    for mask in (1 << names.index(dom), 0):
        s.set_kernel_timing(mask)
        s.set_max_iter(30)
        s.initialize()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = s.solve(fetch_solution=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{cfg} events {'on ' if mask else 'off'}: {1e3 * dt / st.iter:.4f} ms/iter ({st.iter} iters)", flush=True)
