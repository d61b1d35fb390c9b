"""Worker for tests/test_shard_gpu.py::test_multiprocess_sharded_mpc (launched by torch.distributed.run).

Every rank holds one shard of the subtree-sharded LDL^T; the collectives go through HostComm
(torch.distributed gloo, host-staged) because the ranks share one GPU, where RCCL cannot run.  The
replicated MPC state must be bitwise identical on every rank, and match the unsharded solve."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "madipm.jl_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    from madipm_amd import MPCSolver, FixedRegularization, HostComm, standard_form_qp
    from madipm_amd.instances import ex10_standin
    qp = standard_form_qp(ex10_standin(scale=0.05))
    kw = dict(regularization=FixedRegularization(1e-8, -1e-8), max_iter=300)
    comm = HostComm(dist)
    st = MPCSolver(qp, comm=comm, **kw).solve()
    vals = torch.tensor([st.objective, float(st.iter), float(st.status)], dtype=torch.float64)
    allv = [torch.zeros_like(vals) for _ in range(world)]
    dist.all_gather(allv, vals)
    out = {"rank": rank, "objective": st.objective, "iter": st.iter, "status": st.status,
           "identical": all(bool(torch.equal(a, allv[0])) for a in allv)}
    if rank == 0:
        ref = MPCSolver(qp, **kw).solve()
        out.update(ref_objective=ref.objective, ref_iter=ref.iter, ref_status=ref.status)
        print("RESULT " + json.dumps(out), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
