"""Subtree-sharding model of the multi-GPU factorisation, on the host.

For a config and P = 1, 2, 4, 8 shards: the symbolic partition (madipm_symbolic_analyze_shard, the
same analysis every rank runs), the cost-model totals it optimises (top cost, largest shard cost),
the factorisation flops and stored L bytes of the top fronts and of every shard, the bytes the
collectives move (all-reduce of the packed top fronts per factorisation; per solve the all-reduce of
the top rows and the in-place all-gather of the shards' solution slices), and a modelled MPC
iteration time:

  t(P) = (F_shardmax + F_top) / R_f + 2 (B_shardmax + B_top) / R_s + t_comm(P) + t_vec
  t_comm = AR(8 xch_fact) + 2 [AR(8 xch_solve) + AG(8 xch_gather)]
  ring all-reduce of n bytes: 2 (P-1)/P n / BW + 2 (P-1) alpha; all-gather: (P-1)/P n / BW + (P-1) alpha

R_f, R_s (effective factorisation flop rate, solve byte rate) and t_vec are calibrated from the
measured single-GPU iteration (--fact-ms / --solve-ms / --iter-ms: one factorisation, the two solves
and the whole iteration at P = 1, e.g. from a rocprof summary); BW = one xGMI link (153 GB/s, the
ring's per-link bound), alpha = 10 us per ring step.  The top fronts are factorised redundantly on
every rank, so F_top and B_top do not shrink with P.

  python tools/shard_model.py neos --fact-ms 27.4 --solve-ms 5.9 --iter-ms 33.6
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "madipm.jl_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402


def front_costs(first, nrows):
    w = np.diff(first).astype(np.float64)
    r = nrows.astype(np.float64)
    # flops of a front: sum over its pivots t of (r - t - 1)(r - t + 2) (symbolic.cpp's count)
    fl = np.zeros(len(r))
    for k in range(len(r)):
        cc = r[k] - np.arange(w[k])
        fl[k] = np.sum((cc - 1.0) * (cc + 2.0))
    lbytes = 8.0 * (r * w - w * (w - 1) / 2.0)
    return fl, lbytes


def model(config, P, fact_ms, solve_ms, iter_ms, bw=153e9, alpha=10e-6):
    import bench
    from helpers import lp_k2
    from madipm_amd._lib import Symbolic, default_ldl_opts
    qp, _ = bench.build_problem(config)
    K, Lw = lp_k2(qp, 0)
    S1 = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts())
    f1, n1 = S1.supernodes()[0], S1.supernodes()[2]
    fl1, lb1 = front_costs(f1, n1)
    F1, B1 = fl1.sum(), lb1.sum()
    R_f = F1 / (fact_ms * 1e-3)
    R_s = 2 * 2 * B1 / (solve_ms * 1e-3)   # two solves, forward + backward sweep each
    t_vec = (iter_ms - fact_ms - solve_ms) * 1e-3
    rows = []
    for p in P:
        if p == 1:
            rows.append(dict(P=1, flops_top=0.0, flops_shard_max=F1, lbytes_top=0.0, lbytes_shard_max=B1,
                             xch_fact_bytes=0, xch_solve_bytes=0, xch_gather_bytes=0, t_comm_ms=0.0,
                             t_iter_ms=iter_ms, speedup=1.0))
            continue
        S = Symbolic(K.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(), nshards=p, shard=0)
        si, info = S.shard_info(), S.info()
        first, _, nrows = S.supernodes()
        fl, lb = front_costs(first, nrows)
        own = si["owner"]
        top = own < 0
        Ftop, Btop = fl[top].sum(), lb[top].sum()
        Fsh = [fl[own == k].sum() for k in range(p)]
        Bsh = [lb[own == k].sum() for k in range(p)]
        # every shard's analysis lists its own subtrees; shard 0's plan holds the partition (owner) of
        # all fronts, so the per-shard sums come from the one owner array
        xf, xs, xg = 8 * info["xch_fact"], 8 * info["xch_solve"], 8 * info["xch_gather"]
        f = (p - 1) / p
        ar = lambda n: 2 * f * n / bw + 2 * (p - 1) * alpha  # noqa: E731
        ag = lambda n: f * n / bw + (p - 1) * alpha  # noqa: E731
        t_comm = ar(xf) + 2 * (ar(xs) + ag(xg))
        t = (max(Fsh) + Ftop) / R_f + 2 * 2 * (max(Bsh) + Btop) / R_s + t_comm + t_vec
        rows.append(dict(P=p, top_fronts=int(top.sum()), top_cost=si["top_cost"], shard_cost_max=si["shard_cost_max"],
                         shard_cost_sum=si["shard_cost_sum"], flops_top=Ftop, flops_shard_max=max(Fsh),
                         flops_shard_min=min(Fsh), lbytes_top=Btop, lbytes_shard_max=max(Bsh),
                         xch_fact_bytes=xf, xch_solve_bytes=xs, xch_gather_bytes=xg, t_comm_ms=t_comm * 1e3,
                         t_iter_ms=t * 1e3, speedup=iter_ms / (t * 1e3)))
    return dict(config=config, nnzL=int(S1.info()["nnzL"]), flops=F1, lbytes=B1, R_f_tflops=R_f / 1e12,
                R_s_gbs=R_s / 1e9, t_vec_ms=t_vec * 1e3, link_gbs=bw / 1e9, alpha_us=alpha * 1e6, rows=rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--fact-ms", type=float, required=True)
    ap.add_argument("--solve-ms", type=float, required=True)
    ap.add_argument("--iter-ms", type=float, required=True)
    ap.add_argument("--P", default="1,2,4,8")
    a = ap.parse_args()
    out = model(a.config, [int(x) for x in a.P.split(",")], a.fact_ms, a.solve_ms, a.iter_ms)
    print(json.dumps(out, indent=1))
    print(f"\n{a.config}: flops {out['flops']:.3e}, L {out['lbytes'] / 1e9:.2f} GB; calibration R_f "
          f"{out['R_f_tflops']:.2f} TF/s, R_s {out['R_s_gbs']:.0f} GB/s, vector phase {out['t_vec_ms']:.2f} ms")
    print("| P | top fronts | top GFLOP | largest shard GFLOP | smallest | top L MB | largest shard L MB | "
          "all-reduce / fact MB | all-reduce + all-gather / solve MB | t_comm ms | modelled ms/iter | speed-up |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for r in out["rows"]:
        print(f"| {r['P']} | {r.get('top_fronts', 0)} | {r['flops_top'] / 1e9:.1f} | {r['flops_shard_max'] / 1e9:.1f} | "
              f"{r.get('flops_shard_min', r['flops_shard_max']) / 1e9:.1f} | {r['lbytes_top'] / 1e6:.0f} | "
              f"{r['lbytes_shard_max'] / 1e6:.0f} | {r['xch_fact_bytes'] / 1e6:.1f} | "
              f"{(r['xch_solve_bytes'] + r['xch_gather_bytes']) / 1e6:.2f} | {r['t_comm_ms']:.2f} | "
              f"{r['t_iter_ms']:.2f} | {r['speedup']:.2f} |")


if __name__ == "__main__":
    main()
