"""Subtree sharding (SURVEY §8 e), host side: the partition of the front tree computed by the
symbolic analysis (csrc/symbolic.cpp step 8b).  No GPU needed.

Properties: every front is either top (-1) or owned by one shard; the top is closed under parents
(ancestors of a top front are top); a subtree never straddles shards; every shard computes the same
cut; the cut balances the shards on block-angular KKT systems (the structure the north star shards).
"""
import numpy as np
import pytest

from madipm_amd._lib import Symbolic, default_ldl_opts
from tests.helpers import block_angular_k2, dense_k2, random_k2


def _owners(Lw, P, shard=0):
    S = Symbolic(Lw.shape[0], Lw.indptr, Lw.indices, default_ldl_opts(), nshards=P, shard=shard)
    first, parent, _ = S.supernodes()
    return S.shard_info(), parent


@pytest.mark.parametrize("P", [2, 3, 4, 8])
@pytest.mark.parametrize("kind", ["block", "random"])
def test_partition_is_a_valid_subtree_cut(P, kind):
    _, Lw = block_angular_k2(1200, 2400, 24, 3) if kind == "block" else random_k2(300, 600, 0.01, 4)
    info, parent = _owners(Lw, P)
    own = info["owner"]
    assert own.min() >= -1 and own.max() < P
    for s, p in enumerate(parent):
        if p < 0:
            continue
        if own[s] == -1:
            assert own[p] == -1, "a top front's parent must be top"
        elif own[p] != -1:
            assert own[p] == own[s], "a subtree may not straddle shards"
    # identical on every shard
    for r in range(1, P):
        o2, _ = _owners(Lw, P, r)
        assert np.array_equal(o2["owner"], own)


@pytest.mark.parametrize("P", [2, 4, 8])
def test_partition_balances_block_angular(P):
    _, Lw = block_angular_k2(2400, 4800, 48, 5)
    info, _ = _owners(Lw, P)
    avg = info["shard_cost_sum"] / P
    assert info["shard_cost_max"] <= 1.5 * avg
    assert (info["owner"] >= 0).any() and (info["owner"] == -1).any()
    assert set(np.unique(info["owner"][info["owner"] >= 0])) == set(range(P))


def test_unsharded_plan_has_no_top():
    _, Lw = block_angular_k2(600, 1200, 12, 1)
    S = Symbolic(Lw.shape[0], Lw.indptr, Lw.indices, default_ldl_opts())
    assert (S.shard_info()["owner"] == 0).all()


@pytest.mark.parametrize("P", [2, 3, 4])
def test_batched_leaves_dealt_to_shards(P):
    """Dense-column K2: the batched-leaf group under the (top) y front keeps, on each shard, exactly
    that shard's members — every x_j on one shard, balanced within one — and the exchange sizes of
    the sharded plan are shard-independent."""
    K, Lw = dense_k2(150, 1000, 3)
    N = K.shape[0]
    S1 = Symbolic(N, Lw.indptr, Lw.indices, default_ldl_opts(ordering=0))
    assert S1.info()["lb_groups"] == 1 and S1.info()["lb_members"] == 1000
    mem = []
    for r in range(P):
        S = Symbolic(N, Lw.indptr, Lw.indices, default_ldl_opts(ordering=0), nshards=P, shard=r)
        inf, own = S.info(), S.shard_info()["owner"]
        assert inf["lb_groups"] == 1
        mem.append(inf["lb_members"])
        assert (own == -1).sum() >= 1  # the y front is on top
    assert sum(mem) == 1000 and max(mem) - min(mem) <= 1
