"""The assembly's LDS source path (csrc/ldl.hip asm_chunks_lds, `transfer!` / extend-add semantics of
/root/reference/ext/MadIPMCUDAExt/cuda_wrapper.jl:4-24 on the frontal tiles): a tile of <= n windows
of 5120 sources gathers them into LDS window by window and sums each entry there in 8-source chunks,
an entry that straddles a window boundary carrying its running chunk sum to the next.  It must give
the chunk pass's sums (k_asm_chunks + per-entry chunk order) BIT FOR BIT.

By default only launches of >= 256 tiles and k_asm_update tiles use more than one window, so the
small test problems never straddle; MADIPM_ASM_LDS_WIN=n (tests) puts every tile of <= n windows on
the path whatever its launch size.  Each case is factorised and solved with the chunk pass only
(MADIPM_ASM_LDS_SRC=0) and with n = 1, 2, 4, 12 windows: pivots and solution bitwise equal, and the
oracle's pivots to 1e-12 (well conditioned).  MADIPM_ASM_STATS reports how many tiles took the path,
how many needed several windows and how many entries straddled (asserted > 0 where the case has them).

The device guard: a tile whose source count exceeds FrontTab::asm_src_cap (kAsmLdsWinMax windows)
sets the sticky kErrAsmSrc and factorize() raises — MADIPM_DEBUG_ASM_SRC_CAP shrinks the cap."""
import re

import numpy as np
import pytest

from helpers import block_angular_k2, dense_k2, lp_k2
from oracle.ldl import OracleLDL

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _case(name):
    if name == "dense_100_800":  # the round-5 failure's case (test_batched_leaf_columns_parity[100-800-0-128])
        K, Lw = dense_k2(100, 800, 3)
        return K, Lw, dict(ordering=0, small_front_max=128)
    if name == "dense_150_1000_sfm192":
        K, Lw = dense_k2(150, 1000, 3)
        return K, Lw, dict(ordering=0, small_front_max=192)
    if name == "block":
        K, Lw = block_angular_k2(3000, 4000, 20, 7, well=True)
        return K, Lw, {}
    from madipm_amd import standard_form_qp
    from madipm_amd import instances as I
    if name == "neos_0.1":  # big fronts: k_assemble, k_asm_update and big-child records
        K, Lw = lp_k2(standard_form_qp(I.neos5052403_standin(scale=0.1)), 2, well=True)
        return K, Lw, {}
    if name == "supportcase10_0.05":
        K, Lw = lp_k2(standard_form_qp(I.supportcase10_standin(scale=0.05, block_scale=1.0)), 3, well=True)
        return K, Lw, {}
    raise KeyError(name)


def _run(K, Lw, kw, env, monkeypatch, capfd):
    from madipm_amd.linear_solver import HIPLDLSolver
    for k in ("MADIPM_ASM_LDS_SRC", "MADIPM_ASM_LDS_WIN"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("MADIPM_ASM_STATS", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    capfd.readouterr()
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices, **kw)
    err = capfd.readouterr().err
    m = re.search(r"asm lds-src: tiles (\d+) \(multi-window (\d+), straddling entries (\d+), max sources (\d+)\)"
                  r"\s+chunk-path tiles (\d+)", err)
    stats = tuple(int(x) for x in m.groups()) if m else None
    dev = torch.device("cuda:0")
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).to(dev)) == 0
    b = np.random.default_rng(1).standard_normal(K.shape[0])
    x = torch.from_numpy(b.copy()).to(dev)
    ls.solve(x)
    torch.cuda.synchronize()
    return ls.diag().copy(), x.cpu().numpy(), ls, stats


@pytest.mark.parametrize("name", ["dense_100_800", "dense_150_1000_sfm192", "block", "neos_0.1", "supportcase10_0.05"])
def test_asm_lds_windows_bitwise(name, monkeypatch, capfd):
    K, Lw, kw = _case(name)
    d0, x0, ls0, st0 = _run(K, Lw, kw, {"MADIPM_ASM_LDS_SRC": "0"}, monkeypatch, capfd)
    assert st0 is not None and st0[0] == 0, st0  # the reference run: chunk pass only
    ref = OracleLDL(K, ls0.perm())
    assert ref.factorize() == K.shape[0]
    dr = ref.diag()
    assert np.all(np.abs(d0 - dr) <= 1e-12 * np.abs(dr)), "chunk pass vs oracle"
    seen = {}
    for win in ("1", "2", "4", "12"):
        d1, x1, _, st = _run(K, Lw, kw, {"MADIPM_ASM_LDS_WIN": win}, monkeypatch, capfd)
        seen[win] = st
        bad = np.flatnonzero(d0.view(np.uint64) != d1.view(np.uint64))
        assert bad.size == 0, (f"{name} WIN={win} {st}: {bad.size} pivots differ from the chunk pass, first "
                               f"k={bad[0]} lds={d1[bad[0]]:.17e} chunk={d0[bad[0]]:.17e}")
        assert np.array_equal(x0.view(np.uint64), x1.view(np.uint64)), f"{name} WIN={win}: solution differs"
    print(name, seen)
    assert seen["1"][1] == 0  # one window: no tile needs more
    assert seen["12"][0] >= seen["1"][0]
    if name in ("dense_100_800", "block", "neos_0.1", "supportcase10_0.05"):
        # high fan-in tiles: several windows and straddling entries (neos: a >= 256-tile launch)
        assert seen["12"][1] >= 1 and seen["12"][2] >= 1, seen
    if name == "neos_0.1":
        assert seen["12"][1] >= 256 and seen["12"][2] >= 1000, seen


def test_asm_src_cap_guard(monkeypatch):
    """A tile on the LDS source path with more sources than the device cap must raise, not sum silently."""
    from madipm_amd.linear_solver import HIPLDLSolver
    K, Lw, kw = _case("dense_100_800")
    monkeypatch.setenv("MADIPM_ASM_LDS_WIN", "4")
    monkeypatch.setenv("MADIPM_DEBUG_ASM_SRC_CAP", "8")
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices, **kw)
    with pytest.raises(Exception, match="source count"):
        ls.factorize(torch.from_numpy(Lw.data.copy()).cuda())
    monkeypatch.delenv("MADIPM_DEBUG_ASM_SRC_CAP")
    ls = HIPLDLSolver(K.shape[0], Lw.indptr, Lw.indices, **kw)  # a fresh solver factorises normally
    assert ls.factorize(torch.from_numpy(Lw.data.copy()).cuda()) == 0
