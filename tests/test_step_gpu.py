"""GPU tests of the step-length rules (update_step!, src/kernels.jl:291-358) through the C-ABI
`madipm_update_step`, which runs the MPC loop's own step-test kernels (k_alpha + k_final, and k_mu +
k_final for MehrotraAdaptiveStep), against the oracle's restatement (oracle/mpc.py step_on_vectors).

The reference's max-ratio test is `mapreduce(f, (e1, e2) -> e1[1] < e2[1] ? e1 : e2, ...; init =
(1.0, 0))` (kernels.jl:226-272), a left fold: among EXACTLY equal ratios the LAST index wins, and an
element whose ratio is exactly 1.0 replaces the init element.  Only MehrotraAdaptiveStep reads the
index (kernels.jl:335-352), so the tied entries below carry different multipliers: the first-index
rule would give a different step, which the test checks too (it discriminates).
Tolerance: indices exact; alphas 1e-12 relative (the Mehrotra mu_full sum is reduced in a different
order on the GPU).
"""
import numpy as np
import pytest

from oracle.mpc import step_on_vectors

pytestmark = pytest.mark.gpu


def _vectors(seed, nlb=3000, nub=2500, tie_l=(5, 700, 2999), tie_lz=(11, 1500, 2998), tie_u=(17, 300, 2400),
             tie_uz=(40, 1000, 2499), ratio=0.5, lo=0.8):
    """Random interior point + direction whose smallest ratios are EXACT ties (the tied entries have
    bit-identical operands, so every tau gives identical quotients) at the given indices:
    primal ties (tie_l / tie_u) carry distinct multipliers, dual ties (tie_lz / tie_uz) distinct
    primal values — the quantities MehrotraAdaptiveStep reads at the chosen index.  The other entries'
    ratios are >= lo (primal) and >= 1.25 (dual)."""
    rng = np.random.default_rng(seed)
    xl = rng.uniform(-1, 1, nlb)
    x_l = xl + rng.uniform(lo, lo + 1.2, nlb)
    dx_l = rng.uniform(-1.0, 1.0, nlb)
    zl = rng.uniform(0.5, 2.0, nlb)
    dzl = rng.uniform(-1.0, 1.0, nlb) * 0.4
    xu = rng.uniform(-1, 1, nub)
    x_u = xu - rng.uniform(lo, lo + 1.2, nub)
    dx_u = rng.uniform(-1.0, 1.0, nub)
    zu = rng.uniform(0.5, 2.0, nub)
    dzu = -rng.uniform(0.0, 1.0, nub) * 0.4          # zu + dzu > 0: no upper dual candidate
    for k, i in enumerate(tie_l):
        xl[i], x_l[i], dx_l[i] = 0.0, ratio, -1.0     # (-x + xl) tau / dx = ratio tau
        zl[i] = 1.0 + 0.25 * k
    for i in tie_lz:
        zl[i], dzl[i] = 1.0, -2.0                     # -zl tau / dzl = tau / 2
    for k, i in enumerate(tie_u):
        xu[i], x_u[i], dx_u[i] = 0.0, -ratio, 1.0
        zu[i] = 1.5 + 0.25 * k
    for i in tie_uz:
        zu[i], dzu[i] = 1.0, -2.0                     # zu + dzu < 0 holds
    return [x_l, xl, zl, dx_l, dzl, x_u, xu, zu, dx_u, dzu]


def _gpu(rule, tau, mu, vecs):
    import torch
    from madipm_amd.rocm_wrapper import update_step
    dv = [torch.tensor(v, dtype=torch.float64, device="cuda") for v in vecs]
    return update_step(rule, tau, mu, *dv)


def _close(a, b, rtol=1e-12):
    return abs(a - b) <= rtol * max(1.0, abs(b))


@pytest.mark.parametrize("seed", [0, 1])
@pytest.mark.parametrize("rule,tau,mu", [("conservative", 0.995, 0.0), ("adaptive", 0.99, 1e-3),
                                         ("mehrotra", 0.99, 0.0)])
def test_step_rule_ties_match_oracle(seed, rule, tau, mu):
    vecs = _vectors(seed)
    got = _gpu(rule, tau, mu, vecs)
    ref = step_on_vectors((rule, tau), mu, *vecs)
    for k in ("i_xl", "i_xu", "i_zl", "i_zu"):
        assert got[k] == ref[k], (k, got[k], ref[k])
    # the left fold keeps the LAST of the tied indices
    assert (ref["i_xl"], ref["i_xu"], ref["i_zl"], ref["i_zu"]) == (2999, 2400, 2998, 2499)
    for k in ("alpha_p", "alpha_d", "alpha_xl", "alpha_xu", "alpha_zl", "alpha_zu"):
        assert _close(got[k], ref[k]), (k, got[k], ref[k])


def test_mehrotra_tie_choice_changes_the_step():
    """The tie-break is observable: with the first tied index instead, MehrotraAdaptiveStep's alpha_p
    and alpha_d differ from the reference's (and from the GPU's)."""
    vecs = _vectors(3)
    got = _gpu("mehrotra", 0.99, 0.0, vecs)
    ref = step_on_vectors(("mehrotra", 0.99), 0.0, *vecs)
    assert _close(got["alpha_p"], ref["alpha_p"]) and _close(got["alpha_d"], ref["alpha_d"])
    # first-index variant: move the first tie's entry to the end (then it is the last one)
    first = _vectors(3, tie_l=(5,), tie_lz=(11,), tie_u=(17,), tie_uz=(40,))
    alt = step_on_vectors(("mehrotra", 0.99), 0.0, *first)
    assert not _close(alt["alpha_p"], ref["alpha_p"], 1e-9) or not _close(alt["alpha_d"], ref["alpha_d"], 1e-9)


def test_ratio_exactly_one_replaces_init():
    """A ratio of exactly 1.0 is not strictly larger than init (1.0, 0): the element's index is kept;
    ratios above 1 keep the init element (index -1, alpha 1)."""
    vecs = _vectors(4, ratio=1.0, lo=1.5)
    got = _gpu("conservative", 1.0, 0.0, vecs)
    ref = step_on_vectors(("conservative", 1.0), 0.0, *vecs)
    assert got["alpha_xl"] == ref["alpha_xl"] == 1.0
    assert got["i_xl"] == ref["i_xl"] == 2999
    # no candidate at all below or at 1: the init element
    vecs = _vectors(5, ratio=2.0, lo=1.5)
    got = _gpu("conservative", 1.0, 0.0, vecs)
    ref = step_on_vectors(("conservative", 1.0), 0.0, *vecs)
    assert (got["i_xl"], got["alpha_xl"]) == (ref["i_xl"], ref["alpha_xl"]) == (-1, 1.0)


def test_empty_sides():
    """nub = 0 (only lower bounds) and nlb = 0: the empty side is the init element."""
    v = _vectors(6)
    for keep in ("lb", "ub"):
        vecs = [a if (k < 5) == (keep == "lb") else a[:0] for k, a in enumerate(v)]
        got = _gpu("mehrotra", 0.99, 0.0, vecs)
        ref = step_on_vectors(("mehrotra", 0.99), 0.0, *vecs)
        for k in ("i_xl", "i_xu", "i_zl", "i_zu"):
            assert got[k] == ref[k]
        assert _close(got["alpha_p"], ref["alpha_p"]) and _close(got["alpha_d"], ref["alpha_d"])
