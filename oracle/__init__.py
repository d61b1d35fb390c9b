"""ORACLE — test infrastructure, NOT product code.

CPU restatement (numpy/scipy) of the reference MadIPM v0.1.2 Mehrotra predictor-corrector path
(`/root/reference/src/*.jl`) plus the MadNLP 0.8 semantics it delegates to (SURVEY.md Appendix B,
tagged [EXT] below: recalled, not verifiable offline).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker / timed CPU baseline — never as part of the product path.
The product (`madipm.jl_amd/`) must never import it.

Parity pinning: the reference is Julia and cannot run here (no `julia`
in the image).  The oracle is pinned by the analytic answer of the reference's own `simple_lp`
test (objective 1, `test/runtests.jl:29-60,159-164`), by the netlib AFIRO optimum
(-464.75314286, the instance of BASELINE.json configs[0]), and by HiGHS 1.8 (bundled with scipy)
objectives on seeded LPs/QPs.  Per-iteration traces are therefore "parity unpinned" against the
reference itself.
"""
