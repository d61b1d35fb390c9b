import sys, os; sys.path.insert(0,'madipm.jl_amd'); sys.path.insert(0,'.')
from madipm_amd import read_mps, MPCSolver, FixedRegularization
from oracle.mpc import OracleMPC, OracleOptions
qp = read_mps('tests/golden/afiro.mps')
g = MPCSolver(qp, regularization=FixedRegularization(1e-8,-1e-8)).solve()
r = OracleMPC(qp, OracleOptions(regularization=("fixed",1e-8,-1e-8))).solve()
for a,b in zip(g.trace, r.trace):
    print(a['k'], "%.15e %.15e | %.6e %.6e | %.6e %.6e | %.8e %.8e | %.10f %.10f | %.10f %.10f" % (a['obj'], b['obj'], a['inf_pr'], b['inf_pr'], a['inf_du'], b['inf_du'], a['mu'], b['mu'], a['alpha_p'], b['alpha_p'], a['alpha_d'], b['alpha_d']))
