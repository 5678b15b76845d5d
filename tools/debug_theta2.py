"""Debug: the configs[2] sigma = e^18.5 theta - GPU slot state vs the oracle's fp64 statement."""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'auxiliary-pm-mcmc_amd'), os.path.join(REPO, 'oracle')]
import apm_oracle as orc
from gpdemo import _native as nat
from gpdemo.utils import synthetic_gp_data
z = np.load(os.path.join(REPO, 'tests', 'golden', 'config2_ref.npz'))
b = int(sys.argv[1]) if len(sys.argv) > 1 else 2
X, y = synthetic_gp_data(4096, 32, 20151009)
rng = np.random.RandomState(5)
U1, U2 = rng.normal(size=(4096, 256)), rng.normal(size=(4096, 256))
th = z['thetas'][b]
Ls = []
for env in ({}, {'APM_WIDE_Q': '1e30'}, {'APM_WIDE_Q': '0'}):
    for k, v in env.items():
        os.environ[k] = v
    ctx = nat.Context(X, y, nat.KERNEL_ARD, 1e-8, 256, max_batch=1, n_slots=1, n_ubufs=2)
    for k in env:
        del os.environ[k]
    ctx.u_upload(0, U1)
    ctx.u_upload(1, U2)
    out, st, nops = ctx.theta_eval(nat.EST_IS, th[None], [0], [0])
    out2, _ = ctx.u_eval([0], [1])
    L, f, g, cst = ctx.slot_read(0)
    ctx.close()
    Ls.append(L)
    print(env, 'gpu', out[0] - z['logf1'][b], out2[0] - z['logf2'][b], nops[0], 'cst', cst,
          'max|f-fref|/max', np.abs(f - z['f_post'][b]).max() / np.abs(z['f_post'][b]).max(),
          flush=True)
K = np.empty((4096, 4096))
orc.make_kernel_func('ard', 1e-8)(K, X, th)
t0 = time.time()
s = orc.theta_state_pushthrough(K, y)
zz = s['a'] + s['W'] * s['f_post']
print('oracle cst', 0.5 * s['f_post'].dot(zz) - 0.5 * s['logdet_B'], 'logdetB', s['logdet_B'],
      '1/2 fz', 0.5 * s['f_post'].dot(zz), time.time() - t0, flush=True)
# the oracle consistent form with the GPU's fp32 factor and f_post
st2 = dict(s, f_post=f)
print('oracle consistent, GPU f_post, fp64 L', orc.is_estimate_consistent(y, st2, U1) - z['logf1'][b])
print('oracle consistent, GPU L32', orc.is_estimate_consistent(y, s, U1, L) - z['logf1'][b])
print('trace C', (s['C_chol'] ** 2).sum(), 'trace L32', (L ** 2).sum())
C = s['C_chol']
print('max|L_gpu - C_orc| / max|C|', np.abs(Ls[0] - C).max() / np.abs(C).max(),
      'row-rel max', (np.abs(Ls[0] - C).max(1) / np.abs(C).max(1)).max())
print('max|logdiag diff|', np.abs(np.log(np.diagonal(Ls[0])) - np.log(np.diagonal(C))).max())
