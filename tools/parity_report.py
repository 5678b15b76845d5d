"""Print the GPU-vs-reference differences of the estimator values (development tool)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'auxiliary-pm-mcmc_amd'), os.path.join(REPO, 'oracle'),
                os.path.join(REPO, 'tests')]
import apm_oracle as orc  # noqa: E402
from conftest import golden  # noqa: E402
from gpdemo import _native, utils  # noqa: E402

g = golden('estimators')
print('mode', os.environ.get('APM_POSTCOV', 'lk'))
for ci in range(int(g['n_cases'])):
    c = {k[3:]: g[k] for k in g.files if k.startswith('c%d_' % ci)}
    kind = _native.KERNEL_ISO if str(c['kind']) == 'iso' else _native.KERNEL_ARD
    ctx = _native.Context(c['X'], c['y'], kind, 1e-8, c['ns1'].shape[1], n_slots=2, n_ubufs=2)
    ctx.u_upload(0, c['ns1'])
    ctx.u_upload(1, c['ns2'])
    o1, _, _ = ctx.theta_eval(_native.EST_IS, c['theta'][None], [0], [0])
    o2, _ = ctx.u_eval([0], [1])
    L, f, gg, cst = ctx.slot_read(0)
    print('golden case %d: theta-call %+.2e  u-call %+.2e  |dC_chol|max %.2e  |df|max %.2e' % (
        ci, o1[0] - float(c['is_logf1']), o2[0] - float(c['is_logf2']),
        np.abs(L - np.tril(c['C_chol'])).max(), np.abs(f - c['f_post']).max()))
    ctx.close()
for n, d, s, kind in ((700, 5, 32, 'ard'), (1100, 3, 8, 'iso'), (2048, 16, 64, 'ard')):
    X, y = utils.synthetic_gp_data(n, d, 99 + n, kind)
    rng = np.random.RandomState(n)
    P = d + 1 if kind == 'ard' else 2
    for th in (np.r_[0.4, rng.normal(scale=0.3, size=P - 1) + 0.5 * np.log(d)],
               np.r_[1.5, np.full(P - 1, 0.5 * np.log(d) + 1.0)]):
        ns = rng.normal(size=(n, s))
        kf = orc.make_kernel_func(kind, 1e-8)
        r1, rc, _ = orc.is_estimate(X, y, kf, ns, th)
        ctx = _native.Context(X, y, _native.KERNEL_ARD if kind == 'ard' else _native.KERNEL_ISO,
                              1e-8, s, n_slots=1, n_ubufs=1)
        ctx.u_upload(0, ns)
        o, st, _ = ctx.theta_eval(_native.EST_IS, th[None], [0], [0])
        L, f, _, _ = ctx.slot_read(0)
        print('oracle n=%d %s theta0=%.2f: %+.2e (ref %.4f) status %d |dC_chol|max %.2e' % (
            n, kind, th[0], o[0] - r1, r1, st[0], np.abs(L - rc[1]).max()))
        ctx.close()
