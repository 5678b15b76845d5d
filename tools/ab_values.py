"""Values of one library build for a bitwise A/B against another (development tool): the 64-chain
stationary theta-call + cached u-call at N=4096 (and a ragged N=1100 case), the outputs and
slot factors saved to an npz; `--compare a.npz b.npz` prints the largest differences.

    APM_LIB=path/to/libapm.so python tools/ab_values.py out.npz
    python tools/ab_values.py --compare a.npz b.npz
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))


def run(path):
    from gpdemo import _native
    from gpdemo import utils
    out = {}
    X, y = utils.synthetic_gp_data(4096, 32, 20151009)
    th = np.load(os.path.join(REPO, 'tests', 'golden', 'stationary_thetas.npy')).astype(np.float64)
    cases = [('stat', X, y, th, 256, 64)]
    X2, y2 = utils.synthetic_gp_data(1100, 5, 4242, 'ard')
    rng = np.random.RandomState(7)
    th2 = np.array([np.r_[t0, rng.normal(scale=0.3, size=5) + 0.5 * np.log(5)]
                    for t0 in (0.0, 2.0, 4.0)])
    cases.append(('n1100', X2, y2, th2, 32, 3))
    for name, Xc, yc, thc, s, B in cases:
        ctx = _native.Context(Xc, yc, _native.KERNEL_ARD, 1e-8, s, max_batch=B, n_slots=B,
                              n_ubufs=B)
        idx = np.arange(B)
        ctx.u_normal(idx, np.full(B, 7), idx)
        v1, st, nops = ctx.theta_eval(_native.EST_IS, thc, idx, idx)
        v2, st2 = ctx.u_eval(idx, idx)
        out[name + '_v1'], out[name + '_v2'], out[name + '_st'] = v1, v2, st
        for b in range(min(B, 4)):
            L, f, g, c = ctx.slot_read(b)
            out['{0}_L{1}'.format(name, b)] = L.astype(np.float32)
            out['{0}_f{1}'.format(name, b)] = f
        ctx.close()
    np.savez(path, **out)


def compare(a, b):
    za, zb = np.load(a), np.load(b)
    same = True
    for k in za.files:
        d = np.abs(za[k].astype(np.float64) - zb[k].astype(np.float64)).max()
        same &= d == 0
        print('{0:12s} max |a - b| = {1:.3e}'.format(k, d))
    print('bitwise identical' if same else 'DIFFERENT')


if __name__ == '__main__':
    if sys.argv[1] == '--compare':
        compare(sys.argv[2], sys.argv[3])
    else:
        run(sys.argv[1])
