"""Critical-path breakdown of the Newton factor's dataflow panel (k_chol_panel_df32) from a
diagnostic build (-DDF_TRACE, tools/_oldlib/libapm_dftrace.so): wall-clock stamps (100 MHz) of
chain 0's first outer panel in the last factorisation of a 64-chain theta-call. Per column k:
the diagonal tile (update end -> factored -> published) and row k+1's hand-over (published ->
its TRSM wait returns -> TRSM stored -> next diagonal tile's update starts).

    APM_LIB=tools/_oldlib/libapm_dftrace.so python tools/df_trace.py
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'auxiliary-pm-mcmc_amd'))
from gpdemo import _native  # noqa: E402
from gpdemo import utils  # noqa: E402

n, d, s, B = 4096, 32, 256, 64
X, y = utils.synthetic_gp_data(n, d, 20151009)
ctx = _native.Context(X, y, _native.KERNEL_ARD, 1e-8, s, max_batch=B, n_slots=B, n_ubufs=B)
ctx.u_normal(np.arange(B), np.full(B, 7), np.arange(B))
th = np.tile(np.r_[0.0, np.full(d, np.log(np.sqrt(d)))], (B, 1))
th += np.random.RandomState(0).normal(scale=0.1, size=th.shape)
for _ in range(2):
    ctx.theta_eval(_native.EST_IS, th, np.arange(B), np.arange(B))
lib = ctx.lib
fn = lib.apm_debug_df_trace
fn.argtypes = [ctypes.c_void_p]
buf = np.zeros(64 * 16 * 8, dtype=np.uint64)
assert fn(buf.ctypes.data) == 0
T = buf.reshape(64, 16, 8).astype(np.int64)
t0 = T[T > 0].min()
us = lambda v: (v - t0) / 100.0  # noqa: E731  100 MHz -> us
print('col  diag: upd-end  factored  published | row k+1: trsm-wait-ret  trsm-done  next-upd-end')
for k in range(1, 8):
    dg = T[k, k]
    nx = T[k + 1, k] if k + 1 < 64 else None
    nn = T[k + 1, k + 1] if k + 1 < 8 else None
    print('{0:3d}  {1:8.1f} {2:9.1f} {3:10.1f} | {4:14.1f} {5:10.1f} {6:12.1f}'.format(
        k, us(dg[5]), us(dg[6]), us(dg[7]), us(nx[3]) if nx is not None else -1,
        us(nx[4]) if nx is not None else -1, us(nn[2]) if nn is not None else -1))
print('bulk row 40: ' + ' '.join('{0:.1f}/{1:.1f}'.format(us(T[40, c, 3]), us(T[40, c, 2]))
                                 for c in range(8)))
# bulk rows (below the diagonal block) of the same panel: when each row's walk starts, and per
# column step the update (start -> update end) and the TRSM (update end -> stored) times
rows = [r for r in range(8, 64) if T[r, 0, 0] > 0]
if rows:
    st = np.array([us(T[r, 0, 0]) for r in rows])
    print('bulk rows traced: {0}, walk start min/median/max {1:.1f} / {2:.1f} / {3:.1f} us'.format(
        len(rows), st.min(), np.median(st), st.max()))
    upd = np.array([[us(T[r, c, 2]) - us(T[r, c, 0]) for c in range(8)] for r in rows])
    # TRSM + store: update end -> the next column's step start (bulk rows stamp no event 4)
    trs = np.array([[us(T[r, c + 1, 0]) - us(T[r, c, 2]) for c in range(7)] for r in rows])
    wait = np.array([[us(T[r, c, 1]) - us(T[r, c, 0]) if T[r, c, 1] > 0 else 0.0
                      for c in range(8)] for r in rows])
    end = np.array([us(T[r, 7, 2]) for r in rows])
    print('per column (median over rows): wait-for-chain ' +
          ' '.join('%.1f' % v for v in np.median(wait, 0)))
    print('                              update (incl. wait) ' +
          ' '.join('%.1f' % v for v in np.median(upd, 0)))
    print('                              trsm ' + ' '.join('%.1f' % v for v in np.median(trs, 0)))
    print('last update end min/median/max {0:.1f} / {1:.1f} / {2:.1f} us'.format(
        end.min(), np.median(end), end.max()))
