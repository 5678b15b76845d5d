"""Child process of tests/test_gpu_knobs.py (not a test module): one batched IS theta-call and
one cached u-call under the environment it is started with (the knobs read once per process:
APM_DF_SPLIT, APM_UGEMM_W2_MIN); prints a digest of every output's bytes."""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..',
                                'auxiliary-pm-mcmc_amd'))
from gpdemo import _native as nat  # noqa: E402
from gpdemo.utils import synthetic_gp_data  # noqa: E402

n, d, S, B = int(sys.argv[1]), 8, 128, 4
X, y = synthetic_gp_data(n, d, 3)
rng = np.random.RandomState(7)
th = np.tile(np.r_[0.0, np.full(d, np.log(np.sqrt(d)))], (B, 1))
th += rng.normal(scale=0.2, size=th.shape)
th[-1, 0] = 45.0  # extreme theta: fp32 operands, possibly an fp64 rerun
ctx = nat.Context(X, y, nat.KERNEL_ARD, 1e-8, S, max_batch=B, n_slots=B, n_ubufs=2)
try:
    ctx.u_upload(0, rng.normal(size=(n, S)))
    ctx.u_upload(1, rng.normal(size=(n, S)))
    o1, st1, nops = ctx.theta_eval(nat.EST_IS, th, [0] * B, list(range(B)))
    o2, st2 = ctx.u_eval(list(range(B)), [1] * B)
    h = hashlib.sha256()
    for a in (o1, st1, nops, o2, st2):
        h.update(np.ascontiguousarray(a).tobytes())
    for b in range(B):
        if st1[b] == 0:
            L, f = ctx.slot_read(b)[:2]
            h.update(np.ascontiguousarray(f).tobytes())
            h.update(np.ascontiguousarray(L).tobytes())
    print('digest', h.hexdigest(), 'status', [int(v) for v in st1], 'nops', [int(v) for v in nops])
finally:
    ctx.close()
