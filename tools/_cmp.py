import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'auxiliary-pm-mcmc_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'tests'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'oracle'))
from gpdemo import _native as nat
from test_gpu_kernels import _mixed_case

class MP:
    def setenv(self, k, v): os.environ[k] = v
    def delenv(self, k): os.environ.pop(k, None)

def run(**env):
    X, y, thetas, ns = _mixed_case()
    for k, v in env.items(): os.environ[k] = str(v)
    B = len(thetas)
    ctx = nat.Context(X, y, nat.KERNEL_ARD, 1e-8, ns.shape[1], max_batch=B, n_slots=B, n_ubufs=1)
    for k in env: os.environ.pop(k)
    ctx.u_upload(0, ns)
    out, st, nops = ctx.theta_eval(nat.EST_IS, thetas, ubufs=[0] * B, slots=list(range(B)))
    fs = [ctx.slot_read(b)[1] for b in range(B)]
    ctx.close()
    return out, fs

ref_o, ref_f = run(APM_MIXED=0)
for name, env in [('default', {}), ('MW0', {'APM_TRSV_MW': 0}), ('H3=0', {'APM_H3': 0}),
                  ('H3P=0', {'APM_H3_PANEL': 0}), ('MW0,H3=0', {'APM_TRSV_MW': 0, 'APM_H3': 0}),
                  ('FUSED0', {'APM_TRSV_FUSED': 0}), ('default2', {})]:
    o, f = run(**env)
    print(name, ['%.2e' % (np.abs(f[b] - ref_f[b]).max() / np.abs(ref_f[b]).max()) for b in range(3)],
          ['%.2e' % abs(o[b] - ref_o[b]) for b in range(3)])
