"""The reference's own K at the two InvalidCovarianceMatrixError thetas of errors.npz (icm_a,
icm_b: iso N=60 D=3), from the reference's kernels.pyx compiled by `make -C oracle ref` into
oracle/_ref/ (build container only). Nothing from the reference is copied: inputs + the
reference's outputs only.

    python tests/golden/make_golden_icm.py
"""
import glob
import importlib.util
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

_so = glob.glob(os.path.join(REPO, 'oracle', '_ref', 'kernels*.so'))
if not _so:
    raise SystemExit('build the reference Gram first: make -C oracle ref')
_spec = importlib.util.spec_from_file_location('gpdemo.kernels', _so[0])
ref_krn = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(ref_krn)

e = np.load(os.path.join(HERE, 'errors.npz'))
out = {}
for name in ('icm_a', 'icm_b'):
    K = np.empty((e['extreme_X'].shape[0],) * 2)
    ref_krn.isotropic_squared_exponential_kernel(K, e['extreme_X'], e[name + '_theta'], 1e-8)
    out[name + '_K'] = K
np.savez_compressed(os.path.join(HERE, 'icm_k.npz'), **out)
print({k: v.shape for k, v in out.items()})
