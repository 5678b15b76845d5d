import sys, os, numpy as np
sys.path.insert(0, 'auxiliary-pm-mcmc_amd'); sys.path.insert(0, 'oracle')
from gpdemo import _native as nat
import apm_oracle as orc
rng = np.random.RandomState(11)
for n, d, kind in ((200, 3, 'ard'), (150, 40, 'ard'), (130, 6, 'iso'), (300, 32, 'ard')):
    X = rng.normal(size=(n, d)); th = np.r_[0.2, rng.normal(scale=0.5, size=d if kind == 'ard' else 1)]
    Kr = np.empty((n, n)); orc.c_gram(kind, Kr, X, th, 1e-8)
    for mf in ('1', '0'):
        os.environ['APM_GRAM_MFMA'] = mf
        K = np.empty((n, n)); nat.gram(nat.KERNEL_ISO if kind == 'iso' else nat.KERNEL_ARD, K, X, th, 1e-8)
        asym = np.abs(K - K.T); i, j = np.unravel_index(asym.argmax(), asym.shape)
        print(n, d, kind, 'mfma', mf, 'max asym %.3g at (%d,%d) tile (%d,%d)' % (asym.max(), i, j, i // 64, j // 64),
              'n asym', (asym > 0).sum(), 'max rel err vs C %.3g' % (np.abs(K - Kr) / np.abs(Kr)).max())
