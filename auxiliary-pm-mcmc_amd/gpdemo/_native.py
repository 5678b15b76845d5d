"""ctypes binding of libapm.so (include/apm.h) — the only way the Python layer reaches the GPU.

There is deliberately no CPU fallback: if the library is missing or no HIP device is visible,
every estimator / kernel entry point raises :class:`NativeUnavailableError`.
"""
import collections
import ctypes
import os
import threading

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get('APM_LIB', os.path.join(_PKG_ROOT, 'lib', 'libapm.so'))

# include/apm.h constants
KERNEL_ISO, KERNEL_ARD, KERNEL_PRECOMPUTED = 0, 1, 2
EST_IS, EST_PRIORMC, EST_LAPLACE = 0, 1, 2
APM_SUCCESS, APM_E_INVALID, APM_E_HIP, APM_E_NOMEM = 0, -1, -2, -3
STATUS_OK, STATUS_CHOL_K, STATUS_CHOL_B, STATUS_CHOL_C, STATUS_MAXITER = 0, 1, 2, 3, 4
STATUS_GUARD = 5
PROF_GRAM, PROF_CHOL_UPDATE, PROF_UGEMM, PROF_CHOL_UPDATE32, PROF_STATS = 0, 1, 2, 3, 4
PROF_CHOL_UPDATE32_OUTER, PROF_CHOL_UPDATE_OUTER, PROF_DF_TIMEOUTS = 5, 6, 7
PROF_POST32_OUTER, PROF_POST64_RERUNS, PROF_TRSV_TIMEOUTS = 8, 9, 10
PROF_ICM_CHECKS, PROF_GUARD, PROF_NKINDS = 11, 12, 13


class NativeUnavailableError(RuntimeError):
    """libapm.so or a HIP device is missing: the HIP path is mandatory (no CPU fallback)."""


class NativeError(RuntimeError):
    """A C-ABI call returned an APM_E_* code."""


_i64 = ctypes.c_int64
_p = ctypes.c_void_p
_d = ctypes.c_double
_i = ctypes.c_int

_SIGS = {
    'apm_version': (_i, []),
    'apm_device_count': (_i, []),
    'apm_global_error': (ctypes.c_char_p, []),
    'apm_create': (_p, [_i, _i, _p, _i64, _i64, _i64, _p, _d, _i64, _i64, _i64, _i64]),
    'apm_destroy': (None, [_p]),
    'apm_last_error': (ctypes.c_char_p, [_p]),
    'apm_padded_n': (_i64, [_p]),
    'apm_theta_len': (_i64, [_p]),
    'apm_set_newton': (_i, [_p, _d, _i64]),
    'apm_stream': (_p, [_p]),
    'apm_u_upload': (_i, [_p, _i64, _p, _i64]),
    'apm_u_download': (_i, [_p, _i64, _p, _i64]),
    'apm_u_normal': (_i, [_p, _i64, _p, _p, _p]),
    'apm_u_combine': (_i, [_p, _i64, _p, _p, _p, _p, _p]),
    'apm_theta_eval': (_i, [_p, _i, _i64, _p, _i64, _p, _p, _p, _p, _p]),
    'apm_theta_eval_K': (_i, [_p, _i, _p, _i64, _i64, _i64, _p, _p, _p]),
    'apm_u_eval': (_i, [_p, _i64, _p, _p, _p, _p]),
    'apm_slot_read': (_i, [_p, _i64, _p, _i64, _p, _p, _p]),
    'apm_cache_acquire': (_i, [_p, _p]),
    'apm_cache_copy': (_i, [_p, _i64]),
    'apm_cache_release': (_i, [_p, _i64]),
    'apm_cache_refcount': (_i64, [_p, _i64]),
    'apm_gram': (_i, [_i, _i, _p, _i64, _i64, _i64, _p, _i64, _d, _p, _i64]),
    'apm_laplace': (_i, [_i, _p, _i64, _i64, _p, _i, _i, _d, _i64, _p, _p, _i64, _p, _p, _p]),
    'apm_prof_enable': (_i, [_p, _i]),
    'apm_prof_marker': (_i, [_p, _i]),
    'apm_prof_read': (_i, [_p, _i, _p, _p, _p, _i]),
    'apm_guard_read': (_i, [_p, _i64, _p]),
    'apm_selftest_tile': (_i, [_i, _p, _p, _p]),
    'apm_selftest_philox': (_i, [_i, _i64, _p, _p]),
}

_lib = None
_lock = threading.Lock()


def exported_symbols():
    return sorted(_SIGS)


def load_library(check_device=True):
    """Load libapm.so (once). Raises NativeUnavailableError if absent or without a device."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeUnavailableError(
                    'libapm.so not found at {0}: build it with `python -c "import __graft_entry__'
                    ' as g; g.build()"` (no CPU fallback exists)'.format(LIB_PATH))
            lib = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    if check_device and _lib.apm_device_count() <= 0:
        raise NativeUnavailableError('no HIP device visible: the MI355X path is required '
                                     '(no CPU fallback exists)')
    return _lib


def _ptr(a):
    return a.ctypes.data if a is not None else None


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _check(rc, ctx=None):
    if rc != 0:
        lib = load_library(check_device=False)
        msg = (lib.apm_last_error(ctx) if ctx else lib.apm_global_error()) or b''
        raise NativeError('libapm error {0}: {1}'.format(rc, msg.decode(errors='replace')))


def default_device():
    return int(os.environ.get('APM_DEVICE', os.environ.get('LOCAL_RANK', '0')))


# ----------------------------------------------------------------------------- stand-alone calls


def gram(kind, K, X, theta, epsilon, device=None):
    """Fill K (any writable float64 (n, n) array) with the SE Gram matrix computed on the GPU."""
    lib = load_library()
    X = _f64(X)
    theta = _f64(np.atleast_1d(theta))
    n, d = X.shape
    need = 2 if kind == KERNEL_ISO else d + 1
    if theta.shape[0] < need:
        # kernels.pyx indexes theta[k+1] / theta[1] with bounds checking -> IndexError
        raise IndexError('Out of bounds on buffer access (axis 0)')
    out = K if (isinstance(K, np.ndarray) and K.dtype == np.float64 and K.flags.c_contiguous
                and K.flags.writeable) else np.empty((n, n))
    _check(lib.apm_gram(default_device() if device is None else device, kind, _ptr(X), n, d, d,
                        _ptr(theta), theta.shape[0], float(epsilon), out.ctypes.data, n))
    if out is not K:
        K[...] = out
    return None


def laplace(K, y, calc_cov, calc_lml, diff_f_tol, max_iters, device=None):
    lib = load_library()
    K = _f64(K)
    y = _f64(y)
    n = K.shape[0]
    f = np.empty(n)
    C = np.empty((n, n)) if calc_cov else None
    lml = np.zeros(1)
    nit = np.zeros(1, dtype=np.int64)
    st = np.zeros(1, dtype=np.int32)
    _check(lib.apm_laplace(default_device() if device is None else device, _ptr(K), n, n, _ptr(y),
                           int(bool(calc_cov)), int(bool(calc_lml)), float(diff_f_tol),
                           int(max_iters), _ptr(f), _ptr(C), n, _ptr(lml), _ptr(nit), _ptr(st)))
    return f, C, float(lml[0]), int(nit[0]), int(st[0])


def selftest_tile(A, B, C, device=None):
    lib = load_library()
    A, B = _f64(A), _f64(B)
    C = _f64(C).copy()
    _check(lib.apm_selftest_tile(default_device() if device is None else device, _ptr(A), _ptr(B),
                                 _ptr(C)))
    return C


def selftest_philox(blocks, device=None):
    """Philox4x32-10 of (counter[4], key[2]) rows (uint32) through the device round function."""
    lib = load_library()
    inp = np.ascontiguousarray(blocks, dtype=np.uint32).reshape(-1, 6)
    out = np.empty((inp.shape[0], 4), dtype=np.uint32)
    _check(lib.apm_selftest_philox(default_device() if device is None else device, inp.shape[0],
                                   _ptr(inp), _ptr(out)))
    return out


# ----------------------------------------------------------------------------- context


class _Pool(object):
    def __init__(self, n):
        self.free = list(range(n - 1, -1, -1))
        self.refs = {}

    def acquire(self):
        if not self.free:
            raise NativeError('pool exhausted (raise n_slots / n_ubufs)')
        i = self.free.pop()
        self.refs[i] = 1
        return i

    def incref(self, i):
        self.refs[i] += 1

    def release(self, i):
        self.refs[i] -= 1
        if self.refs[i] == 0:
            del self.refs[i]
            self.free.append(i)


class _SlotPool(object):
    """Cache-slot owners kept by the library (apm_cache_acquire / _copy / _release): the same
    interface as _Pool, so a C caller and this layer share one ownership record."""

    def __init__(self, ctx):
        self.ctx = ctx

    def acquire(self):
        s = ctypes.c_int64(-1)
        _check(self.ctx.lib.apm_cache_acquire(self.ctx._h, ctypes.byref(s)), self.ctx._h)
        return int(s.value)

    def incref(self, i):
        _check(self.ctx.lib.apm_cache_copy(self.ctx._h, int(i)), self.ctx._h)

    def release(self, i):
        if self.ctx._h:
            _check(self.ctx.lib.apm_cache_release(self.ctx._h, int(i)), self.ctx._h)

    def refcount(self, i):
        return int(self.ctx.lib.apm_cache_refcount(self.ctx._h, int(i)))


class Context(object):
    """A device-resident problem (X, y, kernel) with workspaces for up to `max_batch` chains."""

    def __init__(self, X, y, kernel_kind, epsilon, n_imp, max_batch=1, n_slots=4, n_ubufs=4,
                 device=None):
        lib = load_library()
        self.lib = lib
        self.device = default_device() if device is None else device
        y = _f64(y)
        self.n = y.shape[0]
        if kernel_kind == KERNEL_PRECOMPUTED:
            Xp, d, ldx = None, 0, 0
        else:
            Xp = _f64(X)
            d, ldx = Xp.shape[1], Xp.shape[1]
        self.d = d
        self.kind = kernel_kind
        self.n_imp = int(n_imp)
        self.max_batch = int(max_batch)
        self._h = lib.apm_create(self.device, kernel_kind, _ptr(Xp), self.n, d, ldx, _ptr(y),
                                 float(epsilon), self.n_imp, self.max_batch, int(n_slots),
                                 int(n_ubufs))
        if not self._h:
            raise NativeError('apm_create failed: ' +
                              (lib.apm_global_error() or b'').decode(errors='replace'))
        self.slots = _SlotPool(self)
        self.ubufs = _Pool(int(n_ubufs))
        # calls per batch size (bench.py reports the timed region's; launch shapes depend on it)
        self.batch_hist = {'u': collections.Counter(), 'theta': collections.Counter()}
        self.theta_len = int(lib.apm_theta_len(self._h))
        self.padded_n = int(lib.apm_padded_n(self._h))

    def close(self):
        if getattr(self, '_h', None):
            self.lib.apm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream_ptr(self):
        return self.lib.apm_stream(self._h)

    def set_newton(self, tol, max_iters):
        _check(self.lib.apm_set_newton(self._h, float(tol), int(max_iters)), self._h)

    # --- U buffers
    def u_upload(self, ubuf, U):
        U = _f64(U)
        if U.shape != (self.n, self.n_imp):
            raise ValueError('u has shape {0}, expected {1}'.format(U.shape, (self.n, self.n_imp)))
        _check(self.lib.apm_u_upload(self._h, ubuf, _ptr(U), U.shape[1]), self._h)

    def u_download(self, ubuf):
        U = np.empty((self.n, self.n_imp))
        _check(self.lib.apm_u_download(self._h, ubuf, _ptr(U), self.n_imp), self._h)
        return U

    def u_normal(self, ubufs, seeds, counters):
        ub = np.ascontiguousarray(ubufs, dtype=np.int64)
        sd = np.ascontiguousarray(seeds, dtype=np.uint64)
        ct = np.ascontiguousarray(counters, dtype=np.uint64)
        _check(self.lib.apm_u_normal(self._h, ub.shape[0], _ptr(ub), _ptr(sd), _ptr(ct)), self._h)

    def u_combine(self, dst, a, b, ca, cb):
        dst, a, b = (np.ascontiguousarray(x, dtype=np.int64) for x in (dst, a, b))
        ca, cb = _f64(ca), _f64(cb)
        _check(self.lib.apm_u_combine(self._h, dst.shape[0], _ptr(dst), _ptr(a), _ptr(b), _ptr(ca),
                                      _ptr(cb)), self._h)

    # --- estimator calls
    def theta_eval(self, est, thetas, ubufs=None, slots=None):
        th = np.atleast_2d(_f64(thetas))
        count = th.shape[0]
        self.batch_hist['theta'][count] += 1
        if th.shape[1] < self.theta_len:
            raise IndexError('Out of bounds on buffer access (axis 0)')
        out = np.full(count, np.nan)
        st = np.zeros(count, dtype=np.int32)
        nops = np.zeros(count, dtype=np.int64)
        ub = None if ubufs is None else np.ascontiguousarray(ubufs, dtype=np.int64)
        sl = None if slots is None else np.ascontiguousarray(slots, dtype=np.int64)
        _check(self.lib.apm_theta_eval(self._h, est, count, _ptr(th), th.shape[1], _ptr(ub),
                                       _ptr(sl), _ptr(out), _ptr(st), _ptr(nops)), self._h)
        return out, st, nops

    def theta_eval_K(self, est, K, ubuf, slot):
        K = _f64(K)
        out = np.full(1, np.nan)
        st = np.zeros(1, dtype=np.int32)
        nops = np.zeros(1, dtype=np.int64)
        _check(self.lib.apm_theta_eval_K(self._h, est, _ptr(K), K.shape[1], int(ubuf), int(slot),
                                         _ptr(out), _ptr(st), _ptr(nops)), self._h)
        return out, st, nops

    def u_eval(self, slots, ubufs):
        sl = np.ascontiguousarray(slots, dtype=np.int64)
        self.batch_hist['u'][sl.shape[0]] += 1
        ub = np.ascontiguousarray(ubufs, dtype=np.int64)
        out = np.full(sl.shape[0], np.nan)
        st = np.zeros(sl.shape[0], dtype=np.int32)
        _check(self.lib.apm_u_eval(self._h, sl.shape[0], _ptr(sl), _ptr(ub), _ptr(out), _ptr(st)),
               self._h)
        return out, st

    def slot_read(self, slot):
        L = np.zeros((self.n, self.n))
        f = np.zeros(self.n)
        g = np.zeros(self.n)
        c = np.zeros(1)
        _check(self.lib.apm_slot_read(self._h, int(slot), _ptr(L), self.n, _ptr(f), _ptr(g),
                                      _ptr(c)), self._h)
        return L, f, g, float(c[0])

    def guard_read(self, count):
        """(count, 4) residuals r1..r4 of the last IS theta-call's guard (include/apm.h)."""
        r = np.zeros((int(count), 4))
        _check(self.lib.apm_guard_read(self._h, int(count), _ptr(r)), self._h)
        return r

    # --- profiling
    def prof_enable(self, on=True):
        """on: False/0 off, True/1 the roofline kinds, 2 every kind (apm.h)."""
        _check(self.lib.apm_prof_enable(self._h, int(on)), self._h)

    def prof_marker(self, marker_id):
        _check(self.lib.apm_prof_marker(self._h, int(marker_id)), self._h)

    def prof_read(self, kind, reset=False):
        ms = np.zeros(1)
        cnt = np.zeros(1, dtype=np.int64)
        wk = np.zeros(1)
        _check(self.lib.apm_prof_read(self._h, kind, _ptr(ms), _ptr(cnt), _ptr(wk), int(reset)),
               self._h)
        return float(ms[0]), int(cnt[0]), float(wk[0])
