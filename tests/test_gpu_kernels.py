"""GPU parity of the HIP building blocks through the C-ABI (libapm.so) against the oracle and
the golden vectors produced by the reference (tests/golden/make_golden.py).

Tolerances: theta-path quantities are fp64 (Gram 1e-13 rel; Laplace f 1e-9 rel);
estimator values go through the fp32 MFMA L.U and are checked to |d log f| <= 5e-4 nats.
"""
import numpy as np
import pytest

import apm_oracle as orc
from conftest import golden

pytestmark = pytest.mark.gpu

TOL_ABS, TOL_REL = 5e-4, 0.0  # nats; no relative term


def _close(v, ref):
    return abs(v - ref) <= TOL_ABS + TOL_REL * abs(ref)


def _assert_gram_close(K, Kref):
    """exp(-s/2) carries the exponent's relative rounding (x s) into K: bound the error relative
    to the exponent, 2e-15 * max(1, |log K|), i.e. a few ulp of s."""
    scale = np.maximum(1.0, np.abs(np.log(np.maximum(Kref, 1e-300))))
    bad = np.abs(K - Kref) > 2e-15 * scale * np.abs(Kref) + 1e-300
    assert not bad.any(), (np.abs(K - Kref)[bad].max(), bad.sum())


@pytest.fixture(scope='module')
def nat(gpu_available):
    from gpdemo import _native
    _native.load_library()
    return _native


def _cases():
    g = golden('estimators')
    out = []
    for ci in range(int(g['n_cases'])):
        pre = 'c{0}_'.format(ci)
        out.append({k[len(pre):]: g[k] for k in g.files if k.startswith(pre)})
    return out


def test_mfma_f64_tile_layout(nat):
    rng = np.random.RandomState(0)
    A = rng.normal(size=(64, 64))
    B = rng.normal(size=(64, 64)) + np.arange(64)[:, None] * 0.01  # asymmetric
    C = rng.normal(size=(64, 64))
    out = nat.selftest_tile(A, B, C)
    np.testing.assert_allclose(out, C + A.dot(B.T), rtol=1e-12, atol=1e-12)


def test_gram_vs_golden(nat):
    g = golden('gram')
    keys = sorted({k.rsplit('_', 1)[0] for k in g.files if k.endswith('_thetas')})
    for key in keys:
        kind = nat.KERNEL_ISO if key.startswith('iso') else nat.KERNEL_ARD
        X = g[key + '_X']
        for th, Kref in zip(g[key + '_thetas'], g[key + '_K']):
            K = np.empty_like(Kref)
            nat.gram(kind, K, X, th, 1e-8)
            _assert_gram_close(K, Kref)


def test_gram_large_ragged_vs_c_oracle(nat):
    rng = np.random.RandomState(5)
    for n, d in ((300, 7), (1000, 32), (129, 64)):
        X = rng.normal(size=(n, d))
        th = np.r_[0.3, rng.normal(size=d)]
        K = np.empty((n, n))
        nat.gram(nat.KERNEL_ARD, K, X, th, 1e-8)
        Kr = np.empty((n, n))
        orc.c_gram('ard', Kr, X, th, 1e-8)
        _assert_gram_close(K, Kr)


def test_gram_near_duplicate_rows_vs_c_oracle(nat):
    """Near-duplicate rows (tiny distances), D within one LDS chunk and beyond it, iso and ARD:
    the direct-form kernel against the C oracle, and K exactly symmetric."""
    rng = np.random.RandomState(11)
    for n, d, kind in ((200, 3, 'ard'), (150, 40, 'ard'), (130, 6, 'iso')):
        base = rng.normal(size=(n // 2, d))
        X = np.concatenate([base, base + 1e-4 * rng.normal(size=base.shape)])[rng.permutation(n)]
        X = np.concatenate([X, 3.0 + 0.01 * rng.normal(size=(n % 2, d))]) if n % 2 else X
        th = np.r_[0.2, rng.normal(scale=0.5, size=d if kind == 'ard' else 1)]
        Kr = np.empty((n, n))
        orc.c_gram(kind, Kr, X, th, 1e-8)
        K = np.empty((n, n))
        nat.gram(nat.KERNEL_ISO if kind == 'iso' else nat.KERNEL_ARD, K, X, th, 1e-8)
        _assert_gram_close(K, Kr)
        assert np.array_equal(K, K.T)


def test_laplace_vs_golden(nat):
    for c in _cases():
        f, C, lml, nit, st = nat.laplace(c['K'], c['y'], True, True, 1e-4, 1000)
        assert st == 0
        assert nit + 1 == int(c['lap_nops_cov_lml'])
        np.testing.assert_allclose(f, c['lap_f'], rtol=1e-9, atol=1e-11)
        np.testing.assert_allclose(C, c['lap_C'], rtol=1e-8, atol=1e-10)
        assert abs(lml - float(c['lap_lml'])) < 1e-8 * max(1., abs(float(c['lap_lml'])))


def _ctx(nat, c, n_slots=4, n_ubufs=4, max_batch=4):
    kind = nat.KERNEL_ISO if str(c['kind']) == 'iso' else nat.KERNEL_ARD
    return nat.Context(c['X'], c['y'], kind, 1e-8, c['ns1'].shape[1], max_batch=max_batch,
                       n_slots=n_slots, n_ubufs=n_ubufs)


def test_is_estimator_vs_golden(nat):
    for ci, c in enumerate(_cases()):
        ctx = _ctx(nat, c)
        ctx.u_upload(0, c['ns1'])
        ctx.u_upload(1, c['ns2'])
        out, st, nops = ctx.theta_eval(nat.EST_IS, c['theta'][None], [0], [0])
        assert st[0] == 0
        assert nops[0] == int(c['is_ops'])
        assert _close(out[0], float(c['is_logf1'])), (ci, out[0], float(c['is_logf1']))
        out2, st2 = ctx.u_eval([0], [1])
        assert _close(out2[0], float(c['is_logf2'])), (ci, out2[0], float(c['is_logf2']))
        L, f, g, cst = ctx.slot_read(0)
        np.testing.assert_allclose(f, c['f_post'], rtol=1e-8, atol=1e-10)
        np.testing.assert_allclose(L, np.tril(c['C_chol']), rtol=0, atol=2e-6 * np.abs(c['C_chol']).max())
        ctx.close()


def test_wide_slot_fp64_path_vs_golden(nat, monkeypatch):
    """The f64-MFMA u-path of wide slots (k_ugemm64, fp64 factor and U; ugemm.hip), forced for
    every slot (APM_WIDE_Q=0), against the reference's own IS estimates (theta-call and cached
    u-call), PriorMC estimates and the default fp32 path; a PriorMC slot goes the same way."""
    for ci, c in enumerate(_cases()):
        res = {}
        for env in ({}, {'APM_WIDE_Q': '0'}):
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            ctx = _ctx(nat, c)
            for k in env:
                monkeypatch.delenv(k)
            ctx.u_upload(0, c['ns1'])
            ctx.u_upload(1, c['ns2'])
            out, st, _ = ctx.theta_eval(nat.EST_IS, c['theta'][None], [0], [0])
            out2, st2 = ctx.u_eval([0], [1])
            pm, st3, _ = ctx.theta_eval(nat.EST_PRIORMC, c['theta'][None], [0], [1])
            pm2, _ = ctx.u_eval([1], [1])
            ctx.close()
            assert st[0] == 0 and st2[0] == 0 and st3[0] == 0
            res[bool(env)] = (out[0], out2[0], pm[0], pm2[0])
        ref = (float(c['is_logf1']), float(c['is_logf2']), float(c['pmc_logf1']),
               float(c['pmc_logf2']))
        for w, r in zip(res[True], ref):
            assert _close(w, r), (ci, w, r)
        for w, f in zip(res[True], res[False]):  # both paths agree far inside the tolerance
            assert abs(w - f) <= 1e-4, (ci, w, f)


def test_wide_buffers_follow_slots(nat, monkeypatch):
    """fp64 factors are attached to slots only while they are wide (capi.cpp attach_l64 /
    detach_l64): a slot that turns narrow gives its buffer back, the next wide slot takes it, and
    every cached u-call afterwards equals a fresh context's - in a batch of wide and narrow
    chains, across the IS (fp32 bottom + fp64 rerun) and PriorMC writers."""
    c = _cases()[0]
    th_n = c['theta'].copy()
    th_w = c['theta'].copy()
    th_w[0] = th_n[0] + 4.0  # trace(C) 23 -> 724, trace(K) 81 -> 4422 (oracle): bound 300
    monkeypatch.setenv('APM_WIDE_Q', '300')
    ctx = _ctx(nat, c, max_batch=2, n_slots=3, n_ubufs=2)
    fresh = _ctx(nat, c, max_batch=1, n_slots=1, n_ubufs=2)
    monkeypatch.delenv('APM_WIDE_Q')
    for x in (ctx, fresh):
        x.u_upload(0, c['ns1'])
        x.u_upload(1, c['ns2'])

    def one(est, th):
        o, st, _ = fresh.theta_eval(est, th[None], [0], [0])
        u, _ = fresh.u_eval([0], [1])
        assert st[0] == 0
        return o[0], u[0]
    seq = [((nat.EST_IS, nat.EST_IS), (th_w, th_n), (0, 1)),
           ((nat.EST_IS, nat.EST_IS), (th_n, th_w), (0, 2)),
           ((nat.EST_PRIORMC, nat.EST_IS), (th_w, th_w), (1, 0)),
           ((nat.EST_IS, nat.EST_PRIORMC), (th_n, th_n), (1, 2))]
    for ests, ths, slots in seq:
        for e, th, sl in zip(ests, ths, slots):
            o, st, _ = ctx.theta_eval(e, th[None], [0], [sl])
            assert st[0] == 0
            u, _ = ctx.u_eval([sl], [1])
            fo, fu = one(e, th)
            assert o[0] == fo and u[0] == fu, (e, sl, o[0], fo, u[0], fu)
        u2, _ = ctx.u_eval(list(slots), [1, 1])  # both slots in one cached call
        for q, (e, th) in enumerate(zip(ests, ths)):
            assert u2[q] == one(e, th)[1]
    ctx.close()
    fresh.close()


def test_cache_tuple_vs_golden(nat):
    """Iterating the API's IS cache yields the reference's (K_chol, C_chol, f_post) tuple
    (estimators.py:166-176); a PriorMC cache converts to the reference's K_chol array
    (estimators.py:311-318). fp32-rounded read-back."""
    import gpdemo.estimators as est
    import gpdemo.kernels as krn
    import gpdemo.latent_posterior_approximations as lpa
    for ci, c in enumerate(_cases()):
        kf = krn.make_kernel_func(str(c['kind']), 1e-8)
        e = est.LogMarginalLikelihoodApproxPosteriorISEstimator(c['X'], c['y'], kf,
                                                                lpa.laplace_approximation)
        _, cache = e(c['ns1'], c['theta'])
        ops = e.n_cubic_ops
        K_chol, C_chol, f_post = cache
        assert e.n_cubic_ops == ops  # inspection is not an estimator op
        for got, ref in ((K_chol, c['K_chol']), (C_chol, c['C_chol'])):
            np.testing.assert_allclose(got, np.tril(ref), rtol=0,
                                       atol=2e-6 * np.abs(ref).max(), err_msg=str(ci))
        np.testing.assert_allclose(f_post, c['f_post'], rtol=1e-8, atol=1e-10)
        # the cache still serves u-calls after the inspection's scratch theta-call
        v2, _ = e(c['ns2'], None, cache)
        assert _close(v2, float(c['is_logf2'])), (ci, v2)
        p = est.LogMarginalLikelihoodPriorMCEstimator(c['X'], c['y'], kf)
        _, kc = p(c['ns1'], c['theta'])
        np.testing.assert_allclose(np.asarray(kc), np.tril(c['K_chol']), rtol=0,
                                   atol=2e-6 * np.abs(c['K_chol']).max(), err_msg=str(ci))


def test_priormc_and_laplace_estimators_vs_golden(nat):
    for ci, c in enumerate(_cases()):
        ctx = _ctx(nat, c)
        ctx.u_upload(0, c['ns1'])
        ctx.u_upload(1, c['ns2'])
        out, st, nops = ctx.theta_eval(nat.EST_PRIORMC, c['theta'][None], [0], [0])
        assert st[0] == 0 and nops[0] == 1
        assert _close(out[0], float(c['pmc_logf1'])), (ci, out[0], float(c['pmc_logf1']))
        out2, _ = ctx.u_eval([0], [1])
        assert _close(out2[0], float(c['pmc_logf2'])), (ci, out2[0], float(c['pmc_logf2']))
        lml, st, nops = ctx.theta_eval(nat.EST_LAPLACE, c['theta'][None])
        assert st[0] == 0 and nops[0] == int(c['lapest_ops'])
        assert abs(lml[0] - float(c['lapest_lml'])) < 1e-8 * max(1, abs(lml[0]))
        ctx.close()


def test_batched_equals_single(nat):
    c = _cases()[1]
    ctx = _ctx(nat, c, n_slots=6, n_ubufs=6, max_batch=3)
    ctx.u_upload(0, c['ns1'])
    ctx.u_upload(1, c['ns2'])
    th = np.stack([c['theta'], c['theta'] + 0.1, c['theta'] - 0.2])
    out, st, nops = ctx.theta_eval(nat.EST_IS, th, [0, 1, 0], [0, 1, 2])
    assert (st == 0).all()
    for b in range(3):
        o1, s1, _ = ctx.theta_eval(nat.EST_IS, th[b][None], [[0, 1, 0][b]], [3])
        assert abs(o1[0] - out[b]) < 1e-9 * max(1., abs(out[b]))
    # reference values at the perturbed thetas
    kf = orc.make_kernel_func('ard', 1e-8)
    for b in range(3):
        ns = c['ns1'] if b != 1 else c['ns2']
        v, _, _ = orc.is_estimate(c['X'], c['y'], kf, ns, th[b])
        assert _close(out[b], v), (b, out[b], v)
    ctx.close()


def test_u_normal_moments(nat):
    c = _cases()[2]
    ctx = _ctx(nat, c)
    ctx.u_normal([0, 1], [123, 123], [0, 1])
    U0, U1 = ctx.u_download(0), ctx.u_download(1)
    assert abs(U0.mean()) < 0.02 and abs(U0.std() - 1) < 0.02
    assert not np.allclose(U0, U1)
    ctx.u_normal([2], [123], [0])
    np.testing.assert_array_equal(ctx.u_download(2), U0)  # counter-based: reproducible
    ctx.u_combine([3], [0], [1], [0.6], [0.8])
    np.testing.assert_allclose(ctx.u_download(3), 0.6 * U0 + 0.8 * U1, rtol=1e-5, atol=1e-5)
    ctx.close()


@pytest.mark.parametrize('n,d,s,kind', [(700, 5, 32, 'ard'), (1100, 3, 8, 'iso')])
def test_estimators_multi_panel_vs_oracle(nat, n, d, s, kind):
    """N spanning several 256-column outer panels (the rank-256 update path) vs the oracle."""
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(n, d, 99 + n, kind)
    rng = np.random.RandomState(n)
    P = d + 1 if kind == 'ard' else 2
    theta = np.r_[0.4, rng.normal(scale=0.3, size=P - 1) + 0.5 * np.log(d)]
    ns1, ns2 = rng.normal(size=(n, s)), rng.normal(size=(n, s))
    kf = orc.make_kernel_func(kind, 1e-8)
    r1, rc, rops = orc.is_estimate(X, y, kf, ns1, theta)
    r2, _, _ = orc.is_estimate(X, y, kf, ns2, None, rc)
    p1, _, _ = orc.priormc_estimate(X, y, kf, ns1, theta)
    lml, lops = orc.laplace_estimate(X, y, kf, theta)
    ctx = nat.Context(X, y, nat.KERNEL_ARD if kind == 'ard' else nat.KERNEL_ISO, 1e-8, s,
                      max_batch=1, n_slots=2, n_ubufs=2)
    ctx.u_upload(0, ns1)
    ctx.u_upload(1, ns2)
    out, st, nops = ctx.theta_eval(nat.EST_IS, theta[None], [0], [0])
    assert st[0] == 0 and nops[0] == rops
    assert _close(out[0], r1), (out[0], r1)
    out2, _ = ctx.u_eval([0], [1])
    assert _close(out2[0], r2), (out2[0], r2)
    _, f, _, _ = ctx.slot_read(0)
    np.testing.assert_allclose(f, rc[2], rtol=1e-7, atol=1e-9)
    out, st, _ = ctx.theta_eval(nat.EST_PRIORMC, theta[None], [0], [1])
    assert _close(out[0], p1), (out[0], p1)
    out, st, nops = ctx.theta_eval(nat.EST_LAPLACE, theta[None])
    assert abs(out[0] - lml) < 1e-7 * max(1., abs(lml)) and nops[0] == lops
    ctx.close()


def _mixed_case(n=700, d=5, s=32):
    from gpdemo import utils
    X, y = utils.synthetic_gp_data(n, d, 4242, 'ard')
    rng = np.random.RandomState(7)
    base = 0.5 * np.log(d)
    thetas = np.array([np.r_[0.0, np.full(d, base)],
                       np.r_[2.0, rng.normal(scale=0.3, size=d) + base - 0.5],
                       np.r_[4.0, rng.normal(scale=0.3, size=d) + base + 0.5]])
    ns = rng.normal(size=(n, s))
    return X, y, thetas, ns


def _run_is(nat, X, y, thetas, ns, monkeypatch, **env):
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    B = len(thetas)
    ctx = nat.Context(X, y, nat.KERNEL_ARD, 1e-8, ns.shape[1], max_batch=B, n_slots=B, n_ubufs=1)
    for k in env:
        monkeypatch.delenv(k)
    ctx.u_upload(0, ns)
    out, st, nops = ctx.theta_eval(nat.EST_IS, thetas, ubufs=[0] * B, slots=list(range(B)))
    fs = [ctx.slot_read(b)[1] for b in range(B)]
    ctx.close()
    return out, st, nops, fs


def test_mixed_newton_matches_fp64(nat, monkeypatch):
    """The fp32 factorisation of B + fp64 refinement (chol32.hip) reproduces the fp64 Newton mode
    within the f_post tolerance, 1e-8 of its maximum (~1e-12 with the dataflow
    walk, ~1e-9 with the explicit-inverse panels, whose fp16x3 product with inv(L_D) leaves a
    less accurate factor for the refinement to correct), and hence the estimate, for
    sigma = e^0..e^4."""
    X, y, thetas, ns = _mixed_case()
    o64, s64, n64, f64 = _run_is(nat, X, y, thetas, ns, monkeypatch, APM_MIXED=0)
    o32, s32, n32, f32 = _run_is(nat, X, y, thetas, ns, monkeypatch, APM_MIXED=1)
    assert (s64 == 0).all() and (s32 == 0).all()
    np.testing.assert_array_equal(n32, n64)
    for b in range(len(thetas)):
        np.testing.assert_allclose(f32[b], f64[b], rtol=0, atol=1e-8 * np.abs(f64[b]).max())
        assert abs(o32[b] - o64[b]) <= 1e-6 * max(1.0, abs(o64[b])), (b, o32[b], o64[b])


def test_fp16x3_updates_match_fp32_operands(nat, monkeypatch):
    """fp16x3 trailing updates of the Newton factor (chol32.hip, default) against fp32 operands
    (APM_H3=0, which also walks every panel: the explicit-inverse panels need the planes): same
    iteration counts, modes within the f_post tolerance (1e-8 of the maximum), estimates to 1e-6.
    The range
    guard is per chain: a chain at theta_0 >= 19 takes fp32 operands (bit-identical to APM_H3=0)
    while the other chains of the same call keep fp16x3 (bit-identical to a call without it), so
    a chain's value does not depend on its batch."""
    X, y, thetas, ns = _mixed_case()
    o0, s0, n0, f0 = _run_is(nat, X, y, thetas, ns, monkeypatch, APM_H3=0)
    o1, s1, n1, f1 = _run_is(nat, X, y, thetas, ns, monkeypatch)
    assert (s0 == 0).all() and (s1 == 0).all()
    np.testing.assert_array_equal(n1, n0)
    for b in range(len(thetas)):
        np.testing.assert_allclose(f1[b], f0[b], rtol=0, atol=1e-8 * np.abs(f0[b]).max())
        assert abs(o1[b] - o0[b]) <= 1e-6 * max(1.0, abs(o0[b])), (b, o1[b], o0[b])
    big = thetas.copy()
    big[2, 0] = 19.5
    ob0, sb0, nb0, fb0 = _run_is(nat, X, y, big, ns, monkeypatch, APM_H3=0)
    ob1, sb1, nb1, fb1 = _run_is(nat, X, y, big, ns, monkeypatch)
    np.testing.assert_array_equal(sb1, sb0)
    np.testing.assert_array_equal(nb1, nb0)
    if sb0[2] == 0:
        np.testing.assert_array_equal(fb1[2], fb0[2])
        assert ob1[2] == ob0[2]
    for b in (0, 1):  # unchanged by the fp32 chain next to them
        np.testing.assert_array_equal(fb1[b], f1[b])
        assert ob1[b] == o1[b]


def _run_is_stats(nat, X, y, thetas, ns, monkeypatch, **env):
    """_run_is plus the context's fp64 Newton-rerun count (APM_PROF_STATS launches)."""
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    B = len(thetas)
    ctx = nat.Context(X, y, nat.KERNEL_ARD, 1e-8, ns.shape[1], max_batch=B, n_slots=B, n_ubufs=1)
    for k in env:
        monkeypatch.delenv(k)
    ctx.u_upload(0, ns)
    ctx.prof_read(nat.PROF_STATS, reset=True)
    out, st, nops = ctx.theta_eval(nat.EST_IS, thetas, ubufs=[0] * B, slots=list(range(B)))
    reruns = ctx.prof_read(nat.PROF_STATS)[1]
    fs = [ctx.slot_read(b)[1] for b in range(B)]
    ctx.close()
    return out, st, nops, fs, reruns


@pytest.mark.parametrize('n', [2048, 1700, 700])
def test_panel_forms_are_batch_independent(nat, monkeypatch, n):
    """The Newton factorisation takes, per chain, the explicit-inverse panel (chol32.hip
    k_zinv_level32 + k_panel_inv_gemm32, chains with 1 + K_ii < 2^15), the dataflow walk with
    fp16x3 operands (1 + K_ii >= 2^15, theta_0 < 19) or the walk with fp32 operands
    (theta_0 >= 19); a batch whose chains all take the first runs compact dataflow launches and
    the far updates on 256x256 quad tiles from the operand planes (k_chol_update32_q256),
    otherwise every row walks or returns by its chain's flag and the far updates run on the
    128-row super-tiles. Both forms perform the same split of the same values in the same MFMA
    order, so a chain's mode and estimate are bitwise those it has in any other batch.
    n = 1700: ragged quad tiles; n = 700: one full panel and a ragged last one (walked)."""
    X, y, thetas, ns = _mixed_case(n=n)
    o1, s1, n1, f1, r1 = _run_is_stats(nat, X, y, thetas, ns, monkeypatch)
    assert (s1 == 0).all() and r1 == 0
    for extra in (12.0, 19.5):  # a walking fp16x3 chain / an fp32-operand chain in the batch
        big = np.vstack([thetas, thetas[1]])
        big[-1, 0] = extra
        ob, sb, nbs, fb, rb = _run_is_stats(nat, X, y, big, ns, monkeypatch)
        np.testing.assert_array_equal(sb[:3], s1)
        np.testing.assert_array_equal(nbs[:3], n1)
        for b in range(3):
            np.testing.assert_array_equal(fb[b], f1[b])
            assert ob[b] == o1[b], (extra, b, ob[b], o1[b])
        if extra == 12.0:  # the walking chain is bitwise its value alone
            oa, sa, na, fa, ra = _run_is_stats(nat, X, y, big[-1:], ns, monkeypatch)
            assert sa[0] == sb[-1] and na[0] == nbs[-1]
            if sa[0] == 0:
                np.testing.assert_array_equal(fa[0], fb[-1])
                assert oa[0] == ob[-1]


@pytest.mark.parametrize('n', [2048, 700])
def test_fp16x3_walk_range_against_fp64(nat, monkeypatch, n):
    """Chains with theta_0 in 11 .. 18 (advisor r05: the explicit-inverse panel's fp16 split of
    Schur-complement entries, bounded by 1 + K_ii, overflowed above theta_0 ~ 11 and sent every
    such call to the fp64 rerun): they now walk their panels with fp16x3 operands (solved
    entries, |L_ij| <= sqrt(1 + K_ii)). Per chain, the default path reruns in fp64 exactly when
    the all-fp32-operand path (APM_H3=0) does - at large sigma cond(B) ~ 1 + W n sigma^2 can
    exceed what any fp32 factor refines, which is the rerun's purpose - and the modes and
    estimates match the all-fp64 Newton iteration (APM_MIXED=0) within the f_post tolerance
    (1e-8 of the maximum) and 1e-6 relative, with the same iteration counts. Short length-scales
    keep K near sigma^2 I, so that cond(B) ~ 1 + W sigma^2 stays within the fp32 factor's reach
    at theta_0 = 11 (there no chain may be rerun) and the fp16x3 walk is what is exercised."""
    X, y, thetas, ns = _mixed_case(n=n)
    for t0 in (11.0, 12.5, 14.0, 17.0):
        th = np.r_[t0, thetas[1, 1:] - 3.0][None]
        o64, s64, n64, f64, _ = _run_is_stats(nat, X, y, th, ns, monkeypatch, APM_MIXED=0)
        o3, s3, n3, f3, r3 = _run_is_stats(nat, X, y, th, ns, monkeypatch, APM_H3=0)
        o32, s32, n32, f32, r32 = _run_is_stats(nat, X, y, th, ns, monkeypatch)
        print('n = {0} theta_0 = {1}: fp64 reruns default {2}, fp32 operands {3}'
              .format(n, t0, r32, r3))
        assert s64[0] == 0 and s32[0] == 0 and s3[0] == 0, (t0, s64, s32, s3)
        assert r32 == r3, (t0, r32, r3)
        if t0 == 11.0:
            assert r32 == 0, 'a chain the fp32 factor handles was rerun in fp64'

        assert n32[0] == n64[0], (t0, n32, n64)
        np.testing.assert_allclose(f32[0], f64[0], rtol=0, atol=1e-8 * np.abs(f64[0]).max())
        assert abs(o32[0] - o64[0]) <= 1e-6 * max(1.0, abs(o64[0])), (t0, o32[0], o64[0])


def _run_is_prof(nat, X, y, thetas, ns, monkeypatch, **env):
    """_run_is plus the slots' factors and the fp64-rerun counter of the posterior bottom block."""
    for k, v in env.items():
        monkeypatch.setenv(k, str(v))
    B = len(thetas)
    ctx = nat.Context(X, y, nat.KERNEL_ARD, 1e-8, ns.shape[1], max_batch=B, n_slots=B, n_ubufs=1)
    for k in env:
        monkeypatch.delenv(k)
    ctx.u_upload(0, ns)
    ctx.prof_read(nat.PROF_POST64_RERUNS, reset=True)
    out, st, nops = ctx.theta_eval(nat.EST_IS, thetas, ubufs=[0] * B, slots=list(range(B)))
    reruns = ctx.prof_read(nat.PROF_POST64_RERUNS, reset=True)[1]
    u_out, u_st = ctx.u_eval(list(range(B)), [0] * B)
    rd = [ctx.slot_read(b) for b in range(B)]
    ctx.close()
    return out, st, nops, rd, reruns, u_out


@pytest.mark.parametrize('n', [700, 1100])
def test_posterior_bottom_fp32_matches_fp64(nat, monkeypatch, n):
    """The posterior factor's bottom block (L_K J) L'^-T in fp32 beside the fp64 factorisation of
    J M J on the second stream (postcov.hip) against its fp64 recomputation (APM_POST32_Q=0: the
    trace bound above which a chain's bottom block is recomputed in fp64 from the intact fp64
    rows, here every chain): Newton modes and log|B| untouched (bitwise equal f_post and cst),
    chol(C) within fp32 accuracy of its maximum, estimates within 1e-4 nats (the fp32 TRSM moves
    log f by ~1e-9 x trace(C)). n = 1100: a ragged last outer panel."""
    X, y, thetas, ns = _mixed_case(n=n)
    o0, s0, n0, r0, k0, u0 = _run_is_prof(nat, X, y, thetas, ns, monkeypatch, APM_POST32_Q=0)
    o1, s1, n1, r1, k1, u1 = _run_is_prof(nat, X, y, thetas, ns, monkeypatch)
    assert (s0 == 0).all() and (s1 == 0).all()
    np.testing.assert_array_equal(n1, n0)
    assert k1 == 0 and k0 == len(thetas)
    for b in range(len(thetas)):
        L0, f0, g0, c0 = r0[b]
        L1, f1, g1, c1 = r1[b]
        np.testing.assert_array_equal(f1, f0)
        assert c1 == c0
        assert np.abs(L1 - L0).max() <= 1e-5 * np.abs(L0).max(), (b, np.abs(L1 - L0).max())
        assert abs(o1[b] - o0[b]) <= 1e-4, (b, o1[b], o0[b])
        assert abs(u1[b] - u0[b]) <= 1e-4, (b, u1[b], u0[b])


@pytest.mark.parametrize('tol', [0.0, 1e-7])
def test_mixed_newton_fp64_fallback(nat, monkeypatch, tol):
    """Chains whose refined fp32 solve fails the acceptance test are rerun in fp64 from f = 0
    while the others keep their mixed-precision modes: tol = 0 sends every chain (Newton modes
    then bit-identical to the fp64 path; the estimate to 1e-9 relative, since the mixed path
    forms h = L_K^-1 f_post as L_K^T a (f_post = K a) from its concurrent chol(K) while the
    all-fp64 path solves for it, which differ by L_K^-1 times the rounding of K a - up to ~1e-10
    relative for an ill-conditioned K), tol = 1e-7 typically some."""
    X, y, thetas, ns = _mixed_case()
    o64, s64, n64, f64 = _run_is(nat, X, y, thetas, ns, monkeypatch, APM_MIXED=0)
    o32, s32, n32, f32 = _run_is(nat, X, y, thetas, ns, monkeypatch, APM_MIXED=1,
                                 APM_REFINE_TOL=tol)
    assert (s32 == 0).all()
    np.testing.assert_array_equal(n32, n64)
    for b in range(len(thetas)):
        if tol == 0.0:
            np.testing.assert_array_equal(f32[b], f64[b])
            assert abs(o32[b] - o64[b]) <= 1e-9 * max(1.0, abs(o64[b])), (b, o32[b], o64[b])
        else:
            np.testing.assert_allclose(f32[b], f64[b], rtol=1e-9, atol=1e-9 * np.abs(f64[b]).max())


def test_philox_known_answers_on_device(nat):
    """The device Philox4x32-10 round function (ugemm.hip) against the published known-answer
    vectors and the oracle on random blocks (bit-exact, integer arithmetic)."""
    blocks = np.array([inp for inp, _ in orc.PHILOX_KAT], dtype=np.uint32)
    out = nat.selftest_philox(blocks)
    np.testing.assert_array_equal(out, np.array([o for _, o in orc.PHILOX_KAT], dtype=np.uint32))
    rnd = np.random.RandomState(3).randint(0, 2 ** 32, size=(1000, 6), dtype=np.uint64)
    np.testing.assert_array_equal(nat.selftest_philox(rnd.astype(np.uint32)),
                                  orc.philox4x32_10(rnd[:, :4], rnd[:, 4:]))


def test_u_normal_matches_philox_box_muller(nat):
    """apm_u_normal's draws for (seed, counter) are the Box-Muller transform of that Philox
    stream (oracle.u_normal, float64) to fp32 transcendental accuracy."""
    c = _cases()[2]
    ctx = _ctx(nat, c)
    n, s = c['ns1'].shape
    seeds = [123, 2 ** 63 + 12345]
    ctrs = [0, 2 ** 33 + 5]
    ctx.u_normal([0, 1], seeds, ctrs)
    for b in range(2):
        ref = orc.u_normal(seeds[b], ctrs[b], n, s)
        np.testing.assert_allclose(ctx.u_download(b), ref, rtol=2e-6, atol=2e-6)
    ctx.close()
