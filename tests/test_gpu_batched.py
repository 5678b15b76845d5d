"""GPU: the lockstep batched APM E-SS + RD-SS driver keeps a consistent per-chain state
(the cached slot, u buffer and log f always describe the current point) and is reproducible."""
import numpy as np
import pytest

import apm_oracle as orc

pytestmark = pytest.mark.gpu


def _sampler(seed=3, chains=3, n=150, d=4, s=16, max_steps_out=0):
    from auxpm.batched import BatchedAPMEllSSPlusRandDirSliceSampler
    from gpdemo.utils import synthetic_gp_data
    X, y = synthetic_gp_data(n, d, 5)
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    return X, y, prior, BatchedAPMEllSSPlusRandDirSliceSampler(
        X, y, chains, s, prior, seed=seed, max_steps_out=max_steps_out)


def test_batched_state_consistent_with_oracle(gpu_available):
    X, y, prior, smp = _sampler()
    th = smp.run(4)
    assert np.isfinite(th).all() and not smp.failed.any()
    kf = orc.make_kernel_func('ard', 1e-8)
    for c in range(smp.n_chains):
        U = smp.ctx.u_download(smp.ub_u[c])  # the fp32 draws the device used
        v, _, _ = orc.is_estimate(X, y, kf, U, smp.theta[c])
        lp = sum(orc.log_gamma_log_pdf(smp.theta[c][k], prior['a_tau'] if k else prior['a_sigma'],
                                       prior['b_tau'] if k else prior['b_sigma'])
                 for k in range(smp.P))
        assert abs(smp.log_f[c] - (v + lp)) < 5e-4, (c, smp.log_f[c], v + lp)
        out, st = smp.ctx.u_eval([smp.slot_cur[c]], [smp.ub_u[c]])
        assert abs(out[0] + lp - smp.log_f[c]) < 1e-9 * max(1, abs(out[0]))


def test_batched_reproducible_and_step_out(gpu_available):
    _, _, _, a = _sampler(seed=11)
    _, _, _, b = _sampler(seed=11)
    np.testing.assert_array_equal(a.run(3), b.run(3))
    _, _, _, c = _sampler(seed=12, max_steps_out=2)
    th = c.run(3)
    assert np.isfinite(th).all()


@pytest.mark.parametrize('max_steps_out', [0, 2])
def test_async_schedule_equals_lockstep(gpu_available, max_steps_out):
    """Per-chain trajectories do not depend on the schedule: every chain makes the same estimator
    calls with the same host-RNG draws (and device u counters) in the same order."""
    _, _, _, a = _sampler(seed=21, chains=4, max_steps_out=max_steps_out)
    _, _, _, b = _sampler(seed=21, chains=4, max_steps_out=max_steps_out)
    a.initialise()
    lock = np.stack([a.step() for _ in range(3)], 1)
    b.initialise()
    traces, done = b.run_async(3)
    assert (done == 3).all()
    np.testing.assert_array_equal(np.array(traces), lock)
    np.testing.assert_array_equal(a.log_f, b.log_f)
    np.testing.assert_array_equal(a.slot_cur, b.slot_cur)
    # throughput mode: at least 2 transitions each, chains that are ahead go on
    traces2, done2 = b.run_async(2, keep_going=True)
    assert (done2 >= 2).all() and all(len(t) == d for t, d in zip(traces2, done2))


def test_checkpoint_restore_continues_bitwise(gpu_available, tmp_path):
    """checkpoint() at a transition boundary, saved with numpy.savez and restored into a fresh
    sampler (u rebuilt on the device from its history), continues every chain bit for bit."""
    _, _, _, a = _sampler(seed=41, chains=4)
    a.initialise()
    a.run_async(3)
    np.savez(tmp_path / 'ck.npz', **a.checkpoint())
    tr_a, _ = a.run_async(3)
    _, _, _, b = _sampler(seed=41, chains=4)
    with np.load(tmp_path / 'ck.npz') as z:
        dlogf = b.restore({k: z[k] for k in z.files})
    assert dlogf == 0.
    tr_b, _ = b.run_async(3)
    np.testing.assert_array_equal(np.array(tr_a), np.array(tr_b))
    np.testing.assert_array_equal(a.log_f, b.log_f)
    for c in range(4):
        np.testing.assert_array_equal(a.ctx.u_download(a.ub_u[c]), b.ctx.u_download(b.ub_u[c]))


def _data(n=150, d=4, kind='ard'):
    from gpdemo.utils import synthetic_gp_data
    X, y = synthetic_gp_data(n, d, 5, kind)
    prior = dict(a_tau=1., b_tau=1. / d ** 0.5, a_sigma=1.1, b_sigma=0.1)
    return X, y, prior


def _current_state_consistent(smp, X, y, prior, kind='ard'):
    """log f of every live chain = u-call at its current (slot, u) + prior, and the oracle's
    estimate on the same (theta, fp32 u) within the estimator tolerance."""
    kf = orc.make_kernel_func(kind, 1e-8)
    for c in np.flatnonzero(~smp.failed):
        lp = smp.log_prior(smp.theta[c][None])[0]
        out, st = smp.ctx.u_eval([smp.slot_cur[c]], [smp.ub_u[c]])
        assert st[0] == 0 and abs(out[0] + lp - smp.log_f[c]) < 1e-9 * max(1, abs(out[0]))
        v, _, _ = orc.is_estimate(X, y, kf, smp.ctx.u_download(smp.ub_u[c]), smp.theta[c])
        assert abs(smp.log_f[c] - (v + lp)) < 5e-4, (c, smp.log_f[c], v + lp)


def test_batched_ess_mh_consistent_and_batch_invariant(gpu_available):
    """configs[1]'s sampler (APMEllSSPlusMHSampler, samplers.py:421-585) batched: consistent
    current state (cache slot, u, log f), accepted moves, and every chain's trajectory equal
    bit for bit to the same chain run alone (first_chain): batch composition changes nothing."""
    from auxpm.batched import BatchedAPMEllSSPlusMHSampler
    X, y, prior = _data()
    th0 = np.tile(np.r_[0.0, np.full(4, np.log(2.))], (4, 1))
    smp = BatchedAPMEllSSPlusMHSampler(X, y, 4, 16, prior, prop_scales=0.1, seed=31)
    th, nrej = smp.get_samples(6, th0)
    assert np.isfinite(th).all() and not smp.failed.any()
    assert (nrej < 5).any()  # some chain accepted moves
    _current_state_consistent(smp, X, y, prior)
    one = BatchedAPMEllSSPlusMHSampler(X, y, 1, 16, prior, prop_scales=0.1, seed=31,
                                       first_chain=2)
    th1, nrej1 = one.get_samples(6, th0[2:3])
    np.testing.assert_array_equal(th1[0], th[2])
    assert nrej1[0] == nrej[2]
    # adaptive phase: per-chain scales follow the accept rates
    ath, sc, rates = smp.adaptive_run(th[:, -1], 4, 2, 0.15, 0.30,
                                      lambda b, n: 1.5)
    assert ath.shape == (4, 8, smp.P) and sc.shape == (4, 2, smp.P)
    for c in range(4):
        f0 = 1.5 if rates[c, 0] > 0.30 else (1 / 1.5 if rates[c, 0] < 0.15 else 1.)
        np.testing.assert_allclose(sc[c, 0], 0.1 * f0)


def test_batched_pmmh_laplace_phase_matches_api_sampler(gpu_available):
    """configs[0]'s PM-MH protocol batched: the deterministic Laplace-estimator adaptive phase
    reproduces, chain by chain and bit for bit, the API-compatible PMMHSampler driven by the GPU
    Laplace estimator with that chain's RandomState (same proposal / uniform draw order)."""
    import auxpm.samplers as smp_api
    import gpdemo.estimators as est
    import gpdemo.kernels as krn
    import gpdemo.utils as utils
    from auxpm.batched import BatchedPMMHSampler, chain_streams
    X, y, prior = _data(200, 3, 'iso')
    C = 3
    th0 = np.array([[0.5, 0.3], [1.0, 0.8], [-0.2, 0.6]])
    b = BatchedPMMHSampler(X, y, C, 1, prior, prop_scales=[0.5, 0.5], kernel='iso', seed=9,
                           estimator='laplace')
    ath, sc, rates = b.adaptive_run(th0, 5, 2, 0.15, 0.30, utils.adapt_factor_func)
    det = est.LogMarginalLikelihoodLaplaceEstimator(X, y, krn.make_kernel_func('iso', 1e-8))
    prngs, _ = chain_streams(9, C)

    for c in range(C):
        prng = prngs[c]

        def log_f(theta):
            return det(theta) + (utils.log_gamma_log_pdf(theta[0], prior['a_sigma'],
                                                         prior['b_sigma']) +
                                 utils.log_gamma_log_pdf(theta[1], prior['a_tau'], prior['b_tau']))
        api = smp_api.PMMHSampler(
            log_f, lambda tp, tc, s: -0.5 * np.sum(((tp - tc) / s) ** 2),
            lambda t, s: t + s * prng.normal(size=t.shape), np.array([0.5, 0.5]), prng)
        a_th, a_sc, a_rates = api.adaptive_run(th0[c], 5, 2, 0.15, 0.30, utils.adapt_factor_func)
        np.testing.assert_array_equal(ath[c], a_th)
        np.testing.assert_array_equal(sc[c], a_sc)
        np.testing.assert_array_equal(rates[c], a_rates)
    # main phase: IS estimator, N_imp = 1, fresh device u per proposal; consistent state
    b.set_estimator('is')
    th, nrej = b.get_samples(6, ath[:, -1])
    assert np.isfinite(th).all() and not b.failed.any()
    _current_state_consistent(b, X, y, prior, 'iso')
    # batch invariance of the IS phase (fresh samplers: same streams for chain 1 alone)
    b2 = BatchedPMMHSampler(X, y, C, 1, prior, prop_scales=[0.3, 0.3], kernel='iso', seed=10)
    th2, nrej2 = b2.get_samples(6, th0)
    one = BatchedPMMHSampler(X, y, 1, 1, prior, prop_scales=[0.3, 0.3], kernel='iso', seed=10,
                             first_chain=1)
    th1, nrej1 = one.get_samples(6, th0[1:2])
    np.testing.assert_array_equal(th1[0], th2[1])
    assert nrej1[0] == nrej2[1]


def test_batched_mi_rdss_consistent_batch_invariant_and_async(gpu_available, tmp_path):
    """APMMetIndPlusRandDirSliceSampler (samplers.py:926-1004) batched: consistent current state
    against the oracle, async == lockstep bit for bit, each chain's trajectory independent of
    its batch (first_chain), and checkpoint / restore replaying the accepted MI draws."""
    from auxpm.batched import BatchedAPMMetIndPlusRandDirSliceSampler as S
    X, y, prior = _data()
    a = S(X, y, 4, 16, prior, seed=51)
    b = S(X, y, 4, 16, prior, seed=51)
    a.initialise()
    lock = np.stack([a.step() for _ in range(4)], 1)
    assert not a.failed.any()
    assert (a.n_reject_u < 4).any() and (a.n_reject_u > 0).any()  # MI moves accepted / rejected
    _current_state_consistent(a, X, y, prior)
    b.initialise()
    traces, done = b.run_async(4)
    np.testing.assert_array_equal(np.array(traces), lock)
    np.testing.assert_array_equal(a.log_f, b.log_f)
    np.testing.assert_array_equal(a.n_reject_u, b.n_reject_u)
    one = S(X, y, 1, 16, prior, seed=51, first_chain=3)
    one.initialise()  # chain 3's own stream: the same prior draw
    tr1, _ = one.run_async(3)
    np.testing.assert_array_equal(np.array(tr1[0]), lock[3, 0:3])
    np.savez(tmp_path / 'ck.npz', **a.checkpoint())
    ta, _ = a.run_async(2)
    c = S(X, y, 4, 16, prior, seed=51)
    with np.load(tmp_path / 'ck.npz') as z:
        assert c.restore({k: z[k] for k in z.files}) == 0.
    tc, _ = c.run_async(2)
    np.testing.assert_array_equal(np.array(ta), np.array(tc))


def test_batched_mi_mh_consistent_and_batch_invariant(gpu_available):
    """APMMetIndPlusMHSampler (samplers.py:265-418) batched: (n_reject_u, n_reject_theta) per
    chain like the reference's tuple, consistent state, batch invariance, and the adaptive run
    driven by the theta rejections (reject_count_index=1)."""
    from auxpm.batched import BatchedAPMMetIndPlusMHSampler as S
    X, y, prior = _data()
    th0 = np.tile(np.r_[0.0, np.full(4, np.log(2.))], (4, 1))
    smp = S(X, y, 4, 16, prior, prop_scales=0.1, seed=61)
    th, (nru, nrt) = smp.get_samples(6, th0)
    assert np.isfinite(th).all() and not smp.failed.any()
    assert (nru < 5).any() and (nrt < 5).any()
    _current_state_consistent(smp, X, y, prior)
    one = S(X, y, 1, 16, prior, prop_scales=0.1, seed=61, first_chain=1)
    th1, (nru1, nrt1) = one.get_samples(6, th0[1:2])
    np.testing.assert_array_equal(th1[0], th[1])
    assert nru1[0] == nru[1] and nrt1[0] == nrt[1]
    with pytest.raises(ValueError):  # a falsy index (the reference ignores 0)
        smp.adaptive_run(th[:, -1], 3, 1, 0.15, 0.30, lambda b, n: 1.5, reject_count_index=0)
    # the reference's default -1 adapts on the last count, the theta step (samplers.py:70, 143)
    ath, sc, rates = smp.adaptive_run(th[:, -1], 4, 2, 0.15, 0.30, lambda b, n: 1.5)
    assert ath.shape == (4, 8, smp.P) and sc.shape == (4, 2, smp.P)
    twin = S(X, y, 4, 16, prior, prop_scales=0.1, seed=61)  # the same calls, explicit index
    twin.get_samples(6, th0)
    with pytest.raises(ValueError):  # (its first batch ran before the index was looked at)
        twin.adaptive_run(th[:, -1], 3, 1, 0.15, 0.30, lambda b, n: 1.5, reject_count_index=0)
    ath1, sc1, rates1 = twin.adaptive_run(th[:, -1], 4, 2, 0.15, 0.30, lambda b, n: 1.5,
                                          reject_count_index=1)
    np.testing.assert_array_equal(rates1, rates)
    np.testing.assert_array_equal(ath1, ath)


def test_run_async_finish_mode_ends_on_boundaries(gpu_available, tmp_path):
    """keep_going='finish' (tools/ess_long.py's throughput mode): chains that are ahead keep
    working until the slowest has n_steps, then every transition in progress is completed - so
    each chain ends at a transition boundary (>= n_steps transitions, traces = done) and a
    checkpoint taken there continues bit for bit."""
    _, _, _, a = _sampler(seed=71, chains=4)
    a.initialise()
    tr, done = a.run_async(3, keep_going='finish')
    assert (done >= 3).all() and all(len(t) == d for t, d in zip(tr, done))
    for c in range(4):
        np.testing.assert_array_equal(tr[c][-1], a.theta[c])
    np.savez(tmp_path / 'ck.npz', **a.checkpoint())
    ta, da = a.run_async(2)
    _, _, _, b = _sampler(seed=71, chains=4)
    with np.load(tmp_path / 'ck.npz') as z:
        assert b.restore({k: z[k] for k in z.files}) == 0.
    tb, db = b.run_async(2)
    np.testing.assert_array_equal(np.array(ta), np.array(tb))
    # u carried by the checkpoint itself (store_u): the replay history restarts there, the
    # rejection counters travel, and the continuation is the same bit for bit
    ck = a.checkpoint(store_u=True)
    assert 'u' in ck and ck['ulog_n'].sum() == 0 and 'n_reject_u' in ck
    np.savez(tmp_path / 'cku.npz', **ck)
    ta2, _ = a.run_async(2)
    _, _, _, c = _sampler(seed=71, chains=4)
    with np.load(tmp_path / 'cku.npz') as z:
        assert c.restore({k: z[k] for k in z.files}) == 0.
    tc2, _ = c.run_async(2)
    np.testing.assert_array_equal(np.array(ta2), np.array(tc2))
    assert 'u' in c.checkpoint()  # later checkpoints keep carrying u (store_u=None)
    with pytest.raises(ValueError):  # a replay checkpoint cannot start from a snapshot
        c.checkpoint(store_u=False)


def test_batched_mi_seqslice_consistent_and_batch_invariant(gpu_available):
    """APMMetIndPlusSeqSliceSampler (samplers.py:844-923) batched: an axis-by-axis linear slice
    step per transition after the MI u-update; consistent state against the oracle, every
    chain's trajectory independent of its batch, and theta moving along every axis."""
    from auxpm.batched import BatchedAPMMetIndPlusSeqSliceSampler as S
    X, y, prior = _data()
    a = S(X, y, 3, 16, prior, ws=0.5, seed=81, max_steps_out=1)
    th = a.run(3)
    assert np.isfinite(th).all() and not a.failed.any()
    assert (np.abs(np.diff(th, axis=1)) > 0).any(axis=(0, 1)).all()  # every axis moved
    _current_state_consistent(a, X, y, prior)
    one = S(X, y, 1, 16, prior, ws=0.5, seed=81, max_steps_out=1, first_chain=2)
    np.testing.assert_array_equal(one.run(3)[0], th[2])


def test_batched_ellss_ellss_consistent_and_batch_invariant(gpu_available):
    """APMEllSSPlusEllSSSampler (samplers.py:1092-1165) batched: E-SS on u and on theta under a
    zero-mean Gaussian prior that the log target excludes; consistent state (log f = the
    estimate alone), batch invariance, and lockstep step() == the asynchronous schedule."""
    from auxpm.batched import BatchedAPMEllSSPlusEllSSSampler as S
    X, y, _ = _data()
    a = S(X, y, 3, 16, theta_prior_std=1.0, seed=91)
    th = a.run(4)
    assert np.isfinite(th).all() and not a.failed.any()
    assert np.array_equal(a.lp_cur, np.zeros(3))
    kf = orc.make_kernel_func('ard', 1e-8)
    for c in range(3):
        out, st = a.ctx.u_eval([a.slot_cur[c]], [a.ub_u[c]])
        assert st[0] == 0 and abs(out[0] - a.log_f[c]) < 1e-9 * max(1, abs(out[0]))
        v, _, _ = orc.is_estimate(X, y, kf, a.ctx.u_download(a.ub_u[c]), a.theta[c])
        assert abs(a.log_f[c] - v) < 5e-4
    one = S(X, y, 1, 16, theta_prior_std=1.0, seed=91, first_chain=1)
    np.testing.assert_array_equal(one.run(4)[0], th[1])
    b = S(X, y, 3, 16, theta_prior_std=1.0, seed=91)
    b.initialise()
    lock = np.stack([b.step() for _ in range(3)], 1)
    np.testing.assert_array_equal(lock, th[:, 1:])
