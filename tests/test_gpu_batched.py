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
        assert abs(smp.log_f[c] - (v + lp)) < 2e-3 + 2e-5 * abs(v), (c, smp.log_f[c], v + lp)
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
