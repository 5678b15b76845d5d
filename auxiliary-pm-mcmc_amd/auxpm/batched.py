# -*- coding: utf-8 -*-
"""Many independent APM / PM chains advanced together on one MI355X.

Three batched twins of the reference samplers share one device context, the per-chain random
streams and the masked-failure bookkeeping (``_BatchedChains``):

* ``BatchedAPMEllSSPlusRandDirSliceSampler`` — ``APMEllSSPlusRandDirSliceSampler`` (reference
  samplers.py:1007-1089; elliptical slice sampling on u, random-direction linear slice sampling
  on theta; mcmc_updates.py:311-400, :403-519; BASELINE configs[2]/[3]). Two schedules:
  ``step()`` lockstep (each shrink round of every still-undecided chain is one batched call) and
  ``run(...)`` / ``run_async(...)`` asynchronous (every round issues ONE batched theta-call for
  all chains whose slice step needs an evaluation, after completing with cheap batched u-calls
  the elliptical slice update of every chain that has just finished a transition).
* ``BatchedAPMEllSSPlusMHSampler`` — ``APMEllSSPlusMHSampler`` (samplers.py:421-585;
  BASELINE configs[1]): E-SS on u (batched u-calls), then one Metropolis(-Hastings) theta step
  per chain — exactly one theta-call per transition, so every theta-call carries the whole batch
  in lockstep; proposal/current cache slots as samplers.py:563-584 (the proposal's slot becomes
  current on accept).
* ``BatchedPMMHSampler`` — ``PMMHSampler`` (samplers.py:159-262; BASELINE configs[0] protocol,
  Pseudo-Marginal MH.ipynb cells 12-14): one batched theta-call per iteration at the proposals,
  with the Laplace estimator (adaptive phase) or the IS estimator on fresh u (main phase).
* ``BatchedAPMMetIndPlusRandDirSliceSampler`` / ``BatchedAPMMetIndPlusMHSampler`` —
  ``APMMetIndPlusRandDirSliceSampler`` (samplers.py:926-1004 over the MI + SS base
  :588-710) and ``APMMetIndPlusMHSampler`` (:265-418): the same theta updates, with u updated
  by a Metropolis independence step (mcmc_updates.py:159-303: a fresh u from the device, one
  batched u-call against the current cache, accept iff U < exp(log f' - log f)).
* ``BatchedAPMMetIndPlusSeqSliceSampler`` — ``APMMetIndPlusSeqSliceSampler`` (:844-923): MI on
  u, then a linear slice step along each theta axis in turn (widths ``ws``).
* ``BatchedAPMEllSSPlusEllSSSampler`` — ``APMEllSSPlusEllSSSampler`` (:1092-1165): E-SS on u and
  E-SS on theta under a zero-mean Gaussian prior (``theta_prior_std``; the log target is the
  estimate alone, as the reference's estimator there excludes that prior).

Per chain the control flow, the cache protocol and the host-RNG draw order are those of the
reference (one ``numpy.random.RandomState`` per chain for slice heights, angles, offsets,
directions, proposals and accept uniforms). Each chain's streams depend only on (seed, chain
index) (``chain_streams``), and every device kernel computes each chain independently of the
others in its batch, so a chain's trajectory does not depend on the batch it runs in
(tests/test_gpu_batched.py). The auxiliary draws u and nu live on the device: Philox4x32-10
(one counter stream per chain) and the E-SS proposal u cos(phi) + nu sin(phi) is formed on the
device, so trajectories are statistically — not bitwise — equivalent to a numpy-u_sampler run
(DESIGN.md §6). The log target is estimator + log-Gamma prior (E-SS+RD-SS.ipynb:167-173), the
tau prior applied to every ARD length-scale (gpdemo.utils.log_prior_ard).
"""
import time
import warnings

import numpy as np

from gpdemo import _native
from gpdemo.utils import log_prior_ard_batch

__all__ = ['BatchedAPMEllSSPlusRandDirSliceSampler', 'BatchedAPMEllSSPlusMHSampler',
           'BatchedPMMHSampler', 'BatchedAPMMetIndPlusRandDirSliceSampler',
           'BatchedAPMMetIndPlusMHSampler', 'BatchedAPMMetIndPlusSeqSliceSampler',
           'BatchedAPMEllSSPlusEllSSSampler', 'chain_streams']

_EST = {'is': _native.EST_IS, 'priormc': _native.EST_PRIORMC, 'laplace': _native.EST_LAPLACE}


def chain_streams(seed, n_chains, first_chain=0):
    """Per-chain random streams: chain c gets numpy.random.SeedSequence(seed, spawn_key=(c,)) —
    the c-th child of SeedSequence(seed).spawn(...), whatever the batch size — which seeds a
    host RandomState (MT19937; slice heights, angles, directions, proposals, accept uniforms)
    and a 64-bit Philox4x32-10 key for its device draws (u, nu). Different `seed`s (bench.py
    derives one per rank) give statistically independent, non-overlapping streams."""
    kids = [np.random.SeedSequence(seed, spawn_key=(first_chain + c,)) for c in range(n_chains)]
    prngs = [np.random.RandomState(np.random.MT19937(k)) for k in kids]
    dev_seeds = np.array([k.generate_state(2, np.uint64)[0] for k in kids], dtype=np.uint64)
    return prngs, dev_seeds


class _BatchedChains(object):
    """Device context, per-chain streams and state shared by the batched samplers.

    Buffers per chain: cache slots ``slot_cur`` / ``slot_prop`` (samplers.py:563-584: the
    current state's cache and the proposal's), u buffers ``ub_u`` (current u), ``ub_nu`` (E-SS
    auxiliary draw) and ``ub_prop`` (proposed u)."""

    def __init__(self, X, y, n_chains, n_imp, prior, kernel='ard', epsilon=1e-8,
                 max_slice_iters=1000, seed=0, estimator='is', device=None, first_chain=0):
        self.n_chains = int(n_chains)
        self.n_imp = int(n_imp)
        self.prior = dict(prior)
        self.max_slice_iters = int(max_slice_iters)
        self.est = _EST[estimator]
        kind = _native.KERNEL_ARD if kernel == 'ard' else _native.KERNEL_ISO
        C = self.n_chains
        self.ctx = _native.Context(X, y, kind, epsilon, n_imp, max_batch=C, n_slots=2 * C,
                                   n_ubufs=3 * C, device=device)
        self.P = self.ctx.theta_len
        self.slot_cur = np.arange(C, dtype=np.int64)
        self.slot_prop = np.arange(C, 2 * C, dtype=np.int64)
        self.ub_u = np.arange(C, dtype=np.int64)
        self.ub_nu = np.arange(C, 2 * C, dtype=np.int64)
        self.ub_prop = np.arange(2 * C, 3 * C, dtype=np.int64)
        self.prngs, self.dev_seeds = chain_streams(seed, C, first_chain)
        self.dev_ctr = np.zeros(C, dtype=np.uint64)
        self.theta = np.zeros((C, self.P))
        self.log_f = np.full(C, -np.inf)
        self.lp_cur = np.zeros(C)  # log prior of the current theta (constant during the u-update)
        self.failed = np.zeros(C, dtype=bool)
        self.fail_status = np.zeros(C, dtype=np.int32)
        self.n_theta_calls = 0
        self.n_u_calls = 0
        self.n_cubic_ops = np.zeros(C, dtype=np.int64)
        # wall seconds inside the device calls (the rest of a run is host-side sampler logic)
        self.wall = {'theta_call': 0., 'u_call': 0., 'u_draw': 0.}
        # per theta-call: (max, mean) over its chains of the cubic-op count (IS: Newton
        # iterations + 3) - the call's wall time follows the max, its work the mean
        self.call_ops = []
        # u history for checkpoint / resume (``checkpoint`` / ``restore``): the Philox counter
        # of the initial draw and, per chain, (counter of nu, cos phi, sin phi) of every
        # accepted elliptical-slice move — u is a deterministic function of these
        self.u_init_ctr = np.zeros(C, dtype=np.uint64)
        self.u_log = [[] for _ in range(C)]
        # set once a checkpoint has carried u itself (checkpoint(store_u=True)): the history
        # then starts at that snapshot, so every later checkpoint carries u too
        self.u_snapshot = False
        self.n_reject_u = np.zeros(C, dtype=np.int64)  # Metropolis independence u-updates

    # ------------------------------------------------------------------ helpers
    def log_prior(self, thetas):
        return log_prior_ard_batch(thetas, self.prior)

    def _normals(self, idx, bufs):
        t0 = time.perf_counter()
        self.ctx.u_normal(bufs[idx], self.dev_seeds[idx], self.dev_ctr[idx])
        self.wall['u_draw'] += time.perf_counter() - t0
        self.dev_ctr[idx] += 1

    def _theta_eval(self, idx, thetas, slots, ubufs=None):
        """Batched theta-call; returns (log target, log prior) of each proposal."""
        t0 = time.perf_counter()
        ub = self.ub_u[idx] if ubufs is None else ubufs
        if self.est == _native.EST_LAPLACE:
            out, st, nops = self.ctx.theta_eval(self.est, thetas)
        else:
            out, st, nops = self.ctx.theta_eval(self.est, thetas, ub, slots)
        self.wall['theta_call'] += time.perf_counter() - t0
        self.n_theta_calls += len(idx)
        self.n_cubic_ops[idx] += nops
        self.call_ops.append((int(nops.max()), float(nops.mean())))
        bad = st != 0
        if bad.any():
            self.failed[idx[bad]] = True
            self.fail_status[idx[bad]] = st[bad]
            out = np.where(bad, -np.inf, out)
        lp = self.log_prior(thetas)
        return out + lp, lp

    def prior_draw(self):
        """theta_init ~ prior per chain, drawn with each chain's RandomState
        (E-SS+RD-SS.ipynb:198-201, extended to every ARD length-scale)."""
        th = np.empty((self.n_chains, self.P))
        for c, rng in enumerate(self.prngs):
            th[c, 0] = np.log(rng.gamma(self.prior['a_sigma'], 1. / self.prior['b_sigma']))
            th[c, 1:] = np.log(rng.gamma(self.prior['a_tau'], 1. / self.prior['b_tau'],
                                         size=self.P - 1))
        return th

    def initialise(self, theta_init=None):
        """u ~ N(0, I) on the device and the first theta-call (reference samplers.py:825-827)."""
        idx = np.arange(self.n_chains)
        self.theta = self.prior_draw() if theta_init is None else np.array(theta_init, float)
        self.u_init_ctr = self.dev_ctr.copy()
        self.u_log = [[] for _ in range(self.n_chains)]
        self.u_snapshot = False
        self._normals(idx, self.ub_u)
        self.log_f, self.lp_cur = self._theta_eval(idx, self.theta, self.slot_cur[idx])
        return self.theta.copy()

    # ------------------------------------------------------------------ checkpoint / resume
    def checkpoint(self, store_u=None):
        """Chain state at a transition boundary as a dict of numpy arrays (``numpy.savez``-able,
        no pickles): theta, log f, log prior, failure flags, rejection counts, device counters,
        each chain's RandomState (MT19937 key and position, cached Gaussian) and the u history.

        Two forms, chosen by ``store_u``:
        * compact (``False``; the default until a snapshot is taken): u itself (N x N_imp fp64 per
          chain) is not stored; ``restore`` rebuilds it on the device from the Philox draws and
          accepted moves since initialisation, bit for bit - a replay that grows with the chain.
          No side effects.
        * snapshot (``True``): u is downloaded (fp64, exact: the device's fp32 mirror is the
          rounding of those values, so an upload restores both bit for bit) and the history
          restarts at this snapshot, so restore time and u-log size stop growing. That restart is
          a side effect on the sampler: the replay base is now this snapshot, which the compact
          form cannot express, so after a snapshot ``store_u=None`` (the default) takes a
          snapshot again and ``store_u=False`` raises ValueError.
        """
        C = self.n_chains
        if store_u is None:
            store_u = self.u_snapshot
        if not store_u and self.u_snapshot:
            raise ValueError('the u history restarts at the last u snapshot: a compact (replay) '
                             'checkpoint cannot rebuild u from it; pass store_u=True or None')
        if store_u:
            u = np.zeros((C, self.ctx.n, self.n_imp))
            for c in np.flatnonzero(~self.failed):
                u[c] = self.ctx.u_download(self.ub_u[c])
            self.u_log = [[] for _ in range(C)]
            self.u_snapshot = True
        keys = np.empty((C, 624), dtype=np.uint32)
        pos = np.empty(C, dtype=np.int64)
        has_g = np.empty(C, dtype=np.int64)
        gauss = np.empty(C)
        for c, rng in enumerate(self.prngs):
            _, key, p, hg, g = rng.get_state(legacy=True)
            keys[c], pos[c], has_g[c], gauss[c] = key, p, hg, g
        n_log = np.array([len(l) for l in self.u_log], dtype=np.int64)
        flat = [r for l in self.u_log for r in l]
        ulog_ctr = np.array([r[0] for r in flat], dtype=np.uint64)
        ulog_cs = np.array([[r[1], r[2]] for r in flat], dtype=np.float64).reshape(-1, 2)
        ck = dict(theta=self.theta.copy(), log_f=self.log_f.copy(), lp_cur=self.lp_cur.copy(),
                  failed=self.failed.copy(), fail_status=self.fail_status.copy(),
                  dev_seeds=self.dev_seeds.copy(), dev_ctr=self.dev_ctr.copy(),
                  rng_key=keys, rng_pos=pos, rng_has_gauss=has_g, rng_gauss=gauss,
                  u_init_ctr=self.u_init_ctr.copy(), ulog_n=n_log, ulog_ctr=ulog_ctr,
                  ulog_cs=ulog_cs, n_reject_u=self.n_reject_u.copy())
        if hasattr(self, 'n_reject'):  # the MH twins' theta rejections
            ck['n_reject'] = np.asarray(self.n_reject).copy()
        if self.u_snapshot:
            ck['u'] = u
        return ck

    def restore(self, ck):
        """Resume from ``checkpoint()`` output (same X, y, chains and seed): host state back,
        u rebuilt on the device by replaying its draws and accepted moves, then one theta-call
        at each live chain's current theta refills its cache slot. Returns the largest
        |log f (recomputed) - log f (saved)| over live chains (0 on a deterministic device)."""
        C = self.n_chains
        if not np.array_equal(np.asarray(ck['dev_seeds'], np.uint64), self.dev_seeds):
            raise ValueError('checkpoint belongs to different chain streams (seed / chains)')
        self.theta = np.array(ck['theta'], dtype=np.float64)
        self.failed = np.array(ck['failed'], dtype=bool)
        self.fail_status = np.array(ck['fail_status'], dtype=np.int32)
        self.dev_ctr = np.array(ck['dev_ctr'], dtype=np.uint64)
        for c, rng in enumerate(self.prngs):
            rng.set_state(('MT19937', np.asarray(ck['rng_key'][c], np.uint32),
                           int(ck['rng_pos'][c]), int(ck['rng_has_gauss'][c]),
                           float(ck['rng_gauss'][c])))
        self.u_init_ctr = np.array(ck['u_init_ctr'], dtype=np.uint64)
        n_log = np.asarray(ck['ulog_n'], dtype=np.int64)
        offs = np.r_[0, np.cumsum(n_log)]
        self.u_log = [[(np.uint64(ck['ulog_ctr'][i]), float(ck['ulog_cs'][i, 0]),
                        float(ck['ulog_cs'][i, 1])) for i in range(offs[c], offs[c + 1])]
                      for c in range(C)]
        if 'n_reject_u' in ck:
            self.n_reject_u = np.array(ck['n_reject_u'], dtype=np.int64)
        if 'n_reject' in ck and hasattr(self, 'n_reject'):
            self.n_reject = np.array(ck['n_reject'], dtype=np.int64)
        idx = np.arange(C)
        self.u_snapshot = 'u' in ck
        if self.u_snapshot:  # u itself (checkpoint(store_u=True)); the history starts there
            for c in idx:
                self.ctx.u_upload(self.ub_u[c], np.asarray(ck['u'][c], dtype=np.float64))
        else:
            self.ctx.u_normal(self.ub_u[idx], self.dev_seeds[idx], self.u_init_ctr[idx])
        for k in range(int(n_log.max()) if C else 0):
            sel = np.flatnonzero(n_log > k)
            rec = [self.u_log[c][k] for c in sel]
            self.ctx.u_normal(self.ub_nu[sel], self.dev_seeds[sel],
                              np.array([r[0] for r in rec], dtype=np.uint64))
            self.ctx.u_combine(self.ub_prop[sel], self.ub_u[sel], self.ub_nu[sel],
                               np.array([r[1] for r in rec]), np.array([r[2] for r in rec]))
            self.ub_u[sel], self.ub_prop[sel] = self.ub_prop[sel].copy(), self.ub_u[sel].copy()
        live = np.flatnonzero(~self.failed)
        self.log_f = np.array(ck['log_f'], dtype=np.float64)
        self.lp_cur = np.array(ck['lp_cur'], dtype=np.float64)
        if live.size == 0:
            return 0.
        saved = self.log_f[live].copy()
        lf, lp = self._theta_eval(live, self.theta[live], self.slot_cur[live])
        self.log_f[live], self.lp_cur[live] = lf, lp
        return float(np.max(np.abs(lf - saved)))

    # ------------------------------------------------------------------ updates
    def _u_update(self, chains=None):
        """The u half of a transition (E-SS here; the MI twins override it)."""
        self._ess_u(chains)

    def _mi_u(self, chains=None):
        """Metropolis independence update of the u of every live chain (or of the given chains)
        (mcmc_updates.py:284-303 with the prior as proposal, as samplers.py:700-705): u' from the
        chain's device stream, one batched u-call against the current cache, then per chain
        accept iff U < exp(log f' - log f) - the reference's draw order. An accepted u' is logged
        for ``restore`` as the combination 0 u + 1 u' (k_u_combine reproduces it bit for bit)."""
        live = np.flatnonzero(~self.failed) if chains is None else \
            np.asarray(chains, dtype=np.int64)[~self.failed[chains]]
        if live.size == 0:
            return
        ctr = self.dev_ctr.copy()
        self._normals(live, self.ub_prop)
        t0 = time.perf_counter()
        out, st = self.ctx.u_eval(self.slot_cur[live], self.ub_prop[live])
        self.wall['u_call'] += time.perf_counter() - t0
        self.n_u_calls += live.size
        lf = np.where(st == 0, out, -np.inf) + self.lp_cur[live]
        with np.errstate(over='ignore'):
            p_acc = np.exp(lf - self.log_f[live])
        for q, c in enumerate(live):
            if self.prngs[c].uniform() < p_acc[q]:
                self.ub_u[c], self.ub_prop[c] = self.ub_prop[c], self.ub_u[c]
                self.log_f[c] = lf[q]
                self.u_log[c].append((ctr[c], 0.0, 1.0))
            else:
                self.n_reject_u[c] += 1

    def _ess_u(self, chains=None):
        """Elliptical slice update of the u of every live chain (or of the given chains),
        mcmc_updates.py:372-400; each shrink round is one batched u-call."""
        live = np.flatnonzero(~self.failed) if chains is None else \
            np.asarray(chains, dtype=np.int64)[~self.failed[chains]]
        if live.size == 0:
            return
        nu_ctr = self.dev_ctr.copy()
        self._normals(live, self.ub_nu)
        log_y = np.empty(self.n_chains)
        phi = np.empty(self.n_chains)
        lo = np.empty(self.n_chains)
        hi = np.empty(self.n_chains)
        for c in live:
            rng = self.prngs[c]
            log_y[c] = self.log_f[c] + np.log(rng.uniform())
            phi[c] = rng.uniform() * 2. * np.pi
            lo[c], hi[c] = phi[c] - 2. * np.pi, phi[c]
        act = live
        it = 0
        while act.size:
            if it >= self.max_slice_iters:
                self.failed[act] = True
                break
            t0 = time.perf_counter()
            cs = np.cos(phi[act]), np.sin(phi[act])
            self.ctx.u_combine(self.ub_prop[act], self.ub_u[act], self.ub_nu[act], cs[0], cs[1])
            out, st = self.ctx.u_eval(self.slot_cur[act], self.ub_prop[act])
            self.wall['u_call'] += time.perf_counter() - t0
            self.n_u_calls += act.size
            lf = np.where(st == 0, out, -np.inf) + self.lp_cur[act]
            keep = []
            for q, c in enumerate(act):
                if lf[q] > log_y[c]:
                    self.ub_u[c], self.ub_prop[c] = self.ub_prop[c], self.ub_u[c]
                    self.log_f[c] = lf[q]
                    self.u_log[c].append((nu_ctr[c], float(cs[0][q]), float(cs[1][q])))
                    continue
                if phi[c] < 0:
                    lo[c] = phi[c]
                elif phi[c] > 0:
                    hi[c] = phi[c]
                else:
                    warnings.warn('Slice collapsed to current value')
                    continue
                phi[c] = lo[c] + self.prngs[c].uniform() * (hi[c] - lo[c])
                keep.append(c)
            act = np.array(keep, dtype=np.int64)
            it += 1


class BatchedAPMEllSSPlusRandDirSliceSampler(_BatchedChains):
    """Batch of APM E-SS(u) + RD-SS(theta) chains on one device.

    Parameters mirror the notebook protocol: ``kernel`` 'ard' | 'iso', ``epsilon`` jitter,
    ``n_imp`` importance samples, slice width ``w`` and ``max_steps_out`` (E-SS+RD-SS.ipynb:64-67),
    ``prior`` the log-Gamma hyper-parameters (a_sigma, b_sigma, a_tau, b_tau).
    """

    def __init__(self, X, y, n_chains, n_imp, prior, kernel='ard', epsilon=1e-8, w=1.,
                 max_steps_out=0, max_slice_iters=1000, seed=0, estimator='is', device=None,
                 first_chain=0):
        super(BatchedAPMEllSSPlusRandDirSliceSampler, self).__init__(
            X, y, n_chains, n_imp, prior, kernel, epsilon, max_slice_iters, seed, estimator,
            device, first_chain)
        self.w = float(w)
        self.max_steps_out = int(max_steps_out)
        C = self.n_chains
        # asynchronous random-direction slice state (one pending theta per chain)
        self._rd_d = np.zeros((C, self.P))
        self._rd_logy = np.zeros(C)
        self._rd_lo = np.zeros(C)
        self._rd_hi = np.zeros(C)
        self._rd_x = np.zeros(C)
        self._rd_mode = np.zeros(C, dtype=np.int64)  # 0: step down, 1: step up, 2: shrink
        self._rd_s = np.zeros(C, dtype=np.int64)
        self._rd_down = np.zeros(C)
        self._rd_up = np.zeros(C)
        self._rd_it = np.zeros(C, dtype=np.int64)
        self._rd_pend = np.zeros((C, self.P))
        # the line of the slice step: theta + x d (axis -1, x_curr = 0) or, for the sequential
        # sampler, theta with component `axis` set to x (x_curr = that component)
        self._rd_axis = np.full(C, -1, dtype=np.int64)
        self._rd_x0 = np.zeros(C)

    def _rdss_theta(self):
        """Random-direction linear slice update of every live chain's theta
        (samplers.py:1071-1089 over mcmc_updates.py:480-519)."""
        live = np.flatnonzero(~self.failed)
        if live.size == 0:
            return
        C = self.n_chains
        d = np.zeros((C, self.P))
        log_y = np.empty(C)
        x_lo = np.empty(C)
        x_hi = np.empty(C)
        for c in live:
            rng = self.prngs[c]
            dd = rng.normal(size=self.P)
            d[c] = dd / dd.dot(dd) ** 0.5
            log_y[c] = np.log(rng.uniform()) + self.log_f[c]
            x_lo[c] = 0. - self.w * rng.uniform()
            x_hi[c] = x_lo[c] + self.w
        if self.max_steps_out > 0:
            self._step_out(live, d, log_y, x_lo, x_hi)
        x_prop = np.empty(C)
        act = live[~self.failed[live]]
        it = 0
        while act.size:
            if it >= self.max_slice_iters:
                self.failed[act] = True
                break
            for c in act:
                x_prop[c] = x_lo[c] + (x_hi[c] - x_lo[c]) * self.prngs[c].uniform()
            th_p = self.theta[act] + x_prop[act, None] * d[act]
            lf, lp = self._theta_eval(act, th_p, self.slot_prop[act])
            keep = []
            for q, c in enumerate(act):
                if lf[q] > log_y[c]:
                    # the accepted call's cache becomes the current one (samplers.py:1079-1086)
                    self.slot_cur[c], self.slot_prop[c] = self.slot_prop[c], self.slot_cur[c]
                    self.theta[c] = th_p[q]
                    self.log_f[c] = lf[q]
                    self.lp_cur[c] = lp[q]
                    continue
                if self.failed[c]:
                    continue
                if x_prop[c] < 0.:
                    x_lo[c] = x_prop[c]
                elif x_prop[c] > 0.:
                    x_hi[c] = x_prop[c]
                else:
                    warnings.warn('Slice collapsed to current value')
                    continue
                keep.append(c)
            act = np.array(keep, dtype=np.int64)
            it += 1

    def _step_out(self, live, d, log_y, x_lo, x_hi):
        """Stepping out (mcmc_updates.py:486-498): split max_steps_out at random, extend each
        end by w while it is inside the slice. Every probe is a theta-call."""
        C = self.n_chains
        down = np.zeros(C)
        up = np.zeros(C)
        for c in live:
            down[c] = np.round(self.prngs[c].uniform() * self.max_steps_out)
            up[c] = self.max_steps_out - down[c]
        for ends, budget, sign in ((x_lo, down, -1.), (x_hi, up, 1.)):
            s = np.zeros(C)
            act = live[(s[live] < budget[live]) & ~self.failed[live]]
            while act.size:
                lf, _ = self._theta_eval(act, self.theta[act] + ends[act, None] * d[act],
                                         self.slot_prop[act])
                inside = log_y[act] < lf
                grow = act[inside]
                ends[grow] += sign * self.w
                s[grow] += 1
                act = grow[s[grow] < budget[grow]]

    def step(self):
        """One lockstep transition (u then theta) of every live chain; returns thetas
        (n_chains, P)."""
        self._u_update()
        self._rdss_theta()
        return self.theta.copy()

    # ------------------------------------------------------------------ asynchronous schedule
    def _theta_begin(self, c):
        """Start the theta half of chain c's transition (the MI / seq / ESS twins override)."""
        self._rd_begin(c)

    def _theta_result(self, c, lf, lp):
        return self._rd_result(c, lf, lp)

    def _rd_begin(self, c):
        """Start chain c's random-direction slice step: the draws of mcmc_updates.py:480-490 in
        the reference order (direction, slice height, bracket offset, step-out split)."""
        rng = self.prngs[c]
        dd = rng.normal(size=self.P)
        self._rd_d[c] = dd / dd.dot(dd) ** 0.5
        self._rd_axis[c] = -1
        self._line_begin(c, 0., self.w)

    def _line_begin(self, c, x0, w):
        """A linear slice step from x0 with bracket width w (mcmc_updates.py:480-490: slice
        height, bracket offset, step-out split, in the reference's draw order)."""
        rng = self.prngs[c]
        self._rd_x0[c] = x0
        self._rd_logy[c] = np.log(rng.uniform()) + self.log_f[c]
        self._rd_lo[c] = x0 - w * rng.uniform()
        self._rd_hi[c] = self._rd_lo[c] + w
        self._rd_s[c] = 0
        self._rd_it[c] = 0
        if self.max_steps_out > 0:
            self._rd_down[c] = np.round(rng.uniform() * self.max_steps_out)
            self._rd_up[c] = self.max_steps_out - self._rd_down[c]
            self._rd_mode[c] = 0
        else:
            self._rd_mode[c] = 2
        self._rd_next(c)

    def _line_point(self, c, x):
        if self._rd_axis[c] < 0:
            return self.theta[c] + x * self._rd_d[c]
        p = self.theta[c].copy()
        p[self._rd_axis[c]] = x
        return p

    def _rd_next(self, c):
        """Set chain c's next theta to evaluate (a step-out probe or a shrink proposal)."""
        if self._rd_mode[c] == 0:
            if self._rd_s[c] < self._rd_down[c]:
                self._rd_pend[c] = self._line_point(c, self._rd_lo[c])
                return
            self._rd_mode[c], self._rd_s[c] = 1, 0
        if self._rd_mode[c] == 1:
            if self._rd_s[c] < self._rd_up[c]:
                self._rd_pend[c] = self._line_point(c, self._rd_hi[c])
                return
            self._rd_mode[c] = 2
        self._rd_x[c] = self._rd_lo[c] + (self._rd_hi[c] - self._rd_lo[c]) * \
            self.prngs[c].uniform()
        self._rd_pend[c] = self._line_point(c, self._rd_x[c])

    def _rd_result(self, c, lf, lp):
        """Consume the estimate lf (log prior lp) at chain c's pending theta; True when the
        transition is done."""
        mode = self._rd_mode[c]
        if mode < 2:  # step out while the bracket end is inside the slice (mcmc_updates.py:491-498)
            if self._rd_logy[c] < lf:
                w = self.w if self._rd_axis[c] < 0 else self.ws[self._rd_axis[c]]
                if mode == 0:
                    self._rd_lo[c] -= w
                else:
                    self._rd_hi[c] += w
                self._rd_s[c] += 1
            else:
                self._rd_mode[c], self._rd_s[c] = mode + 1, 0
            self._rd_next(c)
            return False
        if lf > self._rd_logy[c]:  # accept: the proposal's cache becomes current
            self.slot_cur[c], self.slot_prop[c] = self.slot_prop[c], self.slot_cur[c]
            self.theta[c] = self._rd_pend[c]
            self.log_f[c] = lf
            self.lp_cur[c] = lp
            return True
        if self.failed[c]:
            return True
        x, x0 = self._rd_x[c], self._rd_x0[c]
        if x < x0:
            self._rd_lo[c] = x
        elif x > x0:
            self._rd_hi[c] = x
        else:
            warnings.warn('Slice collapsed to current value')
            return True
        self._rd_it[c] += 1
        if self._rd_it[c] >= self.max_slice_iters:
            self.failed[c] = True
            return True
        self._rd_next(c)
        return False

    def run_async(self, n_steps, keep_going=False, on_round=None):
        """Advance every live chain by at least ``n_steps`` transitions (a number, or one per
        chain) with the asynchronous schedule. keep_going=False: a chain stops after n_steps
        (the call ends with every chain at a transition boundary); True: chains that are ahead
        keep working until the slowest has n_steps (throughput mode; a final partial transition
        is discarded); 'finish': as True, then the transitions in progress are completed, so
        every chain ends at a transition boundary with >= n_steps transitions (throughput mode
        for checkpointed runs). Returns (traces, done): per chain the list of thetas after each
        completed transition and the number of completed transitions. on_round(done): called
        after every batched theta-call (progress reporting)."""
        C = self.n_chains
        n_steps = np.broadcast_to(np.asarray(n_steps, dtype=np.int64), (C,))  # or per chain
        done = np.zeros(C, dtype=np.int64)
        traces = [[] for _ in range(C)]
        need_u = ~self.failed
        in_rd = np.zeros(C, dtype=bool)
        finishing = False
        while True:
            unfinished = (~self.failed) & (done < n_steps)
            if not unfinished.any():
                if keep_going != 'finish':
                    break
                finishing = True  # no new transitions; complete the ones in progress
                if not (in_rd & ~self.failed).any():
                    break
            go = (~self.failed) & (unfinished if not keep_going else True) & (not finishing)
            ess = np.flatnonzero(need_u & go)
            if ess.size:
                self._u_update(ess)
                for c in ess:
                    need_u[c] = False
                    if not self.failed[c]:
                        self._theta_begin(c)
                        in_rd[c] = True
            rd = np.flatnonzero(in_rd & ~self.failed)
            if rd.size == 0:
                break
            lf, lp = self._theta_eval(rd, self._rd_pend[rd], self.slot_prop[rd])
            for q, c in enumerate(rd):
                if self._theta_result(c, lf[q], lp[q]):
                    in_rd[c] = False
                    if not self.failed[c]:
                        done[c] += 1
                        traces[c].append(self.theta[c].copy())
                        need_u[c] = True
            if on_round is not None:
                on_round(done)
        return traces, done

    def run(self, n_steps, theta_init=None, warmup_callback=None):
        """(n_chains, n_steps, P) trace starting at the initial state, asynchronous schedule
        (identical per-chain trajectories to n_steps - 1 lockstep ``step()`` calls)."""
        thetas = np.empty((self.n_chains, n_steps, self.P))
        thetas[:, 0] = self.initialise(theta_init)
        traces, done = self.run_async(n_steps - 1)
        for c in range(self.n_chains):
            k = int(done[c])
            if k:
                thetas[c, 1:1 + k] = np.array(traces[c])
            thetas[c, 1 + k:] = self.theta[c]  # failed chains: frozen at their last state
        return thetas


class _BatchedMHMixin(object):
    """Per-chain Metropolis(-Hastings) decisions of a batch of proposals, in the reference's
    draw order and expressions (mcmc_updates.py:14-156; the notebooks' componentwise Gaussian
    random-walk proposal theta + s * N(0, I) and its log density, e.g. Pseudo-Marginal
    MH.ipynb cell 12). ``prop_scales``: (P,) shared or (n_chains, P) per chain; adapted per
    chain by ``adaptive_run``."""

    def _init_mh(self, prop_scales, metropolis):
        self.prop_scales = np.array(np.broadcast_to(np.asarray(prop_scales, dtype=np.float64),
                                                    (self.n_chains, self.P)))
        self.metropolis = bool(metropolis)
        self.n_reject = np.zeros(self.n_chains, dtype=np.int64)

    def _propose(self, live):
        th = self.theta[live].copy()
        for q, c in enumerate(live):
            th[q] = self.theta[c] + self.prop_scales[c] * self.prngs[c].normal(size=self.P)
        return th

    @staticmethod
    def _log_prop_density(x_to, x_from, s):
        return -0.5 * np.sum(((x_to - x_from) / s) ** 2)

    def _decide(self, live, th_p, lf_p, lp_p, on_accept):
        """accept iff U < exp(log f' - log f) [Metropolis] or the MH ratio (reference
        metropolis_step / met_hastings_step); returns the rejection mask."""
        rej = np.zeros(len(live), dtype=bool)
        for q, c in enumerate(live):
            if self.metropolis:
                p_acc = np.exp(lf_p[q] - self.log_f[c])
            else:
                s = self.prop_scales[c]
                log_q_fwd = self._log_prop_density(th_p[q], self.theta[c], s)
                log_q_bwd = self._log_prop_density(self.theta[c], th_p[q], s)
                p_acc = np.exp(lf_p[q] + log_q_bwd - self.log_f[c] - log_q_fwd)
            if self.prngs[c].uniform() < p_acc:
                self.theta[c] = th_p[q]
                self.log_f[c] = lf_p[q]
                self.lp_cur[c] = lp_p[q]
                on_accept(c)
            else:
                rej[q] = True
                self.n_reject[c] += 1
        return rej

    def get_samples(self, n_sample, theta_init=None):
        """(thetas (n_chains, n_sample, P), n_reject (n_chains,)) from the current state (or a
        fresh start at theta_init), as the reference get_samples (first row = start state);
        failed chains are frozen at their last state."""
        if theta_init is not None or not np.isfinite(self.log_f).any():
            self.initialise(theta_init)
        thetas = np.empty((self.n_chains, n_sample, self.P))
        thetas[:, 0] = self.theta
        self.n_reject[:] = 0
        self.n_reject_u[:] = 0
        for s in range(1, n_sample):
            thetas[:, s] = self.step()
        return thetas, self._rejections()

    def _rejections(self):
        return self.n_reject.copy()

    def adaptive_run(self, theta_init, batch_size, n_batch, low_acc_thr, upp_acc_thr,
                     adapt_factor_func, reject_count_index=-1):
        """BaseAdaptiveMHSampler.adaptive_run (samplers.py:14-156) for every chain: each batch
        restarts get_samples from the previous batch's last state (a fresh estimate there, as
        the reference's get_samples does) and each chain's scales are divided / multiplied by
        adapt_factor_func(b, n_batch) when its batch accept rate is below / above the
        thresholds. Where get_samples returns several rejection counts (MI + MH: u and theta),
        ``reject_count_index`` picks the one the scales drive; as in the reference
        (samplers.py:70, 143-144) it defaults to -1, the last count (the theta step), and a falsy
        index (0, None) leaves the counts unpicked - which the reference then fails on; here that
        raises a ValueError. Returns (thetas (C, n_batch*batch_size, P), scales (C, n_batch, P),
        accept_rates (C, n_batch))."""
        C = self.n_chains
        thetas = np.empty((C, n_batch * batch_size, self.P))
        scales = np.empty((C, n_batch, self.P))
        rates = np.empty((C, n_batch))
        th0 = np.array(theta_init, dtype=np.float64)
        for b in range(n_batch):
            lo, hi = b * batch_size, (b + 1) * batch_size
            thetas[:, lo:hi], n_reject = self.get_samples(batch_size, th0)
            if isinstance(n_reject, tuple):
                if not reject_count_index:
                    raise ValueError('several rejection counts and a falsy reject_count_index '
                                     '(the reference ignores index 0, samplers.py:143): pass -1 '
                                     'or another nonzero index')
                n_reject = n_reject[reject_count_index]
            rates[:, b] = 1. - (n_reject * 1. / batch_size)
            th0 = thetas[:, hi - 1].copy()
            factor = adapt_factor_func(b, n_batch)
            for c in range(C):
                if rates[c, b] < low_acc_thr:
                    self.prop_scales[c] /= factor
                elif rates[c, b] > upp_acc_thr:
                    self.prop_scales[c] *= factor
            scales[:, b] = self.prop_scales
        return thetas, scales, rates


class BatchedAPMEllSSPlusMHSampler(_BatchedMHMixin, _BatchedChains):
    """Batch of APM E-SS(u) + MH(theta) chains (reference APMEllSSPlusMHSampler,
    samplers.py:421-585; BASELINE configs[1]). ``metropolis=False`` uses met_hastings_step with
    the Gaussian proposal density, as the E-SS+MH notebook passes ``log_prop_density``."""

    def __init__(self, X, y, n_chains, n_imp, prior, prop_scales, kernel='ard', epsilon=1e-8,
                 metropolis=False, max_slice_iters=1000, seed=0, estimator='is', device=None,
                 first_chain=0):
        super(BatchedAPMEllSSPlusMHSampler, self).__init__(
            X, y, n_chains, n_imp, prior, kernel, epsilon, max_slice_iters, seed, estimator,
            device, first_chain)
        self._init_mh(prop_scales, metropolis)

    def _mh_theta(self):
        """One batched theta-call at every live chain's proposal (with its current u) into the
        proposal slot; on accept the proposal's slot becomes current (samplers.py:563-584)."""
        live = np.flatnonzero(~self.failed)
        if live.size == 0:
            return
        th_p = self._propose(live)
        lf_p, lp_p = self._theta_eval(live, th_p, self.slot_prop[live])

        def accept(c):
            self.slot_cur[c], self.slot_prop[c] = self.slot_prop[c], self.slot_cur[c]
        self._decide(live, th_p, lf_p, lp_p, accept)

    def step(self):
        """One transition of every live chain (u by E-SS, then theta by MH); returns thetas."""
        self._u_update()
        self._mh_theta()
        return self.theta.copy()


class BatchedPMMHSampler(_BatchedMHMixin, _BatchedChains):
    """Batch of pseudo-marginal MH chains (reference PMMHSampler, samplers.py:159-262; the
    protocol of Pseudo-Marginal MH.ipynb). Every iteration draws each chain's proposal, and with
    the IS estimator a fresh u on the device, and evaluates all proposals in ONE batched
    theta-call; the current state's estimate is recycled. ``set_estimator('laplace')`` gives the
    deterministic Laplace-LML adaptive phase, ``'is'`` the importance-sampling main phase
    (``sampler.log_f_estimator = log_f_estimator_main`` in the notebook)."""

    def __init__(self, X, y, n_chains, n_imp, prior, prop_scales, kernel='iso', epsilon=1e-8,
                 metropolis=False, seed=0, estimator='is', device=None, first_chain=0):
        super(BatchedPMMHSampler, self).__init__(
            X, y, n_chains, n_imp, prior, kernel, epsilon, 1000, seed, estimator, device,
            first_chain)
        self._init_mh(prop_scales, metropolis)

    def set_estimator(self, estimator):
        self.est = _EST[estimator]
        self.log_f[:] = -np.inf  # the next get_samples starts with a fresh estimate

    def initialise(self, theta_init=None):
        """The start state's estimate (PMMHSampler.get_samples: log_f_estimator(theta_init))."""
        idx = np.arange(self.n_chains)
        self.theta = self.prior_draw() if theta_init is None else np.array(theta_init, float)
        if self.est != _native.EST_LAPLACE:
            self._normals(idx, self.ub_u)
        self.log_f, self.lp_cur = self._theta_eval(idx, self.theta, self.slot_cur[idx])
        return self.theta.copy()

    def step(self):
        live = np.flatnonzero(~self.failed)
        if live.size == 0:
            return self.theta.copy()
        th_p = self._propose(live)
        if self.est != _native.EST_LAPLACE:
            self._normals(live, self.ub_prop)  # fresh u for every proposal
        lf_p, lp_p = self._theta_eval(live, th_p, self.slot_prop[live], self.ub_prop[live])

        def accept(c):
            self.slot_cur[c], self.slot_prop[c] = self.slot_prop[c], self.slot_cur[c]
            self.ub_u[c], self.ub_prop[c] = self.ub_prop[c], self.ub_u[c]
        self._decide(live, th_p, lf_p, lp_p, accept)
        return self.theta.copy()


class BatchedAPMMetIndPlusRandDirSliceSampler(BatchedAPMEllSSPlusRandDirSliceSampler):
    """Batch of APM MI(u) + RD-SS(theta) chains (reference APMMetIndPlusRandDirSliceSampler,
    samplers.py:926-1004; get_samples of its base :661-710): ``step()``, ``run`` and
    ``run_async`` as the E-SS twin, the u half of every transition a Metropolis independence
    step (one batched u-call). ``n_reject_u`` counts each chain's rejected u proposals (the
    reference's ``n_reject``)."""

    def _u_update(self, chains=None):
        self._mi_u(chains)


class BatchedAPMMetIndPlusMHSampler(BatchedAPMEllSSPlusMHSampler):
    """Batch of APM MI(u) + MH(theta) chains (reference APMMetIndPlusMHSampler,
    samplers.py:265-418). ``get_samples`` returns (thetas, (n_reject_u, n_reject_theta)) per
    chain like the reference's (n_reject_1, n_reject_2); ``adaptive_run(...,
    reject_count_index=1)`` adapts on the theta step as samplers.py:143-144."""

    def _u_update(self, chains=None):
        self._mi_u(chains)

    def _rejections(self):
        return self.n_reject_u.copy(), self.n_reject.copy()


class BatchedAPMMetIndPlusSeqSliceSampler(BatchedAPMEllSSPlusRandDirSliceSampler):
    """Batch of APM MI(u) + sequential-axis SS(theta) chains (reference
    APMMetIndPlusSeqSliceSampler, samplers.py:844-923): after the Metropolis independence
    u-update, one linear slice step (mcmc_updates.py:403-519) along theta axis j = 0 .. P-1 in
    turn, from x_curr = theta_j with bracket width ws[j], each axis starting from the previous
    axis's state and estimate. Same asynchronous schedule (one batched theta-call per round for
    every chain whose axis step needs an evaluation); ``step()`` is one such transition."""

    def __init__(self, X, y, n_chains, n_imp, prior, ws, kernel='ard', epsilon=1e-8,
                 max_steps_out=0, max_slice_iters=1000, seed=0, estimator='is', device=None,
                 first_chain=0):
        super(BatchedAPMMetIndPlusSeqSliceSampler, self).__init__(
            X, y, n_chains, n_imp, prior, kernel, epsilon, 1., max_steps_out, max_slice_iters,
            seed, estimator, device, first_chain)
        self.ws = np.array(np.broadcast_to(np.asarray(ws, dtype=np.float64), (self.P,)))

    def _u_update(self, chains=None):
        self._mi_u(chains)

    def _theta_begin(self, c):
        self._axis_begin(c, 0)

    def _axis_begin(self, c, j):
        self._rd_axis[c] = j
        self._line_begin(c, self.theta[c, j], self.ws[j])

    def _theta_result(self, c, lf, lp):
        if not self._rd_result(c, lf, lp):
            return False
        j = self._rd_axis[c]
        if self.failed[c] or j + 1 >= self.P:
            return True
        self._axis_begin(c, j + 1)  # the next axis from the state this one left
        return False

    def step(self):
        self.run_async(1)
        return self.theta.copy()


class BatchedAPMEllSSPlusEllSSSampler(BatchedAPMEllSSPlusRandDirSliceSampler):
    """Batch of APM E-SS(u) + E-SS(theta) chains (reference APMEllSSPlusEllSSSampler,
    samplers.py:1092-1165): theta has a zero-mean Gaussian prior with per-component standard
    deviations ``theta_prior_std`` (the reference's theta_sampler draws from it) and the log
    target the estimator sees excludes it (log prior 0 here). The theta update is the elliptical
    slice step of mcmc_updates.py:311-400 with nu = theta_prior_std * N(0, I) from the chain's
    RandomState (drawn first, as samplers.py:1163), on the asynchronous schedule."""

    def __init__(self, X, y, n_chains, n_imp, theta_prior_std, kernel='ard', epsilon=1e-8,
                 max_slice_iters=1000, seed=0, estimator='is', device=None, first_chain=0):
        super(BatchedAPMEllSSPlusEllSSSampler, self).__init__(
            X, y, n_chains, n_imp, {}, kernel, epsilon, 1., 0, max_slice_iters, seed, estimator,
            device, first_chain)
        self.theta_prior_std = np.array(np.broadcast_to(
            np.asarray(theta_prior_std, dtype=np.float64), (self.P,)))
        C = self.n_chains
        self._el_v = np.zeros((C, self.P))
        self._el_phi = np.zeros(C)

    def log_prior(self, thetas):
        return np.zeros(len(thetas))

    def prior_draw(self):
        return np.stack([self.theta_prior_std * rng.normal(size=self.P) for rng in self.prngs])

    def _el_point(self, c):
        phi = self._el_phi[c]
        return self.theta[c] * np.cos(phi) + self._el_v[c] * np.sin(phi)

    def _theta_begin(self, c):
        rng = self.prngs[c]
        self._el_v[c] = self.theta_prior_std * rng.normal(size=self.P)
        self._rd_logy[c] = self.log_f[c] + np.log(rng.uniform())
        self._el_phi[c] = rng.uniform() * 2. * np.pi
        self._rd_lo[c], self._rd_hi[c] = self._el_phi[c] - 2. * np.pi, self._el_phi[c]
        self._rd_it[c] = 0
        self._rd_pend[c] = self._el_point(c)

    def _theta_result(self, c, lf, lp):
        if lf > self._rd_logy[c]:  # accept: the proposal's cache becomes current
            self.slot_cur[c], self.slot_prop[c] = self.slot_prop[c], self.slot_cur[c]
            self.theta[c] = self._rd_pend[c]
            self.log_f[c] = lf
            self.lp_cur[c] = lp
            return True
        if self.failed[c]:
            return True
        phi = self._el_phi[c]
        if phi < 0:
            self._rd_lo[c] = phi
        elif phi > 0:
            self._rd_hi[c] = phi
        else:
            warnings.warn('Slice collapsed to current value')
            return True
        self._rd_it[c] += 1
        if self._rd_it[c] >= self.max_slice_iters:
            self.failed[c] = True
            return True
        self._el_phi[c] = self._rd_lo[c] + self.prngs[c].uniform() * (self._rd_hi[c] - self._rd_lo[c])
        self._rd_pend[c] = self._el_point(c)
        return False

    def step(self):
        self.run_async(1)
        return self.theta.copy()
