"""bench.py's host-side bookkeeping on CPU (no GPU): the ESS block over a chain series with a
burn-in (ESS per transition x timed transitions / time), R-hat, the long-chain ESS record, the
PMC provenance binding (source digest) and the per-call parity inputs."""
import os
import types

import numpy as np

from conftest import REPO


def _bench():
    import sys
    sys.path.insert(0, REPO)
    import bench
    return bench


def test_ess_block_weights_timed_transitions():
    bench = _bench()
    from auxpm.diagnostics import effective_size
    rng = np.random.RandomState(0)
    C, P, L, burn = 3, 2, 160, 50
    series = []
    for c in range(C):  # AR(1) chains of different persistence
        x = np.zeros((L, P))
        for t in range(1, L):
            x[t] = (0.3 + 0.3 * c) * x[t - 1] + rng.normal(size=P)
        series.append(list(x))
    smp = types.SimpleNamespace(n_chains=C, failed=np.zeros(C, dtype=bool))
    done = np.array([20, 30, 40])
    dist = bench.Dist()
    out = bench.ess_block(dist, smp, series, done, burn, 2.0, P)
    ept = [effective_size(np.array(series[c][burn:])).min() / (L - burn) for c in range(C)]
    assert np.isclose(out['ess_per_sec'], np.dot(ept, done) / 2.0)
    assert out['sample']['burn_in_discarded'] == burn
    assert out['sample']['post_burn_transitions_per_chain_min'] == L - burn
    assert out['rhat']['length'] == L - burn and out['rhat']['max'] >= 1.0 - 1e-9
    smp.failed[1] = True  # a failed chain leaves the sums
    out2 = bench.ess_block(dist, smp, series, done, burn, 2.0, P)
    assert np.isclose(out2['ess_per_sec'], (ept[0] * 20 + ept[2] * 40) / 2.0)
    assert out2['sample']['chains'] == 2


def test_long_chain_record_and_provenance():
    bench = _bench()
    a = types.SimpleNamespace(n=4096, d=32, n_imp=256)
    rec = bench.ess_long_record(100.0, a)
    assert rec is not None and rec['source'].startswith('profiles/')
    assert np.isclose(rec['ess_per_sec_estimate'], 100.0 * rec['ess_per_transition_min_component'])
    assert rec['warmup_discarded'] >= 500 and rec['kept_per_chain'] >= 2000
    assert bench.ess_long_record(100.0, types.SimpleNamespace(n=768, d=8, n_imp=1)) is None
    sha = bench.csrc_sha16()
    assert len(sha) == 16 and sha == bench.csrc_sha16()
    prov = bench.pmc_provenance()
    assert prov['this_csrc_sha16'] == sha and prov['stale'] == (prov['profiled_csrc_sha16'] != sha)


def test_parity_inputs_match_reference_fixture():
    """The bench's parity thetas and draws are the ones tests/golden/config2_ref.npz holds the
    reference's outputs for (so that the bench can compare against the reference itself),
    including one stationary chain state of the headline's regime."""
    bench = _bench()
    from conftest import golden
    z = golden('config2_ref')
    th, rows, U1, U2 = bench.parity_inputs(int(z['n']), int(z['d']), int(z['s']))
    assert len(rows) == 3 and th.shape[0] == 3
    np.testing.assert_array_equal(th, z['thetas'][rows])
    assert th[2, 0] > 3.0  # (log sigma of the stationary regime)
    assert int(z['status'][rows].max()) == 0
    rng = np.random.RandomState(int(z['u_seed']))
    np.testing.assert_array_equal(U1, rng.normal(size=U1.shape))
    np.testing.assert_array_equal(U2, rng.normal(size=U2.shape))
    assert os.path.exists(bench.REF_FIXTURE)
