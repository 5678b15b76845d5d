"""ESS / R-hat restatements (auxpm.diagnostics) against closed-form AR(1) behaviour.
coda itself is unavailable (no R): parity with coda is unpinned, see the module docstring."""
import numpy as np

from auxpm import diagnostics as dg


def _ar1(phi, n, seed):
    rng = np.random.RandomState(seed)
    x = np.empty(n)
    x[0] = rng.normal() / np.sqrt(1 - phi ** 2)
    for t in range(1, n):
        x[t] = phi * x[t - 1] + rng.normal()
    return x


def test_yule_walker_recovers_ar1():
    x = _ar1(0.8, 20000, 0)
    ar, vp, order = dg.ar_yule_walker(x)
    assert order >= 1
    assert abs(ar[0] - 0.8) < 0.03
    assert abs(vp - 1.0) < 0.05


def test_ess_ar1_matches_theory():
    for phi in (0.0, 0.5, 0.9):
        ess = np.mean([dg.effective_size(_ar1(phi, 10000, s))[0] for s in range(4)])
        theory = 10000 * (1 - phi) / (1 + phi)
        assert abs(ess / theory - 1) < 0.12, (phi, ess, theory)


def test_ess_constant_chain_is_zero():
    assert dg.effective_size(np.ones(100))[0] == 0.0
    assert dg.effective_size(np.arange(100.))[0] == 0.0  # pure linear trend


def test_gelman_rubin():
    rng = np.random.RandomState(1)
    same = rng.normal(size=(4, 2000, 2))
    r = dg.gelman_rubin(same)
    assert np.all(np.abs(r - 1) < 0.01)
    shifted = same + np.arange(4)[:, None, None]
    assert np.all(dg.gelman_rubin(shifted) > 1.5)


def test_plot_trace_returns_reference_tuple():
    """gpdemo.utils.plot_trace returns (fig, ax1, ax2) like the reference (utils.py:211-242)."""
    import matplotlib
    matplotlib.use('Agg')
    from gpdemo.utils import plot_trace
    fig, ax1, ax2 = plot_trace(np.random.RandomState(0).normal(size=(20, 3)))
    assert len(ax1.lines) == 1 and len(ax2.lines) == 1
    np.testing.assert_array_equal(ax2.lines[0].get_ydata().shape, (20,))
