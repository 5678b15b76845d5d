"""Off-by-default development knobs that DESIGN.md §5 reports as bitwise equal to the default
path, checked in child processes (each knob is read once per process): the two-launch dataflow
Newton panel (APM_DF_SPLIT=1) and the 64x128 L.U tile (APM_UGEMM_W2_MIN=1)."""
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _digest(n, **env):
    e = dict(os.environ)
    for k in ('APM_DF_SPLIT', 'APM_UGEMM_W2_MIN'):
        e.pop(k, None)
    e.update(env)
    out = subprocess.run([sys.executable, os.path.join(HERE, '_knob_child.py'), str(n)], env=e,
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith('digest')][-1]
    return line


@pytest.mark.gpu
@pytest.mark.parametrize('var,val', [('APM_DF_SPLIT', '1'), ('APM_UGEMM_W2_MIN', '1')])
def test_knob_bitwise_equal_to_default(gpu_available, var, val):
    n = 1100  # three outer Newton panels (the last one ragged), two 64-sample blocks
    base = _digest(n)
    alt = _digest(n, **{var: val})
    assert 'status [0, 0, 0' in base, base
    assert alt == base, (var, alt, base)
