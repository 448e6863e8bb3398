"""bench.py's one-line JSON contract (the driver parses it): keys, units, internal consistency.

Runs the default schedule (3 batches in flight) for a few steps on cuda:0 without the CPU baseline."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', '6', '--warmup', '2',
                        '--no-cpu-baseline'], capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]   # exactly one JSON line on stdout
    d = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better', 'scaling',
              'vs_baseline', 'dtype', 'data', 'config', 'roofline'):
        assert k in d, k
    assert d['unit'] == 'images/sec' and d['higher_is_better'] is True and d['scaling'] == 'weak'
    assert d['n_gpus'] == 1 and d['steps'] == 6 and d['dtype'] == 'f16' and d['vs_baseline'] is None
    assert d['config']['global_batch'] == 32 and d['config']['img'] == 640
    # value is whole-job images/s over the timed steps
    assert abs(d['value'] - 32 * 1000.0 / d['ms_per_step']) / d['value'] < 0.02
    rf = d['roofline']
    assert rf['bound'] == 'hbm' and rf['unit'] == 'GB/s' and rf['peak'] == 8000.0
    assert 0.0 < rf['frac'] < 1.0 and abs(rf['frac'] - rf['achieved'] / rf['peak']) < 1e-3
    assert d['detail']['streams'] == 3 and d['detail']['mean_dets_per_image'] > 0
