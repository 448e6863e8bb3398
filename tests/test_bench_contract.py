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
    assert (rf['bound'], rf['unit'], rf['peak']) in (('hbm', 'GB/s', 8000.0), ('mfma', 'TFLOP/s', 2500.0))
    assert 0.0 < rf['frac'] < 1.0 and abs(rf['frac'] - rf['achieved'] / rf['peak']) < 1e-3
    # the dominant kernel is the first of the per-kernel table, and every row's frac = roof / time
    top = rf['kernels_top5']
    assert top[0]['kernel'] == rf['kernel'] and abs(top[0]['us_per_launch'] - rf['mean_launch_us']) < 1e-6
    for r_ in top:
        assert abs(r_['frac'] - r_['roof_us'] / r_['us_per_launch']) < 1e-3 and r_['bound'] in ('hbm', 'mfma')
    assert all(top[i]['us_per_launch'] * top[i]['launches_per_forward'] >=
               top[i + 1]['us_per_launch'] * top[i + 1]['launches_per_forward'] - 1e-6 for i in range(len(top) - 1))
    assert d['detail']['streams'] == 3 and d['detail']['mean_dets_per_image'] > 0
    assert d['config']['resident_input_batches'] >= 4 and isinstance(d['config']['dispatch_env'], dict)
    load = d['detail']['nms_load']
    assert load['conf_0.25']['candidates_per_image'] >= load['conf_0.5']['candidates_per_image'] > 0
