"""Dev diagnostic: force each given conv variant on every conv op of a network, run one forward and
report EVERY op whose output misses the per-op reference (tests/opcheck.py), not just the first.
usage: diag_variants.py MODEL B H W v1,v2,...  (YV7_DUAL etc. from the environment)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402

import opcheck  # noqa: E402
from helpers import fresh_model, frames  # noqa: E402
from yv7 import _lib as L  # noqa: E402

name, B, H, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
variants = [int(v) for v in sys.argv[5].split(',')]
m = fresh_model(name).to('cuda:0').half()
plan = m.plan()
x = frames(B, H, W, seed=31).to('cuda:0').half()
convs = [i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_CONV]
orig = opcheck._ulp_check
for v in variants:
    for i in convs:
        plan.set_op_variant(i, v)
    z, xs = plan.forward(x)
    torch.cuda.synchronize()
    bad = []

    def soft(got, ref, what, fp16, ulps=1):
        try:
            return orig(got, ref, what, fp16, ulps)
        except AssertionError as e:
            bad.append(str(e)[:120])
            return 0.0
    opcheck._ulp_check = soft
    try:
        opcheck.check_ops(plan, x, B, H, W, raw=xs, z=z)
    except AssertionError as e:
        bad.append('hard: ' + str(e)[:120])
    opcheck._ulp_check = orig
    kern = plan.op_kernels(B, H, W) if hasattr(plan, 'op_kernels') else None
    print(f'variant {v}: {len(bad)} bad ops', flush=True)
    for b in bad:
        print('   ', b, flush=True)
    for i in convs:
        plan.set_op_variant(i, 0)
