"""Dev tool: per-op A/B of conv kernel configurations in one process (interleaved rounds).

Every CONV op of the plan is forced to each variant in turn (yv7_set_op_variant; 0 = the tuned
dispatch); ops run one after another on one stream, so each op's HIP-event time under variant v is
that kernel's time on that layer.  Prints, per op, the median time of each variant and the best one,
and the forward total with the default dispatch vs the best variant per op.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT]
import torch  # noqa: E402

from models.yolo import Model  # noqa: E402
from yv7 import _lib as L  # noqa: E402
from yv7.runtime import Plan  # noqa: E402
from yv7.synthetic import synthetic_state_dict  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument('--model', default='yolov7')
ap.add_argument('--b', type=int, default=32)
ap.add_argument('--img', type=int, default=640)
ap.add_argument('--variants', default='0,231,262,270')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--iters', type=int, default=4)
ap.add_argument('--out', default='')
ap.add_argument('--ops', default='', help='comma-separated op indices to force (default: every CONV op)')
ap.add_argument('--fp8', type=int, default=None, help='fp8 plan (this min_cout; 0 = every eligible 1x1): forces '
                'only its fp8 ops (variants 0 = fused quantization, 81 = staged) and adds the fp16 time column')
a = ap.parse_args()
variants = [int(v) for v in a.variants.split(',')]
m = Model(a.model)
synthetic_state_dict(m, seed=0)
m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', torch.float16)
B, H = a.b, a.img
x = torch.rand(B, 3, H, H, device='cuda:0').half()
z = torch.empty(B, plan.num_rows(H, H), plan.no, device='cuda:0')
convs = [i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_CONV]
f16_us = None
if a.fp8 is not None:
    plan.profile_enable(a.iters)
    for _ in range(a.iters + 2):
        plan.forward_into(x, z)
    torch.cuda.synchronize()
    n, ms = plan.profile_read()
    f16_us = [t / n * 1e3 for t in ms]
    plan = Plan.fp8_from_model(m.half().to('cuda:0'), 'cuda:0', min_cout=a.fp8)
    assert len(plan.graph.ops) == len(f16_us)
    convs = [i for i, o in enumerate(plan.graph.ops) if o.get('wfmt', 0) == L.WFMT_FP8]
if a.ops:
    convs = [int(v) for v in a.ops.split(',')]
times = {v: {i: [] for i in range(len(plan.graph.ops))} for v in variants}
for r in range(a.rounds):
    for v in variants:
        for i in convs:
            plan.set_op_variant(i, v)
        for _ in range(2):
            plan.forward_into(x, z)
        torch.cuda.synchronize()
        plan.profile_enable(a.iters)
        for _ in range(a.iters):
            plan.forward_into(x, z)
        torch.cuda.synchronize()
        n, ms = plan.profile_read()
        plan.profile_enable(0)
        for i, t in enumerate(ms):
            times[v][i].append(t / n * 1e3)
    print(f'round {r} done', file=sys.stderr, flush=True)
names = {0: 'INPUT', 1: 'CONV', 2: 'POOL', 3: 'UPS', 4: 'COPY', 5: 'DET', 6: 'STEM'}
med = {v: {i: statistics.median(ts) for i, ts in times[v].items()} for v in variants}
tot_def = sum(med[variants[0]].values())
tot_best = 0.0
rows = []
print(f'{"op":>3} {"desc":34s} ' + ' '.join(f'{v:>8d}' for v in variants) + '   best')
for i, o in enumerate(plan.graph.ops):
    sh = plan.graph.tensors[o['src']][1] if o['kind'] not in (0, 6) else 0
    desc = f"{names[o['kind']]:5s} {o.get('cin', 0):5d}->{o.get('cout', 0):5d} k{o.get('k', 1)} s{o.get('s', 1)} p{o.get('pool', 0)} @{H >> sh}"
    ts = [med[v][i] for v in variants]
    best = variants[min(range(len(ts)), key=lambda k: ts[k])] if i in convs else variants[0]
    tot_best += med[best][i]
    rows.append({'op': i, 'desc': desc, 'us': dict(zip(variants, ts)), 'best': best})
    if f16_us is not None:
        rows[-1]['f16_us'] = f16_us[i]
    if i in convs or not (a.ops or f16_us):
        print(f'{i:3d} {desc:34s} ' + ' '.join(f'{t:8.1f}' for t in ts) + f'   {best}' +
              (f'   f16 {f16_us[i]:8.1f}' if f16_us else ''))
print(f'forward (sum of ops): default {tot_def / 1e3:.3f} ms, best per op {tot_best / 1e3:.3f} ms')
for v in variants:
    print(f'  variant {v}: {sum(med[v].values()) / 1e3:.3f} ms')
if f16_us:
    print(f'  fp16 plan: {sum(f16_us) / 1e3:.3f} ms; fp8 ops only: f16 {sum(f16_us[i] for i in convs) / 1e3:.3f} ms, '
          + ', '.join(f'v{v} {sum(med[v][i] for i in convs) / 1e3:.3f} ms' for v in variants))
if a.out:
    with open(a.out, 'w') as f:
        json.dump({'model': a.model, 'b': B, 'img': H, 'variants': variants, 'rows': rows,
                   'total_default_ms': tot_def / 1e3, 'total_best_ms': tot_best / 1e3}, f, indent=1)
