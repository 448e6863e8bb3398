"""Dev tool: per-layer kernel-configuration sweep with ONE op forced at a time (the rest of the network
on the tuned dispatch), so each candidate is timed in its real neighbourhood (same clocks, same L2 /
MALL contents from the producing layer) rather than with every layer switched at once (ab_ops.py).

For each CONV op and candidate variant: 2 warm forwards, then `--iters` profiled forwards; the op's
median HIP-event time over `--rounds` interleaved rounds.  Prints per op the default time, the best
candidate and its gain, and writes the table as JSON.
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
from yv7.runtime import Plan, kernel_key  # noqa: E402
from yv7.synthetic import synthetic_state_dict  # noqa: E402

RING = [100 + 10 * c + s for c in range(6) for s in (0, 2, 4)]
DEFAULT_CANDS = [201, 202, 203, 204, 205, 206, 231, 232, 262, 270, 271, 4, 5, 6, 7, 8] + RING

ap = argparse.ArgumentParser()
ap.add_argument('--model', default='yolov7')
ap.add_argument('--b', type=int, default=32)
ap.add_argument('--img', type=int, default=640)
ap.add_argument('--cands', default='')
ap.add_argument('--rounds', type=int, default=3)
ap.add_argument('--iters', type=int, default=3)
ap.add_argument('--ops', default='')
ap.add_argument('--out', default='')
a = ap.parse_args()
cands = [int(v) for v in a.cands.split(',')] if a.cands else DEFAULT_CANDS
m = Model(a.model)
synthetic_state_dict(m, seed=0)
m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', torch.float16)
B, H = a.b, a.img
x = torch.rand(B, 3, H, H, device='cuda:0').half()
z = torch.empty(B, plan.num_rows(H, H), plan.no, device='cuda:0')
convs = [i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_CONV and not o.get('pool', 0)]
if a.ops:
    convs = [int(v) for v in a.ops.split(',')]


def timed(op):
    for _ in range(2):
        plan.forward_into(x, z)
    torch.cuda.synchronize()
    plan.profile_enable(a.iters)
    for _ in range(a.iters):
        plan.forward_into(x, z)
    torch.cuda.synchronize()
    n, ms = plan.profile_read()
    plan.profile_enable(0)
    return ms[op] / n * 1e3, sum(ms) / n * 1e3


names = {1: 'CONV', 5: 'DET'}
rows = []
for i in convs:
    o = plan.graph.ops[i]
    sh = plan.graph.tensors[o['src']][1]
    desc = f"{o['cin']:5d}->{o['cout']:5d} k{o['k']} s{o['s']} @{H >> sh}"
    t = {v: [] for v in [0] + cands}
    tot = {v: [] for v in [0] + cands}
    for r in range(a.rounds):
        for v in [0] + cands:
            try:
                plan.set_op_variant(i, v)
                a_, b_ = timed(i)
            except RuntimeError:
                continue
            t[v].append(a_)
            tot[v].append(b_)
    med = {v: statistics.median(ts) for v, ts in t.items() if ts}
    totm = {v: statistics.median(ts) for v, ts in tot.items() if ts}
    best = min(med, key=med.get)
    # the kernel the winner actually launches (a forced variant the shape does not support falls back
    # to another kernel, which may be what won)
    plan.set_op_variant(i, best)
    kern = ','.join(kernel_key(k) for k in plan.op_kernels(B, H, H, torch.float16)[i])
    plan.set_op_variant(i, 0)
    rows.append({'op': i, 'desc': desc, 'us': med, 'fwd_us': totm, 'best': best, 'best_kernel': kern})
    print(f'{i:3d} {desc:28s} default {med[0]:7.1f}  best {best:4d} {med[best]:7.1f}  gain {med[0] - med[best]:6.1f}'
          f'   fwd {totm[0] / 1e3:.3f} -> {totm[best] / 1e3:.3f} ms   top3 '
          + ' '.join(f'{v}:{med[v]:.1f}' for v in sorted(med, key=med.get)[:3]) + f'   [{kern}]', flush=True)
print(f'sum of per-op gains: {sum(r["us"][0] - r["us"][r["best"]] for r in rows):.1f} us')
if a.out:
    with open(a.out, 'w') as f:
        json.dump({'model': a.model, 'b': B, 'img': H, 'rows': rows}, f, indent=1)
