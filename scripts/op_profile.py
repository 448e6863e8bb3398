"""Dev tool: per-op event timing of one plan forward (bs32 640 fp16 yolov7 by default) with rooflines."""
import os, sys, argparse
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT]
import torch
from models.yolo import Model
from yv7.runtime import Plan
from yv7.synthetic import synthetic_state_dict
from yv7 import _lib as L
ap = argparse.ArgumentParser(); ap.add_argument('--model', default='yolov7'); ap.add_argument('--b', type=int, default=32)
ap.add_argument('--img', type=int, default=640); ap.add_argument('--dtype', default='f16'); ap.add_argument('--iters', type=int, default=10)
ap.add_argument('--csv', default=''); ap.add_argument('--top', type=int, default=40)
ap.add_argument('--dump', default='', help='JSON of every op: desc, kernels, us, algorithmic bytes (scripts/pmc_ops.py)')
a = ap.parse_args()
dt = torch.float32 if a.dtype == 'f32' else torch.float16
m = Model(a.model); synthetic_state_dict(m, seed=0); m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', 'fp8' if a.dtype == 'fp8' else dt)
B, H = a.b, a.img
x = torch.rand(B, 3, H, H, device='cuda:0').to(dt)
z = torch.empty(B, plan.num_rows(H, H), plan.no, device='cuda:0')
for _ in range(3): plan.forward_into(x, z)
torch.cuda.synchronize()
plan.profile_enable(a.iters)
for _ in range(a.iters): plan.forward_into(x, z)
torch.cuda.synchronize()
n, ms = plan.profile_read()
costs = plan.op_costs(B, H, H, x_bytes=x.element_size(), with_raw=False)
names = {0: 'INPUT', 1: 'CONV', 2: 'POOL', 3: 'UPS', 4: 'COPY', 5: 'DET', 6: 'STEM'}
tot = sum(ms) / n
# An op without a kernel of its own (the second op of the dual 1x1 launch, the later pools of the SPPCSPC
# cascade) runs inside the launch of the op before it: its bytes, FLOPs and (zero-length) event time are
# credited to that op, and it is listed as part of it — no per-op frac above 1 (the
# bench's kernel table does the same).
ks = plan.op_kernels(B, H, H)
costs = [list(c) for c in costs]
ms = list(ms)
merged = {}
for i in range(len(costs)):
    if not ks[i] and costs[i][0] not in (0,):
        j = i - 1
        while j >= 0 and not ks[j]:
            j -= 1
        if j >= 0:
            costs[j][1] += costs[i][1]
            costs[j][2] += costs[i][2]
            ms[j] += ms[i]
            merged.setdefault(j, []).append(i)
rows = []
for i, ((kind, fl, by), t, o) in enumerate(zip(costs, ms, plan.graph.ops)):
    if any(i in v for v in merged.values()):
        continue
    t = t / n
    sh = plan.graph.tensors[o['src']][1] if o['kind'] not in (0, 6) else 0
    hw = H >> sh
    desc = f"{names[kind]:5s} {o.get('cin',0):5d}->{o.get('cout',0):5d} k{o.get('k',1)} s{o.get('s',1)} @{hw}"
    if i in merged:
        desc += ' +op' + ','.join(str(j) for j in merged[i])
    tf = fl / (t * 1e-3) / 1e12 if t > 0 else 0
    gb = by / (t * 1e-3) / 1e9 if t > 0 else 0
    # roofline-limited time at 8 TB/s and 2.5 PF
    tmin = max(by / 8e12, fl / 2.5e15) * 1e3
    rows.append((t, i, desc, tf, gb, tmin))
if a.dump:
    import json
    json.dump([{'op': i, 'desc': desc, 'us': t * 1e3, 'roof_us': tmin * 1e3, 'bytes': costs[i][2], 'flops': costs[i][1],
                'kernels': ks[i]} for t, i, desc, tf, gb, tmin in sorted(rows, key=lambda r: r[1])], open(a.dump, 'w'), indent=0)
print(f'forward {tot:.3f} ms over {n} forwards; sum of roofline minima {sum(r[5] for r in rows):.3f} ms')
import csv
if a.csv:
    with open(a.csv, 'w') as f:
        wr = csv.writer(f); wr.writerow(['op', 'desc', 'us', 'tflops', 'gbs', 'roof_us'])
        for t, i, desc, tf, gb, tmin in sorted(rows, key=lambda r: r[1]):
            wr.writerow([i, desc, round(t * 1e3, 2), round(tf, 1), round(gb, 1), round(tmin * 1e3, 2)])
for t, i, desc, tf, gb, tmin in sorted(rows, reverse=True)[:a.top]:
    print(f'{i:3d} {desc:40s} {t*1e3:8.1f} us  {tf:7.1f} TF/s  {gb:7.1f} GB/s  roof {tmin*1e3:7.1f} us  frac {tmin/t:5.2f}')
by_kind = {}
for t, i, desc, tf, gb, tmin in rows:
    o = plan.graph.ops[i]
    k = desc.split()[0] + (f" k{o.get('k', 1)}s{o.get('s', 1)}" if desc.startswith('CONV') else '')
    by_kind.setdefault(k, [0, 0, 0]); by_kind[k][0] += t; by_kind[k][1] += tmin; by_kind[k][2] += 1
for k, (t, tm, c) in sorted(by_kind.items(), key=lambda kv: -kv[1][0]):
    print(f'{k:10s} n={c:3d} {t:7.3f} ms roof {tm:7.3f} ms frac {tm/t:5.2f}')
