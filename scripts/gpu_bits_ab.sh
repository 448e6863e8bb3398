#!/bin/bash
# Bitwise comparison of the fp16 plan's z between two builds (abtmp/libyv7_base.so, abtmp/libyv7_new.so),
# per op: the first op whose output differs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
export PYTHONPATH=$R/yolo-series_amd:$R
L=yolo-series_amd/yv7/libyv7.so
for v in base new; do
  cp abtmp/libyv7_$v.so $L
  timeout -k 10 200 python -u - gpurun_out/bits_$v.pt <<'PY' || exit 1
import sys, torch
from models.yolo import Model
from yv7.runtime import Plan
from yv7.synthetic import synthetic_frames, synthetic_state_dict
m = Model('yolov7'); synthetic_state_dict(m, seed=0); m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', torch.float16)
B, H = 4, 640
x = synthetic_frames(B, H, H, seed=3).to('cuda:0').half()
z, _ = plan.forward(x, want_raw=False)
torch.cuda.synchronize()
outs = {}
for i, o in enumerate(plan.graph.ops):
    if o['kind'] in (2, 3, 8):   # CONV, DETECT? (store every dst tensor we can read)
        pass
for t in range(len(plan.graph.tensors)):
    try:
        outs[t] = plan.tensor_view(t, B, H, H).detach().cpu().clone()
    except Exception:
        pass
torch.save({'z': z.cpu(), 't': outs}, sys.argv[1])
print('saved', len(outs))
PY
done
cp abtmp/libyv7_new.so $L
python3 - <<'PY'
import torch
a = torch.load('gpurun_out/bits_base.pt'); b = torch.load('gpurun_out/bits_new.pt')
print('z equal:', torch.equal(a['z'], b['z']), 'max |dz|', (a['z'] - b['z']).abs().max().item())
for t in sorted(a['t']):
    x, y = a['t'][t], b['t'][t]
    if not torch.equal(x, y):
        d = (x.float() - y.float()).abs()
        print('tensor', t, 'differs in', int((d > 0).sum()), 'of', d.numel(), 'max', d.max().item())
PY
