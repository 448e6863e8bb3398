"""Dev check: force one conv kernel configuration on every CONV op of a network and run the per-op
checker (tests/opcheck.py) against plain PyTorch fp32 references.  usage: check_variant.py V [model B H W]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402

from helpers import fresh_model, frames  # noqa: E402
from opcheck import check_ops, kernel_summary  # noqa: E402
from yv7 import _lib as L  # noqa: E402

v = int(sys.argv[1])
name = sys.argv[2] if len(sys.argv) > 2 else 'yolov7'
B, H, W = (int(a) for a in sys.argv[3:6]) if len(sys.argv) > 5 else (2, 256, 256)
torch.backends.cudnn.enabled = False
m = fresh_model(name).to('cuda:0').half()
plan = m.plan()
x = frames(B, H, W, seed=31).to('cuda:0').half()
for i, o in enumerate(plan.graph.ops):
    if o['kind'] == L.OP_CONV:
        plan.set_op_variant(i, v)
z, xs = plan.forward(x)
torch.cuda.synchronize()
out = check_ops(plan, x, B, H, W, raw=xs, z=z)
print(f'{name} B{B} {H}x{W} variant {v}: ' + kernel_summary(out), flush=True)
