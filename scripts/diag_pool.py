"""Dev diagnostic: where the dual 1x1's pooled output differs from the reference (per column, row and
channel position), on yolov7 2x256x256 fp16.  usage: diag_pool.py OP"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import opcheck  # noqa: E402
from helpers import fresh_model, frames  # noqa: E402

op = int(sys.argv[1])
B, H, W = 2, 256, 256
m = fresh_model('yolov7').to('cuda:0').half()
plan = m.plan()
x = frames(B, H, W, seed=31).to('cuda:0').half()
plan.forward(x)
torch.cuda.synchronize()
g = plan.graph
o = g.ops[op]
blob = g.weight_blob().to('cuda:0')
tv = lambda t: plan.tensor_view(t, B, H, W)  # noqa: E731
xin = tv(o['src'])[..., o['src_coff']:o['src_coff'] + o['cin']].float()
xin = F.max_pool2d(xin.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
w, b = opcheck._weights(plan, blob, o)
ref = opcheck.conv_ref(xin, w, b, 1, o['act'])
got = tv(o['dst'])[..., o['dst_coff']:o['dst_coff'] + o['cout']].float()
d = (got - ref).abs()
bad = d > (ref.abs() * 2 ** -10 + 1e-3)
print('shape', tuple(got.shape), 'bad frac', bad.float().mean().item())
print('by col mod 8  ', [round(bad[:, :, c::8].float().mean().item(), 3) for c in range(8)])
print('by row mod 4  ', [round(bad[:, r::4].float().mean().item(), 3) for r in range(4)])
print('by chan mod 32', [round(bad[..., c::32].float().mean().item(), 2) for c in range(32)])
print('by chan /32   ', [round(bad[..., c * 32:(c + 1) * 32].float().mean().item(), 3) for c in range(4)])
# is got equal to the reference at a shifted position / another pooling?
for name, alt in (('no pool (top-left px)', tv(o['src'])[:, ::2, ::2, o['src_coff']:o['src_coff'] + o['cin']].float()),
                  ('row max only', torch.maximum(tv(o['src'])[:, ::2, ::2, o['src_coff']:o['src_coff'] + o['cin']],
                                                 tv(o['src'])[:, 1::2, ::2, o['src_coff']:o['src_coff'] + o['cin']]).float()),
                  ('col max only', torch.maximum(tv(o['src'])[:, ::2, ::2, o['src_coff']:o['src_coff'] + o['cin']],
                                                 tv(o['src'])[:, ::2, 1::2, o['src_coff']:o['src_coff'] + o['cin']]).float())):
    r2 = opcheck.conv_ref(alt, w, b, 1, o['act'])
    print(name, 'bad frac', ((got - r2).abs() > (r2.abs() * 2 ** -10 + 1e-3)).float().mean().item())
