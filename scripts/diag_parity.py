"""Dev tool: GPU fp32 plan vs oracle fp32 vs oracle fp64 — where does the z error come from?"""
import sys, os, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT, os.path.join(ROOT, 'tests')]
import torch
from helpers import fresh_model, frames, oracle_net
from oracle import yolo_ref

def fwd64(net, fused, x):
    f64 = {}
    for k, v in fused.items():
        if isinstance(v, tuple): f64[k] = (v[0].double(), v[1].double())
        elif isinstance(v, dict): f64[k] = {j: (a.double(), b.double()) for j, (a, b) in v.items()}
        else: f64[k] = [(a.double(), b.double()) for a, b in v]
    ag = net.anchor_grid; net.anchor_grid = ag.double()
    z, xs = yolo_ref.forward(net, f64, x.double())
    net.anchor_grid = ag
    return z

for name, H in [('yolov7-tiny', 640), ('yolov7', 640)]:
    x = frames(1, H, H, seed=4)
    net, fused = oracle_net(name)
    z32, _ = yolo_ref.forward(net, fused, x)
    z64 = fwd64(net, fused, x)
    m = fresh_model(name).to('cuda:0')
    zg, _ = m(x.cuda()); zg = zg.cpu().double()
    z32 = z32.double()
    den = z64.abs().clamp(min=1)
    for lab, sl in [('xy', slice(0, 2)), ('wh', slice(2, 4)), ('conf', slice(4, None))]:
        e_ref = ((z32 - z64)[..., sl].abs() / (den[..., sl] if lab != 'conf' else 1)).max().item()
        e_gpu = ((zg - z64)[..., sl].abs() / (den[..., sl] if lab != 'conf' else 1)).max().item()
        e_rg = ((zg - z32)[..., sl].abs() / (den[..., sl] if lab != 'conf' else 1)).max().item()
        print(f'{name} {lab}: oracle32-vs-64 {e_ref:.3g}  gpu-vs-64 {e_gpu:.3g}  gpu-vs-oracle32 {e_rg:.3g}')
    # timing fp16 plan at bs32
for name in ['yolov7']:
    for dt in (torch.float32, torch.float16):
        m = fresh_model(name).to('cuda:0').to(dt)
        x = frames(32, 640, 640, seed=1).cuda().to(dt)
        plan = m.plan()
        z = torch.empty(32, plan.num_rows(640, 640), 85, device='cuda:0')
        for _ in range(3): plan.forward_into(x, z)
        torch.cuda.synchronize(); t = time.time()
        for _ in range(10): plan.forward_into(x, z)
        torch.cuda.synchronize(); dtm = (time.time() - t) / 10
        print(f'{name} {dt} bs32: {dtm*1e3:.2f} ms/batch, {32/dtm:.0f} img/s')
