import sys, torch
sys.path.insert(0, 'yolo-series_amd')
from models.yolo import Model
from yv7.synthetic import synthetic_state_dict
from yv7.runtime import Plan
m = Model('yolov7'); synthetic_state_dict(m, seed=0); m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', torch.float16)
g = torch.Generator(device='cuda:0').manual_seed(1000)
x = (torch.randint(0, 256, (32, 3, 640, 640), generator=g, device='cuda:0', dtype=torch.uint8).half() / 255.0)
z = plan.forward(x)
z = z[0] if isinstance(z, tuple) else z
obj = z[..., 4]
print('rows', z.shape, 'obj>0.25 frac', (obj > 0.25).float().mean().item())
conf = (z[..., 5:] * obj[..., None]).amax(-1)
print('cand frac', ((obj > 0.25) & (conf > 0.25)).float().mean().item(), 'per image', ((obj > 0.25) & (conf > 0.25)).sum(1).tolist()[:8])
