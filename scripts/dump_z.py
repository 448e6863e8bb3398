"""Dev tool: fp16 plan forward of seeded frames -> z saved to a file (A/B of kernel variants selected by
environment variables, which libyv7 reads once per process).  usage: python scripts/dump_z.py OUT.pt"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT]
import torch
from models.yolo import Model
from yv7.runtime import Plan
from yv7.synthetic import synthetic_frames, synthetic_state_dict
m = Model('yolov7'); synthetic_state_dict(m, seed=0); m = m.float().fuse().eval()
plan = Plan.from_model(m, 'cuda:0', torch.float16)
x = synthetic_frames(8, 640, 640, seed=3).to('cuda:0').half()
z, _ = plan.forward(x, want_raw=False)
torch.cuda.synchronize()
torch.save(z.cpu(), sys.argv[1])
print('saved', tuple(z.shape), float(z.abs().sum()))
