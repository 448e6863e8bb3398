"""Regenerates the golden fixtures in tests/golden/ from the oracle (run from the repo root).

The reference ships no tests, vectors or weights and could not be imported or run here
(SURVEY §8c), so these vectors come from the oracle (the CPU restatement) on seeded inputs; they
pin the oracle (tests/test_golden.py) and the HIP path (tests/test_gpu_golden.py) against
regressions.  Inputs are stored with the expected outputs.
  nms_cases.npz       z [2, 800, 13] (nc 8, clustered boxes, exact ties, values at the threshold)
                      + for each case: det rows / kept anchor rows / counts
  tiny64.npz          yolov7-tiny, synthetic weights seed 0, frames seed 1 [1,3,64,96]: z and the
                      per-level raw logits (fp32)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'yolo-series_amd'), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

NMS_CASES = [
    dict(conf_thres=0.25, iou_thres=0.45),
    dict(conf_thres=0.25, iou_thres=0.45, agnostic=True),
    dict(conf_thres=0.3, iou_thres=0.6, multi_label=True),
    dict(conf_thres=0.25, iou_thres=0.45, classes=[1, 3, 7]),
    dict(conf_thres=0.05, iou_thres=0.3, multi_label=True, agnostic=True),
]


def nms_input(seed=21, B=2, N=800, nc=8):
    g = torch.Generator().manual_seed(seed)
    z = torch.zeros(B, N, nc + 5)
    centers = torch.rand(B, 30, 2, generator=g) * 600 + 20
    which = torch.randint(0, 30, (B, N), generator=g)
    z[..., 0:2] = torch.gather(centers, 1, which[..., None].expand(B, N, 2)) + torch.randn(B, N, 2, generator=g) * 5
    z[..., 2:4] = torch.rand(B, N, 2, generator=g) * 60 + 8
    z[..., 4] = torch.rand(B, N, generator=g)
    z[..., 5:] = torch.rand(B, N, nc, generator=g)
    z[:, 1::37, 4:] = z[:, 0::37, 4:][:, :z[:, 1::37].shape[1]]    # exact score ties
    z[:, 3::41, 4] = 0.25                                           # exactly at conf_thres
    return z


def main():
    from oracle import nms_ref, yolo_ref
    from models.yolo import Model
    from yv7.synthetic import synthetic_frames, synthetic_state_dict
    out = os.path.dirname(os.path.abspath(__file__))
    z = nms_input()
    arrs = {'z': z.numpy()}
    for i, kw in enumerate(NMS_CASES):
        dets, rows = nms_ref.non_max_suppression(z, return_rows=True, **kw)
        arrs[f'case{i}_count'] = np.array([d.shape[0] for d in dets], dtype=np.int32)
        arrs[f'case{i}_det'] = np.concatenate([d.numpy() for d in dets], 0).astype(np.float32)
        arrs[f'case{i}_rows'] = np.concatenate([r.numpy() for r in rows], 0).astype(np.int64)
    np.savez_compressed(os.path.join(out, 'nms_cases.npz'), **arrs)

    m = Model('yolov7-tiny')
    sd = synthetic_state_dict(m, seed=0)
    net = yolo_ref.parse(m.yaml)
    fused = yolo_ref.fuse(net, sd)
    x = synthetic_frames(1, 64, 96, seed=1)
    zt, xs = yolo_ref.forward(net, fused, x)
    np.savez_compressed(os.path.join(out, 'tiny64.npz'), x=x.numpy(), z=zt.numpy(),
                        **{f'raw{i}': t.numpy() for i, t in enumerate(xs)})
    print('wrote', sorted(os.listdir(out)))


if __name__ == '__main__':
    main()
