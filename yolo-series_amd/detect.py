"""detect.py — the reference's PyTorch inference loop (detect.py:25-230, its `else` branch: no ONNX/TRT)
on the MI355X path: attempt_load -> LoadImages (GPU letterbox) -> model(img)[0] -> non_max_suppression
-> scale_coords().round(), with the reference's call sites unchanged (detect.py:41, 144, 152, 183).

Differences, all forced by the environment: frames are decoded by PIL (cv2 is absent; decode parity
unpinned), there are no checkpoints offline so `--cfg NAME --synthetic-seed S` builds seeded synthetic
weights instead of `--weights`, and drawing/saving annotated images (utils/plots.py, cv2) is out of
scope — `--save-txt` writes the reference's label format.  There is no CPU execution path.

    python detect.py --cfg yolov7-tiny --source ../tests/golden/bus.jpg --img-size 640
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from models.experimental import attempt_load  # noqa: E402
from utils.datasets import LoadImages  # noqa: E402
from utils.general import check_img_size, non_max_suppression, scale_coords, xyxy2xywh  # noqa: E402
from utils.torch_utils import select_device, time_synchronized  # noqa: E402


def load_model(opt, device):
    if opt.weights:
        return attempt_load(opt.weights, map_location=device, cfg=opt.cfg)   # load FP32 model (detect.py:41)
    from models.yolo import Model
    from yv7.synthetic import synthetic_state_dict
    m = Model(opt.cfg or 'yolov7')
    synthetic_state_dict(m, seed=opt.synthetic_seed)
    return attempt_load(m, map_location=device)


def detect(opt):
    """Returns [(path, det)] with det [n, 6] (x1, y1, x2, y2, conf, cls) in original-image pixels (CPU)."""
    device = select_device(opt.device)
    if device.type == 'cpu':
        raise RuntimeError('detect.py: the MI355X path has no CPU execution (oracle/ holds the CPU reference)')
    half = not opt.fp32                                   # detect.py:38 (half on every GPU device)
    model = load_model(opt, device)
    stride = int(model.stride.max())
    imgsz = check_img_size(opt.img_size, s=stride)
    if half:
        model.half()
    dataset = LoadImages(opt.source, img_size=imgsz, stride=stride)
    names = model.module.names if hasattr(model, 'module') else model.names
    model(torch.zeros(1, 3, imgsz, imgsz).to(device).type_as(next(model.parameters())))  # run once
    save_dir = Path(opt.project) / opt.name
    if opt.save_txt:
        (save_dir / 'labels').mkdir(parents=True, exist_ok=True)
    results = []
    t0 = time.time()
    for path, img, im0s, vid_cap, ratio, dwdh in dataset:
        img = torch.from_numpy(img).to(device)
        img = img.half() if half else img.float()          # uint8 to fp16/32
        img /= 255.0                                       # 0 - 255 to 0.0 - 1.0
        if img.ndimension() == 3:
            img = img.unsqueeze(0)
        t1 = time_synchronized()
        with torch.no_grad():
            pred = model(img, augment=opt.augment)[0]
        t2 = time_synchronized()
        pred = non_max_suppression(pred, opt.conf_thres, opt.iou_thres, classes=opt.classes, agnostic=opt.agnostic_nms)
        t3 = time_synchronized()
        for i, det in enumerate(pred):
            p, s, im0 = Path(path), '', im0s
            gn = torch.tensor(im0.shape)[[1, 0, 1, 0]]      # normalization gain whwh
            if len(det):
                det[:, :4] = scale_coords(img.shape[2:], det[:, :4], im0.shape).round()
                for c in det[:, -1].unique():
                    n = (det[:, -1] == c).sum()
                    s += f"{n} {names[int(c)]}{'s' * (n > 1)}, "
                if opt.save_txt:
                    with open(save_dir / 'labels' / (p.stem + '.txt'), 'a') as f:
                        for *xyxy, conf, cls in reversed(det.cpu()):
                            xywh = (xyxy2xywh(torch.tensor(xyxy).view(1, 4)) / gn).view(-1).tolist()
                            line = (cls, *xywh, conf) if opt.save_conf else (cls, *xywh)
                            f.write(('%g ' * len(line)).rstrip() % line + '\n')
            if not opt.quiet:
                print(f'{s}Done. ({(1E3 * (t2 - t1)):.1f}ms) Inference, ({(1E3 * (t3 - t2)):.1f}ms) NMS')
            results.append((path, det.cpu()))
    if not opt.quiet:
        print(f'Done. ({time.time() - t0:.3f}s)')
    return results


def parse_opt(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--weights', nargs='+', type=str, default=None, help='model.pt path(s)')
    ap.add_argument('--cfg', type=str, default=None, help='architecture (yolov7, yolov7-tiny, yolov7-w6, ...) for '
                    'state_dict checkpoints or synthetic weights')
    ap.add_argument('--synthetic-seed', type=int, default=0, help='seeded synthetic weights when --weights is absent')
    ap.add_argument('--source', type=str, default='inference/images', help='file/folder')
    ap.add_argument('--img-size', type=int, default=640, help='inference size (pixels)')
    ap.add_argument('--conf-thres', type=float, default=0.25, help='object confidence threshold')
    ap.add_argument('--iou-thres', type=float, default=0.45, help='IOU threshold for NMS')
    ap.add_argument('--device', default='', help='cuda device, i.e. 0 or 0,1,2,3')
    ap.add_argument('--save-txt', action='store_true', help='save results to *.txt')
    ap.add_argument('--save-conf', action='store_true', help='save confidences in --save-txt labels')
    ap.add_argument('--classes', nargs='+', type=int, help='filter by class: --class 0, or --class 0 2 3')
    ap.add_argument('--agnostic-nms', action='store_true', help='class-agnostic NMS')
    ap.add_argument('--augment', action='store_true', help='augmented inference')
    ap.add_argument('--project', default='runs/detect', help='save results to project/name')
    ap.add_argument('--name', default='exp', help='save results to project/name')
    ap.add_argument('--fp32', action='store_true', help='run the fp32 plan instead of half()')
    ap.add_argument('--quiet', action='store_true')
    return ap.parse_args(argv)


if __name__ == '__main__':
    detect(parse_opt())
