"""Post-processing API — mirror of the reference's utils/general.py subset on the inference path.

non_max_suppression keeps the reference signature and return type (utils/general.py:628-720) but
runs the whole batch as HIP kernels (libyv7 yv7_nms: candidate filter, conf product, argmax or
multi-label expansion, class filter, class-offset boxes, stable score sort, greedy IoU
suppression, max_det) in one stream-ordered call; the only host sync is reading the per-image
counts to build the returned list, exactly where the reference's semantics need it.
The small box helpers below are plain tensor math on the caller's device.
"""
from __future__ import annotations

import math

import torch

from yv7 import _lib

MAX_WH = 4096      # general.py:640
MAX_DET = 300      # general.py:641
MAX_NMS = 30000    # general.py:642


def make_divisible(x, divisor):  # general.py:177-179
    return math.ceil(x / divisor) * divisor


def check_img_size(img_size, s=32):  # general.py:124-129
    new_size = make_divisible(img_size, int(s))
    if new_size != img_size:
        print('WARNING: --img-size %g must be multiple of max stride %g, updating to %g' % (img_size, s, new_size))
    return new_size


def xyxy2xywh(x):  # general.py:256-263
    y = x.clone()
    y[:, 0] = (x[:, 0] + x[:, 2]) / 2
    y[:, 1] = (x[:, 1] + x[:, 3]) / 2
    y[:, 2] = x[:, 2] - x[:, 0]
    y[:, 3] = x[:, 3] - x[:, 1]
    return y


def xywh2xyxy(x):  # general.py:275-282
    y = x.clone()
    y[:, 0] = x[:, 0] - x[:, 2] / 2
    y[:, 1] = x[:, 1] - x[:, 3] / 2
    y[:, 2] = x[:, 0] + x[:, 2] / 2
    y[:, 3] = x[:, 1] + x[:, 3] / 2
    return y


def clip_coords(boxes, img_shape):  # general.py:356-361
    boxes[:, 0].clamp_(0, img_shape[1])
    boxes[:, 1].clamp_(0, img_shape[0])
    boxes[:, 2].clamp_(0, img_shape[1])
    boxes[:, 3].clamp_(0, img_shape[0])


def scale_coords(img1_shape, coords, img0_shape, ratio_pad=None):  # general.py:340-353
    if ratio_pad is None:
        gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
        pad = (img1_shape[1] - img0_shape[1] * gain) / 2, (img1_shape[0] - img0_shape[0] * gain) / 2
    else:
        gain = ratio_pad[0][0]
        pad = ratio_pad[1]
    coords[:, [0, 2]] -= pad[0]
    coords[:, [1, 3]] -= pad[1]
    coords[:, :4] /= gain
    clip_coords(coords, img0_shape)
    return coords


def box_iou(box1, box2):  # general.py:464-486
    def box_area(box):
        return (box[2] - box[0]) * (box[3] - box[1])

    area1 = box_area(box1.T)
    area2 = box_area(box2.T)
    inter = (torch.min(box1[:, None, 2:], box2[:, 2:]) - torch.max(box1[:, None, :2], box2[:, :2])).clamp(0).prod(2)
    return inter / (area1[:, None] + area2 - inter)


class _NmsWorkspace:
    """Device scratch for yv7_nms, grown on demand and reused across calls — one buffer per (device,
    stream): calls on one stream are ordered, calls on different streams (several batches in flight)
    may run concurrently and must not share scratch."""

    def __init__(self):
        self.buf = {}

    def get(self, device, nbytes, stream=0):
        key = (device, stream)
        t = self.buf.get(key)
        if t is None or t.numel() < nbytes:
            t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device)
            self.buf[key] = t
        return t


_WS = _NmsWorkspace()


def nms_batched(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False, multi_label=False,
                max_det=MAX_DET, max_nms=MAX_NMS, out=None, rowbest=None):
    """Stream-ordered batched NMS: returns device tensors (det [B,max_det,6], src_row [B,max_det], count [B]).

    rowbest: the forward's per-row score records (Plan.forward_into(..., rowbest=)); found automatically
    for a z returned by Model.forward / Plan.forward that has not been modified since."""
    if not prediction.is_cuda:
        raise RuntimeError('non_max_suppression runs on a ROCm device (libyv7); got a CPU tensor')
    if rowbest is None:
        from yv7.runtime import row_scores
        rowbest = row_scores.lookup(prediction)
    z = prediction.detach()
    if z.dtype != torch.float32:
        z = z.float()
    z = z.contiguous()
    B, N, no = z.shape
    dev = z.device
    if out is None:
        det = torch.empty((B, max_det, 6), dtype=torch.float32, device=dev)
        src = torch.empty((B, max_det), dtype=torch.int64, device=dev)
        cnt = torch.empty((B,), dtype=torch.int32, device=dev)
    else:
        det, src, cnt = out
    cls_t = None
    ncls = 0
    if classes is not None:
        cls_t = torch.tensor(list(classes), dtype=torch.int32, device=dev)
        ncls = cls_t.numel()
    L = _lib.lib()
    multi = int(bool(multi_label))
    nbytes = L.yv7_nms_workspace_bytes(B, N, no, multi, max_nms)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ws = _WS.get(dev, nbytes, stream)
    with torch.cuda.device(dev):
        rc = L.yv7_nms(z.data_ptr(), rowbest.data_ptr() if rowbest is not None else None, B, N, no,
                       float(conf_thres), float(iou_thres), multi, int(bool(agnostic)),
                       cls_t.data_ptr() if cls_t is not None else None, ncls, max_det, max_nms, det.data_ptr(),
                       src.data_ptr(), cnt.data_ptr(), ws.data_ptr(), ws.numel(), stream)
    _lib.check(rc, 'yv7_nms')
    return det, src, cnt


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False, multi_label=False,
                        labels=(), return_rows=False):
    """Runs NMS on inference results.  Returns a list of [n_i, 6] tensors (xyxy, conf, cls) per image;
    with return_rows=True also the anchor-row index of every kept box."""
    if labels and any(len(l) for l in labels):
        raise NotImplementedError('autolabelling (labels=...) is not part of the MI355X inference path')
    det, src, cnt = nms_batched(prediction, conf_thres, iou_thres, classes, agnostic, multi_label)
    counts = cnt.tolist()  # the one host sync: variable-length outputs
    out = [det[i, :n] for i, n in enumerate(counts)]
    if return_rows:
        return out, [src[i, :n] for i, n in enumerate(counts)]
    return out


def end2end(prediction, conf_thres=0.25, iou_thres=0.45, topk=100):
    """EfficientNMS_TRT-shaped outputs (models/experimental.py:111-156, End2End 226-241):
    (num_dets int32 [B,1], det_boxes [B,topk,4], det_scores [B,topk], det_classes int32 [B,topk])."""
    if not prediction.is_cuda:
        raise RuntimeError('end2end runs on a ROCm device (libyv7); got a CPU tensor')
    z = prediction.detach().float().contiguous()
    B, N, no = z.shape
    dev = z.device
    num = torch.empty((B, 1), dtype=torch.int32, device=dev)
    boxes = torch.empty((B, topk, 4), dtype=torch.float32, device=dev)
    scores = torch.empty((B, topk), dtype=torch.float32, device=dev)
    cls = torch.empty((B, topk), dtype=torch.int32, device=dev)
    L = _lib.lib()
    nbytes = L.yv7_end2end_workspace_bytes(B, N, no, topk)
    stream = torch.cuda.current_stream(dev).cuda_stream
    ws = _WS.get(dev, nbytes, stream)
    with torch.cuda.device(dev):
        rc = L.yv7_end2end(z.data_ptr(), B, N, no, float(conf_thres), float(iou_thres), topk, num.data_ptr(),
                           boxes.data_ptr(), scores.data_ptr(), cls.data_ptr(), ws.data_ptr(), ws.numel(), stream)
    _lib.check(rc, 'yv7_end2end')
    return num, boxes, scores, cls
