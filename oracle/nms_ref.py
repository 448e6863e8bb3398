"""TEST INFRASTRUCTURE ONLY — CPU restatement of non_max_suppression (utils/general.py:628-720).

The per-image filtering runs the same torch CPU ops in the same order as the reference
(obj > conf mask :637/:653, cls *= obj :669-673, xywh2xyxy :676 / general.py:275-282, single-label
first-max :683-684 or multi-label row-major nonzero :680-681, class filter :687-688, max_nms
truncation :698-699, class offset max_wh=4096 :702-703, max_det :705-706).  torchvision.ops.nms
(:704) is restated in C (oracle/nms_ref.c); `nms_py` is a pure-Python version for small cases.

Besides the reference's list of [n,6] tensors, `non_max_suppression(..., return_rows=True)` also
returns the anchor-row index of every kept detection (the "kept-box indices" the north star
requires bit-exact).  Deliberate differences from the reference, documented in DESIGN.md:
  * the 10 s wall-clock time limit (:716-718) is not restated (it makes outputs timing-dependent);
  * the max_nms truncation uses a stable sort (the reference's argsort is unstable, so its tie order
    there is implementation-defined);
  * `labels` (autolabelling) is supported as in :657-663.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, 'build', 'liboracle_nms.so')
        if not os.path.exists(path):
            subprocess.check_call(['make', '-s', '-C', _HERE])
        lib = ctypes.CDLL(path)
        lib.oracle_nms.restype = ctypes.c_int64
        lib.oracle_nms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_float,
                                   ctypes.c_void_p]
        _LIB = lib
    return _LIB


def nms(boxes: torch.Tensor, scores: torch.Tensor, iou_thres: float) -> torch.Tensor:
    """torchvision.ops.nms restated (C). boxes [n,4] xyxy fp32, scores [n] -> int64 kept indices."""
    b = np.ascontiguousarray(boxes.detach().cpu().numpy(), dtype=np.float32)
    s = np.ascontiguousarray(scores.detach().cpu().numpy(), dtype=np.float32)
    n = b.shape[0]
    keep = np.empty(max(n, 1), dtype=np.int64)
    k = _lib().oracle_nms(b.ctypes.data, s.ctypes.data, n, ctypes.c_float(iou_thres), keep.ctypes.data)
    return torch.from_numpy(keep[:k].copy())


def nms_py(boxes, scores, iou_thres):
    """Pure-Python torchvision.ops.nms restatement (fp32 via numpy scalars); small n only."""
    b = np.asarray(boxes, dtype=np.float32)
    s = np.asarray(scores, dtype=np.float32)
    n = len(s)
    order = sorted(range(n), key=lambda i: (-float(s[i]), i))
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    supp = [False] * n
    keep = []
    f32 = np.float32
    for a, i in enumerate(order):
        if supp[i]:
            continue
        keep.append(i)
        for j in order[a + 1:]:
            if supp[j]:
                continue
            w = max(f32(0), f32(min(b[i, 2], b[j, 2]) - max(b[i, 0], b[j, 0])))
            h = max(f32(0), f32(min(b[i, 3], b[j, 3]) - max(b[i, 1], b[j, 1])))
            inter = f32(w * h)
            if f32(inter / f32(f32(area[i] + area[j]) - inter)) > f32(iou_thres):
                supp[j] = True
    return keep


def xywh2xyxy(x):  # utils/general.py:275-282
    y = x.clone()
    y[:, 0] = x[:, 0] - x[:, 2] / 2
    y[:, 1] = x[:, 1] - x[:, 3] / 2
    y[:, 2] = x[:, 0] + x[:, 2] / 2
    y[:, 3] = x[:, 1] + x[:, 3] / 2
    return y


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), return_rows=False, max_det=300, max_nms=30000):
    prediction = prediction.detach().cpu().float()
    nc = prediction.shape[2] - 5
    xc = prediction[..., 4] > conf_thres
    max_wh = 4096
    multi_label &= nc > 1
    output = [torch.zeros((0, 6))] * prediction.shape[0]
    rows_out = [torch.zeros((0,), dtype=torch.int64)] * prediction.shape[0]
    for xi, x in enumerate(prediction):
        rows = torch.nonzero(xc[xi]).view(-1)
        x = x[xc[xi]]
        if labels and len(labels[xi]):
            lab = labels[xi]
            v = torch.zeros((len(lab), nc + 5))
            v[:, :4] = lab[:, 1:5]
            v[:, 4] = 1.0
            v[range(len(lab)), lab[:, 0].long() + 5] = 1.0
            x = torch.cat((x, v), 0)
            rows = torch.cat((rows, torch.full((len(lab),), -1, dtype=torch.int64)))
        if not x.shape[0]:
            continue
        if nc == 1:
            x[:, 5:] = x[:, 4:5]
        else:
            x[:, 5:] *= x[:, 4:5]
        box = xywh2xyxy(x[:, :4])
        if multi_label:
            i, j = (x[:, 5:] > conf_thres).nonzero(as_tuple=False).T
            x = torch.cat((box[i], x[i, j + 5, None], j[:, None].float()), 1)
            rows = rows[i]
        else:
            conf, j = x[:, 5:].max(1, keepdim=True)
            m = conf.view(-1) > conf_thres
            x = torch.cat((box, conf, j.float()), 1)[m]
            rows = rows[m]
        if classes is not None:
            m = (x[:, 5:6] == torch.tensor(classes)).any(1)
            x, rows = x[m], rows[m]
        n = x.shape[0]
        if not n:
            continue
        elif n > max_nms:
            o = torch.sort(x[:, 4], descending=True, stable=True).indices[:max_nms]
            x, rows = x[o], rows[o]
        c = x[:, 5:6] * (0 if agnostic else max_wh)
        boxes, scores = x[:, :4] + c, x[:, 4]
        i = nms(boxes, scores, iou_thres)
        if i.shape[0] > max_det:
            i = i[:max_det]
        output[xi] = x[i]
        rows_out[xi] = rows[i]
    return (output, rows_out) if return_rows else output


def scale_coords(img1_shape, coords, img0_shape):
    """utils/general.py:340-361 (ratio_pad=None): letterboxed xyxy -> original-image pixels, clipped.
    detect.py:183 then applies .round()."""
    gain = min(img1_shape[0] / img0_shape[0], img1_shape[1] / img0_shape[1])
    padw, padh = (img1_shape[1] - img0_shape[1] * gain) / 2, (img1_shape[0] - img0_shape[0] * gain) / 2
    c = coords.clone()
    c[:, [0, 2]] -= padw
    c[:, [1, 3]] -= padh
    c[:, :4] /= gain
    c[:, 0].clamp_(0, img0_shape[1])
    c[:, 1].clamp_(0, img0_shape[0])
    c[:, 2].clamp_(0, img0_shape[1])
    c[:, 3].clamp_(0, img0_shape[0])
    return c


def end2end(prediction, conf_thres=0.25, iou_thres=0.45, topk=100, max_nms=65536):
    """The End2End / EfficientNMS_TRT output contract (models/experimental.py:195-241, TRT_NMS
    111-156; inf_onnx_trt.py:27-36 reads it): ONNX_TRT hands the plugin boxes = z[..., :4] (xywh,
    box_coding 1) and scores = z[..., 5:] * z[..., 4:5] (z[..., 4:5] when nc == 1); the plugin keeps
    every (box, class) with score > score_threshold, suppresses within a class only (no class
    offset, background_class -1) where IoU > iou_threshold on the corner boxes, and returns the top
    max_output_boxes by score: num_dets int32 [B,1], det_boxes [B,topk,4] xyxy, det_scores [B,topk],
    det_classes int32 [B,topk], zero-padded.  The TensorRT plugin is not in the reference (nor this
    image), so this restates its published algorithm; ties resolve like the rest of the oracle (stable
    descending score order, candidates row-major then class) and at most max_nms candidates enter
    the suppression.  Parity unpinned at the plugin boundary."""
    z = prediction.detach().cpu().float()
    B, N, no = z.shape
    nc = no - 5
    num = torch.zeros((B, 1), dtype=torch.int32)
    boxes = torch.zeros((B, topk, 4))
    scores = torch.zeros((B, topk))
    classes = torch.zeros((B, topk), dtype=torch.int32)
    for b in range(B):
        x = z[b]
        box = xywh2xyxy(x[:, :4])
        sc = x[:, 4:5].clone() if nc == 1 else x[:, 5:] * x[:, 4:5]
        i, j = (sc > conf_thres).nonzero(as_tuple=False).T
        if not i.numel():
            continue
        s = sc[i, j]
        o = torch.sort(s, descending=True, stable=True).indices[:max_nms]
        i, j, s = i[o], j[o], s[o]
        kept = []
        for c in j.unique().tolist():
            idx = (j == c).nonzero().view(-1)       # ascending = score order within the class
            k = nms(box[i[idx]], s[idx], iou_thres)
            kept.append(idx[k])
        kept = torch.sort(torch.cat(kept)).values[:topk]   # back to the global score order
        n = kept.numel()
        num[b, 0] = n
        boxes[b, :n] = box[i[kept]]
        scores[b, :n] = s[kept]
        classes[b, :n] = j[kept].to(torch.int32)
    return num, boxes, scores, classes
