"""mAP evaluation — the "mAP@0.5 parity" half of the metric.

Mirrors the reference's test.py statistics and utils/metrics.py:
  match_predictions  test.py:181-208: per image, per class, every prediction (in the NMS output's
                     descending-confidence order) takes its best-IoU target; a target already taken by
                     an earlier prediction is not taken again; correct at 10 IoU thresholds 0.5:0.95.
                     Vectorised on the device: the first claimant of a target (lowest prediction index
                     among those with IoU > 0.5) is the one the reference's sequential loop accepts.
  ap_per_class       utils/metrics.py:18-78   (host numpy, as the reference)
  compute_ap         utils/metrics.py:81-110  (101-point interpolation, v5_metric=False sentinel)
  map_from_lists     test.py:218-227          mAP@0.5 and mAP@0.5:0.95 over a set of images
"""
from __future__ import annotations

import numpy as np
import torch

_trapz = getattr(np, 'trapezoid', None) or np.trapz


def iou_thresholds(device=None):
    return torch.linspace(0.5, 0.95, 10, device=device)   # test.py:92


def box_iou(box1, box2):
    """utils/general.py:464-486: pairwise IoU of xyxy boxes [N,4] x [M,4] -> [N,M]."""
    def area(b):
        return (b[2] - b[0]) * (b[3] - b[1])
    a1, a2 = area(box1.T), area(box2.T)
    inter = (torch.min(box1[:, None, 2:], box2[:, 2:]) - torch.max(box1[:, None, :2], box2[:, :2])).clamp(0).prod(2)
    return inter / (a1[:, None] + a2 - inter)


def match_predictions(pred, labels, iouv=None):
    """pred [n,6] (xyxy, conf, cls) in NMS order, labels [m,5] (cls, xyxy) -> correct [n, 10] bool."""
    dev = pred.device
    iouv = iou_thresholds(dev) if iouv is None else iouv.to(dev)
    n, m = pred.shape[0], labels.shape[0]
    correct = torch.zeros(n, iouv.numel(), dtype=torch.bool, device=dev)
    if n == 0 or m == 0:
        return correct
    labels = labels.to(dev)
    iou = box_iou(pred[:, :4], labels[:, 1:5])
    iou = torch.where(pred[:, 5:6] == labels[None, :, 0], iou, torch.full_like(iou, -1.0))  # same class only
    best, tgt = iou.max(1)            # each prediction's best target (first maximum, as torch .max)
    valid = best > iouv[0]
    # the first valid claimant of every target wins (test.py:197-204 'detected' bookkeeping)
    idx = torch.arange(n, device=dev)
    first = torch.full((m,), n, dtype=torch.long, device=dev)
    first.scatter_reduce_(0, tgt[valid], idx[valid], reduce='amin')
    win = valid & (first[tgt] == idx)
    correct[win] = best[win, None] > iouv
    return correct


def compute_ap(recall, precision, v5_metric=False):
    """utils/metrics.py:81-110."""
    mrec = np.concatenate(([0.], recall, [1.0] if v5_metric else [recall[-1] + 0.01]))
    mpre = np.concatenate(([1.], precision, [0.]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    return _trapz(np.interp(x, mrec, mpre), x), mpre, mrec


def ap_per_class(tp, conf, pred_cls, target_cls, v5_metric=False):
    """utils/metrics.py:18-78 (plots omitted): (p, r, ap [nc, 10], f1, classes)."""
    i = np.argsort(-conf)
    tp, conf, pred_cls = tp[i], conf[i], pred_cls[i]
    unique_classes = np.unique(target_cls)
    nc = unique_classes.shape[0]
    px = np.linspace(0, 1, 1000)
    ap, p, r = np.zeros((nc, tp.shape[1])), np.zeros((nc, 1000)), np.zeros((nc, 1000))
    for ci, c in enumerate(unique_classes):
        i = pred_cls == c
        n_l = (target_cls == c).sum()
        n_p = i.sum()
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[i]).cumsum(0)
        tpc = tp[i].cumsum(0)
        recall = tpc / (n_l + 1e-16)
        r[ci] = np.interp(-px, -conf[i], recall[:, 0], left=0)
        precision = tpc / (tpc + fpc)
        p[ci] = np.interp(-px, -conf[i], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j], _, _ = compute_ap(recall[:, j], precision[:, j], v5_metric=v5_metric)
    f1 = 2 * p * r / (p + r + 1e-16)
    i = f1.mean(0).argmax()
    return p[:, i], r[:, i], ap, f1[:, i], unique_classes.astype('int32')


def map_from_lists(preds, labels):
    """preds: per image [n,6] (xyxy, conf, cls); labels: per image [m,5] (cls, xyxy) ->
    (mAP@0.5, mAP@0.5:0.95) as test.py:218-227 computes them."""
    stats = []
    for pred, lab in zip(preds, labels):
        tcls = lab[:, 0].tolist()
        if pred.shape[0] == 0:
            if len(tcls):
                stats.append((np.zeros((0, 10), bool), np.zeros(0), np.zeros(0), tcls))
            continue
        c = match_predictions(pred.float(), lab.float())
        stats.append((c.cpu().numpy(), pred[:, 4].float().cpu().numpy(), pred[:, 5].float().cpu().numpy(), tcls))
    stats = [np.concatenate(x, 0) for x in zip(*stats)]
    if len(stats) and stats[0].any():
        _, _, ap, _, _ = ap_per_class(*stats)
        return float(ap[:, 0].mean()), float(ap.mean(1).mean())
    return 0.0, 0.0


def dets_as_labels(dets):
    """Detections [n,6] (xyxy, conf, cls) of a reference run -> labels [n,5] (cls, xyxy), the parity
    check's ground truth."""
    return torch.cat((dets[:, 5:6], dets[:, :4]), 1)
