"""TEST INFRASTRUCTURE ONLY — restatement of the reference's mAP evaluation (see oracle/__init__.py).

  match_image     test.py:181-208   per-class IoU matching of predictions to targets at 10 IoU thresholds
  ap_per_class    utils/metrics.py:18-78
  compute_ap      utils/metrics.py:81-110 (101-point interpolation, default non-v5 sentinel recall[-1]+0.01)
  map_from_lists  test.py:218-227   mAP@0.5 and mAP@0.5:0.95 over a set of images
"""
from __future__ import annotations

import numpy as np
import torch

IOUV = torch.linspace(0.5, 0.95, 10)

_trapz = getattr(np, 'trapezoid', None) or np.trapz


def box_iou(box1, box2):  # utils/general.py:464-486
    def area(b):
        return (b[2] - b[0]) * (b[3] - b[1])
    a1, a2 = area(box1.T), area(box2.T)
    inter = (torch.min(box1[:, None, 2:], box2[:, 2:]) - torch.max(box1[:, None, :2], box2[:, :2])).clamp(0).prod(2)
    return inter / (a1[:, None] + a2 - inter)


def match_image(pred, labels, iouv=IOUV):
    """pred [n,6] (xyxy, conf, cls), labels [m,5] (cls, xyxy) -> correct [n, len(iouv)] bool."""
    correct = torch.zeros(pred.shape[0], len(iouv), dtype=torch.bool)
    nl = labels.shape[0]
    if nl and pred.shape[0]:
        detected = []
        tcls = labels[:, 0]
        tbox = labels[:, 1:5]
        for cls in torch.unique(tcls):
            ti = (cls == tcls).nonzero(as_tuple=False).view(-1)
            pi = (cls == pred[:, 5]).nonzero(as_tuple=False).view(-1)
            if pi.shape[0]:
                ious, i = box_iou(pred[pi, :4], tbox[ti]).max(1)
                detected_set = set()
                for j in (ious > iouv[0]).nonzero(as_tuple=False):
                    d = ti[i[j]]
                    if d.item() not in detected_set:
                        detected_set.add(d.item())
                        detected.append(d)
                        correct[pi[j]] = ious[j] > iouv
                        if len(detected) == nl:
                            break
    return correct


def compute_ap(recall, precision, v5_metric=False):
    mrec = np.concatenate(([0.], recall, [1.0] if v5_metric else [recall[-1] + 0.01]))
    mpre = np.concatenate(([1.], precision, [0.]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    return _trapz(np.interp(x, mrec, mpre), x), mpre, mrec


def ap_per_class(tp, conf, pred_cls, target_cls, v5_metric=False):
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
    """preds: list of [n,6] tensors per image; labels: list of [m,5] (cls, xyxy) -> (mAP@0.5, mAP@0.5:0.95)."""
    stats = []
    for pred, lab in zip(preds, labels):
        pred, lab = pred.detach().cpu().float(), lab.detach().cpu().float()
        tcls = lab[:, 0].tolist()
        if pred.shape[0] == 0:
            if len(tcls):
                stats.append((torch.zeros(0, len(IOUV), dtype=torch.bool), torch.Tensor(), torch.Tensor(), tcls))
            continue
        stats.append((match_image(pred, lab), pred[:, 4], pred[:, 5], tcls))
    stats = [np.concatenate(x, 0) for x in zip(*stats)]
    if len(stats) and stats[0].any():
        p, r, ap, f1, ap_class = ap_per_class(*stats)
        return float(ap[:, 0].mean()), float(ap.mean(1).mean())
    return 0.0, 0.0


def dets_as_labels(dets):
    """Turn reference detections [n,6] (xyxy, conf, cls) into labels [n,5] (cls, xyxy)."""
    dets = dets.detach().cpu().float()
    return torch.cat((dets[:, 5:6], dets[:, :4]), 1)
