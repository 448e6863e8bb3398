"""Decision-margin filter for end-to-end NMS index parity (SURVEY §7.2 hard part 4).

Two fp32 forwards of the same network (the GPU plan and the CPU oracle) sum in different orders, so
their z differ by float noise (tests/parity.py).  non_max_suppression (utils/general.py:628-720) turns
z into discrete decisions — obj > conf_thres (:653), class argmax and obj*cls > conf_thres (:683-684),
the stable descending score order and IoU(offset boxes) > iou_thres (:702-704, torchvision.ops.nms) —
and a decision whose operands sit within that noise of its threshold (or of each other) can legitimately
come out either way.  Every other decision must agree, so after removing the candidates involved in a
noise-level decision the two kept-index lists must be EQUAL (north_star: "kept-box indices bit-exact").

Noise per element is anchored on the float64 forward: e = |z_ref32 - z64| + |z_gpu - z64|, each
implementation's own distance from exact arithmetic, and a decision is "within noise" when its float64
operand lies within 2x the propagated e of the threshold.  IoU decisions are judged the way the
reference computes them: fp32 on class-offset boxes (max_wh = 4096), whose rounding at offsets up to
79 * 4096 is part of the noise (|IoU_32 - IoU_64| of both sides).
Test infrastructure only (tests/ imports it); the product never does.
"""
from __future__ import annotations

import torch

MAX_WH = 4096


def _xyxy(b):
    return torch.stack((b[:, 0] - b[:, 2] / 2, b[:, 1] - b[:, 3] / 2, b[:, 0] + b[:, 2] / 2, b[:, 1] + b[:, 3] / 2), 1)


def _iou32(bx, cls):
    """Pairwise IoU the reference's way: fp32 xyxy boxes + class * 4096 (general.py:702-703), inter /
    (area_i + area_j - inter) as torchvision's CPU kernel evaluates it."""
    b = _xyxy(bx.float()) + (cls.float() * MAX_WH)[:, None]
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = torch.maximum(b[:, None, :2], b[None, :, :2])
    rb = torch.minimum(b[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area[:, None] + area[None, :] - inter)


def _iou64(bx):
    b = _xyxy(bx.double())
    area = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    lt = torch.maximum(b[:, None, :2], b[None, :, :2])
    rb = torch.minimum(b[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    return inter / (area[:, None] + area[None, :] - inter)


def noise_rows(zr, z64, zg, conf_thres, iou_thres, factor=2.0):
    """One image's z [N, no] from the oracle (fp32), the oracle in float64 and the GPU (fp32).
    Returns (drop: bool [N] — rows involved in a noise-level NMS decision, stats dict).  Single-label
    NMS with class offsets (detect.py's call)."""
    zr, z64, zg = zr.double(), z64.double(), zg.double()
    e = (zr - z64).abs() + (zg - z64).abs()
    N, no = z64.shape
    obj64, cls64 = z64[:, 4], z64[:, 5:]
    eo, ec = e[:, 4], e[:, 5:]
    tiny = 1e-7   # ~1 fp32 ulp at 1: the product obj * cls is rounded once more
    conf64 = cls64 * obj64[:, None]
    econf = ec * obj64[:, None] + cls64 * eo[:, None] + tiny
    drop = (obj64 - conf_thres).abs() <= factor * eo + tiny
    live = obj64 > conf_thres
    best64, bi = conf64.max(1)
    eb = econf.gather(1, bi[:, None]).view(-1)
    drop |= live & ((best64 - conf_thres).abs() <= factor * eb)
    # argmax: the runner-up within noise of the best (general.py:683, first maximum)
    second = conf64.clone()
    second.scatter_(1, bi[:, None], -1.0)
    s2, si = second.max(1)
    es2 = econf.gather(1, si[:, None]).view(-1)
    drop |= live & (best64 > conf_thres) & (best64 - s2 <= factor * (eb + es2))
    cand = live & (best64 > conf_thres) & ~drop
    stats = {'rows_noise_conf': int(drop.sum())}
    # pairs within one class: IoU within noise of iou_thres, or interacting (IoU near or above the
    # threshold) with scores within noise of each other (their greedy order can flip)
    idx = cand.nonzero().view(-1)
    cls = bi[idx]
    n_iou = n_ord = 0
    for c in cls.unique():
        m = idx[cls == c]
        if len(m) < 2:
            continue
        i64 = _iou64(z64[m, :4])
        ir = _iou32(zr[m, :4], cls.new_full((len(m),), int(c)))
        ig = _iou32(zg[m, :4], cls.new_full((len(m),), int(c)))
        ie = (ir.double() - i64).abs() + (ig.double() - i64).abs() + 1e-7
        amb = (i64 - iou_thres).abs() <= factor * ie
        s = best64[m]
        es = eb[m]
        close = (s[:, None] - s[None, :]).abs() <= factor * (es[:, None] + es[None, :])
        inter = i64 + factor * ie > iou_thres
        ordr = close & inter
        amb.fill_diagonal_(False)
        ordr.fill_diagonal_(False)
        n_iou += int(amb.triu(1).sum())
        n_ord += int((ordr & ~amb).triu(1).sum())
        bad = amb | ordr
        if bad.any():
            a, b = bad.triu(1).nonzero().T
            # drop the lower-scored member of every noise-level pair (rank by float64 score, then row)
            lo = torch.where(s[a] < s[b], a, torch.where(s[a] > s[b], b, torch.maximum(a, b)))
            drop[m[lo]] = True
    stats.update(pairs_noise_iou=n_iou, pairs_noise_order=n_ord, rows_dropped=int(drop.sum()),
                 candidates=int(cand.sum()))
    return drop, stats


def tail_tied(scores, factor_noise):
    """True where a kept row's score is within noise of its successor's (their output order may swap)."""
    if len(scores) < 2:
        return torch.zeros(len(scores), dtype=torch.bool)
    d = (scores[:-1] - scores[1:]).abs() <= factor_noise[:-1] + factor_noise[1:]
    return torch.cat((d, d.new_zeros(1)))
