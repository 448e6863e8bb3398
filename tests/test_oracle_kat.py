"""Known-answer tests that pin the oracle to the reference's documented semantics (CPU only).

The reference ships no tests, fixtures or weights and could not be imported here, so
these cases are derived by hand from the reference source (file:line in each test) and from the
published torchvision.ops.nms algorithm.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import metrics_ref, nms_ref, yolo_ref


def _z(rows, nc=3):
    """rows: (cx, cy, w, h, obj, [cls...]) -> z [1, n, nc+5]."""
    z = torch.zeros(1, len(rows), nc + 5)
    for i, r in enumerate(rows):
        z[0, i, :5] = torch.tensor(r[:5])
        z[0, i, 5:5 + len(r[5])] = torch.tensor(r[5])
    return z


# ------------------------------------------------------------------ torchvision.ops.nms semantics

def test_nms_strict_greater_than_threshold():
    # two 10x10 boxes overlapping in a 10x5 strip: inter 50, union 150, IoU = 1/3 exactly
    boxes = torch.tensor([[0., 0., 10., 10.], [0., 5., 10., 15.]])
    scores = torch.tensor([0.9, 0.8])
    assert nms_ref.nms(boxes, scores, 1 / 3).tolist() == [0, 1]        # IoU == thr: kept (strict >)
    assert nms_ref.nms(boxes, scores, 0.33).tolist() == [0]            # IoU > thr: suppressed
    assert nms_ref.nms_py(boxes, scores, 1 / 3) == [0, 1]


def test_nms_stable_ties_and_order():
    boxes = torch.tensor([[0., 0., 1., 1.], [10., 10., 11., 11.], [20., 20., 21., 21.], [0., 0., 1., 1.]])
    scores = torch.tensor([0.5, 0.7, 0.7, 0.5])
    # descending score, ties in input order; box 3 duplicates box 0 (IoU 1) and is suppressed
    assert nms_ref.nms(boxes, scores, 0.5).tolist() == [1, 2, 0]


def test_nms_no_plus_one_area_and_touching_boxes():
    # touching boxes: inter 0 -> never suppressed; degenerate zero-area box kept
    boxes = torch.tensor([[0., 0., 10., 10.], [10., 0., 20., 10.], [5., 5., 5., 5.]])
    scores = torch.tensor([0.9, 0.8, 0.7])
    assert nms_ref.nms(boxes, scores, 0.0).tolist() == [0, 1, 2]


@pytest.mark.parametrize('seed', range(5))
def test_nms_c_matches_python(seed):
    g = torch.Generator().manual_seed(seed)
    n = 300
    xy = torch.rand(n, 2, generator=g) * 100
    wh = torch.rand(n, 2, generator=g) * 30 + 1
    boxes = torch.cat((xy, xy + wh), 1)
    scores = (torch.rand(n, generator=g) * 20).floor() / 20  # many exact ties
    for thr in (0.1, 0.45, 0.7):
        assert nms_ref.nms(boxes, scores, thr).tolist() == nms_ref.nms_py(boxes, scores, thr)


# ------------------------------------------------------------------ non_max_suppression (general.py:628-720)

def test_nms_pipeline_conf_product_argmax_and_offset():
    z = _z([
        (50, 50, 20, 20, 0.9, [0.1, 0.8, 0.8]),   # conf = 0.72 class 1 (first max of a tie)
        (52, 50, 20, 20, 0.9, [0.7, 0.1, 0.1]),   # conf = 0.63 class 0, overlaps row 0, other class
        (51, 50, 20, 20, 0.8, [0.1, 0.7, 0.1]),   # conf = 0.56 class 1, overlaps row 0 -> suppressed
        (200, 200, 10, 10, 0.25, [1.0, 0.0, 0.0]),  # obj == conf_thres: dropped by strict >
        (300, 300, 10, 10, 0.9, [0.2, 0.2, 0.2]),   # best conf 0.18 < 0.25: dropped
    ])
    out, rows = nms_ref.non_max_suppression(z, 0.25, 0.45, return_rows=True)
    assert rows[0].tolist() == [0, 1]
    d = out[0]
    assert d[:, 5].tolist() == [1.0, 0.0]
    assert d[0, 4].item() == pytest.approx(0.9 * 0.8)
    assert d[0, :4].tolist() == [40.0, 40.0, 60.0, 60.0]     # xywh2xyxy (general.py:275-282)
    # agnostic: the class-0 box overlapping row 0 is suppressed too
    out_a, rows_a = nms_ref.non_max_suppression(z, 0.25, 0.45, agnostic=True, return_rows=True)
    assert rows_a[0].tolist() == [0]


def test_nms_multi_label_order_and_class_filter():
    z = _z([(50, 50, 20, 20, 0.9, [0.5, 0.0, 0.9]),
            (400, 400, 20, 20, 0.8, [0.0, 0.6, 0.0])])
    out, rows = nms_ref.non_max_suppression(z, 0.3, 0.45, multi_label=True, return_rows=True)
    # candidates (row0,c0)=.45 (row0,c2)=.81 (row1,c1)=.48 -> sorted by score, class offset keeps both row0 boxes
    assert rows[0].tolist() == [0, 1, 0]
    assert out[0][:, 5].tolist() == [2.0, 1.0, 0.0]
    out_c = nms_ref.non_max_suppression(z, 0.3, 0.45, multi_label=True, classes=[1])
    assert out_c[0][:, 5].tolist() == [1.0]


def test_nms_single_class_model_and_max_det():
    z = torch.zeros(1, 400, 6)
    z[0, :, 0] = torch.arange(400) * 30.0 + 15
    z[0, :, 1] = 15
    z[0, :, 2:4] = 10
    z[0, :, 4] = torch.linspace(0.3, 0.9, 400)
    z[0, :, 5] = 0.01                       # ignored when nc == 1: conf = obj (general.py:669-670)
    out, rows = nms_ref.non_max_suppression(z, 0.25, 0.45, return_rows=True)
    assert out[0].shape[0] == 300           # max_det (general.py:705-706)
    assert rows[0][:3].tolist() == [399, 398, 397]
    assert torch.all(out[0][:, 4] == z[0, rows[0], 4])


# ------------------------------------------------------------------ decode (models/yolo.py:52-57)

def test_detect_decode_known_answer():
    net = yolo_ref.Net(layers=[], save=[], nc=1, na=1, no=6, nl=1, anchors=[[10, 20]])
    net.stride = [8.0]
    net.anchor_grid = torch.tensor([[[10.0, 20.0]]])
    raw = torch.zeros(1, 6, 2, 3)            # [bs, na*no, ny, nx], logits 0 -> sigmoid 0.5
    raw[0, 0, 1, 2] = math.log(3.0)          # sigmoid = 0.75 at (gy=1, gx=2)
    z, xs = yolo_ref.detect_decode(net, [raw])
    row = 1 * 3 + 2                          # (a*ny + gy)*nx + gx
    # xy = (0.75*2 - 0.5 + gx) * stride = (1 + 2) * 8 ; y = (0.5*2 - 0.5 + 1) * 8 = 12
    assert z[0, row, 0].item() == pytest.approx(24.0)
    assert z[0, row, 1].item() == pytest.approx(12.0)
    # wh = (0.5*2)**2 * anchor
    assert z[0, row, 2].item() == pytest.approx(10.0)
    assert z[0, row, 3].item() == pytest.approx(20.0)
    assert z[0, row, 4].item() == pytest.approx(0.5)
    assert xs[0].shape == (1, 1, 2, 3, 6)


# ------------------------------------------------------------------ folding identities

def _bn(c, g):
    bn = nn.BatchNorm2d(c, eps=1e-3).eval()
    bn.weight.data = torch.rand(c, generator=g) + 0.5
    bn.bias.data = torch.randn(c, generator=g)
    bn.running_mean.data = torch.randn(c, generator=g)
    bn.running_var.data = torch.rand(c, generator=g) + 0.5
    return bn


def test_fuse_conv_and_bn_matches_unfused():
    g = torch.Generator().manual_seed(0)
    conv = nn.Conv2d(16, 24, 3, 1, 1, bias=False)
    bn = _bn(24, g)
    w, b = yolo_ref.fuse_conv_and_bn(conv.weight.data, bn.weight.data, bn.bias.data, bn.running_mean.data,
                                     bn.running_var.data)
    x = torch.randn(2, 16, 9, 9, generator=g)
    with torch.no_grad():
        assert torch.allclose(F.conv2d(x, w, b, 1, 1), bn(conv(x)), atol=1e-5)


def test_repconv_fold_matches_branches():
    g = torch.Generator().manual_seed(1)
    c3, c1 = nn.Conv2d(8, 12, 3, 1, 1, bias=False), nn.Conv2d(8, 12, 1, 1, 0, bias=False)
    b3, b1 = _bn(12, g), _bn(12, g)
    w3, bb3 = yolo_ref._repconv_branch(c3.weight.data, b3.weight, b3.bias, b3.running_mean, b3.running_var)
    w1, bb1 = yolo_ref._repconv_branch(c1.weight.data, b1.weight, b1.bias, b1.running_mean, b1.running_var)
    w = w3 + F.pad(w1, [1, 1, 1, 1])
    x = torch.randn(1, 8, 7, 7, generator=g)
    with torch.no_grad():
        assert torch.allclose(F.conv2d(x, w, bb3 + bb1, 1, 1), b3(c3(x)) + b1(c1(x)), atol=1e-5)


def test_maxpool_cascade_equals_direct():
    """pool9 = pool5(pool5), pool13 = pool5(pool9) with -inf padding: exact (the SPPCSPC rewrite)."""
    x = torch.randn(2, 4, 20, 20, generator=torch.Generator().manual_seed(2))
    p5 = F.max_pool2d(x, 5, 1, 2)
    p9 = F.max_pool2d(p5, 5, 1, 2)
    p13 = F.max_pool2d(p9, 5, 1, 2)
    assert torch.equal(p9, F.max_pool2d(x, 9, 1, 4))
    assert torch.equal(p13, F.max_pool2d(x, 13, 1, 6))


# ------------------------------------------------------------------ mAP (utils/metrics.py:81-110)

def test_compute_ap_known_answer():
    ap, _, _ = metrics_ref.compute_ap(np.array([0.5, 1.0]), np.array([1.0, 0.5]))
    # envelope: precision 1 up to recall 0.5, 0.5 up to 1.0, 0 beyond 1.01 -> 101-pt trapezoid
    x = np.linspace(0, 1, 101)
    ref = np.trapezoid(np.interp(x, [0, 0.5, 1.0, 1.01], [1, 1, 0.5, 0]), x)
    assert ap == pytest.approx(ref)
    # one perfect detection: recall 1 at precision 1 -> the 101-point AP with the recall+0.01 sentinel
    perfect = [torch.tensor([[0., 0., 10., 10., 0.9, 1.]])]
    m50, _ = metrics_ref.map_from_lists(perfect, [torch.tensor([[1., 0., 0., 10., 10.]])])
    assert m50 == pytest.approx(1.0)
