"""BASELINE.json configs[0]: yolov7-tiny 640x640 bs=1 on the reference's samples/bus.jpg (copied as a
data fixture, tests/golden/bus.jpg) through detect.py's path (detect.py:41-183).

CPU (not gpu): the oracle's restatement of the reference CPU path on bus.jpg — decode, letterbox
(auto=False, datasets.py:196: 1080x810 -> 480x640 + 80 px each side), forward, NMS, scale_coords.
GPU: the product's detect.py (GPU letterbox, libyv7 forward, GPU NMS, scale_coords) on the same file:
fp32 plan z within the parity criterion and NMS bit-exact on identical z; the final boxes against the
oracle's; fp16 (detect.py's half default) by mAP@0.5 against the oracle's fp32 detections.
The frame is decoded by PIL (cv2 absent: decode parity unpinned) — identically for both sides."""
import os

import numpy as np
import pytest
import torch

from helpers import oracle_net

BUS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'bus.jpg')


def _oracle_bus(name='yolov7-tiny'):
    from oracle import letterbox_ref as R, nms_ref, yolo_ref
    from utils.datasets import imread
    img0 = imread(BUS)
    lb, ratio, dwdh = R.letterbox(img0, 640, auto=False)
    x = R.to_input(lb, half=False)[None]
    net, fused = oracle_net(name)
    with torch.no_grad():
        z, _ = yolo_ref.forward(net, fused, x)
    det = nms_ref.non_max_suppression(z, 0.25, 0.45)[0]
    det[:, :4] = nms_ref.scale_coords(x.shape[2:], det[:, :4], img0.shape).round()
    return img0, lb, x, z, det


def test_bus_jpg_oracle_path():
    img0, lb, x, z, det = _oracle_bus()
    assert img0.shape == (1080, 810, 3) and img0.dtype == np.uint8
    assert lb.shape == (640, 640, 3) and (lb[:, :80] == 114).all() and (lb[:, 560:] == 114).all()
    assert x.shape == (1, 3, 640, 640) and z.shape == (1, 25200, 85)
    assert det.shape[1] == 6 and 0 < len(det) <= 300
    # boxes live inside the original frame, sorted by descending confidence (general.py:704-706)
    assert (det[:, [0, 2]] >= 0).all() and (det[:, [0, 2]] <= 810).all()
    assert (det[:, [1, 3]] >= 0).all() and (det[:, [1, 3]] <= 1080).all()
    assert (det[1:, 4] <= det[:-1, 4]).all()


def _detect(fp32):
    import detect
    opt = detect.parse_opt(['--cfg', 'yolov7-tiny', '--source', BUS, '--quiet'] + (['--fp32'] if fp32 else []))
    return detect.detect(opt)


@pytest.mark.gpu
def test_bus_jpg_detect_fp32():
    from oracle import letterbox_ref as R, nms_ref
    from utils.datasets import letterbox_batch
    from utils.general import non_max_suppression
    from helpers import fresh_model
    from parity import check_z
    from oracle import yolo_ref
    img0, lb, x, zr, det_r = _oracle_bus()
    # model input: GPU letterbox + conversion == oracle's, bit for bit
    xg, _, _ = letterbox_batch(torch.from_numpy(img0).cuda(), 640, half=False)
    assert torch.equal(xg.cpu(), x)
    net, fused = oracle_net('yolov7-tiny')
    z64, _ = yolo_ref.forward64(net, fused, x)
    m = fresh_model('yolov7-tiny').cuda()
    z, _ = m(xg)
    print('\n' + check_z(z, zr, z64, 'bus.jpg yolov7-tiny fp32'))
    out_g, rows_g = non_max_suppression(z, 0.25, 0.45, return_rows=True)
    out_r, rows_r = nms_ref.non_max_suppression(z.cpu(), 0.25, 0.45, return_rows=True)
    assert torch.equal(rows_g[0].cpu(), rows_r[0]) and torch.equal(out_g[0].cpu(), out_r[0])
    # the whole detect.py loop against the oracle's own chain
    (path, det), = _detect(fp32=True)
    assert det.shape == det_r.shape, (det.shape, det_r.shape)
    assert torch.equal(det[:, 5], det_r[:, 5])
    assert (det[:, :4] - det_r[:, :4]).abs().max() <= 1.0          # .round() of coords within 1e-4 rel
    assert (det[:, 4] - det_r[:, 4]).abs().max() <= 1e-4


@pytest.mark.gpu
def test_bus_jpg_detect_fp16_map():
    """detect.py's default half() path, judged like the reference's own half() path: mAP@0.5 of the
    detections against the oracle's fp32 ones, next to the oracle's fp16-storage emulation of the
    reference half path on the same frame (bus.jpg lights up ~20k candidate rows of this synthetic
    head, so the 300-detection cut falls among near-tied scores and costs both paths the same)."""
    from oracle import metrics_ref, nms_ref, yolo_ref
    img0, _, x, _, det_r = _oracle_bus()
    net, fused = oracle_net('yolov7-tiny')
    with torch.no_grad():
        ze, _ = yolo_ref.forward(net, fused, x, half_storage=True)
    de = nms_ref.non_max_suppression(ze, 0.25, 0.45)[0]
    de[:, :4] = nms_ref.scale_coords(x.shape[2:], de[:, :4], img0.shape).round()
    truth = [metrics_ref.dets_as_labels(det_r)]
    emu, _ = metrics_ref.map_from_lists([de], truth)
    (path, det), = _detect(fp32=False)
    m50, _ = metrics_ref.map_from_lists([det], truth)
    print(f'\nbus.jpg yolov7-tiny fp16: {len(det)} dets (oracle fp32 {len(det_r)}), mAP@0.5 {m50:.4f} '
          f'(reference-half emulation {emu:.4f})')
    assert m50 >= emu - 0.02
