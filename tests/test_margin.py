"""The decision-margin filter (tests/margin.py) is sound: two z tensors that differ only by float noise
give IDENTICAL kept rows from the same NMS (the oracle's restatement of general.py:628-720) once the
rows involved in noise-level decisions are removed from both.  CPU only: the oracle's fp32 forward vs
its float64 forward rounded to fp32 (a second "implementation" whose distance from exact arithmetic is
one rounding), on the synthetic yolov7-tiny at 640."""
import torch

from helpers import frames, oracle_net
from margin import noise_rows


def _kept(z, conf, iou):
    from oracle import nms_ref
    out, rows = nms_ref.non_max_suppression(z, conf, iou, return_rows=True, max_det=30000)
    return out, rows


def test_margin_filter_makes_noisy_z_agree():
    from oracle import yolo_ref
    net, fused = oracle_net('yolov7-tiny')
    x = frames(2, 640, 640, seed=41)
    zr, _ = yolo_ref.forward(net, fused, x)
    z64, _ = yolo_ref.forward64(net, fused, x)
    zo = z64.float()                      # the other "implementation"
    for conf, iou in ((0.25, 0.45), (0.1, 0.6)):
        zr2, zo2 = zr.clone(), zo.clone()
        dropped = 0
        for b in range(2):
            drop, st = noise_rows(zr[b], z64[b], zo[b], conf, iou)
            zr2[b, drop, 4] = 0.0
            zo2[b, drop, 4] = 0.0
            dropped += st['rows_dropped']
            assert st['candidates'] > 50, st
        out_r, rows_r = _kept(zr2, conf, iou)
        out_o, rows_o = _kept(zo2, conf, iou)
        for b in range(2):
            assert set(rows_r[b].tolist()) == set(rows_o[b].tolist()), (conf, b)
            cr = dict(zip(rows_r[b].tolist(), out_r[b][:, 5].tolist()))
            co = dict(zip(rows_o[b].tolist(), out_o[b][:, 5].tolist()))
            assert cr == co
        print(f'conf {conf} iou {iou}: kept {[len(r) for r in rows_r]}, rows dropped {dropped}')


def test_margin_filter_flags_threshold_cases():
    """Hand-built rows: a score exactly at noise distance from conf_thres is dropped, a robust one is
    kept; two boxes with IoU on the threshold are resolved by dropping the lower-scored one."""
    N, nc = 6, 3
    z64 = torch.zeros(N, 5 + nc, dtype=torch.float64)
    z64[:, :4] = torch.tensor([[100, 100, 20, 20]] * N, dtype=torch.float64)
    z64[:, 0] += torch.arange(N, dtype=torch.float64) * 200          # disjoint boxes
    z64[:, 4] = 0.9
    z64[:, 5] = torch.tensor([0.9, 0.25 / 0.9 + 1e-9, 0.5, 0.9, 0.9, 0.9], dtype=torch.float64)
    # rows 4 and 5: same class, IoU exactly 0.45 (x shift d: (20 - d) / (20 + d) = 0.45)
    d = 20 * 0.55 / 1.45
    z64[5, :4] = z64[4, :4]
    z64[5, 0] += d
    zr = z64.float()
    zg = (z64 + 1e-6).float()
    drop, st = noise_rows(zr, z64, zg, 0.25, 0.45)
    assert drop[1] and not drop[0] and not drop[2] and not drop[3]
    assert drop[5] != drop[4] and st['pairs_noise_iou'] == 1
