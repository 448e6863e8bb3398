"""GPU parity of the forward pass (HIP kernels through the C ABI) against the CPU oracle.

Tolerances (north_star: "box coords/conf within 1e-4 fp32"): see tests/parity.py — 1e-4 wherever
the reference's own fp32 result is stable to 1e-4, else within twice the reference's own fp32
error (|z32 - z64|), and never less accurate than the reference vs float64.  Every intermediate
layer must match within 1e-4 of its own scale (max|ref|).
fp16 plan: judged like the reference's half() path — by detections / layer rms, not bits.
"""
import pytest
import torch

from helpers import fresh_model, frames, oracle_net
from parity import check_z

pytestmark = pytest.mark.gpu

DEV = 'cuda:0'


def _oracle(name, x):
    from oracle import yolo_ref
    net, fused = oracle_net(name)
    (z, xs), outs = yolo_ref.forward(net, fused, x, return_all=True)
    return z, xs, outs


def _z_err(z, zr):
    coord = ((z[..., :4] - zr[..., :4]).abs() / zr[..., :4].abs().clamp(min=1.0)).max().item()
    conf = (z[..., 4:] - zr[..., 4:]).abs().max().item()
    return coord, conf


@pytest.mark.parametrize('name,B,H,W', [('yolov7-tiny', 2, 128, 160), ('yolov7', 2, 128, 128),
                                        ('yolov7-w6', 1, 128, 192), ('yolov7-train', 1, 96, 128)])
def test_forward_fp32_layerwise(name, B, H, W):
    x = frames(B, H, W, seed=3)
    zr, xsr, outs = _oracle(name, x)
    m = fresh_model(name).to(DEV)
    plan = m.plan()
    z, xs = m(x.to(DEV))
    torch.cuda.synchronize()
    worst = (0.0, None)
    for i, (t, coff, c) in sorted(plan.graph.layer_tensor.items()):
        ref = outs[i]
        if not isinstance(ref, torch.Tensor):
            continue
        got = plan.layer_output(i, B, H, W).cpu()
        assert got.shape == ref.shape, (i, got.shape, ref.shape)
        err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
        if err > worst[0]:
            worst = (err, i)
    print(f'\n{name}: worst layer rel err {worst[0]:.3g} at layer {worst[1]}')
    assert worst[0] <= 1e-4, worst
    from oracle import yolo_ref
    net, fused = oracle_net(name)
    z64, xs64 = yolo_ref.forward64(net, fused, x)
    print(check_z(z, zr, z64, name))
    for a, b, c in zip(xs, xsr, xs64):
        assert a.shape == b.shape
        a = a.cpu().double()
        tol = 1e-4 * b.abs().clamp(min=1.0) + 2 * (b.double() - c).abs()
        assert ((a - b.double()).abs() <= tol).all()


@pytest.mark.parametrize('name,B,H,W', [('yolov7', 1, 640, 640), ('yolov7-tiny', 1, 640, 640)])
def test_forward_fp32_full_size(name, B, H, W):
    x = frames(B, H, W, seed=4)
    from oracle import yolo_ref
    net, fused = oracle_net(name)
    zr, xsr = yolo_ref.forward(net, fused, x)
    z64, _ = yolo_ref.forward64(net, fused, x)
    m = fresh_model(name).to(DEV)
    z, xs = m(x.to(DEV))
    print('\n' + check_z(z, zr, z64, f'{name} @{H}'))


@pytest.mark.parametrize('name,B,H,W', [('yolov7', 2, 128, 128), ('yolov7-w6', 1, 256, 320)])
def test_forward_fp16_layerwise_scale(name, B, H, W):
    """fp16 plan (the bench path): every layer within fp16 precision of the fp32 oracle (rms).  Small
    frames put the deep 3x3 layers on the split-K ring (two and four K parts)."""
    x = frames(B, H, W, seed=5)
    zr, xsr, outs = _oracle(name, x)
    m = fresh_model(name).to(DEV).half()
    plan = m.plan()
    z, xs = m(x.to(DEV).half())
    torch.cuda.synchronize()
    worst = 0.0
    for i, (t, coff, c) in sorted(plan.graph.layer_tensor.items()):
        ref = outs[i]
        if not isinstance(ref, torch.Tensor):
            continue
        got = plan.layer_output(i, B, H, W).cpu()
        rms = ref.pow(2).mean().sqrt().item()
        err = (got - ref).pow(2).mean().sqrt().item() / max(rms, 1e-3)
        worst = max(worst, err)
    print(f'\n{name} fp16: worst layer rms-rel err {worst:.3g}')
    assert worst < 0.05


@pytest.mark.parametrize('name', ['yolov7', 'yolov7-tiny', 'yolov7-w6'])
def test_forward_fp16_map_parity(name):
    """fp16 plan judged like the reference's half() path (BASELINE metric: mAP@0.5 parity vs ref):
    mAP@0.5 of the GPU fp16 detections against the oracle's fp32 detections taken as ground truth
    (both conf 0.25 / iou 0.45), on 8 frames.  The bar is the oracle's own fp16-storage emulation of
    the reference's half() path (oracle.yolo_ref.forward(half_storage=True)) scored the same way,
    minus 0.01: the fp16 plan is at least as faithful as the reference's half() path."""
    from oracle import metrics_ref, nms_ref, yolo_ref
    from utils.general import non_max_suppression
    x = frames(8, 640, 640, seed=8)
    net, fused = oracle_net(name)
    zr, _ = yolo_ref.forward(net, fused, x)
    z16e, _ = yolo_ref.forward(net, fused, x, half_storage=True)
    gt = [metrics_ref.dets_as_labels(d) for d in nms_ref.non_max_suppression(zr, 0.25, 0.45)]
    emu_map, _ = metrics_ref.map_from_lists(nms_ref.non_max_suppression(z16e, 0.25, 0.45), gt)
    m = fresh_model(name).to(DEV).half()
    z, _ = m(x.to(DEV).half())
    pred = non_max_suppression(z, 0.25, 0.45)
    m50, m5095 = metrics_ref.map_from_lists(pred, gt)
    zc = z.cpu().double()
    sc = zr.double().abs().clamp(min=1)
    print(f'\n{name} fp16: mAP@0.5 {m50:.4f} (reference-half emulation {emu_map:.4f}), mAP@.5:.95 {m5095:.4f}; '
          f'z vs fp32 oracle: coord rel {((zc - zr.double()).abs() / sc)[..., :4].max():.3g}, '
          f'vs half emulation {((zc - z16e.double()).abs() / sc)[..., :4].max():.3g}')
    assert m50 >= emu_map - 0.01 and m50 >= 0.95


@pytest.mark.gpu
@pytest.mark.parametrize('name,H,W', [('yolov7', 128, 192), ('yolov7-w6', 256, 192)])
def test_fp16_plan_fp32_input_matches_fp16_input(name, H, W):
    """The fused stems read the image in either precision (csrc/stem.hip: stem2_kernel's fp32 single-pixel
    loads, stem_reorg_kernel's fp32 pixel pairs); converting in the kernel must give the same fp16 patch
    as converting on the host (round to nearest even both ways), so z is bit-identical."""
    x = frames(2, H, W, seed=11)
    m = fresh_model(name).to(DEV).half()
    z16, _ = m(x.to(DEV).half())
    z32, _ = m(x.to(DEV).float())
    torch.cuda.synchronize()
    assert torch.equal(z16, z32)
