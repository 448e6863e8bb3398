"""GPU parity of the forward pass (HIP kernels through the C ABI) against the CPU oracle.

Tolerances (north_star: "box coords/conf within 1e-4 fp32"):
  fp32 plan: z coordinates |d| <= 1e-4 * max(1, |ref|), objectness / class conf |d| <= 1e-4,
             raw head logits |d| <= 1e-4 * max(1, |ref|); every intermediate layer within 1e-4
             of its own scale (max|ref|).
  fp16 plan: judged like the reference's half() path — detections, not bits (see test_gpu_fp16_*).
"""
import pytest
import torch

from helpers import fresh_model, frames, oracle_net

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
    coord, conf = _z_err(z.cpu(), zr)
    print(f'{name}: z coord rel err {coord:.3g}, conf abs err {conf:.3g}')
    assert coord <= 1e-4 and conf <= 1e-4
    for a, b in zip(xs, xsr):
        assert a.shape == b.shape
        assert ((a.cpu() - b).abs() / b.abs().clamp(min=1.0)).max().item() <= 1e-4


@pytest.mark.parametrize('name,B,H,W', [('yolov7', 1, 640, 640), ('yolov7-tiny', 1, 640, 640)])
def test_forward_fp32_full_size(name, B, H, W):
    x = frames(B, H, W, seed=4)
    from oracle import yolo_ref
    net, fused = oracle_net(name)
    zr, xsr = yolo_ref.forward(net, fused, x)
    m = fresh_model(name).to(DEV)
    z, xs = m(x.to(DEV))
    coord, conf = _z_err(z.cpu(), zr)
    print(f'\n{name} @{H}: z coord rel err {coord:.3g}, conf abs err {conf:.3g}')
    assert coord <= 1e-4 and conf <= 1e-4


def test_forward_fp16_layerwise_scale():
    """fp16 plan (the bench path): every layer within fp16 precision of the fp32 oracle."""
    name, B, H, W = 'yolov7', 2, 128, 128
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
    coord, conf = _z_err(z.cpu(), zr)
    print(f'\nfp16: worst layer rms-rel err {worst:.3g}; z coord rel {coord:.3g} conf abs {conf:.3g}')
    assert worst < 0.05
