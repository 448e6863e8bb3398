"""BASELINE.json configs[4]: yolov7 640x640 with fp8 weights — the fp16 plan whose 1x1 convs run on
OCP e4m3 weights and activations through the block-scaled fp8 MFMA (csrc/conv_f8.hip).

The reference has no fp8 path; parity is anchored on (i) the e4m3 rounding itself (known answers for
torch.float8_e4m3fn, RNE with saturation, and the GPU quantizer bit-exact against it), (ii) the oracle's
restatement of the fp8 plan's arithmetic (oracle.yolo_ref.fp8_fused: per-channel e4m3 weights,
per-tensor e4m3 activations, fp32 accumulation) — the CPU plan interpreter and the GPU plan against it —
and (iii) the metric's mAP@0.5 parity of the GPU fp8 detections against the oracle's fp32 ones."""
import math

import pytest
import torch

import plan_interp
from helpers import fresh_model, frames, oracle_net
from oracle import metrics_ref, nms_ref, yolo_ref
from yv7 import _lib as L
from yv7.graph import compile_model, fp8_candidates, fp8_weight_scales


def test_e4m3_known_answers():
    f = yolo_ref.fp8_e4m3
    t = torch.tensor([1.0, 0.3, 448.0, 500.0, -1000.0, 2.0 ** -9, 2.0 ** -10, 3 * 2.0 ** -10, 17.0, 19.0, 0.28125])
    want = [1.0, 0.3125, 448.0, 448.0, -448.0, 2.0 ** -9, 0.0, 2.0 ** -8, 16.0, 20.0, 0.28125]
    assert f(t).tolist() == want   # RNE: 2^-10 and 17 are ties to the even neighbour, 19 -> 20


def _entries(g):
    return [(tuple(tag), o['xscale']) for o in g.ops if o.get('wfmt', 0) == L.WFMT_FP8 for tag in o['layers']]


def _calibrated_fp8_graph(m, x):
    """fp8 graph with activation scales from the CPU interpreter's fp16-graph tensors (the GPU plan
    takes them from its own fp16 forward, yv7.runtime.Plan.fp8_from_model)."""
    g16 = compile_model(m, L.DT_F16)
    _, T = plan_interp.run(g16, x, return_tensors=True)
    scales = {}
    for i in fp8_candidates(g16, 0):   # every eligible 1x1 (the product plan marks the wide ones)
        o = g16.ops[i]
        amax = float(T[o['src']][:, o['src_coff']:o['src_coff'] + o['cin']].abs().max())
        scales[i] = 2.0 ** math.ceil(math.log2(amax / 448.0)) if amax > 0 else 1.0
    return g16, compile_model(m, L.DT_F16, fp8=scales)


def test_fp8_graph_packing():
    m = fresh_model('yolov7')
    x = frames(1, 64, 64, seed=2)
    g16, g8 = _calibrated_fp8_graph(m, x)
    f8 = [o for o in g8.ops if o.get('wfmt', 0) == L.WFMT_FP8]
    assert len(f8) == len(fp8_candidates(g16, 0)) > 25 and len(fp8_candidates(g16)) > 10
    assert all(o['kind'] == L.OP_CONV and o['k'] == 1 for o in f8)
    assert not any(o.get('wfmt', 0) for o in g8.ops if o['kind'] == L.OP_DETECT)
    for o in f8:
        xs = o['xscale']
        assert xs > 0 and math.log2(xs) == round(math.log2(xs))       # power of two
    # one op's packed e4m3 weights and scales == the per-channel quantization of the fused weights
    blob = g8.weight_blob()
    o = f8[3]
    (layer, sub), = o['layers'][:1] if len(o['layers']) == 1 else [o['layers'][0]]
    conv = m.model[layer] if sub is None else getattr(m.model[layer], f'cv{sub}')
    w, _ = conv.fused_weight_bias()
    wk = w.reshape(w.shape[0], -1)[:o['cout']]
    ws = fp8_weight_scales(wk)
    got = plan_interp._weights_f8(blob, o['w_off'], o['cout'], o['cin'], o['s_off']).reshape(o['cout'], -1)
    want = yolo_ref.fp8_e4m3(wk / ws[:, None]) * ws[:, None]
    assert torch.equal(got[:wk.shape[0], :wk.shape[1]], want)


@pytest.mark.parametrize('name', ['yolov7', 'yolov7-tiny'])
def test_fp8_plan_semantics_vs_oracle_emulation(name):
    """Every fp8 op of the compiled plan, run by the CPU interpreter, against the oracle's restatement
    (oracle.yolo_ref.fp8_fused: its own per-channel e4m3 quantization of the fused fp32 weights, e4m3
    input on the op's scale) applied to the same input tensor.  Per op, because e4m3 rounding makes the
    whole random-weight network chaotic: a 1e-6 upstream difference flips roundings that compound over
    40 quantized layers (end-to-end z differs by several %; mAP is the end-to-end criterion)."""
    import torch.nn.functional as F
    m = fresh_model(name)
    x = frames(1, 128, 128, seed=3)
    _, g8 = _calibrated_fp8_graph(m, x)
    net, fused = oracle_net(name)
    emu = yolo_ref.fp8_fused(fused, _entries(g8))
    with torch.no_grad():
        _, T = plan_interp.run(g8, x, return_tensors=True)
    acts = {L.ACT_SILU: F.silu, L.ACT_LEAKY: lambda t: F.leaky_relu(t, 0.1), L.ACT_NONE: lambda t: t}
    n = 0
    for o in g8.ops:
        if o.get('wfmt', 0) != L.WFMT_FP8:
            continue
        parts = [emu[l] if sub is None else emu[l][sub] for l, sub in o['layers']]
        w = torch.cat([p[0] for p in parts], 0)
        b = torch.cat([p[1] for p in parts], 0)
        assert all(p[2] == o['xscale'] for p in parts)
        xin = T[o['src']][:, o['src_coff']:o['src_coff'] + o['cin']]
        want = acts[o['act']](F.conv2d(yolo_ref.fp8_e4m3(xin / o['xscale']) * o['xscale'], w, b))
        got = T[o['dst']][:, o['dst_coff']:o['dst_coff'] + o['cout']]
        torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5 * float(want.abs().max()))
        n += 1
    assert n > 20


# ------------------------------------------------------------------------------------------ GPU
def _gpu_fp8_plan(name, calib, min_cout=None):
    """min_cout=0: every eligible 1x1 conv in fp8 (kernel coverage); None: the product plan's choice."""
    from yv7.runtime import Plan
    m = fresh_model(name).cuda().half()
    return Plan.fp8_from_model(m, 'cuda:0', calib=calib, min_cout=min_cout)


@pytest.mark.gpu
def test_gpu_fp8_quantizer_bit_exact():
    """The GPU quantizer (v_cvt_pk_fp8_f32 after a power-of-two scale and +-448 clamp) writes exactly
    torch.float8_e4m3fn's bytes for the fp16 input it read (checked on the last fp8 op of a forward)."""
    B, H, W = 2, 128, 160
    x = frames(B, H, W, seed=5)
    plan = _gpu_fp8_plan('yolov7', x, 0)
    ops = [i for i, o in enumerate(plan.graph.ops) if o.get('wfmt', 0) == L.WFMT_FP8]
    for i in ops:
        plan.set_op_variant(i, 81)   # the staged configuration: a separate quantize pass into the buffer
    z = torch.empty(B, plan.num_rows(H, W), plan.no, device='cuda:0')
    plan.forward_into(x.cuda().half(), z)
    torch.cuda.synchronize()
    o = plan.graph.ops[ops[-1]]
    src = plan.tensor_view(o['src'], B, H, W)[..., o['src_coff']:o['src_coff'] + o['cin']].float().cpu()
    M, cin = src.numel() // o['cin'], o['cin']
    kp = (cin + 127) // 128 * 128
    want = torch.zeros(M, kp, dtype=torch.uint8)
    want[:, :cin] = (src.reshape(M, cin) / o['xscale']).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    got = plan.f8_scratch(B, H, W)[:M * kp].view(M, kp).cpu()
    assert torch.equal(got, want), int((got != want).sum())


@pytest.mark.gpu
@pytest.mark.parametrize('name,B,H,W', [('yolov7', 2, 128, 160), ('yolov7-tiny', 3, 96, 224)])
def test_gpu_fp8_fused_quantize_matches_staged(name, B, H, W):
    """Variant 82 quantizes the fp16 input in registers on the way into LDS; variant 81 (staged) writes
    the e4m3 copy with the separate, bit-exact quantizer first.  Same bytes in LDS, same MFMA order: the
    two forwards agree bit for bit on every tensor (and the default dispatch mixes the two per layer)."""
    x = frames(B, H, W, seed=12)
    plan = _gpu_fp8_plan(name, x, 0)
    ops = [i for i, o in enumerate(plan.graph.ops) if o.get('wfmt', 0) == L.WFMT_FP8]
    xd = x.cuda().half()
    for i in ops:
        plan.set_op_variant(i, 82)
    z0, r0 = plan.forward(xd)
    t0 = [plan.tensor_view(t, B, H, W).clone() for t in range(len(plan.graph.tensors))]
    for i in ops:
        plan.set_op_variant(i, 81)
    z1, r1 = plan.forward(xd)
    torch.cuda.synchronize()
    for t, a in enumerate(t0):
        assert torch.equal(a, plan.tensor_view(t, B, H, W)), f'tensor {t}'
    assert torch.equal(z0, z1) and all(torch.equal(a, b) for a, b in zip(r0, r1))


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['yolov7', 'yolov7-tiny'])
def test_gpu_fp8_map_parity(name):
    """configs[4] parity: mAP@0.5 of the GPU fp8 plan's detections against the oracle's fp32 detections
    (the metric's ground truth), next to the oracle's restatement of the fp8 arithmetic on the same scales
    (fp16 storage elsewhere) scored the same way; conf 0.25 / iou 0.45, 32 frames at 640 in ONE batch of
    32 (the bench's fp8 dispatch).

    Why 32 frames: e4m3 rounding is chaotic — an fp16 input one ulp away rounds to
    the neighbouring e4m3 value — so the GPU plan and the restatement agree with each other only at mAP
    ~0.6-0.85, and on 2 frames their scores against the fp32 oracle differed by up to 0.04 either way
    (round 4: 0.539 vs 0.560 for yolov7).  Over 32 frames that per-frame chaos averages out, so the
    round-3 bar is back: the GPU plan may trail the restatement of its own arithmetic by at most 0.02.
    The absolute floors only catch a collapse (they are not fitted: e4m3 on both operands costs this
    random-weight network about half its detections)."""
    NF = 32
    x = frames(NF, 640, 640, seed=8)
    plan = _gpu_fp8_plan(name, None)
    z, _ = plan.forward(x.cuda().half(), want_raw=False)
    pred = [d.cpu() for d in nms_ref.non_max_suppression(z.cpu(), 0.25, 0.45)]
    net, fused = oracle_net(name)
    f8 = yolo_ref.fp8_fused(fused, _entries(plan.graph))
    with torch.no_grad():
        zr = torch.cat([yolo_ref.forward(net, fused, x[i:i + 4])[0] for i in range(0, NF, 4)])
        ze = torch.cat([yolo_ref.forward(net, f8, x[i:i + 4], half_storage=True)[0] for i in range(0, NF, 4)])
    gt = [metrics_ref.dets_as_labels(d) for d in nms_ref.non_max_suppression(zr, 0.25, 0.45)]
    ge = [metrics_ref.dets_as_labels(d) for d in nms_ref.non_max_suppression(ze, 0.25, 0.45)]
    m32, _ = metrics_ref.map_from_lists(pred, gt)
    memu, _ = metrics_ref.map_from_lists(pred, ge)
    emu32, _ = metrics_ref.map_from_lists([d for d in nms_ref.non_max_suppression(ze, 0.25, 0.45)], gt)
    print(f'\n{name} fp8 ({NF} frames): mAP@0.5 vs fp32 oracle {m32:.4f} (oracle fp8 restatement vs fp32: '
          f'{emu32:.4f}), vs fp8 restatement {memu:.4f}; dets/frame {sum(len(d) for d in pred) / NF:.1f}')
    assert m32 >= emu32 - 0.02
    # absolute floors = the 32-frame values measured on MI355X (round 5: yolov7 0.467, tiny 0.592,
    # profiles/r5_lines/fp8_map.log) minus 0.05 of noise margin (VERDICT r5 item 6 / ADVICE r5); do not
    # lower them without a failing run that explains why
    assert m32 >= {'yolov7': 0.42, 'yolov7-tiny': 0.54}[name]


@pytest.mark.gpu
@pytest.mark.parametrize('name', ['yolov7', 'yolov7-tiny'])
def test_gpu_fp8_layerwise(name):
    """Every fp8 op of a GPU forward against the restatement applied to the very fp16 input the op read
    (so the comparison does not depend on upstream rounding): e4m3 input on the op's scale, the plan's
    e4m3 weights and scales, fp32 accumulation, bias, activation.  Output within 2e-3 of max|y| (fp16
    output rounding plus accumulation order)."""
    import torch.nn.functional as F
    B, H, W = 1, 128, 128
    x = frames(B, H, W, seed=9)
    plan = _gpu_fp8_plan(name, x, 0)
    z = torch.empty(B, plan.num_rows(H, W), plan.no, device='cuda:0')
    plan.forward_into(x.cuda().half(), z)
    torch.cuda.synchronize()
    blob = plan.graph.weight_blob()
    acts = {L.ACT_SILU: F.silu, L.ACT_LEAKY: lambda t: F.leaky_relu(t, 0.1), L.ACT_NONE: lambda t: t}
    worst = 0.0
    n = 0
    for o in plan.graph.ops:
        if o.get('wfmt', 0) != L.WFMT_FP8:
            continue
        xin = plan.tensor_view(o['src'], B, H, W)[..., o['src_coff']:o['src_coff'] + o['cin']].float().cpu()
        xq = yolo_ref.fp8_e4m3(xin / o['xscale']) * o['xscale']
        w = plan_interp._weights_f8(blob, o['w_off'], o['cout'], o['cin'], o['s_off']).reshape(o['cout'], -1)
        b = plan_interp._bias(blob, o['b_off'], o['cout'])
        want = acts[o['act']](xq @ w.t() + b)
        got = plan.tensor_view(o['dst'], B, H, W)[..., o['dst_coff']:o['dst_coff'] + o['cout']].float().cpu()
        err = ((got - want).abs().max() / want.abs().max().clamp(min=1e-3)).item()
        worst = max(worst, err)
        n += 1
    print(f'\n{name}: {n} fp8 ops, worst max-norm rel err {worst:.3g}')
    assert n > 10 and worst < 2e-3
