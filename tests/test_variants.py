"""Every kernel configuration of the fp16 conv dispatch, forced onto every conv op of a real network
(yv7_set_op_variant), checked op by op against a plain PyTorch fp32 reference of the same op on the
op's own input (tests/opcheck.py).

The tuned dispatch (csrc/conv_f16.hip launch_conv_f16 / choose) picks among these by tile count, so
a small frame exercises only some of them; forcing each one on every layer shape of yolov7 /
yolov7-tiny covers them all: the generic tile kernels (1, 2, 8), the 8-wave LDS-DMA rings (4-7),
the halo and weight-stationary 3x3 kernels (10, 11, and 15: its half-patch ring form), every ring configuration with 1, 2 and 4 K
splits (1CS: configuration C, S splits; the split-K hand-off of splitk_reduce), the persistent rings
(201-206), the 8-phase rings (231: 256 x 256, 232: 256 x 128), the weight-stationary 1x1 rings (234-236,
and 239: N-split), the column-group 3x3 halo ring (262), the
low-resolution 3x3 kernel (270-273: 80 / 64-pixel tiles of 4 images x 4 columns, 128 / 64 channels;
274 / 277-279: stride 2; 275 / 276: 160-pixel tiles), the register-weight 3x3 kernel (280-284: stride 2,
285-288: stride 1; cin 64 / 128, 2-5 ring slots, 2-8-row tiles, with and without the stagger), the register-weight 1x1 kernel (290-295: cin 128 / 256 / 512, with and
without the stagger; 302 / 303: cin 256 with 128-channel N slices) and
the alternative Detect heads (92, 97, and 99: the 64 x 256 ring that was the default before the
persistent head).  A variant a layer's shape
does not support falls back to the tuned kernel, which the check then covers again.
Reference computation: models/common.py:110-111 (Conv.fuseforward), models/yolo.py:46-57 (Detect).
"""
import pytest
import torch

from helpers import fresh_model, frames
from opcheck import check_ops, kernel_summary
from yv7 import _lib as L

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'

CONV_VARIANTS = [1, 2, 4, 5, 6, 7, 8, 10, 11, 15, 17,
                 100, 102, 104, 110, 112, 114, 120, 122, 124, 130, 132, 134, 140, 142, 144, 150, 152, 154,
                 201, 202, 203, 204, 205, 206, 231, 232, 234, 235, 236, 239, 262, 270, 271, 272, 273, 274, 275, 276,
                 277, 278, 279, 280, 281, 282, 283, 284, 285, 286, 287, 288, 290, 291, 292, 293,
                 294, 295, 302, 303]
DET_VARIANTS = [92, 94, 97, 99]


@pytest.fixture(scope='module', autouse=True)
def _no_miopen():
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    yield
    torch.backends.cudnn.enabled = prev


@pytest.mark.parametrize('name,B,H,W', [('yolov7', 2, 256, 256), ('yolov7-tiny', 2, 192, 256)])
def test_every_conv_variant(name, B, H, W):
    m = fresh_model(name).to(DEV).half()
    plan = m.plan()
    x = frames(B, H, W, seed=31).to(DEV).half()
    convs = [i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_CONV]
    dets = [i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_DETECT]
    lines = []
    for v in CONV_VARIANTS + DET_VARIANTS:
        for i in (dets if v in DET_VARIANTS else convs):
            plan.set_op_variant(i, v)
        z, xs = plan.forward(x)
        torch.cuda.synchronize()
        out = check_ops(plan, x, B, H, W, raw=xs, z=z)
        lines.append(f'variant {v}: ' + kernel_summary(out))
        for i in (dets if v in DET_VARIANTS else convs):
            plan.set_op_variant(i, 0)
    print('\n' + '\n'.join(lines))


# A net with the shapes the fragment kernels mask: 3x3 layers with cout % 32 == 16 (cout = 80:
# the permlane16 pair store of the 32-channel pair 64..95 is half masked), stride-2 layers with cin 64
# and 128 (conv_s2.hip's two weight layouts), and batches with a partial trailing 4-image group after
# full ones (B = 5, 6).  ADVICE r5: 1x1 layers with the register-weight kernel's input widths (cin 128 /
# 256 / 512, conv_w1.hip) and outputs of 80 / 144 channels (cout % 32 == 16: masked pair store), so the
# forced w1 variants really launch on a half-masked N slice and a partial pixel tile (layers 8, 10, 12).
RAGGED = {'nc': 3, 'depth_multiple': 1.0, 'width_multiple': 1.0,
          'anchors': [[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]],
          'backbone': [[-1, 1, 'Conv', [32, 3, 1]],    # 0  @1
                       [-1, 1, 'Conv', [64, 3, 2]],    # 1  @2
                       [-1, 1, 'Conv', [80, 3, 1]],    # 2  lr, cin 64 -> 80
                       [-1, 1, 'Conv', [64, 1, 1]],    # 3
                       [-1, 1, 'Conv', [80, 3, 2]],    # 4  @4: s2, cin 64 -> 80
                       [-1, 1, 'Conv', [128, 1, 1]],   # 5
                       [-1, 1, 'Conv', [80, 3, 2]],    # 6  @8: s2, cin 128 -> 80
                       [-1, 1, 'Conv', [128, 1, 1]],   # 7
                       [-1, 1, 'Conv', [80, 1, 1]],    # 8  w1, cin 128 -> 80
                       [-1, 1, 'Conv', [256, 1, 1]],   # 9
                       [-1, 1, 'Conv', [144, 1, 1]],   # 10 w1, cin 256 -> 144
                       [-1, 1, 'Conv', [512, 1, 1]],   # 11
                       [-1, 1, 'Conv', [80, 1, 1]],    # 12 w1, cin 512 -> 80
                       [-1, 1, 'Conv', [128, 1, 1]],   # 13
                       [-1, 1, 'Conv', [80, 3, 1]],    # 14 lr, cin 128 -> 80 (P3)
                       [-1, 1, 'Conv', [64, 1, 1]],    # 15
                       [-1, 1, 'Conv', [80, 3, 2]],    # 16 @16: s2, cin 64 (P4)
                       [-1, 1, 'Conv', [128, 1, 1]],   # 17
                       [-1, 1, 'Conv', [96, 3, 2]]],   # 18 @32: s2, cin 128 (P5)
          'head': [[[14, 16, 18], 1, 'Detect', ['nc', 'anchors']]]}
# register-weight 1x1 configurations (conv_w1.hip W1_CFGS) -> the input width each one takes
W1_CIN = {290: 128, 291: 256, 292: 512, 293: 256, 294: 128, 295: 512, 302: 256, 303: 256}


@pytest.mark.parametrize('B', [5, 6])
def test_fragment_kernels_ragged(B):
    """The fragment kernels (conv_lr.hip 270-279, conv_s2.hip 280-288, conv_w1.hip 290-295, 302-303) on partial
    trailing image groups / pixel tiles and half-masked channel pairs, op by op against fp32 torch.  A forced
    w1 variant must actually launch conv1x1_rw_kernel on every 1x1 layer of its input width (no silent
    fallback to the tuned kernel)."""
    import copy
    from models.yolo import Model
    from yv7.synthetic import synthetic_state_dict
    m = Model(copy.deepcopy(RAGGED))
    m.load_state_dict(synthetic_state_dict(m, seed=3, calib_hw=256))
    m = m.float().eval().fuse().to(DEV).half()
    plan = m.plan()
    H = W = 256
    x = frames(B, H, W, seed=7).to(DEV).half()
    convs = [i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_CONV]
    lines = []
    for v in [0, 270, 271, 272, 273, 274, 275, 276, 277, 278, 279, 280, 281, 282, 283, 284, 285, 286, 287, 288,
              290, 291, 292, 293, 294, 295, 302, 303]:
        for i in convs:
            plan.set_op_variant(i, v)
        if v in W1_CIN:
            ks = plan.op_kernels(B, H, W)
            want = [i for i in convs if plan.graph.ops[i].get('k', 1) == 1 and plan.graph.ops[i]['cin'] == W1_CIN[v]
                    and plan.graph.ops[i]['cout'] % 32 == 16]
            assert want, f'variant {v}: no 1x1 layer with cin {W1_CIN[v]} and a half-masked channel pair'
            for i in want:
                assert any('conv1x1_rw_kernel' in k for k in ks[i]), (v, i, ks[i])
        z, xs = plan.forward(x)
        torch.cuda.synchronize()
        out = check_ops(plan, x, B, H, W, raw=xs, z=z)
        lines.append(f'variant {v}: ' + kernel_summary(out))
        for i in convs:
            plan.set_op_variant(i, 0)
    print('\n' + '\n'.join(lines))


def test_variant_api_rejects_hooks():
    """Microbenchmark hooks (which skip work on purpose) and unchecked experiment schedules (the
    round-2 ws64 / 8-phase scheduling experiments 18-19, 241-255) cannot be forced through the ABI (17 is
    now the 8-wave ws64 form, a kernel configuration)."""
    m = fresh_model('yolov7-tiny').to(DEV).half()
    plan = m.plan()
    conv = next(i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_CONV)
    for v in (12, 13, 14, 16, 18, 19, 90, 91, 93, 94, 298, 160, 190, 105, 211, 221, 233, 237, 238, 240, 241,
              248, 255, 259, 260, 261, 263, 289, 296, 299, 300, 301, 304, 911):
        with pytest.raises(RuntimeError):
            plan.set_op_variant(conv, v)
    # the Detect op: the detbench hooks (91, 93, 95, 96, 98 reach launch_det_pring) are refused, the
    # alternative heads the suite checks (92, 94, 97, 99) are accepted
    det = next(i for i, o in enumerate(plan.graph.ops) if o['kind'] == L.OP_DETECT)
    for v in (91, 93, 95, 96, 98):
        with pytest.raises(RuntimeError):
            plan.set_op_variant(det, v)
    for v in DET_VARIANTS:
        plan.set_op_variant(det, v)
    plan.set_op_variant(det, 0)
    with pytest.raises(RuntimeError):
        plan.set_op_variant(len(plan.graph.ops) + 3, 0)
