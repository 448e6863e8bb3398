"""The MP block's two readers of one tensor run as ONE register-streamed launch (csrc/conv_rs.hip, the
runtime's pair fusion in yv7_forward): `MP -> 1x1` (the plan's pool = 2 op) and the plain `1x1` beside
it (cfg/deploy/yolov7.yaml:27-30 and the head's P3 pair; MP = models/common.py:30-36, Conv =
common.py:110-111).

Checks that the default dispatch really takes the dual path on yolov7 and yolov7-tiny where the shapes
allow it (the kernel name the dry run reports for the pooled op, nothing for its partner), and that both
outputs then match plain fp32 references of the two ops on their own input (tests/opcheck.py) — at a
small frame and at a second shape with more units than waves (several units per wave: the rolling
prefetch's steady state).  Forcing a kernel variant on either op disables the pair (each op then runs
alone), which the variant sweep (test_variants.py) covers.
"""
import pytest
import torch

from helpers import fresh_model, frames
from opcheck import check_ops
from yv7 import _lib as L

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


@pytest.fixture(scope='module', autouse=True)
def _no_miopen():
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False
    yield
    torch.backends.cudnn.enabled = prev


def _pairs(g):
    """(pooled op, plain op) index pairs: adjacent 1x1 convs reading the same input slice."""
    out = []
    for i in range(len(g.ops) - 1):
        a, b = g.ops[i], g.ops[i + 1]
        if a['kind'] == b['kind'] == L.OP_CONV and a['src'] == b['src'] and a['src_coff'] == b['src_coff'] and \
                a['k'] == b['k'] == 1 and (a.get('pool', 0) == 2) != (b.get('pool', 0) == 2):
            out.append((i, i + 1) if a.get('pool', 0) == 2 else (i + 1, i))
    return out


@pytest.mark.parametrize('name,B,H,W', [('yolov7', 2, 256, 256), ('yolov7', 4, 512, 640), ('yolov7-tiny', 2, 256, 320)])
def test_dual_launch_and_parity(name, B, H, W):
    m = fresh_model(name).to(DEV).half()
    plan = m.plan()
    g = plan.graph
    pairs = _pairs(g)
    kern = plan.op_kernels(B, H, W)
    dual = []
    for pi, fi in pairs:
        first = min(pi, fi)
        if any('conv1x1_rs_kernel' in k for k in kern[first]):
            assert kern[max(pi, fi)] == [], (pi, fi, kern[max(pi, fi)])
            dual.append((pi, fi))
    if name == 'yolov7':
        # both MP blocks whose 1x1 reads <= 256 channels (128-channel consumers, W % 16 == 0 at this frame)
        assert len(dual) == 2, (pairs, [kern[min(p)] for p in pairs])
    x = frames(B, H, W, seed=7).to(DEV).half()
    z, xs = plan.forward(x)
    torch.cuda.synchronize()
    out = check_ops(plan, x, B, H, W, raw=xs, z=z)
    for pi, fi in dual:
        assert pi in out and fi in out
