"""Model-level paths on the GPU against the oracle: workspace layouts that alternate between calls,
test-time augmentation (models/yolo.py:582-597), Ensemble (models/experimental.py:69-81) and a
reference-format pickled checkpoint through attempt_load (experimental.py:247-270).

Workspace: libyv7 trusts the zero frame of a workspace it has already cleared for a layout
(include/yv7.h).  (B, H, W) and (B, W, H) have the same byte size, so when the plan drops one and
allocates the other the caching allocator hands back the same block — the frame must be cleared
again for the new layout, or the 3x3 convs read the old layout's activations as padding.  TTA runs
three shapes per call, so it walks exactly this path.
"""
import pytest
import torch

from helpers import fresh_model, frames, model_and_weights, oracle_net
from parity import check_z

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'


@pytest.fixture(scope='module', autouse=True)
def _no_miopen():
    prev = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False   # TTA's bilinear resize etc. on native kernels
    yield
    torch.backends.cudnn.enabled = prev


def _check(m, name, x, label):
    from oracle import yolo_ref
    net, fused = oracle_net(name)
    z, _ = m(x.to(DEV))
    zr, _ = yolo_ref.forward(net, fused, x)
    z64, _ = yolo_ref.forward64(net, fused, x)
    return check_z(z, zr, z64, label)


def test_workspace_layouts_alternate():
    name = 'yolov7-tiny'
    m = fresh_model(name).to(DEV)
    shapes = [(2, 128, 160), (2, 160, 128), (2, 128, 160), (1, 192, 128), (2, 160, 128)]
    for k, (B, H, W) in enumerate(shapes):
        print('\n' + _check(m, name, frames(B, H, W, seed=40 + k), f'{name} {B}x{H}x{W} (call {k})'))


def test_workspace_layouts_alternate_fp16():
    """fp16 plan (the bench path): a transposed layout after another must give the same z as a fresh
    plan on that layout (bit for bit: same kernels, same data)."""
    name = 'yolov7'
    x1, x2 = frames(2, 128, 192, seed=50).to(DEV).half(), frames(2, 192, 128, seed=51).to(DEV).half()
    z1_ref, _ = fresh_model(name).to(DEV).half()(x1)     # each layout on a plan that never saw another
    z2_ref, _ = fresh_model(name).to(DEV).half()(x2)
    m = fresh_model(name).to(DEV).half()
    for rep in range(2):
        z1, _ = m(x1)
        z2, _ = m(x2)
        assert torch.equal(z1, z1_ref) and torch.equal(z2, z2_ref), rep


def test_tta_matches_oracle_twice():
    from oracle import yolo_ref
    name = 'yolov7-tiny'
    net, fused = oracle_net(name)
    m = fresh_model(name).to(DEV)
    x = frames(2, 160, 224, seed=44)
    zr = yolo_ref.forward_augment(net, fused, x)
    z64 = yolo_ref.forward_augment(net, fused, x, f64=True)
    for rep in range(2):
        z, none = m(x.to(DEV), augment=True)
        assert none is None and z.shape == zr.shape
        print('\n' + check_z(z, zr, z64, f'{name} TTA call {rep}'))
        # a plain forward between TTA calls still matches
        print(_check(m, name, x, f'{name} plain after TTA {rep}'))


def test_ensemble_matches_oracle(tmp_path):
    from models.experimental import Ensemble, attempt_load
    from oracle import nms_ref, yolo_ref
    from utils.general import non_max_suppression
    names = [('yolov7-tiny', 0), ('yolov7-tiny', 1)]
    paths = []
    for k, (name, seed) in enumerate(names):
        m0, sd = model_and_weights(name, seed)
        p = tmp_path / f'm{k}.pt'
        torch.save({'model': sd, 'cfg': name}, p)
        paths.append(str(p))
    ens = attempt_load(paths, map_location=DEV)
    assert isinstance(ens, Ensemble) and len(ens) == 2 and ens.stride is ens[-1].stride
    x = frames(2, 160, 192, seed=45)
    z, none = ens(x.to(DEV))
    members = [oracle_net(n, s) for n, s in names]
    zr = yolo_ref.ensemble_forward(members, x)
    z64 = yolo_ref.ensemble_forward(members, x, f64=True)
    print('\n' + check_z(z, zr, z64, 'Ensemble of two yolov7-tiny'))
    out_g, rows_g = non_max_suppression(z, 0.25, 0.45, return_rows=True)
    out_x, rows_x = nms_ref.non_max_suppression(z.cpu(), 0.25, 0.45, return_rows=True)
    for a, b, ra, rb in zip(out_g, out_x, rows_g, rows_x):
        assert torch.equal(ra.cpu(), rb) and torch.equal(a.cpu(), b)


def test_pickled_checkpoint_forward(tmp_path):
    """A reference-format checkpoint (pickled fp16 models.yolo.Model under 'model', train.py:465-472)
    loaded by attempt_load and run on the GPU == the oracle on the same (fp16-rounded) weights."""
    from checkpoint_fixture import write_reference_checkpoint
    from models.experimental import attempt_load
    from oracle import yolo_ref
    path, sd16 = write_reference_checkpoint(tmp_path, 'yolov7-train', seed=0)
    m = attempt_load(str(path), map_location=DEV)
    x = frames(1, 160, 192, seed=46)
    z, _ = m(x.to(DEV))
    m0, _ = model_and_weights('yolov7-train', 0)
    net = yolo_ref.parse(m0.yaml)
    fused = yolo_ref.fuse(net, sd16)
    zr, _ = yolo_ref.forward(net, fused, x)
    z64, _ = yolo_ref.forward64(net, fused, x)
    print('\n' + check_z(z, zr, z64, 'pickled yolov7-train fp16 checkpoint'))


def test_profile_events_span_kernels():
    """Live per-op timing (yv7_profile_enable / _read, the bench roofline's source): every op gets a
    (start, stop) pair from its own kernel dispatches (hipExtLaunchKernel), an op without a kernel of
    its own (the later pools of the SPP cascade) reads 0, and the per-op sum of a serial forward stays
    within the forward's wall time; with three forwards in flight on three streams the recorded
    durations are still finite and positive for every conv."""
    from yv7 import _lib as L
    from yv7.runtime import Plan
    model = fresh_model('yolov7')
    plan = Plan.from_model(model, torch.device(DEV), torch.float16)
    B, H, W = 2, 256, 256
    x = frames(B, H, W, seed=7).to(DEV).half()
    N = plan.num_rows(H, W)
    z = torch.empty((B, N, plan.no), dtype=torch.float32, device=DEV)
    plan.forward_into(x, z)          # warm-up (workspace clear, code load)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    plan.profile_enable(1)
    e0.record()
    plan.forward_into(x, z)
    e1.record()
    torch.cuda.synchronize()
    nf, ms = plan.profile_read()
    plan.profile_enable(0)
    assert nf == 1 and all(v >= 0.0 for v in ms)
    costs = plan.op_costs(B, H, W, x_bytes=2, with_raw=False)
    convs = [v for (kind, _, _), v in zip(costs, ms) if kind in (L.OP_CONV, L.OP_DETECT)]
    assert convs and all(v > 0.0 for v in convs)
    wall = e0.elapsed_time(e1)
    assert sum(ms) <= wall * 1.05 + 0.05, (sum(ms), wall)
    # three forwards in flight on three streams, each with its own workspace
    streams = [torch.cuda.Stream() for _ in range(3)]
    zs = [torch.empty_like(z) for _ in range(3)]
    plan.profile_enable(3)
    for k, s in enumerate(streams):
        s.wait_stream(torch.cuda.current_stream())
        plan.forward_into(x, zs[k], stream=s, ws_slot=k)
    torch.cuda.synchronize()
    nf, ms3 = plan.profile_read()
    plan.profile_enable(0)
    assert nf == 3
    convs3 = [v for (kind, _, _), v in zip(costs, ms3) if kind in (L.OP_CONV, L.OP_DETECT)]
    assert all(0.0 < v < 1e3 for v in convs3)
    for k in range(3):
        assert torch.equal(zs[k], z)
