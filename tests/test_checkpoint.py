"""attempt_load on a reference-format checkpoint (pickled fp16 models.yolo.Model, train.py:465-472;
experimental.py:247-270: `ckpt['ema' if ckpt.get('ema') else 'model'].float().fuse().eval()`) — CPU
side: the loaded model is the fused fp32 network of the checkpoint's weights, bit for bit the same
packed plan as building the model from the same state_dict, and its folds equal the oracle's."""
import torch

from checkpoint_fixture import write_reference_checkpoint
from helpers import model_and_weights
from yv7 import _lib as L
from yv7.graph import compile_model


def test_pickled_reference_checkpoint_loads_and_fuses(tmp_path):
    from models.experimental import attempt_load
    from models.yolo import IDetect, Model
    path, sd16 = write_reference_checkpoint(tmp_path, 'yolov7-train', seed=0)
    m = attempt_load(str(path), map_location='cpu')
    assert isinstance(m, Model) and not m.training
    assert next(m.parameters()).dtype == torch.float32
    assert not any(isinstance(x, torch.nn.BatchNorm2d) for x in m.modules())
    assert not hasattr(m.model[-1], 'ia') and isinstance(m.model[-1], IDetect)
    assert m.stride.tolist() == [8.0, 16.0, 32.0] and len(m.names) == 80
    direct = Model('yolov7-train')
    direct.load_state_dict(sd16)
    direct = direct.float().fuse().eval()
    for dt in (L.DT_F32, L.DT_F16):
        a, b = compile_model(m, dt), compile_model(direct, dt)
        assert [o['kind'] for o in a.ops] == [o['kind'] for o in b.ops]
        assert torch.equal(a.weight_blob(), b.weight_blob())


def test_pickled_checkpoint_folds_match_oracle(tmp_path):
    """Every fused conv of the loaded checkpoint == the oracle's fold of the same fp16 weights
    (torch_utils.py:181-201, common.py:584-643, yolo.py:178-190), at the packed fp32 plan."""
    from models.experimental import attempt_load
    from oracle import yolo_ref
    path, sd16 = write_reference_checkpoint(tmp_path, 'yolov7-train', seed=1)
    m = attempt_load(str(path))
    m0, _ = model_and_weights('yolov7-train', 1)
    net = yolo_ref.parse(m0.yaml)
    fused = yolo_ref.fuse(net, sd16)
    checked = 0
    for layer in m.model:
        f = fused.get(layer.i)
        if isinstance(f, tuple) and hasattr(layer, 'fused_weight_bias'):
            w, b = layer.fused_weight_bias()
            assert torch.equal(w, f[0]) and torch.equal(b, f[1]), layer.i
            checked += 1
        elif isinstance(f, dict):   # SPPCSPC: cv1..cv7
            for j, (fw, fb) in f.items():
                w, b = getattr(layer, f'cv{j}').fused_weight_bias()
                assert torch.equal(w, fw) and torch.equal(b, fb), (layer.i, j)
                checked += 1
    head = m.model[-1]
    for j in range(head.nl):
        w, b = head.head_weights(j)
        assert torch.equal(w, fused[head.i][j][0]) and torch.equal(b, fused[head.i][j][1])
    assert checked == 89   # yolov7: 82 Conv / RepConv layers + SPPCSPC's 7


# Instance attribute trees the reference's constructors create (plain attributes, submodules,
# parameters, buffers), read from the reference source: Conv models/common.py:101-105, SPPCSPC
# common.py:264-274, ImplicitA / ImplicitM common.py:433-453, RepConv common.py:468-496 (training form;
# rbr_identity is a BatchNorm2d when c1 == c2 and s == 1, else a plain None attribute), Detect
# models/yolo.py:30-40, IDetect yolo.py:104-117 (+ `stride`, set on the head by Model.__init__,
# yolo.py:545), MP / SP common.py:30-45, Concat common.py:56-59, nn.Upsample (torch's own).  Every
# top-level layer also carries parse_model's i, f, type, np (yolo.py:806-808).
REF_TREES = {
    'Conv': (set(), {'conv', 'bn', 'act'}, set(), set()),
    'SPPCSPC': (set(), {'cv1', 'cv2', 'cv3', 'cv4', 'cv5', 'cv6', 'cv7', 'm'}, set(), set()),
    'ImplicitA': ({'channel', 'mean', 'std'}, set(), {'implicit'}, set()),
    'ImplicitM': ({'channel', 'mean', 'std'}, set(), {'implicit'}, set()),
    'RepConv': ({'deploy', 'groups', 'in_channels', 'out_channels'}, {'act', 'rbr_dense', 'rbr_1x1'}, set(), set()),
    'Detect': ({'nc', 'no', 'nl', 'na', 'grid', 'stride'}, {'m'}, set(), {'anchors', 'anchor_grid'}),
    'IDetect': ({'nc', 'no', 'nl', 'na', 'grid', 'stride'}, {'m', 'ia', 'im'}, set(), {'anchors', 'anchor_grid'}),
    'MP': (set(), {'m'}, set(), set()),
    'SP': (set(), {'m'}, set(), set()),
    'Concat': ({'d'}, set(), set(), set()),
}
PARSE_ATTRS = {'i', 'f', 'type', 'np'}


def _tree(mod):
    plain = {k for k in vars(mod) if not k.startswith('_') and k != 'training'}
    return plain, set(mod._modules), set(mod._parameters), set(mod._buffers)


def test_module_attribute_trees_match_reference():
    """Every module of the product's unfused Model (what a training checkpoint pickles, train.py:468-469)
    has exactly the reference constructor's attribute tree: unpickling a reference checkpoint gives the
    product's classes nothing less (a method of this package needing an attribute the reference does not
    create would fail on load) and nothing more.  yolov7-train (IDetect, RepConv), yolov7 (Detect),
    yolov7-tiny (MP / SP / LeakyReLU Convs)."""
    from models.yolo import Model
    seen = set()
    for name in ('yolov7-train', 'yolov7', 'yolov7-tiny'):
        m = Model(name)
        top = {id(x) for x in m.model}
        for mod in m.modules():
            cls = type(mod).__name__
            if cls not in REF_TREES and cls != 'Upsample':
                continue
            plain, subs, params, bufs = _tree(mod)
            if id(mod) in top:
                assert PARSE_ATTRS <= plain, (name, cls, PARSE_ATTRS - plain)
                plain -= PARSE_ATTRS
            if cls == 'Upsample':
                continue
            rp, rs, rpar, rb = (set(v) for v in REF_TREES[cls])
            if cls == 'RepConv':   # rbr_identity: a BatchNorm2d (c1 == c2, s == 1) or a plain None
                (rs if isinstance(mod.rbr_identity, torch.nn.BatchNorm2d) else rp).add('rbr_identity')
            assert (plain, subs, params, bufs) == (rp, rs, rpar, rb), (name, cls, plain, subs, params, bufs)
            seen.add(cls)
    assert seen == set(REF_TREES), set(REF_TREES) - seen
