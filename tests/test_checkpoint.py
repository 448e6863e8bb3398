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
