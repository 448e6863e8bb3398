"""The reference's model/loader/NMS API surface (CPU-side behaviour; no compute without a GPU)."""
import pytest
import torch

from helpers import model_and_weights
from models.common import Conv, RepConv
from models.experimental import attempt_load
from models.yolo import IDetect, Model
from utils.general import non_max_suppression


def test_state_dict_keys_follow_reference_layout():
    m = Model('yolov7-train')
    keys = set(m.state_dict())
    for k in ('model.0.conv.weight', 'model.0.bn.running_var', 'model.102.rbr_dense.0.weight',
              'model.102.rbr_1x1.1.running_mean', 'model.51.cv7.conv.weight', 'model.105.anchors',
              'model.105.anchor_grid', 'model.105.m.2.bias', 'model.105.ia.0.implicit', 'model.105.im.1.implicit'):
        assert k in keys, k
    assert isinstance(m.model[-1], IDetect)
    assert m.model[0].bn.eps == 1e-3          # initialize_weights (torch_utils.py:150)


def test_fuse_removes_bn_and_branches():
    m = Model('yolov7-train')
    m.fuse()
    assert not any(isinstance(x, torch.nn.BatchNorm2d) for x in m.modules())
    assert all(hasattr(x, 'rbr_reparam') for x in m.modules() if isinstance(x, RepConv))
    assert not hasattr(m.model[-1], 'ia')
    assert all(x.conv.bias is not None for x in m.modules() if type(x) is Conv)


def test_attempt_load_state_dict_checkpoint(tmp_path):
    _, sd = model_and_weights('yolov7-tiny')
    path = tmp_path / 'tiny.pt'
    torch.save({'model': sd, 'cfg': 'yolov7-tiny'}, path)
    m = attempt_load(str(path))
    assert not m.training
    assert m.stride.tolist() == [8.0, 16.0, 32.0]
    assert len(m.names) == 80
    assert next(m.parameters()).dtype == torch.float32
    assert not any(isinstance(x, torch.nn.BatchNorm2d) for x in m.modules())


def test_no_cpu_fallback():
    m = Model('yolov7-tiny').fuse().eval()
    with pytest.raises(RuntimeError, match='ROCm'):
        m(torch.zeros(1, 3, 64, 64))
    with pytest.raises(RuntimeError, match='ROCm'):
        non_max_suppression(torch.zeros(1, 10, 85))
    with pytest.raises(RuntimeError):
        m.model[0](torch.zeros(1, 3, 8, 8))
