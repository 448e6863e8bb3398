"""Graph definitions: the generated cfgs equal the reference YAML files, and both parsers agree."""
import os

import pytest
import yaml

from models.yolo import Model
from oracle import yolo_ref
from yv7.arch import REGISTRY, get_cfg

REF = '/root/reference/cfg'
PAIRS = {'yolov7': 'deploy/yolov7', 'yolov7-tiny': 'deploy/yolov7-tiny', 'yolov7-w6': 'deploy/yolov7-w6',
         'yolov7-train': 'training/yolov7', 'yolov7-tiny-train': 'training/yolov7-tiny',
         'yolov7-w6-train': 'training/yolov7-w6'}


@pytest.mark.parametrize('name', sorted(PAIRS))
def test_generated_cfg_equals_reference_yaml(name):
    path = os.path.join(REF, PAIRS[name] + '.yaml')
    if not os.path.exists(path):
        pytest.skip('reference cfg not present (GPU box)')
    ref = yaml.safe_load(open(path))
    mine = get_cfg(name)
    for k in ('nc', 'depth_multiple', 'width_multiple', 'anchors', 'backbone', 'head'):
        assert ref[k] == mine[k], k


@pytest.mark.parametrize('name,nlayers,stride', [('yolov7', 106, [8, 16, 32]), ('yolov7-tiny', 78, [8, 16, 32]),
                                                 ('yolov7-w6', 119, [8, 16, 32, 64]),
                                                 ('yolov7-w6-train', 123, [8, 16, 32, 64])])
def test_product_and_oracle_parse_agree(name, nlayers, stride):
    m = Model(name)
    net = yolo_ref.parse(get_cfg(name))
    assert len(m.model) == len(net.layers) == nlayers
    assert m.save == net.save
    assert m.stride.tolist() == net.stride == stride
    det = m.model[-1]
    assert det.anchor_grid.view(-1).tolist() == net.anchor_grid.view(-1).tolist()
    # anchors are in grid units (anchor_grid / stride), models/yolo.py:546
    assert (det.anchors * m.stride.view(-1, 1, 1)).view(-1).tolist() == det.anchor_grid.view(-1).tolist()
    for L, mod in zip(net.layers, m.model):
        assert L.type == mod.type and L.f == mod.f


def test_registry_names_and_yaml_paths():
    assert {'yolov7', 'yolov7-tiny', 'yolov7-w6'} <= set(REGISTRY)
    assert get_cfg('yolov7.yaml') == get_cfg('cfg/deploy/yolov7.yaml')
    with pytest.raises(KeyError):
        get_cfg('yolov7x')
