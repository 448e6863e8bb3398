"""Product mAP evaluation (utils/metrics.py) against the oracle's restatement of test.py / utils/metrics.py."""
import numpy as np
import pytest
import torch

from oracle import metrics_ref as R
from utils import metrics as M


def _case(seed, n=60, m=25, nc=4):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(m, 2, generator=g) * 100
    wh = torch.rand(m, 2, generator=g) * 30 + 2
    labels = torch.cat((torch.randint(0, nc, (m, 1), generator=g).float(), xy, xy + wh), 1)
    # predictions: jittered copies of targets (some duplicated, some wrong class) + clutter
    k = torch.randint(0, m, (n,), generator=g)
    jit = torch.randn(n, 4, generator=g) * 3
    boxes = labels[k, 1:5] + jit
    boxes[:, 2:] = torch.maximum(boxes[:, 2:], boxes[:, :2] + 1)
    cls = torch.where(torch.rand(n, generator=g) < 0.85, labels[k, 0], torch.randint(0, nc, (n,), generator=g).float())
    conf = torch.rand(n, generator=g).sort(descending=True).values
    pred = torch.cat((boxes, conf[:, None], cls[:, None]), 1)
    return pred, labels


@pytest.mark.parametrize('seed', range(8))
def test_match_predictions_equals_reference_loop(seed):
    pred, labels = _case(seed)
    assert torch.equal(M.match_predictions(pred, labels), R.match_image(pred, labels))


def test_match_edge_cases():
    pred, labels = _case(0)
    assert M.match_predictions(pred[:0], labels).shape == (0, 10)
    assert not M.match_predictions(pred, labels[:0]).any()
    # two predictions on one target: only the first (higher confidence) is a true positive
    lab = torch.tensor([[1., 0., 0., 10., 10.]])
    p = torch.tensor([[0., 0., 10., 10., .9, 1.], [0., 0., 10., 10., .8, 1.]])
    c = M.match_predictions(p, lab)
    assert c[0].all() and not c[1].any()


def test_map_equals_reference():
    preds, labels = zip(*[_case(s) for s in range(5)])
    assert M.map_from_lists(list(preds), list(labels)) == pytest.approx(R.map_from_lists(list(preds), list(labels)),
                                                                       abs=1e-12)
    # predictions identical to the labels (conf 1): mAP@0.5 = 1
    lab = labels[0]
    perfect = torch.cat((lab[:, 1:5], torch.ones(len(lab), 1), lab[:, :1]), 1)
    assert M.map_from_lists([perfect], [lab])[0] == pytest.approx(1.0, abs=1e-9)


def test_compute_ap_known_value():
    ap, _, _ = M.compute_ap(np.array([0.5, 1.0]), np.array([1.0, 0.5]))
    ap_r, _, _ = R.compute_ap(np.array([0.5, 1.0]), np.array([1.0, 0.5]))
    assert ap == ap_r
