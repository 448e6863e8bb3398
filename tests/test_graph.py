"""Graph compiler: op lists, zero-copy concat placement, weight packing, algorithmic costs (CPU)."""
import collections

import pytest
import torch

from helpers import fresh_model
from models.yolo import Model
from yv7 import _lib as L
from yv7.graph import _rup, compile_model


@pytest.mark.parametrize('name', ['yolov7', 'yolov7-tiny', 'yolov7-w6', 'yolov7-train', 'yolov7-w6-train'])
@pytest.mark.parametrize('dtype', [L.DT_F32, L.DT_F16])
def test_compile_structure(name, dtype):
    g = compile_model(Model(name), dtype)
    V = 8 if dtype == L.DT_F16 else 4
    kinds = collections.Counter(o['kind'] for o in g.ops)
    assert kinds[L.OP_INPUT] + kinds[L.OP_STEM] == 1 and kinds[L.OP_DETECT] == g.nl
    assert kinds[L.OP_COPY] == 0          # every concat of the yolov7 family is written in place
    assert g.ops[0]['kind'] in (L.OP_INPUT, L.OP_STEM)
    # the fused stem is used exactly for the fp16 plans (w6: ReOrg + its two convs, stem_reorg_kernel)
    assert (kinds[L.OP_STEM] == 1) == (dtype == L.DT_F16)
    for c, s in g.tensors:
        assert c % V == 0 and 0 <= s <= g.max_shift
    for o in g.ops:
        if o['kind'] in (L.OP_CONV, L.OP_DETECT):
            assert o['cin'] % V == 0 and o['w_off'] % 256 == 0 and o['b_off'] % 256 == 0
            src_c = g.tensors[o['src']][0]
            assert o['src_coff'] + o['cin'] <= src_c
        if o['kind'] == L.OP_CONV:
            assert o['dst_coff'] + o['cout'] <= g.tensors[o['dst']][0]


def test_flops_match_baseline():
    """Conv FLOPs per image at 640 (1280 for w6) equal BASELINE.md §2 (2*MAC, padded channels excluded)."""
    from yv7.runtime import Plan
    want = {'yolov7': (640, 104.51), 'yolov7-tiny': (640, 13.70), 'yolov7-w6': (1280, 359.72)}
    for name, (hw, gflops) in want.items():
        g = compile_model(Model(name), L.DT_F16)
        p = Plan.__new__(Plan)
        p.graph, p.dtype = g, g.dtype
        tot = 0.0
        for (kind, fl, by), o in zip(p.op_costs(1, hw, hw), g.ops):
            if kind == L.OP_STEM:
                tot += fl
            if kind in (L.OP_CONV, L.OP_DETECT):
                cin_real = 3 if o['src'] == 0 and not (g.ops[0]['k'] == 2) else (12 if o['src'] == 0 else o['cin'])
                tot += fl * cin_real / o['cin']
        assert tot / 1e9 == pytest.approx(gflops, rel=2e-3), name


def test_weight_packing_round_trip():
    m = fresh_model('yolov7-tiny')
    g = compile_model(m, L.DT_F32)
    blob = g.weight_blob()
    layer1 = m.model[1]
    w, b = layer1.fused_weight_bias()
    op = [o for o in g.ops if o['kind'] == L.OP_CONV][1]   # op 0 is layer 0, op 1 is layer 1
    cout, cin, k = w.shape[0], op['cin'], op['k']
    kpad = _rup(k * k * cin, 64)
    W = blob[op['w_off']:op['w_off'] + _rup(cout, 32) * kpad * 4].view(torch.float32).view(-1, kpad)
    unpacked = W[:cout, :k * k * cin].view(cout, k, k, cin).permute(0, 3, 1, 2)
    assert torch.equal(unpacked, w)
    assert torch.equal(blob[op['b_off']:op['b_off'] + cout * 4].view(torch.float32), b)
    assert torch.all(W[:, k * k * cin:] == 0) and torch.all(W[cout:] == 0)


@pytest.mark.parametrize('name', ['yolov7-tiny', 'yolov7', 'yolov7-w6'])
def test_plan_semantics_vs_oracle(name):
    """The compiled fp32 plan, executed op by op on the CPU (tests/plan_interp.py), reproduces the
    oracle's z: concat placement, pool cascade, sibling merging and detect rows are all exercised."""
    import plan_interp
    from helpers import frames, oracle_net
    from oracle import yolo_ref
    m = fresh_model(name)
    g = compile_model(m, L.DT_F32)
    assert any('merged' in o for o in g.ops)
    s = 128 if 'w6' in name else 64
    x = frames(1, s, s)
    net, fused = oracle_net(name)
    with torch.no_grad():
        want = yolo_ref.forward(net, fused, x)[0]
        got = plan_interp.run(g, x)
    assert got.shape == want.shape
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-3)


def test_sibling_merge(monkeypatch):
    """ELAN entry pairs fold into one GEMM whose packed weights are the two convs' rows back to back,
    written where the pair's concat slices sit, and sibling 1x1 convs writing separate tensors fold the
    same way once their tensors are fused side by side; the f16 plan (fused stem) keeps its semantics
    bit for bit (plan interpreter)."""
    import plan_interp
    from helpers import frames
    m = fresh_model('yolov7')
    g = compile_model(m, L.DT_F16)
    merged = [o for o in g.ops if 'merged' in o]
    # 4 backbone ELAN + 4 head ELAN-H entry pairs (adjacent concat slices), and 3 pairs whose outputs
    # were separate tensors (_merge_sibling_tensors: layers 27 + 66, 40 + 54, SPPCSPC 51 cv1 + cv2)
    assert len(merged) == 11
    pairs = sorted(tuple(sorted(l for l, _ in o['layers'])) for o in merged if len({l for l, _ in o['layers']}) == 2
                   and abs(o['layers'][0][0] - o['layers'][1][0]) > 1)
    assert pairs == [(27, 66), (40, 54)]
    assert any(o['layers'] == [(51, 2), (51, 1)] for o in merged)
    for a, b in ((27, 66), (40, 54)):   # the two layers now live side by side in one tensor
        (ta, oa, ca), (tb, ob, cb) = g.layer_tensor[a], g.layer_tensor[b]
        assert ta == tb and oa + ca == ob
    monkeypatch.setenv('YV7_NO_MERGE', '1')
    g0 = compile_model(m, L.DT_F16)
    assert len(g0.ops) == len(g.ops) + 11 and not any('merged' in o for o in g0.ops)
    assert len(g0.tensors) == len(g.tensors) + 3
    x = frames(1, 64, 64)
    with torch.no_grad():
        z0 = plan_interp.run(g0, x)
        # the tensor-fused pairs run as wider CPU convolutions, whose fp32 summation order may differ
        # (oneDNN blocks by output channels): equal within fp32 rounding of the conv sums
        torch.testing.assert_close(plan_interp.run(g, x), z0, rtol=2e-5, atol=1e-5)
        # the adjacent-slice merges alone: bit for bit
        monkeypatch.setenv('YV7_NO_MERGE', '0')
        monkeypatch.setenv('YV7_NO_TMERGE', '1')
        g1 = compile_model(m, L.DT_F16)
        assert len(g1.ops) == len(g.ops) + 3
        torch.testing.assert_close(plan_interp.run(g1, x), z0, rtol=0, atol=0)


def test_pool_fold(monkeypatch):
    """The MPs of yolov7 whose 1x1 conv reads <= 512 channels (backbone 2 + head 2; the 1024-channel one
    stays separate) fold into that conv (pool = 2, s = 2): the pooled tensors are never written, and the
    fp16 plan computes the same network."""
    import plan_interp
    from helpers import frames
    m = fresh_model('yolov7')
    g = compile_model(m, L.DT_F16)
    pooled = [o for o in g.ops if o.get('pool', 0) == 2]
    assert len(pooled) == 4 and all(o['k'] == 1 and o['s'] == 2 and o['kind'] == L.OP_CONV for o in pooled)
    assert sum(o['kind'] == L.OP_MAXPOOL and o['k'] == 2 for o in g.ops) == 1
    for o in pooled:   # the conv reads the MP's input: one level finer than its output
        assert g.tensors[o['src']][1] + 1 == g.tensors[o['dst']][1]
    monkeypatch.setenv('YV7_NO_POOLFOLD', '1')
    g0 = compile_model(m, L.DT_F16)
    assert len(g0.ops) == len(g.ops) + 4
    x = frames(1, 64, 64)
    with torch.no_grad():
        torch.testing.assert_close(plan_interp.run(g, x), plan_interp.run(g0, x), rtol=0, atol=0)


def test_reorg_stem_op():
    """yolov7-w6's fp16 front end (ReOrg, cfg/deploy/yolov7-w6.yaml:14-16 layers 1-2) compiles to ONE stem
    op for csrc/stem.hip's stem_reorg_kernel: conv A packed with K = tap * 16 + ci (ci 12-15 zero), conv B
    with K = tap * 64 + ci, written into layer 2's tensor; and the fp16 plan, interpreted on the CPU
    (tests/plan_interp.py), agrees with the fp32 plan (which keeps ReOrg in the INPUT op) to fp16 precision."""
    import plan_interp
    from helpers import frames
    m = fresh_model('yolov7-w6')
    g = compile_model(m, L.DT_F16)
    st = g.ops[0]
    assert st['kind'] == L.OP_STEM and (st['cin'], st['cout'], st['cout2'], st['s']) == (12, 64, 128, 1)
    assert not any(o['kind'] == L.OP_INPUT for o in g.ops)
    blob = g.weight_blob()
    for (w_off, b_off, layer, cin_pad) in ((st['w_off'], st['b_off'], 1, 16), (st['w2_off'], st['b2_off'], 2, 64)):
        w, b = m.model[layer].fused_weight_bias()
        cout, cin = w.shape[:2]
        kpad = _rup(9 * cin_pad, 64)
        W = blob[w_off:w_off + _rup(cout, 32) * kpad * 2].view(torch.float16).float().view(-1, kpad)
        unpacked = W[:cout, :9 * cin_pad].view(cout, 3, 3, cin_pad).permute(0, 3, 1, 2)
        torch.testing.assert_close(unpacked[:, :cin], w.half().float(), rtol=0, atol=0)
        assert torch.all(unpacked[:, cin:] == 0) and torch.all(W[:, 9 * cin_pad:] == 0)
        assert torch.equal(blob[b_off:b_off + cout * 4].view(torch.float32), b)
    x = frames(1, 128, 128)
    with torch.no_grad():
        want = plan_interp.run(compile_model(m, L.DT_F32), x)
        got = plan_interp.run(g, x)
    torch.testing.assert_close(got, want, rtol=2e-2, atol=2e-2)
