"""The chained low-resolution 3x3 launch (csrc/conv_lr.hip conv3x3_chain_kernel, runtime.cpp find_chain):
an ELAN block's 3x3 stack (cfg/deploy/yolov7.yaml:65-68, 84-87, 98-101, 113-116, 128-131 — Conv.fuseforward,
models/common.py:110-111, four times in a row) as ONE launch whose layers hand rows to each other through
per-band ready counters.  Measured slower than the per-layer launches (profiles/r6_chain/), so it is
not in the default dispatch: variant 305 on a stack's first op forces it.

The chain runs the same tile body and the same per-element summation order as the single-layer kernel, so its
outputs must equal the default dispatch's BIT FOR BIT — any hand-off race (a tile reading rows before their
producer finished) shows up as a difference.
The races the hand-off could have only show under uneven load (MI355X_MICROARCH.md, inter-workgroup
visibility), so the comparison is repeated with three forwards in flight on three streams."""
import copy

import pytest
import torch

from helpers import fresh_model, frames
from opcheck import check_ops, kernel_summary
from yv7 import _lib as L

pytestmark = pytest.mark.gpu
DEV = 'cuda:0'
B, H, W = 32, 640, 640


def stacks(plan):
    """[first op] of every run of >= 2 chainable 3x3 stride-1 convs (each reading the previous one's output),
    up to 4 ops from each start."""
    ops = plan.graph.ops
    k3 = lambda o: o['kind'] == L.OP_CONV and o.get('k', 1) == 3 and o.get('s', 1) == 1   # noqa: E731
    out, i = [], 0
    while i < len(ops):
        j = i
        while j + 1 < len(ops) and j - i < 3 and k3(ops[i]) and k3(ops[j + 1]) and ops[j + 1]['src'] == ops[j]['dst'] \
                and ops[j + 1]['src_coff'] == ops[j]['dst_coff']:
            j += 1
        if j > i:
            out.append(i)
        i = j + 1
    return out


def force_chains(plan, starts, on=True):
    for i in starts:
        plan.set_op_variant(i, 305 if on else 0)


def chains(plan, B, H, W):
    """[(first op, ops)] of the chained launches the dispatch makes (op_kernels: the first op carries the
    chain kernel, the others no kernel of their own)."""
    ks = plan.op_kernels(B, H, W)
    out = []
    for i, k in enumerate(ks):
        if any('conv3x3_chain_kernel' in n for n in k):
            j = i + 1
            while j < len(ks) and not ks[j] and plan.graph.ops[j]['kind'] == L.OP_CONV:
                j += 1
            out.append((i, list(range(i, j))))
    return out


def snapshot(plan, ops, B, H, W):
    g = plan.graph
    return {i: plan.tensor_view(g.ops[i]['dst'], B, H, W)[..., g.ops[i]['dst_coff']:g.ops[i]['dst_coff'] + g.ops[i]['cout']].clone()
            for i in ops}


def test_yolov7_bs32_chains_bit_exact():
    """The bench configuration (yolov7 640 bs 32 fp16): the dispatch chains the 20^2 stacks (256 -> 256 x 4;
    512 -> 256, 256 -> 256 x 3) and the 128-channel 40^2 stacks; every chained layer's output and z equal the
    unchained forward exactly."""
    m = fresh_model('yolov7').to(DEV).half()
    plan = m.plan()
    assert not chains(plan, B, H, W)   # not in the default dispatch
    force_chains(plan, stacks(plan))
    found = chains(plan, B, H, W)
    print('\nchains:', [(i, len(ops), plan.graph.ops[i]['cin'], plan.graph.ops[i]['cout']) for i, ops in found])
    # the 20^2 stacks (256 -> 256 x 4; 512 -> 256 then 256 -> 256 x 3) and the 128-channel 40^2 ones
    assert len(found) >= 4 and all(len(ops) == 4 for _, ops in found), found
    x = frames(B, H, W, seed=5).to(DEV).half()
    z1, _ = plan.forward(x, want_raw=False)
    torch.cuda.synchronize()
    allops = [i for _, ops in found for i in ops]
    got = snapshot(plan, allops, B, H, W)
    z1 = z1.clone()
    force_chains(plan, stacks(plan), False)
    assert not chains(plan, B, H, W)
    z0, _ = plan.forward(x, want_raw=False)
    torch.cuda.synchronize()
    want = snapshot(plan, allops, B, H, W)
    for i in allops:
        assert torch.equal(got[i], want[i]), f'op {i}: {(got[i].float() - want[i].float()).abs().max().item()}'
    assert torch.equal(z1, z0)


def test_chains_under_streams_repeat():
    """Three forwards in flight on three streams with their own workspaces, eight rounds: every z equals the
    serial forward of the same input bit for bit (the chain's counters re-arm between launches; contention from
    the other streams makes the hand-offs uneven)."""
    m = fresh_model('yolov7').to(DEV).half()
    plan = m.plan()
    N = plan.num_rows(H, W)
    xs = [frames(B, H, W, seed=40 + k).to(DEV).half() for k in range(3)]
    ref = []
    for x in xs:
        z = torch.empty(B, N, plan.no, device=DEV)
        plan.forward_into(x, z)
        ref.append(z)
    torch.cuda.synchronize()
    force_chains(plan, stacks(plan))
    assert chains(plan, B, H, W)
    streams = [torch.cuda.Stream(DEV) for _ in range(3)]
    zs = [torch.empty(B, N, plan.no, device=DEV) for _ in range(3)]
    for r in range(8):
        for k in range(3):
            zs[k].fill_(float('nan'))
        torch.cuda.synchronize()
        for k in range(3):
            plan.forward_into(xs[k], zs[k], stream=streams[k], ws_slot=k + 1)
        torch.cuda.synchronize()
        for k in range(3):
            assert torch.equal(zs[k], ref[k]), (r, k)


# a net whose 3x3 stack meets the chain's masked cases: a partial trailing image group (B = 5: images 5-7 of
# the second group read zeros and store nothing) and 192-channel layers (six 32-channel chunks, three 64-channel
# N slices) at 40 x 40 (8 000 output pixels: 480 tiles per layer)
CHAINED = {'nc': 3, 'depth_multiple': 1.0, 'width_multiple': 1.0,
           'anchors': [[10, 13, 16, 30, 33, 23], [30, 61, 62, 45, 59, 119], [116, 90, 156, 198, 373, 326]],
           'backbone': [[-1, 1, 'Conv', [64, 3, 2]],     # 0  @2
                        [-1, 1, 'Conv', [128, 3, 2]],    # 1  @4
                        [-1, 1, 'Conv', [192, 3, 2]],    # 2  @8
                        [-1, 1, 'Conv', [192, 3, 1]],    # 3  chained 3..6
                        [-1, 1, 'Conv', [192, 3, 1]],    # 4
                        [-1, 1, 'Conv', [192, 3, 1]],    # 5
                        [-1, 1, 'Conv', [192, 3, 1]],    # 6  (P3)
                        [-1, 1, 'Conv', [256, 3, 2]],    # 7  @16 (P4)
                        [-1, 1, 'Conv', [256, 3, 2]]],   # 8  @32 (P5)
           'head': [[[6, 7, 8], 1, 'Detect', ['nc', 'anchors']]]}


@pytest.mark.parametrize('Bn', [5, 8])
def test_chain_ragged_every_op(Bn):
    """The chain on a partial image group and 192-channel layers: every op against fp32 torch on its own input
    (tests/opcheck.py) and the chained outputs equal the unchained ones."""
    from models.yolo import Model
    from yv7.synthetic import synthetic_state_dict
    m = Model(copy.deepcopy(CHAINED))
    m.load_state_dict(synthetic_state_dict(m, seed=4, calib_hw=320))
    m = m.float().eval().fuse().to(DEV).half()
    plan = m.plan()
    Hs = 320
    force_chains(plan, stacks(plan))
    found = chains(plan, Bn, Hs, Hs)
    assert len(found) == 1 and len(found[0][1]) == 4, found
    x = frames(Bn, Hs, Hs, seed=9).to(DEV).half()
    z, xs = plan.forward(x)
    torch.cuda.synchronize()
    out = check_ops(plan, x, Bn, Hs, Hs, raw=xs, z=z)
    print('\n' + kernel_summary(out))
    ops = found[0][1]
    got = snapshot(plan, ops, Bn, Hs, Hs)
    z = z.clone()
    force_chains(plan, stacks(plan), False)
    z0, _ = plan.forward(x)
    torch.cuda.synchronize()
    want = snapshot(plan, ops, Bn, Hs, Hs)
    for i in ops:
        assert torch.equal(got[i], want[i]), i
    assert torch.equal(z, z0)
