"""CPU tests of the ISA invariants the hand-scheduled kernels' correctness rests on (tests/isa_check.py):
hipcc's gfx950 assembly of csrc/conv_hring.hip and csrc/conv_rs.hip, checked without a GPU, so a
toolchain change that re-introduces the round-3 races fails here instead of intermittently on a GPU
under three streams of contention."""
import collections
import os
import re
import shutil
import subprocess

import pytest

import isa_check as I

pytestmark = pytest.mark.skipif(not os.path.exists(I.HIPCC), reason='hipcc not available')
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def asm_dir(tmp_path_factory):
    return tmp_path_factory.mktemp('isa')


def dma_blocks_by_rsrc(lines):
    """LDS-DMA instructions after the kernel's first barrier, counted per basic block and grouped by the
    buffer resource they read through: {rsrc: Counter(DMAs in one block -> number of such blocks)}."""
    first = lines.index('s_barrier')
    per = collections.defaultdict(collections.Counter)
    bid = 0
    for i, ln in enumerate(lines):
        if ln.endswith(':') or (i and lines[i - 1].split()[0].startswith(('s_branch', 's_cbranch'))):
            bid += 1
        if i > first and I.is_lds_dma(ln):
            per[ln.split(',')[1].strip()][bid] += 1
    return {rs: collections.Counter(c.values()) for rs, c in per.items()}


def hring2_violations(asm):
    """Every halo-ring phase issues 3 weight-stage DMAs and 1 patch DMA on each of its paths (live or
    dummy past the block's last tile): per resource, every DMA-issuing basic block must issue the same
    number, 3 for the weights and 1 for the patch."""
    bad, checked = [], 0
    for name, (lines, _) in I.functions(asm).items():
        if not re.search(r'conv3x3_hring2_kernelILi\dELi0EE', name):
            continue
        checked += 1
        per = dma_blocks_by_rsrc(lines)
        sizes = sorted(tuple(sorted(c)) for c in per.values())
        if sizes != [(1,), (3,)]:
            bad.append((name, {rs: dict(c) for rs, c in per.items()}))
    return checked, bad


def test_hring2_dma_count_per_phase(asm_dir):
    asm = I.device_asm(os.path.join(I.CSRC, 'conv_hring.hip'), str(asm_dir / 'hring.s'))
    checked, bad = hring2_violations(asm)
    assert checked == 3 and not bad, bad


def test_hring2_check_catches_the_round3_race(asm_dir):
    """Negative control: the source of commit 324c6e0, before the fix (8c5e7f4) that gave every dummy DMA
    of a phase its own LDS slot — hipcc merged a block's three dummy weight DMAs into one."""
    if not shutil.which('git') or not os.path.isdir(os.path.join(ROOT, '.git')):
        pytest.skip('no git history')
    r = subprocess.run(['git', '-C', ROOT, 'show', '324c6e0:yolo-series_amd/csrc/conv_hring.hip'],
                       capture_output=True, text=True)
    if r.returncode:
        pytest.skip('commit 324c6e0 not in this history')
    src = asm_dir / 'conv_hring_324c6e0.hip'
    src.write_text(r.stdout)
    checked, bad = hring2_violations(I.device_asm(str(src), str(asm_dir / 'hring_324c6e0.s')))
    assert checked == 3 and len(bad) == 3
    # the weight resource shows blocks of 1 DMA (the merged dummies) beside the blocks of 3
    assert all(any(set(c) == {1, 3} for c in per.values()) for _, per in bad)


def test_conv_rs_asm_loads_waited(asm_dir):
    """The register-streamed 1x1: no instruction reads a register of an inline-asm buffer_load before
    the next s_waitcnt vmcnt, and no wave ends with such a load in flight (the next kernel's waves
    inherited the VGPRs)."""
    asm = I.device_asm(os.path.join(I.CSRC, 'conv_rs.hip'), str(asm_dir / 'rs.s'))
    fns = {n: v for n, v in I.functions(asm).items() if 'conv1x1_rs_kernel' in n}
    assert fns
    for name, (lines, asm_idx) in fns.items():
        loads = {i for i in asm_idx if lines[i].startswith('buffer_load_dwordx4')}
        assert loads, name
        assert not I.early_async_reads(lines, loads), name
        last = max(loads)
        for j, ln in enumerate(lines):
            if ln == 's_endpgm' and j > last:
                between = lines[last + 1:j]
                assert any(re.match(r's_waitcnt vmcnt\(0\)', b) for b in between), name


def test_early_read_detector():
    """The detector itself: a use before the wait is flagged, a use after it is not."""
    lines = ['buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen', 'v_mov_b32 v8, v5', 's_waitcnt vmcnt(0)']
    assert I.early_async_reads(lines, {0})
    lines = ['buffer_load_dwordx4 v[4:7], v1, s[0:3], 0 offen', 'v_mov_b32 v8, v9', 's_waitcnt vmcnt(0)',
             'v_mov_b32 v8, v5']
    assert not I.early_async_reads(lines, {0})


def ws64_wide_ors(asm):
    """Per conv3x3_ws64_kernel instantiation: the v_or_b32 with a constant of 64 KiB or more (an LDS address
    past the ds_read offset field, built per read instead of folded into the offset)."""
    return {n: sum(1 for ln in lines if re.match(r'v_or_b32_e32 v\d+, 0x[0-9a-f]{5,}', ln))
            for n, (lines, _) in I.functions(asm).items() if 'conv3x3_ws64_kernel' in n}


def test_ws64_weight_reads_fold_their_offsets(asm_dir):
    """Round 6 (profiles/r6_ws64/): the weight reads of the 8-wave ws64 kernel take one opaque
    base per (tap column, K half) and carry the tap / fragment offsets in the ds_read offset field; the
    compiler's `base | constant` form cost a v_or per read (114 in the 8-wave kernel) and 42 VGPRs."""
    ors = ws64_wide_ors(I.device_asm(os.path.join(I.CSRC, 'conv_ws.hip'), str(asm_dir / 'ws.s')))
    eight = {n: c for n, c in ors.items() if n.endswith('ELi8EEEvNS_10ConvParamsE')}
    assert eight and all(c <= 16 for c in eight.values()), eight


def test_ws64_check_catches_the_per_read_ors(asm_dir):
    """Negative control: the round-5 source (before commit 1aba2fd) builds its weight addresses per read."""
    if not shutil.which('git') or not os.path.isdir(os.path.join(ROOT, '.git')):
        pytest.skip('no git history')
    r = subprocess.run(['git', '-C', ROOT, 'show', '1aba2fd~1:yolo-series_amd/csrc/conv_ws.hip'],
                       capture_output=True, text=True)
    if r.returncode:
        pytest.skip('commit 1aba2fd not in this history')
    src = asm_dir / 'conv_ws_before.hip'
    src.write_text(r.stdout)
    ors = ws64_wide_ors(I.device_asm(str(src), str(asm_dir / 'ws_before.s')))
    eight = {n: c for n, c in ors.items() if n.endswith('ELi8EEEvNS_10ConvParamsE')}
    assert eight and all(c > 60 for c in eight.values()), eight
