"""ISA-level invariants of the hand-scheduled kernels, checked on the gfx950 assembly hipcc emits
(CPU only: `hipcc --cuda-device-only -S`).  Two kinds of correctness in these kernels rest on the
instruction stream rather than on the source:

* counted `s_waitcnt vmcnt(N)`: the halo ring (csrc/conv_hring.hip, variant 262) waits for "all but the
  N youngest" vector-memory ops, so every phase must issue the same number of LDS-DMA ops on every path
  (3 weight stages + 1 patch piece); the round-3 race came from hipcc merging a block's identical dummy
  DMAs, after which a wait retired one stage too few;
* asm-issued register loads: the register-streamed 1x1 (csrc/conv_rs.hip) loads its activations with
  inline-asm `buffer_load_dwordx4`, invisible to the compiler's wait insertion, so no instruction may
  read such a register before the next `s_waitcnt vmcnt`.
"""
from __future__ import annotations

import os
import re
import subprocess

HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'yolo-series_amd', 'csrc')


def device_asm(src: str, out: str, include: str = CSRC) -> str:
    """gfx950 device assembly of one .hip file (same flags as the product build)."""
    subprocess.run([HIPCC, '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off', '-x', 'hip',
                    '--cuda-device-only', '-S', '-I', include, src, '-o', out],
                   check=True, capture_output=True)
    return open(out).read()


def functions(asm: str) -> dict[str, tuple[list[str], set[int]]]:
    """Kernel symbol -> (its instruction / label lines with comments and directives dropped, the indices
    of the instructions that came from inline asm: between ;;#ASMSTART and ;;#ASMEND)."""
    out = {}
    for m in re.finditer(r'^(_Z\S+):.*?\n(.*?)^\.Lfunc_end', asm, re.S | re.M):
        lines, asm_idx, in_asm = [], set(), False
        for raw in m.group(2).split('\n'):
            if ';;#ASMSTART' in raw:
                in_asm = True
                continue
            if ';;#ASMEND' in raw:
                in_asm = False
                continue
            ln = raw.split(';')[0].strip()
            if not ln or (ln.startswith('.') and not re.match(r'^\.LBB\d+_\d+:$', ln)):
                continue
            if in_asm:
                asm_idx.add(len(lines))
            lines.append(ln)
        out[m.group(1)] = (lines, asm_idx)
    return out


def _successors(lines):
    labels = {ln[:-1]: i for i, ln in enumerate(lines) if ln.endswith(':')}
    succ = []
    for i, ln in enumerate(lines):
        op = ln.split()[0] if not ln.endswith(':') else ''
        if op == 's_branch':
            succ.append([labels[ln.split()[1]]])
        elif op.startswith('s_cbranch'):
            succ.append([labels[ln.split()[1]], i + 1])
        elif op in ('s_endpgm', 's_setpc_b64'):
            succ.append([])
        else:
            succ.append([i + 1] if i + 1 < len(lines) else [])
    return succ


def is_lds_dma(ln: str) -> bool:
    return ln.startswith('buffer_load_') and re.search(r'\blds\b', ln) is not None


def barrier_region_counts(lines, pred=is_lds_dma, cap=32):
    """For every s_barrier, the set of counts of `pred` instructions on the control-flow paths from it to
    the next s_barrier (or the end of the kernel).  Returns {barrier line index: set(counts)}."""
    succ = _successors(lines)
    out = {}
    for b, ln in enumerate(lines):
        if ln != 's_barrier':
            continue
        counts, seen, stack = set(), set(), [(b + 1, 0)]
        while stack:
            i, n = stack.pop()
            if (i, n) in seen:
                continue
            seen.add((i, n))
            if i >= len(lines):
                counts.add(n)
                continue
            cur = lines[i]
            if cur == 's_barrier':
                counts.add(n)
                continue
            n2 = min(n + (1 if pred(cur) else 0), cap)
            nxt = succ[i]
            if not nxt:
                counts.add(n2)
            for j in nxt:
                stack.append((j, n2))
        out[b] = counts
    return out


def _regs(txt: str) -> set[int]:
    out = set()
    for a, b in re.findall(r'\bv\[(\d+):(\d+)\]', txt):
        out.update(range(int(a), int(b) + 1))
    for x in re.findall(r'(?<![\w\[:])v(\d+)\b', txt):
        out.add(int(x))
    return out


def early_async_reads(lines, asm_loads: set[int]):
    """Instructions that read a register written by one of the asm register loads (line indices in
    `asm_loads`) before the next `s_waitcnt` with a vmcnt, in straight-line order.  (scripts/
    check_async_loads.py, as a function.)"""
    bad = []
    for i in sorted(asm_loads):
        m = re.match(r'buffer_load_dwordx4 v\[(\d+):(\d+)\]', lines[i])
        live = set(range(int(m.group(1)), int(m.group(2)) + 1))
        for ln in lines[i + 1:]:
            if ln.startswith('s_waitcnt') and 'vmcnt' in ln:
                break
            if ln.endswith(':'):
                continue
            op = ln.split()[0]
            rest = ln[len(op):]
            if op.startswith(('buffer_store', 's_', 'ds_write', 'global_store')):
                srcs, dst = _regs(rest), set()
            else:
                parts = rest.split(',', 1)
                dst = _regs(parts[0])
                srcs = _regs(parts[1]) if len(parts) > 1 else set()
                if op.startswith('buffer_load') and len(parts) > 1:
                    srcs = _regs(parts[1].split(',')[0])
            if srcs & live:
                bad.append((lines[i], ln))
                break
            live -= dst
            if not live:
                break
    return bad
