"""Per-basic-block instruction mix of one kernel in hipcc's gfx950 assembly (CPU only).

usage: python scripts/isa_blocks.py FILE.hip KERNEL_REGEX [--asm OUT.s] [--min N]

For every basic block of the first kernel whose symbol matches KERNEL_REGEX: its MFMA, VALU (v_* other
than MFMA), SALU (s_* other than the waitcnt / barrier / setprio / nop / branch class), SOPP (those),
LDS (ds_*) and vector-memory (buffer_* / global_*) counts, the loop depth read from hipcc's
"Loop Depth" comments, and the same per MFMA for the blocks that hold MFMAs.  VERDICT r5 item 2 asked
for p8's SALU per MFMA by basic block (the PMC figure 1.16 counts every dynamic SALU issue).
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys

HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
SOPP = ('s_waitcnt', 's_barrier', 's_setprio', 's_nop', 's_branch', 's_cbranch', 's_endpgm',
        's_sleep', 's_sethalt', 's_trap', 's_delay_alu')


def kind(op: str) -> str:
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith(SOPP):
        return 'sopp'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer_', 'global_', 'flat_', 'scratch_')):
        return 'vmem'
    return 'other'


def blocks(asm: str, pattern: str):
    m = None
    for mm in re.finditer(r'^(_Z\S+):.*?\n(.*?)^\.Lfunc_end', asm, re.S | re.M):
        if re.search(pattern, mm.group(1)):
            m = mm
            break
    if m is None:
        sys.exit(f'no kernel matches {pattern}')
    out, cur = [], {'label': 'entry', 'depth': 0, 'n': {}, 'ops': []}
    for raw in m.group(2).split('\n'):
        lab = re.match(r'^(\.LBB\d+_\d+):', raw)
        if lab:
            out.append(cur)
            d = re.search(r'Loop Depth=(\d+)', raw)
            cur = {'label': lab.group(1), 'depth': int(d.group(1)) if d else 0, 'n': {}, 'ops': []}
            continue
        ln = raw.split(';')[0].strip()
        if not ln or ln.startswith('.') or ln.endswith(':'):
            continue
        op = ln.split()[0]
        k = kind(op)
        cur['n'][k] = cur['n'].get(k, 0) + 1
        cur['ops'].append(op)
    out.append(cur)
    return m.group(1), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('src')
    ap.add_argument('kernel')
    ap.add_argument('--asm', default='/tmp/isa_blocks.s')
    ap.add_argument('--min', type=int, default=1, help='skip blocks with fewer instructions')
    ap.add_argument('--ops', action='store_true', help='list the SALU / VALU opcodes of MFMA blocks')
    a = ap.parse_args()
    if a.src.endswith('.s'):
        asm = open(a.src).read()
    else:
        inc = os.path.dirname(os.path.abspath(a.src))
        subprocess.run([HIPCC, '-O3', '-std=c++17', '--offload-arch=gfx950', '-ffp-contract=off', '-x', 'hip',
                        '--cuda-device-only', '-S', '-I', inc, a.src, '-o', a.asm], check=True)
        asm = open(a.asm).read()
    name, bl = blocks(asm, a.kernel)
    print(name)
    cols = ('mfma', 'valu', 'salu', 'sopp', 'lds', 'vmem')
    print(f'{"block":>12} {"depth":>5} ' + ' '.join(f'{c:>5}' for c in cols))
    tot = {c: 0 for c in cols}
    for b in bl:
        n = sum(b['n'].values())
        if n < a.min:
            continue
        print(f'{b["label"]:>12} {b["depth"]:>5} ' + ' '.join(f'{b["n"].get(c, 0):>5}' for c in cols))
        if a.ops and b['n'].get('mfma'):
            from collections import Counter
            for k in ('salu', 'valu'):
                cnt = Counter(o for o in b['ops'] if kind(o) == k)
                print(f'{"":>19}{k}: ' + ', '.join(f'{o} {c}' for o, c in cnt.most_common()))
        for c in cols:
            tot[c] += b['n'].get(c, 0)
    print(f'{"static":>12} {"":>5} ' + ' '.join(f'{tot[c]:>5}' for c in cols))


if __name__ == '__main__':
    main()
