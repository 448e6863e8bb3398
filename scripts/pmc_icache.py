"""Summarise scripts/pmc_icache.sh per kernel family: instruction-cache miss rate, instruction fetches per issued
instruction, the share of wave cycles waiting to issue (SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES)."""
import collections
import csv
import glob
import re
import sys


def family(name):   # (as scripts/pmc_summary.py, which runs on import)
    n = re.sub(r'yv7::\(anonymous namespace\)::', '', name)
    m = re.match(r'(?:void )?([A-Za-z0-9_]+)(<[^(]*>)?', n)
    base = m.group(1) if m else n[:40]
    if base.startswith('_ZN3yv7'):
        base = re.sub(r'^_ZN3yv712_GLOBAL__N_1\d+', '', base).split('I')[0]
    return base + (m.group(2) if m and m.group(2) and 'conv' in base else '')

D = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f'{D}/p*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        acc[family(r['Kernel_Name'])][r['Counter_Name']] += float(r['Counter_Value'])
print(f'{"kernel family":72s} {"icache miss%":>12s} {"ifetch/inst":>11s} {"waitinst%":>9s} {"insts(M)":>9s}')
rows = []
for k, c in acc.items():
    h, m = c.get('SQC_ICACHE_HITS', 0), c.get('SQC_ICACHE_MISSES', 0)
    ins = sum(c.get(n, 0) for n in ('SQ_INSTS_VALU', 'SQ_INSTS_SALU', 'SQ_INSTS_MFMA', 'SQ_INSTS_LDS'))
    rows.append((c.get('SQ_WAVE_CYCLES', 0), k, 100 * m / max(h + m, 1), c.get('SQ_IFETCH', 0) / max(ins, 1),
                 100 * c.get('SQ_WAIT_INST_ANY', 0) / max(c.get('SQ_WAVE_CYCLES', 0), 1), ins / 1e6))
for _, k, mr, fi, wi, ins in sorted(rows, reverse=True):
    print(f'{k[:72]:72s} {mr:12.2f} {fi:11.3f} {wi:9.1f} {ins:9.1f}')
