"""Summarise the PMC passes of scripts/pmc_net.sh: per kernel family of one yolov7 bs32 640 fp16
forward — time, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA-busy share of the CU
cycles, stall shares, HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, the gfx950 FETCH correction of
MI355X_MICROARCH.md)."""
import collections
import csv
import json
import re
import sys

D = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out'


def load(path):
    rows = collections.defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        d = int(r['Dispatch_Id'])
        rows[d][r['Counter_Name']] = float(r['Counter_Value'])
        meta[d] = (r['Kernel_Name'], int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    return rows, meta


def family(name):
    n = re.sub(r'yv7::\(anonymous namespace\)::', '', name)
    m = re.match(r'(?:void )?([A-Za-z0-9_]+)(<[^(]*>)?', n)
    base = m.group(1) if m else n[:40]
    if base.startswith('_ZN3yv7'):
        base = re.sub(r'^_ZN3yv712_GLOBAL__N_1\d+', '', base).split('I')[0]
    return base + (m.group(2) if m and m.group(2) and 'conv' in base else '')


p1, meta = load(f'{D}/pmcnet1/pmc_counter_collection.csv')
p2, _ = load(f'{D}/pmcnet2/pmc_counter_collection.csv')
p3, _ = load(f'{D}/pmcnet3/pmc_counter_collection.csv')
p4, _ = load(f'{D}/pmcnet4/pmc_counter_collection.csv')
ids = sorted(meta)
# the last forward: op_profile runs 3 + 2 forwards; keep the dispatches of the last fifth of yv7 kernels
yv = [d for d in ids if 'rocclr' not in meta[d][0] and 'at::' not in meta[d][0] and 'elementwise' not in meta[d][0]]
per_fwd = len(yv) // 5
last = yv[-per_fwd:]
fam = collections.OrderedDict()
for d in last:
    name, dur = meta[d]
    f = family(name)
    a = fam.setdefault(f, collections.Counter())
    a['n'] += 1
    a['ns'] += dur
    for src in (p1, p2, p3, p4):
        for k, v in src.get(d, {}).items():
            a[k] += v
out = []
tot_ns = sum(a['ns'] for a in fam.values())
print(f'{"kernel family":70s} {"n":>3} {"us":>8} {"%":>5} {"GHz":>5} {"mfma%":>6} {"waitany%":>8} {"waitinst%":>9} {"MB":>8}')
for f, a in sorted(fam.items(), key=lambda kv: -kv[1]['ns']):
    cyc = a['GRBM_GUI_ACTIVE'] / 8 / 2   # two passes carry GRBM_GUI_ACTIVE: per-XCD cycles of one
    ghz = cyc / a['ns'] if a['ns'] else 0
    simd_cycles = cyc * 1024            # 256 CUs x 4 SIMDs
    mfma = a['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles if simd_cycles else 0
    wave = a['SQ_WAVE_CYCLES'] or 1
    mb = (2 * a['FETCH_SIZE'] + a['WRITE_SIZE']) / 1e3   # FETCH/WRITE_SIZE are in KB
    r = dict(family=f, launches=int(a['n']), us=round(a['ns'] / 1e3, 1), share=round(a['ns'] / tot_ns, 4),
             clock_ghz=round(ghz, 3), mfma_busy=round(mfma, 4), wait_any=round(a['SQ_WAIT_ANY'] / wave, 4),
             wait_inst_any=round(a['SQ_WAIT_INST_ANY'] / wave, 4), hbm_mb=round(mb, 1),
             mfma_insts=int(a['SQ_INSTS_MFMA']), mfma_busy_cycles=int(a['SQ_VALU_MFMA_BUSY_CYCLES']),
             lds_bank_conflict=int(a['SQ_LDS_BANK_CONFLICT']))
    out.append(r)
    print(f'{f[:70]:70s} {r["launches"]:3d} {r["us"]:8.1f} {100 * r["share"]:5.1f} {ghz:5.2f} {100 * mfma:6.1f} '
          f'{100 * r["wait_any"]:8.1f} {100 * r["wait_inst_any"]:9.1f} {mb:8.1f}')
print(f'total {tot_ns / 1e3:.1f} us (profiled forward)')
if len(sys.argv) > 2:
    json.dump({'source': 'rocprofv3 --pmc passes of scripts/pmc_net.sh (scripts/op_profile.py, yolov7 bs32 640 '
                         'fp16, default dispatch; the last of 5 forwards)', 'families': out,
               'notes': 'clock = GRBM_GUI_ACTIVE / 8 / duration; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / '
                        '(cycles x 1024 SIMDs); hbm = 2 x FETCH_SIZE + WRITE_SIZE'}, open(sys.argv[2], 'w'), indent=1)
