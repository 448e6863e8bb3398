"""Per-kernel summary of rocprofv3 --pmc passes (each DIR one pass of scripts/pmc_cb.sh): dispatches
grouped by kernel name, counters averaged per dispatch; clock = GRBM_GUI_ACTIVE / 8 XCDs / duration,
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs), wait shares of SQ_WAVE_CYCLES."""
import collections
import csv
import glob
import re
import sys


def short(name):
    n = re.sub(r'yv7::\(anonymous namespace\)::', '', name)
    n = re.sub(r'^void ', '', n)
    return n.split('(')[0][:90]


agg = collections.defaultdict(collections.Counter)
durs = collections.defaultdict(dict)
for d in sys.argv[1:]:
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r['Kernel_Name'])
            key = (d, int(r['Dispatch_Id']))
            durs[k][key] = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
            agg[k][r['Counter_Name'] + '@' + d] += float(r['Counter_Value'])
for k, c in agg.items():
    if 'fill_rand' in k or 'rocclr' in k:
        continue
    n_by_pass = collections.Counter(d for (d, _) in durs[k])
    tot = collections.Counter()
    for ck, v in c.items():
        name, d = ck.split('@')
        tot[name] += v / max(n_by_pass[d], 1)
    us = sum(durs[k].values()) / len(durs[k]) / 1e3
    cyc = tot['GRBM_GUI_ACTIVE'] / 8
    ghz = cyc / (us * 1e3) if us else 0
    mfma = tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024) if cyc else 0
    wave = tot['SQ_WAVE_CYCLES'] or 1
    print(f'{k}\n   {us:8.1f} us/dispatch  clock {ghz:4.2f} GHz  MFMA busy {100 * mfma:5.1f}%  '
          f'wait_any {100 * tot["SQ_WAIT_ANY"] / wave:5.1f}%  wait_inst {100 * tot["SQ_WAIT_INST_ANY"] / wave:5.1f}%  '
          f'active {100 * tot["SQ_ACTIVE_INST_ANY"] / wave:5.1f}%  lds_wait {100 * tot["SQ_WAIT_INST_LDS"] / wave:5.1f}%\n'
          f'   insts/MFMA: VALU {tot["SQ_INSTS_VALU"] / max(tot["SQ_INSTS_MFMA"], 1):.2f} LDS {tot["SQ_INSTS_LDS"] / max(tot["SQ_INSTS_MFMA"], 1):.2f} '
          f'SALU {tot["SQ_INSTS_SALU"] / max(tot["SQ_INSTS_MFMA"], 1):.2f} VMEM {tot["SQ_INSTS_VMEM"] / max(tot["SQ_INSTS_MFMA"], 1):.2f}  '
          f'LDS bank-conflict / active {tot["SQ_LDS_BANK_CONFLICT"] / max(tot["SQ_LDS_IDX_ACTIVE"], 1):.3f}  '
          f'LDS active / cycle {tot["SQ_LDS_IDX_ACTIVE"] / max(cyc * 256, 1):.3f}')
