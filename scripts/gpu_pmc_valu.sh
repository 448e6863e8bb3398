#!/bin/bash
# Instruction mix per kernel family over whole yolov7 forwards (scripts/op_profile.py, bs32 640
# fp16): one rocprofv3 --pmc pass, then VALU / LDS / SALU wave-instructions per MFMA per family.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmcvalu -o pmc -- python3 $R/scripts/op_profile.py --iters 2 --top 0 > $R/gpurun_out/pmcvalu.log 2>&1 || { echo "pmc pass failed"; tail $R/gpurun_out/pmcvalu.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections, re
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob('gpurun_out/pmcvalu/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name']
        k = re.sub(r'^void yv7::\(anonymous namespace\)::', '', k)
        k = re.sub(r'\(yv7::.*$', '', k)
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == 'SQ_INSTS_MFMA': n[k] += 1
rows = sorted(acc.items(), key=lambda kv: -kv[1]['SQ_WAVE_CYCLES'])
print(f"{'family':70s} {'n':>4s} {'VALU/MFMA':>9s} {'LDS/MFMA':>8s} {'SALU/MFMA':>9s} {'aVALU/wave':>10s} {'mfmaBusy/GUI':>12s}")
for k, c in rows[:22]:
    m = c['SQ_INSTS_MFMA'] or 1
    print(f"{k[:70]:70s} {n[k]:4d} {c['SQ_INSTS_VALU']/m:9.2f} {c['SQ_INSTS_LDS']/m:8.2f} {c['SQ_INSTS_SALU']/m:9.2f} {c['SQ_ACTIVE_INST_VALU']/max(c['SQ_WAVE_CYCLES'],1):10.3f} {c['SQ_VALU_MFMA_BUSY_CYCLES']/max(c['GRBM_GUI_ACTIVE']/8*1024,1):12.3f}")
PY
