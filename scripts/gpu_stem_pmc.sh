#!/bin/bash
# PMC passes over the fused stem microbenchmark (scripts/stembench.hip, bs32 640 fp16), one rocprofv3
# --pmc run per counter set under its own time limit, then a per-counter summary of stem2_kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/stembench.hip -I yolo-series_amd/csrc -L yolo-series_amd/yv7 -lyv7 -Wl,-rpath,$R/yolo-series_amd/yv7 -o gpurun_out/stembench || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/stempmc$i -o pmc -- $R/gpurun_out/stembench 0 > $R/gpurun_out/stempmc$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $R/gpurun_out/stempmc$i.log; }
done
cd $R && python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob('gpurun_out/stempmc*/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'stem2_kernel' in r.get('Kernel_Name', ''):
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k in sorted(acc):
    v = acc[k]
    print(f'{k:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}')
PY
