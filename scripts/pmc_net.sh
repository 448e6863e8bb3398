#!/bin/bash
# PMC passes over whole yolov7 forwards (scripts/op_profile.py, bs32 640 fp16, default dispatch):
# one rocprofv3 --pmc run per counter set, each under its own time limit; a kernel-trace run for the
# durations.  Summaries: scripts/pmc_summary.py.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA" \
           "GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmcnet$i -o pmc -- python3 $R/scripts/op_profile.py --iters 2 --top 0 > $R/gpurun_out/pmcnet$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/pmcnet_kt -o kt -- python3 $R/scripts/op_profile.py --iters 2 --top 0 > $R/gpurun_out/pmcnet_kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
echo done
