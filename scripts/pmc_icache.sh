#!/bin/bash
# Instruction-supply probe of a serial yolov7 bs32 640 fp16 forward (scripts/op_profile.py): instruction-cache
# hits / misses and instruction fetches against issued instructions, per kernel, one rocprofv3 --pmc pass per
# counter set under its own time limit.  Summary: scripts/pmc_icache.py.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmc_icache}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" \
           "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $O/p$i -o pmc -- python3 $R/scripts/op_profile.py --iters 2 --top 0 > $O/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $O/p$i.log; exit 1; }
done
echo done
