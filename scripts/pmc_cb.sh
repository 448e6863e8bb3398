#!/bin/bash
# PMC passes on the conv microbenchmark: one shape, the given variants; then a per-kernel summary.
# usage: bash scripts/pmc_cb.sh "<shape substring>" OUTDIR variant [variant ...]
set -o pipefail
R=$GRAFT_REPO_ROOT
SHAPE="$1"; OUT="$2"; shift 2
mkdir -p $R/$OUT
cd /tmp && export TMPDIR=/tmp
export CB_SHAPE="$SHAPE"
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/p$i -o pmc -- $R/scripts/convbench "$@" > $R/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
cd $R && python3 scripts/pmc_kernels.py $OUT/p1 $OUT/p2 $OUT/p3 > $OUT/summary.txt && cat $OUT/summary.txt
