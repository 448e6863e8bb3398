#!/bin/bash
# p8 issue A/B (round 6): convbench timings and the instruction-mix PMC pass of the
# 8-phase ring on its yolov7 shapes, for the library built from the previous tree (libyv7_base.so) and this
# tree's; the outputs land in gpurun_out/TAG/.
# usage: [LIBS="base v1 cur"] bash scripts/gpu_p8ab.sh TAG   (libyv7_NAME.so each; cur = this tree's)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=$1
O=$R/gpurun_out/$TAG
LIBD=$R/yolo-series_amd/yv7
mkdir -p $O
cp $LIBD/libyv7.so $LIBD/libyv7_cur.so || exit 1
cd /tmp && export TMPDIR=/tmp
LIBS=${LIBS:-base cur}
for lib in $LIBS $LIBS; do
  cp $LIBD/libyv7_$lib.so $LIBD/libyv7.so || exit 1
  for shape in "1x1 1024->1024 @40" "1x1 2048->512 @20" "1x1 1024->1024 @20"; do
    f=$O/cb_${lib}_$(echo "$shape" | tr -cd '0-9a-z_').txt
    CB_SHAPE="$shape" timeout -k 10 120 $R/scripts/convbench 0 >> $f 2>&1 || { tail $f; exit 1; }
    grep -E "^ *variant|us" $f | tail -2
  done
done
for lib in $LIBS; do
  cp $LIBD/libyv7_$lib.so $LIBD/libyv7.so || exit 1
  CB_SHAPE="1x1 1024->1024 @40" timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $O/pmc_$lib -o pmc \
    -- $R/scripts/convbench 0 > $O/pmc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail $O/pmc_$lib.log; exit 1; }
  CB_SHAPE="1x1 1024->1024 @40" timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
    SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --output-format csv -d $O/pmc2_$lib -o pmc -- $R/scripts/convbench 0 > $O/pmc2_$lib.log 2>&1 \
    || { echo "pmc2 $lib failed"; tail $O/pmc2_$lib.log; exit 1; }
  CB_SHAPE="1x1 1024->1024 @40" timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT \
    SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE --output-format csv -d $O/pmc3_$lib -o pmc -- $R/scripts/convbench 0 \
    > $O/pmc3_$lib.log 2>&1 || { echo "pmc3 $lib failed"; tail $O/pmc3_$lib.log; exit 1; }
  (cd $R && python3 scripts/pmc_kernels.py gpurun_out/$TAG/pmc_$lib gpurun_out/$TAG/pmc2_$lib gpurun_out/$TAG/pmc3_$lib \
    > $O/summary_$lib.txt) && grep -A2 "p8_kernel" $O/summary_$lib.txt
done
cp $LIBD/libyv7_cur.so $LIBD/libyv7.so
