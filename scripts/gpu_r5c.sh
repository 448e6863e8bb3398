#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5c; mkdir -p $O; cd $R
CB_SHAPE="3x3s2 64->128" timeout -k 10 120 ./scripts/convbench 0 280 285 286 287 > $O/cb_s2.txt 2>&1 || exit 1
CB_SHAPE="3x3s2 128->128 @160" timeout -k 10 120 ./scripts/convbench 0 282 288 289 >> $O/cb_s2.txt 2>&1 || exit 1
cat $O/cb_s2.txt
cd /tmp && export TMPDIR=/tmp
for v in 0 280 285; do
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_TA_BUSY_sum"; do
    tag=$(echo $c | cut -d' ' -f1)
    CB_SHAPE="3x3s2 64->128" timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${v}_$tag -o pmc -- $R/scripts/convbench $v > $O/pmc_${v}_$tag.log 2>&1 || echo "pmc $v $c failed"
  done
done
rocprofv3 -L > $O/counters.txt 2>&1 || true
