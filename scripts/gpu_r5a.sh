#!/bin/bash
# Round-5 probe: stride-2 register-weight kernel hooks + PMC, lr N-grouped tile order A/B (time + FETCH).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r5a; mkdir -p $O; cd $R
CB_SHAPE="3x3s2 64->128" timeout -k 10 120 ./scripts/convbench 0 280 285 286 287 283 > $O/cb_s2.txt 2>&1 || exit 1
CB_SHAPE="3x3s2 128->128 @160" timeout -k 10 120 ./scripts/convbench 0 282 288 289 >> $O/cb_s2.txt 2>&1 || exit 1
cat $O/cb_s2.txt
for n in 1 2 4; do
  YV7_LR_NGX=$n CB_SHAPE="3x3 512->" timeout -k 10 120 ./scripts/convbench 0 > $O/cb_lr_ngx$n.txt 2>&1 || exit 1
  YV7_LR_NGX=$n CB_SHAPE="3x3 256->256 @20" timeout -k 10 120 ./scripts/convbench 0 >> $O/cb_lr_ngx$n.txt 2>&1 || exit 1
  echo "ngx $n"; cat $O/cb_lr_ngx$n.txt
done
cd /tmp && export TMPDIR=/tmp
for n in 1 2 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    YV7_LR_NGX=$n CB_SHAPE="3x3 512->512 @20" timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/pmc_lr_${n}_$c -o pmc -- $R/scripts/convbench 0 > $O/pmc_lr_${n}_$c.log 2>&1 || { echo "pmc $n $c failed"; exit 1; }
  done
done
cd $R && bash scripts/pmc_cb.sh "3x3s2 64->128" gpurun_out/r5a/pmc_s2 280 2>&1 | tail -30
