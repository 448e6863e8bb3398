# PMC passes on the conv microbenchmark (one shape, default dispatch): instruction mix and stall mix.
# usage: bash scripts/pmc_conv.sh "<shape substring>" [variant]
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
export CB_SHAPE="$1"
V=${2:-0}
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- $R/scripts/convbench $V > $R/gpurun_out/pmc$i.log 2>&1
done
echo done
