# PMC passes over a microbenchmark binary: instruction mix, stall mix, HBM traffic (one pass each).
# usage: bash scripts/pmc_bin.sh <binary> [args...]
set -e
R=$GRAFT_REPO_ROOT
BIN=$R/$1; shift
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/pmc$i -o pmc -- $BIN "$@" > $R/gpurun_out/pmc$i.log 2>&1
done
echo done
