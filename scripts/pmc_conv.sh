set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
export CB_SHAPE="64->64 @160"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES -d $R/gpurun_out/pmc1 -o pmc -- $R/scripts/convbench 0 4 > $R/gpurun_out/pmc1.log 2>&1
echo done
