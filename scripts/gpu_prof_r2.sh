#!/bin/bash
# Round-2 profiles: PMC HBM traffic of the bench workload (FETCH_SIZE / WRITE_SIZE passes), PMC per
# kernel family over whole forwards (pmc_net.sh), and the rocprofv3 kernel trace + stats of the bench
# command.  Each rocprofv3 run under its own time limit; any failure ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
bash $R/scripts/pmc_traffic.sh || exit 1
cd $R && python3 scripts/pmc_traffic.py gpurun_out gpurun_out/r2_pmc_traffic.json || exit 1
bash $R/scripts/pmc_net.sh || exit 1
cd $R && python3 scripts/pmc_summary.py gpurun_out gpurun_out/r2_pmc_families.json > gpurun_out/r2_pmc_families.txt || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2f_kt -o kt -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r2f_kt_bench.json 2> $R/gpurun_out/r2f_kt.err || exit 1
cd $R && python3 scripts/rocprof_timed.py gpurun_out/r2f_kt/kt_kernel_trace.csv gpurun_out/r2f_kt_bench.json gpurun_out/r2f_rocprof_vs_bench.json
echo done
