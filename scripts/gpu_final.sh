#!/bin/bash
# Round-end evidence: smoke + GPU tests + bench + rocprof kernel stats, then the PMC traffic passes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_round.sh && cd $R && bash $R/scripts/pmc_traffic.sh && cd $R && python scripts/pmc_traffic.py gpurun_out gpurun_out/pmc_traffic.json
