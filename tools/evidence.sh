#!/bin/bash
# Round evidence on one GPU box: parity tests, smoke, bench (+ CPU baseline, latency probes),
# rocprofv3 kernel stats, then PMC passes (SQ decomposition, LDS bank conflicts, HBM bytes).
# Every GPU step has its own limit; the first failure ends the script.   TAG=r02ab
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ev} bash tools/gpu_round.sh
TAG=${TAG:-ev}/pmcv bash tools/pmc_vote.sh
TAG=${TAG:-ev} bash tools/pmc_round.sh
echo done > gpurun_out/${TAG:-ev}/evidence_ok
