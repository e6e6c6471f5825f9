#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${TAG}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --steps 30 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1
echo ok > $OUT/ok
