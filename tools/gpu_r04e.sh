#!/bin/bash
# r04e: occupancy A/B (tools/occupancy_ab.py), the -m gpu tests, the bench.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/occupancy_ab.py > "$OUT/occupancy_ab.json" 2> "$OUT/occupancy_ab.err"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 400 python -u bench.py --steps 30 --warmup 2 > "$OUT/bench.log" 2>&1
echo ok > "$OUT/ok"
