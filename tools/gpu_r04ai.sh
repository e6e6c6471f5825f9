#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04ai}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/occupancy_real.py > "$OUT/occ_real.json" 2> "$OUT/occ_real.err"
timeout -k 10 240 python -u bench.py --warmup 3 --no-cpu-baseline --no-latency --steps 30 > "$OUT/bench.log" 2>&1
echo ok > "$OUT/ok"
