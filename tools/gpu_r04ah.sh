#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04ah}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/occupancy_real.py > "$OUT/occ_real.json" 2> "$OUT/occ_real.err"
timeout -k 10 200 python -u tools/occupancy_ab.py > "$OUT/occ_zero.json" 2> "$OUT/occ_zero.err"
echo ok > "$OUT/ok"
