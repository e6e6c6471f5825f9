#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04v}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/occupancy_ab.py > "$OUT/occupancy_ab.json" 2> "$OUT/occupancy_ab.err"
echo ok > "$OUT/ok"
