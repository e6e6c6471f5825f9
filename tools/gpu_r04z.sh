#!/bin/bash
# r04z: occupancy diag of the spilled vote with one shared scratch vs two slots' scratch.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04z}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/occupancy_ab.py > "$OUT/occ_shared.json" 2> "$OUT/occ_shared.err"
OVH_DIAG_SCR_ALT=1 timeout -k 10 200 python -u tools/occupancy_ab.py > "$OUT/occ_alt.json" 2> "$OUT/occ_alt.err"
echo ok > "$OUT/ok"
