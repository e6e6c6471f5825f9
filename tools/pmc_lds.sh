#!/bin/bash
# LDS / wait PMC pass over a short bench run (names filtered against `rocprofv3 -L`).
set -e -o pipefail
OUT=gpurun_out/${TAG:-pmc}/pmc_lds
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 -L > "$OUT/list.txt" 2>&1
WANT="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVE_CYCLES"
HAVE=""
for c in $WANT; do grep -qw "$c" "$OUT/list.txt" && HAVE="$HAVE $c"; done
echo "$HAVE" > "$OUT/counters.txt"
timeout -s KILL 300 rocprofv3 --pmc $HAVE -d "$OUT/run" -o lds --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/run.log" 2>&1
echo done > "$OUT/ok"
