#!/bin/bash
# PMC passes over the vote pool (one rocprofv3 --pmc run per counter group: <= 8 SQ counters,
# FETCH_SIZE and WRITE_SIZE alone) on tools/pool_probe.py's pre-published mode (prog 2: six
# 4,096-vote batches published before the grids start, so the counters hold no idle wait),
# then tools/pmc_pool_summary.py. TAG=r05x bash tools/pmc_pool.sh   (GPU box, repo root)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-pmc}/pmcpool
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
P="python3 $R/tools/pool_probe.py 4096 6 2 1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY -d "$OUT/a" -o a --output-format csv -- $P > "$OUT/a.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_INT64 \
  SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d "$OUT/b" -o b --output-format csv \
  -- $P > "$OUT/b.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- $P > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- $P > "$OUT/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- $P > "$OUT/kt.log" 2>&1
echo done > "$OUT/ok"
