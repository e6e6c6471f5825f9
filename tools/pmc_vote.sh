#!/bin/bash
# SQ counter passes (one rocprofv3 run per counter group) over a short bench run, for the
# per-wave VALU / SALU / LDS / wait decomposition of k_vm_vote.  TAG=r02s bash tools/pmc_vote.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --clock-seconds 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/a" -o a --output-format csv -- $B > "$OUT/a.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
  SQ_INSTS_BRANCH -d "$OUT/b" -o b --output-format csv -- $B > "$OUT/b.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT \
  SQ_LDS_UNALIGNED_STALL -d "$OUT/c" -o c --output-format csv -- $B > "$OUT/c.log" 2>&1
echo done > "$OUT/ok"
