#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter group, gfx950 slot
# limits: <= 8 SQ, FETCH_SIZE and WRITE_SIZE in separate passes), then a summary per kernel.
#   TAG=r01i bash tools/pmc_round.sh      (on the GPU box, from the repo root)
set -e -o pipefail
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
RUN="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-latency --clock-seconds 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/sq" -o sq --output-format csv -- $RUN > "$OUT/sq.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o fetch --output-format csv -- $RUN > "$OUT/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o write --output-format csv -- $RUN > "$OUT/write.log" 2>&1
echo done > "$OUT/ok"
