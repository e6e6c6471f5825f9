#!/bin/bash
# Shard-path A/B of OVH_SHARD_SPAN (the grid per shard batch also claims the next SPAN batches):
# bench.py --shard-path at world 1 for each span, and the single-GPU path, ROUNDS times.
#   TAG=r06n ROUNDS=1 SPANS="0 1 2" bash tools/gpu_span_ab.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/${TAG:-spanab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-1}); do
  for sp in single ${SPANS:-0 1 2}; do
    if [ "$sp" = single ]; then a=""; else a="--shard-path"; fi
    OVH_SHARD_SPAN=${sp/single/0} timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline \
      --no-latency --clock-seconds 0 $a > "$OUT/bench_${sp}_$r.log" 2>&1
    echo "$sp $r $(python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['vote_spans'].get('concurrency'), d.get('batch_latency_ms'))" "$OUT/bench_${sp}_$r.log")" >> "$OUT/summary.txt"
  done
done
echo done > "$OUT/ok"
