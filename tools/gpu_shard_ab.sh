#!/bin/bash
# Shard-path A/B on one GPU box: the pool tests, then bench.py ROUNDS times
# interleaved as the single-GPU path, the shard path (partials + RCCL all-gather at world 1) on an
# OVH_FLAG_POOL_RESERVE context, the same with 8 pool workgroups per CU, and the shard path with
# a pool grid per batch (without --pool-reserve). Each step has its own limit; the first failure ends
# the script.   TAG=r06e ROUNDS=2 STEPS=30 bash tools/gpu_shard_ab.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-shardab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pool.py tests/test_gpu_parity.py -x -v --timeout 120 \
    --timeout-method thread > "$OUT/pytest_pool.log" 2>&1
fi
run() {  # name, env, bench args
  local name=$1 envs=$2
  shift 2
  env $envs timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-latency \
    --clock-seconds 0 "$@" > "$OUT/bench_${name}_$r.log" 2>&1
  echo "$name $r $(python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['stage_ms'])" "$OUT/bench_${name}_$r.log")" >> "$OUT/summary.txt"
}
for r in $(seq 1 ${ROUNDS:-2}); do
  run single "X=1"
  run shard_rsv "X=1" --shard-path --pool-reserve
  run shard_rsv8 "OVH_POOL_PER_CU=8" --shard-path --pool-reserve
  run shard_grid "X=1" --shard-path
  if [ -n "${SINGLE_RSV:-}" ]; then
    run single_rsv "X=1" --pool-reserve
    run single_rsv8 "OVH_POOL_PER_CU=8" --pool-reserve
  fi
done
echo done > "$OUT/ok"
