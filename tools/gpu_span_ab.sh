#!/bin/bash
# Shard-path A/B on one GPU box: bench.py at world 1 for each variant "name:ENV=VALUE[,ENV=VALUE]"
# (a name starting with "single" runs the single-GPU path, the others --shard-path; a name containing
# "rsv" adds --pool-reserve, one containing "lat" also runs the latency probes), ROUNDS times.
#   TAG=r06n ROUNDS=2 VARIANTS="single:X=1 grid:X=1 span1:OVH_SHARD_SPAN=1" bash tools/gpu_span_ab.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out/${TAG:-spanab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-1}); do
  for v in ${VARIANTS:-single:X=1 grid:X=1}; do
    name=${v%%:*}
    envs=${v#*:}
    case $name in single*) a="" ;; *) a="--shard-path" ;; esac
    case $name in *rsv*) a="$a --pool-reserve" ;; esac
    case $name in *lat*) lat="--profile-steps 1" ;; *) lat="--no-latency" ;; esac
    env ${envs//,/ } timeout -k 10 250 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline \
      $lat --clock-seconds 0 $a > "$OUT/bench_${name}_$r.log" 2>&1
    echo "$name $r $(python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); l=d.get('latency') or {}; print(d['value'], d['ms_per_step'], d['roofline']['vote_spans'].get('concurrency'), d.get('batch_latency_ms'), l.get('samemsg4096_pipelined_ms_per_batch'), l.get('verify_ms'), l.get('cfg5_ms'))" "$OUT/bench_${name}_$r.log")" >> "$OUT/summary.txt"
  done
done
echo done > "$OUT/ok"
