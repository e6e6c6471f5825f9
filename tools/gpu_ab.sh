#!/bin/bash
# A/B pass on one GPU box: the fp_mul microbenchmark, bench with the default library and with
# the A/B build (libovhip_ab.so), and the shard (RCCL) path at one rank. Each step has its
# own limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 60 tools/ubench/fp_mul28 > "$OUT/fp_mul28.log" 2>&1
timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline > "$OUT/bench.log" 2>&1
OVH_LIBPATH=$R/consensus_overlord_amd/libovhip_ab.so timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline > "$OUT/bench_ab.log" 2>&1
timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-latency --shard-path > "$OUT/bench_shard.log" 2>&1
timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --multi-device 0 > "$OUT/bench_multi1.log" 2>&1
timeout -k 10 200 python -u bench.py --steps ${STEPS:-30} --warmup 2 --multi-device 0,0 > "$OUT/bench_multi2.log" 2>&1
echo done > "$OUT/ok"
