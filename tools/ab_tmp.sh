set -e
TAG=$1 TESTS=1 SMOKE=1 BENCH=1 PROF=1 STEPS=30 bash tools/gpu.sh
timeout -k 10 200 python -u bench.py --steps 30 --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0 --shard-path > gpurun_out/$1/shard.log 2>&1
