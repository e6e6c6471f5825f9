set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pool or parity or configs" > $O/pytest.log 2>&1
timeout -k 10 120 python -u tools/pool_timeline.py 1 4 > $O/tl1.json 2> $O/tl1.err
timeout -k 10 300 python -u bench.py --steps 30 --warmup 2 --no-cpu-baseline > $O/bench30.log 2>&1
