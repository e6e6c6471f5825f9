set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 150 python -u tools/pool_timeline.py 1 6 > $O/tl1.json 2> $O/tl1.err
