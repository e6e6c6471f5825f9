set -e
O=gpurun_out/$1; mkdir -p $O; shift
L=$PWD/consensus_overlord_amd
B="timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-latency --clock-seconds 0"
for i in 1 2 3; do
  for v in "$@"; do
    if [ "$v" = base ]; then $B > $O/${v}_$i.log 2>&1; else OVH_LIBPATH=$L/libovhip_$v.so $B > $O/${v}_$i.log 2>&1; fi
  done
done
