#!/bin/bash
# Kernel trace of the pipelined same-message loop (tools/samemsg_pipe.py).  TAG=r04m bash tools/gpu_pipe_trace.sh
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04m}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/samemsg_pipe.py 24 4096 > "$OUT/pipe.json" 2> "$OUT/pipe.err"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o pipe -- python3 -u tools/samemsg_pipe.py 12 4096 > "$OUT/trace.log" 2>&1
echo ok > "$OUT/ok"
