#!/bin/bash
# C3 (16384x16384x4 int16, tile 512, 1 GPU): kernel-trace stats and a bench line, then the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/c3; mkdir -p gpurun_out/c3
B="python3 bench.py --height 16384 --width 16384 --steps 10 --warmup 2 --no-cpu --queries 200"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c3/kt -o run -- $B > gpurun_out/c3/kt.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --height 16384 --width 16384 --steps 10 --warmup 2 --cpu-tiles 256 > gpurun_out/c3/bench_c3.log 2>&1 || exit 1
echo done
