#!/bin/bash
# HIP API + kernel trace of a short bench run (host-overhead diagnosis); no counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/ht; mkdir -p gpurun_out/ht
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d gpurun_out/ht/out -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --queries 0 > gpurun_out/ht/log.txt 2>&1 || exit 1
echo done
