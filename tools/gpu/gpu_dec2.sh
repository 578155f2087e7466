#!/bin/bash
# C5 decode timing per library variant (variants/lib*.so, FRS_LIB_PATH), 200 queries each.
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dec2
for lib in variants/lib*.so; do
  n=$(basename $lib .so)
  FRS_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --queries 200 > gpurun_out/dec2/$n.log 2>&1 || exit 1
done
echo done
