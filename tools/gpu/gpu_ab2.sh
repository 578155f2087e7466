#!/bin/bash
# A/B of decode variants: C5 queries only (small encode), no CPU baseline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for lib in variants/lib*.so; do
  n=$(basename $lib .so)
  FRS_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --queries 300 > gpurun_out/ab/$n.log 2>&1 || exit 1
done
echo done
