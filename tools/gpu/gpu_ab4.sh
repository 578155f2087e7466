#!/bin/bash
# Variant A/B (variants/lib*.so), then the in-tree library: GPU parity suite and encode bench with and
# without FRS_ABLATE=128 (zig-zag residual cache off).
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/ab4; mkdir -p gpurun_out/ab4
for lib in variants/lib*.so; do
  n=$(basename $lib .so)
  FRS_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ab4/$n.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab4/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ab4/tree.log 2>&1 || exit 1
FRS_ABLATE=128 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ab4/tree_a128.log 2>&1 || exit 1
echo done
