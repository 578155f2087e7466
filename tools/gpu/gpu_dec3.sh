#!/bin/bash
# C5 decode timing per library variant (variants/lib*.so, FRS_LIB_PATH), 300 queries each; a variant that
# breaks losslessness (ablations) still reports its kernel times.
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/dec3
for lib in variants/lib*.so; do
  n=$(basename $lib .so)
  FRS_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu --queries 300 > gpurun_out/dec3/$n.log 2>&1
  rc=$?
  echo "$n rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
echo done
