#!/bin/bash
# A/B of library variants under variants/ (FRS_LIB_PATH) on the C4 encode, no C5 queries, no CPU leg;
# the base library is also run with FRS_ABLATE=256 (previous analysis kernel).
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab3
for lib in variants/lib*.so; do
  n=$(basename $lib .so)
  FRS_LIB_PATH=$PWD/$lib timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ab3/$n.log 2>&1 || exit 1
done
FRS_ABLATE=256 FRS_LIB_PATH=$PWD/variants/libbase.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ab3/base_v2.log 2>&1 || exit 1
echo done
