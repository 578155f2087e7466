#!/bin/bash
# Run one test per prebuilt variant library (FRS_LIB_PATH), each under its own time limit.
# usage: VARIANTS="base cur" TEST=tests/x.py::test_y ./tools/gpu/gpu_isolate.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/iso
for v in ${VARIANTS:-base}; do
  echo "== $v"
  FRS_LIB_PATH=variants/lib$v.so timeout -k 10 ${TLIM:-60} python -u -m pytest -x -q -m gpu --timeout ${TLIM:-60} --timeout-method thread $TEST > gpurun_out/iso/$v.log 2>&1
  rc=$?
  tail -3 gpurun_out/iso/$v.log
  [ $rc -eq 0 ] || { echo "variant $v rc=$rc"; exit 1; }
done
