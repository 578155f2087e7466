#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pytest_gpu15.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu15.log
[ $rc -eq 0 ] || exit $rc
for ab in 0 1; do
  FRS_ABLATE=$ab timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench15_ab$ab.log 2>&1 || exit 1
done
echo done
