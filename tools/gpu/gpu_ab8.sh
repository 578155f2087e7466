#!/bin/bash
# GPU parity suite on the in-tree library, then alternating A/B of variants/libhead.so and variants/libnew.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/ab8; mkdir -p gpurun_out/ab8
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab8/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  for n in head mid new; do
    FRS_LIB_PATH=$PWD/variants/lib$n.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 >> gpurun_out/ab8/$n.log 2>&1 || exit 1
  done
done
echo done
