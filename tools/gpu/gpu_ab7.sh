#!/bin/bash
# GPU parity suite on the in-tree library, then alternating A/B of variants/libhead.so and variants/libnew.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/ab7; mkdir -p gpurun_out/ab7
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ab7/pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  for n in head new; do
    FRS_LIB_PATH=$PWD/variants/lib$n.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 >> gpurun_out/ab7/$n.log 2>&1 || exit 1
  done
done
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d gpurun_out/ab7/ht -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu --queries 0 > gpurun_out/ab7/ht.log 2>&1 || exit 1
echo done
