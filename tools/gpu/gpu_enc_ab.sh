#!/bin/bash
# Encode A/B on one library: default vs FRS_ABLATE=2048 (encoder normalises through the LUT), then the GPU parity suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/encab; mkdir -p gpurun_out/encab
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/encab/pytest.log 2>&1 || exit 1
for a in 0 0 0; do
  FRS_ABLATE=$a timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 >> gpurun_out/encab/a$a.log 2>&1 || exit 1
done
echo done
