#!/bin/bash
# encode/decode parity files with per-test time limits (progress printed per test), then the variant A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab1
timeout -k 10 500 python -u -m pytest ${AB_TESTS:-tests/test_gpu_encode_parity.py tests/test_gpu_configs.py tests/test_gpu_stereo.py tests/test_gpu_decode.py} -x -v --timeout 60 --timeout-method thread > gpurun_out/ab1/tests.log 2>&1 || { tail -60 gpurun_out/ab1/tests.log; exit 1; }
tail -2 gpurun_out/ab1/tests.log
[ -n "$AB_NOBENCH" ] && exit 0
VARIANTS="${VARIANTS:-base cur base cur}" ./tools/gpu/gpu_variants.sh
timeout -k 10 120 ./tools/micro/pcie_rates2 3200 8 > gpurun_out/ab1/pcie.txt 2>&1 || { cat gpurun_out/ab1/pcie.txt; exit 1; }
cat gpurun_out/ab1/pcie.txt
