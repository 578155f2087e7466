#!/bin/bash
# Analysis at 5 waves/SIMD (variants/libana16.so, libana32.so) against the base build: parity of the 16-chunk form
# (encode parity + C3/C4 configs), then the C4 step alternating base / ana16 / ana32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ana5
FRS_LIB_PATH=$PWD/variants/libana16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ana5/p16.log 2>&1 || { echo "ana16 parity FAILED"; tail -30 gpurun_out/ana5/p16.log; exit 1; }
tail -1 gpurun_out/ana5/p16.log
for v in base ana16 ana32 base ana16 ana32; do
  FRS_LIB_PATH=$PWD/variants/lib$v.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/ana5/b_$v.json 2> gpurun_out/ana5/b_$v.err || { tail -5 gpurun_out/ana5/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ana5/b_$v.json'));print('$v', d['ms_per_step'], d['kernels_ms'])"
done
