#!/bin/bash
# Encoder CRC slice-by-16 (variants/libecrc16.so) against the base build: encode parity (incl. all 6241 C4 tiles),
# then the C4 step alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ecrc
FRS_LIB_PATH=$PWD/variants/libecrc16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_configs.py tests/test_gpu_files.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/ecrc/p.log 2>&1 || { echo "ecrc16 parity FAILED"; tail -30 gpurun_out/ecrc/p.log; exit 1; }
tail -1 gpurun_out/ecrc/p.log
for v in ebase ecrc16 ebase ecrc16 ebase ecrc16; do
  FRS_LIB_PATH=$PWD/variants/lib$v.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --queries 0 --steps 20 > gpurun_out/ecrc/b_$v.json 2> gpurun_out/ecrc/b_$v.err || { tail -5 gpurun_out/ecrc/b_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ecrc/b_$v.json'));print('$v', d['ms_per_step'], d['kernels_ms'])"
done
