#!/bin/bash
# round 6 call j: encoder taking the next ticket after its frame publishes (variants/libeC.so) -- parity (encode, stereo, multi-channel,
# configs C3) under its own time limit first, then the C4 step alternating with the tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6j
mkdir -p $O
export FRS_LIB_PATH=$PWD/variants/libeC.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_stereo.py tests/test_gpu_configs.py -x -v -m gpu -k "not c4 and not c5" --timeout 120 --timeout-method thread > $O/pytest_eC.log 2>&1 || { tail -30 $O/pytest_eC.log; exit 1; }
tail -2 $O/pytest_eC.log
for lib in variants/libeC.so tree variants/libeC.so tree variants/libeC.so tree; do
  if [ "$lib" = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-extras --queries 0 --steps 20 > $O/ab.json 2> $O/ab.err || { tail -30 $O/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab.json'));print('$lib', d['ms_per_step'], d['kernels_ms'])"
done
