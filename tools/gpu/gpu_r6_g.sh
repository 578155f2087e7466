#!/bin/bash
# round 6 call g: encoder A/B (tree vs variants/libeA.so: one barrier per ticket) and batched-decode A/B
# (persistent k_sync_count_p vs FRS_SYNC_P=0), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_configs.py -x -q -m gpu -k "decode or c3 or large_range" --timeout 200 --timeout-method thread > $O/pytest_dec.log 2>&1 || { tail -30 $O/pytest_dec.log; exit 1; }
tail -2 $O/pytest_dec.log
timeout -k 10 300 env FRS_LIB_PATH=$PWD/variants/libeA.so python -u -m pytest tests/test_gpu_encode_parity.py tests/test_gpu_stereo.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_eA.log 2>&1 || { tail -30 $O/pytest_eA.log; exit 1; }
tail -2 $O/pytest_eA.log
for lib in tree variants/libeA.so tree variants/libeA.so tree variants/libeA.so; do
  if [ "$lib" = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-extras --queries 0 --steps 20 > $O/ab.json 2> $O/ab.err || { tail -30 $O/ab.err; exit 1; }
  python -c "import json;d=json.load(open('$O/ab.json'));print('$lib', d['ms_per_step'], d['kernels_ms'])"
done
unset FRS_LIB_PATH
for sp in 1 0 1 0; do
  export FRS_SYNC_P=$sp
  timeout -k 10 300 python -u bench.py --no-cpu --steps 3 --queries 0 --legs batched_decode > $O/dec.json 2> $O/dec.err || { tail -30 $O/dec.err; exit 1; }
  python -c "import json;d=json.load(open('$O/dec.json'));print('SYNC_P=$sp', json.dumps(d['batched_decode']))"
done
