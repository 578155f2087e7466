#!/bin/bash
# round 6 call f: prefetching analysis for small jobs -- parity, then C3 / Sentinel-2 timings with and without it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_encode_parity.py -x -v -m gpu -k "prefetch or c3 or partial or sentinel or parity" --timeout 200 --timeout-method thread > $O/pytest_pf.log 2>&1 || { tail -40 $O/pytest_pf.log; exit 1; }
tail -3 $O/pytest_pf.log
for pf in 1 0 1; do
  export FRS_ANA_PF=$pf
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --queries 0 --legs c3_streaming,sentinel2 > $O/legs$pf.json 2> $O/legs$pf.err || { tail -30 $O/legs$pf.err; exit 1; }
  python -c "import json;d=json.load(open('$O/legs$pf.json'));print('PF=$pf C4', d['ms_per_step'], d['kernels_ms']);[print(k, d[k]['ms_per_step'], d[k]['kernels_ms']) for k in ('c3_streaming','sentinel2')]"
done
