#!/bin/bash
# round 6 call e: lag-split analysis -- parity tests first, the full suite, then C3 / Sentinel-2 / C4 timings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu -k "lag_split or c3" --timeout 200 --timeout-method thread > $O/pytest_ls.log 2>&1 || { tail -40 $O/pytest_ls.log; exit 1; }
tail -3 $O/pytest_ls.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --queries 0 --legs c3_streaming,sentinel2 > $O/legs.json 2> $O/legs.err || { tail -30 $O/legs.err; exit 1; }
python -c "import json;d=json.load(open('$O/legs.json'));print(d['ms_per_step'], d['kernels_ms']);[print(k, json.dumps(d[k])) for k in ('c3_streaming','sentinel2')]"
export FRS_ANA_LSPLIT=0
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --queries 0 --legs c3_streaming,sentinel2 > $O/legs0.json 2> $O/legs0.err || { tail -30 $O/legs0.err; exit 1; }
python -c "import json;d=json.load(open('$O/legs0.json'));print('LSPLIT=0', d['ms_per_step'], d['kernels_ms']);[print(k, json.dumps(d[k])) for k in ('c3_streaming','sentinel2')]"
