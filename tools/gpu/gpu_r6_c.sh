#!/bin/bash
# round 6 call c: GPU suite + smoke (new raw-frames tests first); the raw-frames leg; the C4 step + C5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_raw_frames.py tests/test_gpu_files.py -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_raw.log 2>&1 || { tail -40 $O/pytest_raw.log; exit 1; }
tail -3 $O/pytest_raw.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --queries 0 --legs raw_frames > $O/raw.json 2> $O/raw.err || { tail -30 $O/raw.err; exit 1; }
python -c "import json;d=json.load(open('$O/raw.json'));print(json.dumps(d['raw_frames']))"
timeout -k 10 300 python -u bench.py --no-cpu --no-extras --steps 20 > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
python -c "import json;d=json.load(open('$O/c4.json'));print(d['ms_per_step'], d['kernels_ms'], json.dumps(d['roofline']), d['bbox_extract']['p50_ms'])"
