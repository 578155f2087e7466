#!/bin/bash
# round 6 call b: restore micro; GPU suite + smoke; C5 restore-form A/B (tree = form B, variants/libdA.so, libdC.so);
# the raw-frames leg
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 60 ./tools/micro/restore_chain 300 > $O/restore_chain.txt 2>&1 || { cat $O/restore_chain.txt; exit 1; }
cat $O/restore_chain.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=15 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
for lib in tree variants/libdA.so variants/libdC.so tree; do
  if [ "$lib" = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 300 python -u bench.py --no-cpu --no-extras --steps 10 > $O/c5.json 2> $O/c5.err || { tail -30 $O/c5.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c5.json'));b=d['bbox_extract'];print('$lib', d['ms_per_step'], b['p50_ms'], b['p90_ms'], b['kernels_ms_rank0'])"
done
unset FRS_LIB_PATH
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --queries 0 --legs raw_frames > $O/raw.json 2> $O/raw.err || { tail -30 $O/raw.err; exit 1; }
python -c "import json;d=json.load(open('$O/raw.json'));print(json.dumps(d['raw_frames']))"
