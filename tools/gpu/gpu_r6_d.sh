#!/bin/bash
# round 6 call d: C3 create-streaming leg + Sentinel-2 + batched decode; rocprofv3 kernel trace of the batched decode
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp FRS_BENCH_TMP=/dev/shm
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --queries 0 --legs c3_streaming,sentinel2,batched_decode > $O/legs.json 2> $O/legs.err || { tail -30 $O/legs.err; exit 1; }
python -c "import json;d=json.load(open('$O/legs.json'));[print(k, json.dumps(d[k])) for k in ('c3_streaming','sentinel2','batched_decode')]"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --no-cpu --steps 2 --warmup 1 --queries 0 --legs batched_decode > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
python3 tools/rocprof_summary.py $(find $O/kt -name "*kernel_stats.csv" | head -1) > $O/dec_kernel_stats.md
cat $O/dec_kernel_stats.md
