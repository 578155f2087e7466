#!/bin/bash
# Round-3 profile: kernel-trace stats of the default bench workload (C4 + C5), separate FETCH_SIZE / WRITE_SIZE /
# SQ_INSTS_VALU passes (one counter block per run), summaries under gpurun_out/prof_r3/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/prof_r3
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extras --queries 200"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d $O/valu -o run -- $B > $O/valu.log 2>&1 || exit 1
python3 tools/rocprof_summary.py $(find $O/kt -name "*kernel_stats.csv" | head -1) > $O/kernel_stats.md
python3 tools/pmc_traffic.py $O/fetch $O/write $O/pmc_traffic.json --label r3 --pixels 1600000000 --valu $O/valu --lib flac_raster_amd/libflac_raster_amd.so > $O/pmc.txt
tail -3 $O/kt.log
cat $O/kernel_stats.md $O/pmc.txt
