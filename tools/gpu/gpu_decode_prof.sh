#!/bin/bash
# Batched-decode profile: kernel trace + SQ counter passes of tools/decode_probe.py (C3-sized band).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/decprof
mkdir -p $O
B="python3 tools/decode_probe.py ${PROBE_N:-16384} 3"
timeout -k 10 300 $B > $O/probe.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o run -- $B > $O/sq.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit 1
cat $O/probe.log
python3 tools/rocprof_summary.py $(find $O/kt -name "*kernel_stats.csv" | head -1)
python3 tools/pmc_summary.py $O/sq 2>/dev/null | head -40
python3 tools/pmc_traffic.py $O/fetch $O/write $O/traffic.json | grep -i decode
