#!/bin/bash
# Round-6 closing run on the final library: GPU suite + smoke, the default bench line, then the profiles --
# kernel-trace stats of the C4 step + 200 C5 queries (with the timed steps' encoder average), separate FETCH_SIZE /
# WRITE_SIZE / SQ_INSTS_VALU passes (pmc_traffic.json stamped with the library hash), two SQ counter passes, and a
# kernel trace of the batched decode.  Every GPU step bounded; outputs under gpurun_out/final_r6/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final_r6
mkdir -p $O
sha256sum flac_raster_amd/libflac_raster_amd.so > $O/lib.sha256
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=12 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
B="python3 bench.py --steps 5 --warmup 2 --no-cpu --no-extras --queries 200"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d $O/valu -o run -- $B > $O/valu.log 2>&1 || exit 1
S="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-extras --queries 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/sqa -o run -- $S > $O/sqa.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sqb -o run -- $S > $O/sqb.log 2>&1 || exit 1
D="python3 bench.py --steps 2 --warmup 1 --no-cpu --queries 0 --legs batched_decode"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dkt -o run -- $D > $O/dkt.log 2>&1 || exit 1
python3 tools/rocprof_summary.py $(find $O/kt -name "*kernel_stats.csv" | head -1) --trace $(find $O/kt -name "*kernel_trace.csv" | head -1) --last 5 --kernels k_encode_v4,k_analyze_v3 > $O/kernel_stats.md
python3 tools/rocprof_summary.py $(find $O/dkt -name "*kernel_stats.csv" | head -1) > $O/decode_kernel_stats.md
python3 tools/pmc_traffic.py $O/fetch $O/write $O/pmc_traffic.json --label r6 --pixels 1600000000 --valu $O/valu --lib flac_raster_amd/libflac_raster_amd.so > $O/pmc.txt
for k in k_encode_v4 k_analyze_v3 k_decode_frames_pipe; do echo "## $k"; python3 tools/pmc_by_kernel.py $O/sqa $O/sqb -k $k; done > $O/sq_counters.md 2>&1 || true
cat $O/kernel_stats.md $O/pmc.txt $O/decode_kernel_stats.md
head -40 $O/sq_counters.md
