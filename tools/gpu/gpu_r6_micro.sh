#!/bin/bash
# round 6: re-read micro (+ pmc FETCH_SIZE of it)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 120 ./tools/micro/reread > $O/reread.txt 2>&1 || { cat $O/reread.txt; exit 1; }
cat $O/reread.txt
