#!/bin/bash
# round 6 call w: the C5 pipe decode with the consumer's restore skipped (variants/libdprod.so: the producer's pace
# alone, outputs wrong) against the tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6w
mkdir -p $O
for v in tree dprod tree dprod; do
  if [ $v = tree ]; then unset FRS_LIB_PATH; else export FRS_LIB_PATH=$PWD/variants/lib$v.so; fi
  timeout -k 10 200 python -u tools/gpu/c5_split.py > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
  echo $v; cat $O/$v.json
done
