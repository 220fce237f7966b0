#!/bin/bash
# A/B of library builds on one workload: tools/ab_libs.sh TAG "bench args" lib1 lib2 ...
# ("product" = y-crdt_amd/lib/libymerge.so); each lib benched 3 times, interleaved.
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in "$@"; do
    if [ $v = product ]; then unset YMERGE_LIB; else export YMERGE_LIB=$GRAFT_REPO_ROOT/diag/$v; fi
    n=$(basename $v .so)
    timeout -k 10 300 python -u $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/${n}_$rep.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/${n}_$rep.log; exit 1; }
    echo "$n rep $rep: $(grep -o '"k_lean_ms": [0-9.]*' $OUT/${n}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/${n}_$rep.log | head -1)"
  done
done
exit 0
