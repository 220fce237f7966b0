#!/bin/bash
# one command under rocprofv3 --kernel-trace --stats; summary CSV copied next to its log.
# usage: tools/gpu_prof.sh TAG NAME cmd...
set -o pipefail
TAG=$1; NAME=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$NAME -o p --output-format csv -- "$@" > $OUT/$NAME.log 2>&1 || { echo "prof $NAME failed"; tail -30 $OUT/$NAME.log; exit 1; }
f=$(ls $OUT/prof_$NAME/*/p_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && cp "$f" $OUT/${NAME}_kernel_stats.csv && cut -d, -f1-4 "$f" | head -16
tail -1 $OUT/$NAME.log | cut -c1-400
exit 0
