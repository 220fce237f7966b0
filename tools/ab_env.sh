#!/bin/bash
# A/B of environment settings on one workload: tools/ab_env.sh TAG "bench args" "ENV=.. ENV=.." "ENV=.." ...
# (each setting benched 3 times, interleaved; "-" = no extra environment)
set -o pipefail
TAG=$1; ARGS=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    E=""; [ "$v" != "-" ] && E="$v"
    timeout -k 10 300 env $E python -u $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/env${i}_$rep.log 2>&1 || { echo "bench [$v] failed"; tail -20 $OUT/env${i}_$rep.log; exit 1; }
    echo "[$v] rep $rep: $(grep -o '"k_lean_ms": [0-9.]*' $OUT/env${i}_$rep.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/env${i}_$rep.log | head -1)"
  done
done
exit 0
