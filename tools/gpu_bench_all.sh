#!/bin/bash
# One bench line per BASELINE.json workload.  usage: tools/gpu_bench_all.sh TAG [workloads...]
set -o pipefail
TAG=${1:-b}; shift
WL=${@:-c2 c4 c3 c5 c1}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for w in $WL; do
  case $w in
    c1) ARGS="--steps 2 --warmup 1" ;;
    *) ARGS="--steps 5 --warmup 2" ;;
  esac
  echo "== $w" 
  timeout -k 10 420 python -u bench.py --workload $w $ARGS > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed rc=$?"; tail -20 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-400
done
