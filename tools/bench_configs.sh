#!/bin/bash
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r06fin3}; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for w in c1 c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 10 --warmup 3 > $OUT/bench_$w.log 2>&1 || { echo "$w failed"; tail -20 $OUT/bench_$w.log; exit 1; }
  echo "$w $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_$w.log) $(grep -o '"frac": [0-9.]*' $OUT/bench_$w.log | head -1) $(grep -o '"cpu_baseline": {"value": [0-9.]*' $OUT/bench_$w.log)"
done
