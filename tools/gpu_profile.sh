#!/bin/bash
# One GPU-box profiling session for one workload: bench line (with CPU baseline),
# rocprofv3 kernel trace + stats, then the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE)
# on the same bench command.  Every GPU step has its own time limit; steps are chained.
# usage: tools/gpu_profile.sh TAG WORKLOAD [pmc]
set -o pipefail
TAG=${1:-run}; WL=${2:-c2}; PMC=${3:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
case $WL in c1) S="--steps 2 --warmup 1" ;; *) S="--steps 5 --warmup 2" ;; esac
timeout -k 10 420 python bench.py --workload $WL $S > $OUT/bench_$WL.log 2>&1 \
&& timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $OUT/kt_$WL -o kt --output-format csv -- python3 bench.py --workload $WL --no-cpu-baseline --no-e2e --no-compact --no-v2 $S > $OUT/kt_$WL.log 2>&1 \
&& if [ -n "$PMC" ]; then \
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$WL -o pmc --output-format csv -- python3 bench.py --workload $WL --no-cpu-baseline --no-e2e --no-compact --no-v2 --steps 2 --warmup 1 > $OUT/pmc_fetch_$WL.log 2>&1 \
  && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$WL -o pmc --output-format csv -- python3 bench.py --workload $WL --no-cpu-baseline --no-e2e --no-compact --no-v2 --steps 2 --warmup 1 > $OUT/pmc_write_$WL.log 2>&1; fi
rc=$?
echo "exit $rc ($WL)"
tail -1 $OUT/bench_$WL.log | cut -c1-300
exit $rc
