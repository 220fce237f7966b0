#!/bin/bash
# GPU parity suite (+ optional bench workloads).  usage: tools/gpu_tests.sh TAG [pytest selector] [workloads...]
set -o pipefail
TAG=${1:-t}; SEL=${2:-tests}; shift 2 2>/dev/null
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -15 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for w in "$@"; do
  timeout -k 10 420 python -u bench.py --workload $w --no-cpu-baseline > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $OUT/bench_$w.log; exit 1; }
  tail -1 $OUT/bench_$w.log | cut -c1-300
done
