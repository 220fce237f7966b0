#!/bin/bash
# full GPU parity suite, then bench lines for the listed workloads (no CPU baseline).
# usage: tools/gpu_round.sh TAG [workloads...]
set -o pipefail
TAG=${1:-r}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
for w in "$@"; do
  timeout -k 10 420 python -u bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $OUT/bench_$w.log; exit 1; }
  grep '^{' $OUT/bench_$w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["config"]["workload"][:12], round(d["ms_per_step"],3), "ms", round(d["value"],1), d["unit"], "frac", round(r["frac"],4), {k: (round(v,2) if isinstance(v,float) else v) for k,v in r.items() if k.endswith("ms") or k.startswith("docs")})'
done
