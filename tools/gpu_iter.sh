#!/bin/bash
# Iteration run: full GPU parity suite, C2 bench + stamps, then short bench lines for more
# workloads.  usage: tools/gpu_iter.sh TAG [workloads...]
set -o pipefail
TAG=${1:-i}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
summ() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d['roofline']; print('$2', round(d['ms_per_step'],3), 'ms', round(d['value'],1), d['unit'], 'frac', round(r['frac'],4), {k: round(v,3) for k,v in r.items() if k.endswith('_ms')})"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_c2.log 2>&1 || exit 1
summ $OUT/bench_c2.log c2
timeout -k 10 120 python tools/stamps.py 2000 > $OUT/stamps.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/stamps.log
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 > $OUT/bench_$w.log 2>&1 || exit 1
  summ $OUT/bench_$w.log $w
done
