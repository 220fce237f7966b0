#!/bin/bash
# Lean-kernel iteration: lean + parity tests, C2 bench (lean on / off).  usage: tools/gpu_lean.sh TAG [workloads...]
set -o pipefail
TAG=${1:-l}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
summ() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d['roofline']; print('$2', round(d['ms_per_step'],3), 'ms', round(d['value'],1), d['unit'], 'frac', round(r['frac'],4), {k: round(v,3) for k,v in r.items() if k.endswith('_ms')}, 'lean', r.get('docs_lean'))"; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_lean.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 > $OUT/bench_c2.log 2>&1 || exit 1
summ $OUT/bench_c2.log c2
YMERGE_LEAN=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 10 > $OUT/bench_c2_nolean.log 2>&1 || exit 1
summ $OUT/bench_c2_nolean.log c2_nolean
for w in "$@"; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-e2e --steps 5 --warmup 2 > $OUT/bench_$w.log 2>&1 || exit 1
  summ $OUT/bench_$w.log $w
done
