#!/bin/bash
# C2 A/B over an environment knob: bench + stamps per value.  usage: tools/gpu_c2_ab.sh TAG VAR v1 v2 ...
set -o pipefail
TAG=$1; VAR=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for v in "$@"; do
  env $VAR=$v timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_c2_$v.log 2>&1 || exit 1
  env $VAR=$v timeout -k 10 120 python tools/stamps.py 2000 > $OUT/stamps_$v.log 2>&1 || exit 1
  echo "$VAR=$v"
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_c2_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],3), 'ms', 'frac', round(r['frac'],4), {k: round(v,3) for k,v in r.items() if k.endswith('_ms')})"
  grep -v amdgpu.ids $OUT/stamps_$v.log | head -8
done
