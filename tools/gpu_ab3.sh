#!/bin/bash
# Round-3 iteration: full GPU parity suite, C2 bench A/B (current / env variant / base library),
# k_lean stamps, then bench lines for the listed workloads.
# usage: tools/gpu_ab3.sh TAG "ENV=VAL ..." [workloads...]
set -o pipefail
TAG=${1:-ab}; VAR=${2:-}; shift; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
summ() { python3 -c "import json; d=json.loads([l for l in open('$1') if l.startswith('{')][-1]); r=d['roofline']; print('$2', round(d['ms_per_step'],3), 'ms', round(d['value'],1), d['unit'], 'frac', round(r['frac'],4), {k: (round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.endswith('_ms') or k.startswith('docs')})"; }
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 20 > $OUT/bench_c2.log 2>&1 || exit 1
summ $OUT/bench_c2.log c2
IFS=';' read -ra VARS <<< "$VAR"
k=0
for v in "${VARS[@]}"; do
  k=$((k+1))
  env $v timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 20 > $OUT/bench_c2_var$k.log 2>&1 || exit 1
  summ $OUT/bench_c2_var$k.log "c2[$v]"
done
if [ -f y-crdt_amd/lib/libymerge_base.so ]; then
  YMERGE_LIB=$PWD/y-crdt_amd/lib/libymerge_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 20 > $OUT/bench_c2_base.log 2>&1 || exit 1
  summ $OUT/bench_c2_base.log c2_base
fi
timeout -k 10 120 python tools/stamps.py lean c2 10000 > $OUT/stamps_lean_c2.log 2>&1 || exit 1
cat $OUT/stamps_lean_c2.log
for w in "$@"; do
  timeout -k 10 420 python -u bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 $OUT/bench_$w.log; exit 1; }
  summ $OUT/bench_$w.log $w
done
