#!/bin/bash
# round-4 iteration: selected GPU tests, then bench lines.  usage: tools/gpu_r04.sh TAG "TESTS" [bench args ;; ...]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  tail -4 $OUT/pytest.log
  [ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $OUT/pytest.log | head -30; exit $rc; }
fi
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 env $args > $OUT/bench_$i.log 2>&1 || { echo "bench $i failed: $args"; tail -20 $OUT/bench_$i.log; exit 1; }
  echo "== $args"
  grep '^{' $OUT/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],3), "ms", round(d["value"],1), d["unit"], "frac", round(r["frac"],4), {k: (round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.endswith("ms") or k.startswith("docs")})'
done
