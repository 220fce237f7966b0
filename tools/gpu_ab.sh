#!/bin/bash
# A/B: the in-tree library vs y-crdt_amd/lib/exp/base.so on one workload, alternating.
# usage: tools/gpu_ab.sh TAG WORKLOAD [rounds]
set -o pipefail
TAG=${1:-ab}; WL=${2:-c2}; N=${3:-3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for k in $(seq 1 $N); do
  for v in base new; do
    if [ $v = base ]; then export YMERGE_LIB=$PWD/y-crdt_amd/lib/exp/base.so; else unset YMERGE_LIB; fi
    timeout -k 10 300 python -u bench.py --workload $WL --no-cpu-baseline --no-e2e --steps 10 --warmup 3 > $OUT/${v}_$k.log 2>&1 || { echo "$v failed"; tail -3 $OUT/${v}_$k.log; exit 1; }
    echo "$v $k $(grep '^{' $OUT/${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(round(d["ms_per_step"],3), {k: round(v,3) for k,v in r.items() if k.endswith("_ms")})')"
  done
done
