#!/bin/bash
# C3 with small documents routed to the exact engine (YMERGE_TINY=T: documents of <= T updates)
set -o pipefail
OUT=gpurun_out/${1:-tiny}
mkdir -p $OUT
for T in 0 1 2 4 8 16; do
  YMERGE_TINY=$T timeout -k 10 400 python -u bench.py --workload c3 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $OUT/c3_tiny$T.log 2>&1 || exit 1
  echo "T=$T $(grep '^{' $OUT/c3_tiny$T.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("stages"))' 2>&1 | cut -c1-400)"
done
