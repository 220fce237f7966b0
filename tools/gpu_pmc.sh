#!/bin/bash
# SQ counter pass over the merge bench (one rocprofv3 --pmc run, <= 8 SQ counters).
# usage: tools/gpu_pmc.sh TAG "COUNTERS" [bench args]
set -o pipefail
TAG=$1; shift; CNT=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc $CNT -d $OUT/pmc -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > $OUT/pmc.log 2>&1
rc=$?
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections
f = glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "k_fast_merge" in r["Kernel_Name"] or "k_plan" in r["Kernel_Name"] or "k_exec" in r["Kernel_Name"]:
        agg[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, sum(v) / len(v))
PY
exit $rc
