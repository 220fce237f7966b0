#!/bin/bash
# One rocprofv3 --pmc pass over a short bench run (<= 8 SQ, <= 4 TCC counters per pass).
# usage: tools/gpu_pmc.sh TAG PASSNAME "COUNTERS" [bench args]
set -o pipefail
TAG=$1; shift; PASS=$1; shift; CNT=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc $CNT -d $OUT/pmc_$PASS -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --no-e2e --steps 2 --warmup 1 "$@" > $OUT/pmc_$PASS.log 2>&1
rc=$?
python3 tools/pmc_summary.py $OUT/pmc_$PASS > $OUT/pmc_$PASS.txt
cat $OUT/pmc_$PASS.txt
exit $rc
