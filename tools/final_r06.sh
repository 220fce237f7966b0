#!/bin/bash
# round-6 closing measurements: bench lines, rocprofv3 kernel stats, PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ instruction mix) on C2; kernel stats on C1 / C3 / C4 / C5 / corpus.
# usage: tools/final_r06.sh TAG
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
B="--no-cpu-baseline --no-e2e"
run() { local name=$1; shift; ( cd $R && timeout -k 10 400 "$@" > $OUT/$name.log 2>&1 ) || { echo "$name failed"; tail -20 $OUT/$name.log; exit 1; }; echo "== $name: $(tail -1 $OUT/$name.log | cut -c1-300)"; }
run bench_c2 python -u bench.py
tools/gpu_prof.sh $TAG c2 python3 bench.py --steps 20 --warmup 3 $B --no-compact --no-v2 || exit 1
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  n=$(echo $pass | cut -d' ' -f1)
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $pass -d $OUT/pmc_$n -o p --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 $B --no-compact --no-v2 > $OUT/pmc_$n.log 2>&1 ) || { echo "pmc $n failed"; tail -10 $OUT/pmc_$n.log; exit 1; }
  echo "== pmc $n done"
done
for w in c1 c3 c4 c5; do
  tools/gpu_prof.sh $TAG $w python3 bench.py --workload $w --steps 10 --warmup 3 $B || exit 1
done
run bench_corpus python -u bench.py --workload corpus --steps 5 --warmup 2 --no-cpu-baseline
exit 0
