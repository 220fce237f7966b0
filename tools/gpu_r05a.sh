#!/bin/bash
# round 5 first call: corpus bench + b4 device timings under rocprofv3
set -o pipefail
OUT=gpurun_out/r05a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload corpus --steps 5 --warmup 2 > $OUT/bench_corpus.log 2>&1 || { tail -30 $OUT/bench_corpus.log; exit 1; }
grep '^{' $OUT/bench_corpus.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/b4prof -o b4 -- python3 $GRAFT_REPO_ROOT/tools/b4_time.py > $GRAFT_REPO_ROOT/$OUT/b4.log 2>&1 || { tail -30 $GRAFT_REPO_ROOT/$OUT/b4.log; exit 1; }
grep -E "merge b4|state vector" $GRAFT_REPO_ROOT/$OUT/b4.log
