#!/bin/bash
# k_lean per-phase cost on C2: the product library and the YM_LEAN_STOP=1/2/3 builds in diag/
# (documents end after decode / layout / copy); for each, the bench's k_lean time and one
# SQ-counter pass.  usage: tools/lean_phases.sh TAG
set -o pipefail
TAG=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-compact --no-v2"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
for v in ${VARIANTS:-full stop1 stop2 stop3}; do
  if [ $v = full ]; then unset YMERGE_LIB; else export YMERGE_LIB=$GRAFT_REPO_ROOT/diag/libymerge_$v.so; fi
  timeout -k 10 300 python -u $B > $OUT/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $OUT/bench_$v.log; exit 1; }
  grep -o '"k_lean_ms": [0-9.]*' $OUT/bench_$v.log | head -1
  ( cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_$v -o p --output-format csv -- python3 $B > $OUT/pmc_$v.log 2>&1 ) || { echo "pmc $v failed"; tail -20 $OUT/pmc_$v.log; exit 1; }
  echo "== $v done"
done
exit 0
