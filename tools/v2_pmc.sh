#!/bin/bash
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r06x
mkdir -p $OUT
export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-compact"
cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VMEM_WR -d $OUT/pmc1 -o p --output-format csv -- python3 $B > $OUT/pmc1.log 2>&1 || { tail -20 $OUT/pmc1.log; exit 1; }
cd /tmp && timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM -d $OUT/pmc2 -o p --output-format csv -- python3 $B > $OUT/pmc2.log 2>&1 || { tail -20 $OUT/pmc2.log; exit 1; }
echo done
