#!/bin/bash
# SQ counter pass (instruction mix, wave cycles, waits) over one bench workload.  usage: tools/gpu_sqpmc.sh TAG WORKLOAD [bench args]
set -o pipefail
TAG=${1:-sq}; WL=${2:-c5}; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT/sq_$WL -o pmc --output-format csv -- python3 bench.py --workload $WL --no-cpu-baseline --no-e2e --steps 2 --warmup 1 "$@" > $OUT/sq_$WL.log 2>&1 \
&& timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES -d $OUT/sq2_$WL -o pmc --output-format csv -- python3 bench.py --workload $WL --no-cpu-baseline --no-e2e --steps 2 --warmup 1 "$@" > $OUT/sq2_$WL.log 2>&1
rc=$?
echo "exit $rc"
exit $rc
