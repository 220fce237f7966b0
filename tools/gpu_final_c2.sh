#!/bin/bash
# Final C2 evidence in one session: smoke, bench line with CPU baseline, rocprofv3 kernel
# stats, FETCH/WRITE passes, two SQ passes (occupancy, LDS bank conflicts), stamps.
set -o pipefail
TAG=${1:-fin}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
&& bash tools/gpu_profile.sh $TAG c2 pmc \
&& bash tools/gpu_pmc.sh $TAG sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
&& bash tools/gpu_pmc.sh $TAG sq2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
&& timeout -k 10 120 python tools/stamps.py 2000 > $OUT/stamps.log 2>&1
rc=$?
cat $OUT/smoke.log; echo "exit $rc"
exit $rc
