#!/bin/bash
# one rocprofv3 PMC pass per call: tools/pmc_pass.sh TAG N "COUNTERS" cmd...
set -o pipefail
TAG=$1; N=$2; C=$3; shift 3
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $C -d $OUT/pmc_$N -o p --output-format csv -- "$@" > $OUT/pmc_$N.log 2>&1
