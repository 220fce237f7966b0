#!/bin/bash
# One GPU-box profiling session: gpu parity tests, bench line, rocprofv3 kernel
# trace + stats, then the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE) on the same
# bench command.  Every GPU step has its own time limit; steps are chained with &&.
# usage: tools/gpu_profile.sh TAG [bench args...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BARGS="$@"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
&& timeout -k 10 300 python bench.py $BARGS > $OUT/bench.log 2>&1 \
&& timeout -k 10 120 python tools/stamps.py 2000 > $OUT/stamps.log 2>&1 \
&& timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv rocpd -- python3 bench.py --no-cpu-baseline $BARGS > $OUT/kt.log 2>&1 \
&& timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $BARGS > $OUT/pmc_fetch.log 2>&1 \
&& timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $BARGS > $OUT/pmc_write.log 2>&1
rc=$?
echo "exit $rc"
tail -3 $OUT/pytest_gpu.log
cat $OUT/bench.log | tail -2
exit $rc
