#!/bin/bash
# round-5 iteration: selected GPU tests (one pytest process), then optional profiled commands.
# usage: tools/gpu_r05.sh TAG "TESTS" [cmd ;; ...]   (each cmd runs under rocprofv3 --kernel-trace --stats)
set -o pipefail
TAG=$1; TESTS=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 700 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  tail -4 $OUT/pytest.log
  [ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $OUT/pytest.log | head -40; exit $rc; }
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  ( cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$i -o p --output-format csv -- $cmd > $OUT/cmd_$i.log 2>&1 ) || { echo "cmd $i failed: $cmd"; tail -30 $OUT/cmd_$i.log; exit 1; }
  echo "== $cmd"; tail -6 $OUT/cmd_$i.log
  f=$(ls $OUT/prof_$i/*/p_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && cut -d, -f1-4 "$f" | head -14
done
exit 0
