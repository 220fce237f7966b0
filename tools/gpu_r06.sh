#!/bin/bash
# round-6 iteration: selected GPU tests (one pytest process), then plain commands (no profiler).
# usage: tools/gpu_r06.sh TAG "TESTS" [cmd ...]
set -o pipefail
TAG=$1; TESTS=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?
  tail -4 $OUT/pytest.log
  [ $rc -ne 0 ] && { grep -E "^E |Error|FAILED" $OUT/pytest.log | head -40; exit $rc; }
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  ( cd $GRAFT_REPO_ROOT && timeout -k 10 300 $cmd > $OUT/cmd_$i.log 2>&1 ) || { echo "cmd $i failed: $cmd"; tail -30 $OUT/cmd_$i.log; exit 1; }
  echo "== $cmd"; tail -12 $OUT/cmd_$i.log
done
exit 0
