#!/bin/bash
# round-4 diagnostic sweep: planner tests, k_lean / lane-planner / tiled-kernel stamps, C5 planner
# knob sweep, C2 line with the lib0_v2 stage split.  Every GPU step under its own time limit.
set -o pipefail
OUT=gpurun_out/r04n
mkdir -p $OUT
export TMPDIR=/tmp
tools/gpu_r04.sh r04n "tests/test_gpu_diff.py tests/test_gpu_corpus.py tests/test_sync.py tests/test_b4.py tests/test_move_weak.py" || exit 1
timeout -k 10 200 python tools/stamps.py lean c2 10000 > $OUT/lean_stamps.log 2>&1 || exit 1
tail -14 $OUT/lean_stamps.log
timeout -k 10 300 python tools/stamps.py c4 2000 > $OUT/c4_stamps.log 2>&1 || exit 1
tail -12 $OUT/c4_stamps.log
YMERGE_PLANNER=lane timeout -k 10 200 python tools/stamps.py c5 20000 > $OUT/lane_stamps.log 2>&1 || exit 1
tail -3 $OUT/lane_stamps.log
for v in 0 1536 393216 525824 787968; do
  YMERGE_PLANNER=lane YMERGE_LANE_DBG=$v timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline --no-e2e > $OUT/c5_$v.log 2>&1 || exit 1
  echo $v $(tail -1 $OUT/c5_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['k_plan_ms'])")
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-e2e > $OUT/c2_v2.log 2>&1 || exit 1
tail -1 $OUT/c2_v2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['k_lean_ms'], d['lib0_v2'])"
