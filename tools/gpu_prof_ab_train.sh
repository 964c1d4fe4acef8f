#!/bin/bash
# Per-kernel durations of the training step for several library builds: one
# rocprofv3 kernel trace per build, weight-gradient passes serialised
# (ENFLOW_SERIAL_BWD=1) so the durations are not inflated by stream overlap.
# Usage (via gpurun): bash tools/gpu_prof_ab_train.sh <tag> lib1.so lib2.so ...
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for LIB in "$@"; do
  case "$LIB" in /*) ;; *) LIB="$ROOT/$LIB" ;; esac
  ENFLOW_LIB="$LIB" ENFLOW_SERIAL_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/prof_$i" -o run -- python3 "$ROOT/bench.py" --mode train --steps 5 --warmup 2 --no-cpu-baseline \
    > "$OUT/bench_$i.json" 2> "$OUT/prof_$i.err"
  echo "$i $LIB" >> "$OUT/libs.txt"
  i=$((i + 1))
done
echo done
