#!/bin/bash
# A/B of the forward kernel against a previous build, then the training step's
# true per-kernel durations: rocprofv3 kernel trace with the weight-gradient
# passes serialised (ENFLOW_SERIAL_BWD=1, no stream overlap inflating durations).
# Usage (via gpurun): bash tools/gpu_prof_train.sh <tag> [old.so]
set -euo pipefail
TAG=${1:-rXX}; OLD=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$OLD" ]; then
  timeout -k 10 300 python -u tools/ab_libs.py "$OLD" enflow_amd/libenflow_hip.so > "$OUT/ab_forward.txt" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
ENFLOW_SERIAL_BWD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_train_serial" -o run -- \
  python3 "$ROOT/bench.py" --mode train --steps 5 --warmup 3 > "$OUT/bench_train_serial.json" 2> "$OUT/prof_train_serial.err"
echo done
