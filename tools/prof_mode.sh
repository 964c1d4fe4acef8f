#!/bin/bash
# rocprofv3 kernel-trace summary of one bench mode (env passes through, e.g.
# ENFLOW_LARGE_MIN_ATOMS / ENFLOW_LARGE_ROWS for A/B runs).
# Usage: bash tools/prof_mode.sh <tag> <mode> [steps]
set -euo pipefail
TAG=$1; MODE=$2; STEPS=${3:-5}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/bench.py" --mode "$MODE" --steps "$STEPS" --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/prof.err"
echo done
