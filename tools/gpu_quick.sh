#!/bin/bash
# Quick GPU pass: GPU tests, forward + train bench lines (default warmup).
# Usage (via gpurun): bash tools/gpu_quick.sh <tag> [pytest-args...]
set -euo pipefail
TAG=${1:-rXX}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread "$@" > "$OUT/gpu_tests.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/bench_train.json" 2> "$OUT/train.err"
echo done
