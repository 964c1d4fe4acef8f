#!/bin/bash
# One GPU-box pass: GPU tests (errors printed), bench lines for every mode,
# rocprofv3 kernel-trace summary of the headline bench.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [pytest-args...]
set -euo pipefail
TAG=${1:-rXX}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread "$@" > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 200 python -u bench.py --mode generate --steps 20 --warmup 3 > "$OUT/bench_generate.json" 2> "$OUT/generate.err"
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 > "$OUT/bench_train.json" 2> "$OUT/train.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 "$ROOT/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_under_profiler.json" 2> "$OUT/prof.err"
echo done
