#!/bin/bash
# GPU pass for the training path: full GPU test suite, train-mode bench, kernel-trace profile.
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 > "$OUT/bench_train.json" 2> "$OUT/bench_train.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_train" -o run -- \
  python3 "$ROOT/bench.py" --mode train --steps 3 --warmup 1 > "$OUT/bench_train_under_profiler.json" 2> "$OUT/prof_train.err"
echo done
