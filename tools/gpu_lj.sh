#!/bin/bash
# Large-system check on one GPU: full GPU tests, headline bench, the LJ-box
# generate bench and its rocprofv3 kernel-trace summary.  Usage: bash tools/gpu_lj.sh <tag>
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 200 python -u bench.py --mode lj --steps 10 --warmup 2 > "$OUT/bench_lj.json" 2> "$OUT/lj.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_lj" -o run -- \
  python3 "$ROOT/bench.py" --mode lj --steps 5 --warmup 1 > "$OUT/bench_lj_under_profiler.json" 2> "$OUT/prof_lj.err"
echo done
