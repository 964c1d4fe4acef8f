#!/bin/bash
# One GPU-box evaluation of the in-tree build (run via gpurun):
#   GPU test suite, interleaved A/B of the forward against the given library
#   builds, the strong-scaling probe (4-wave vs latency instances), forward and
#   training bench lines.
# Usage: bash tools/gpu_eval.sh TAG [other.so ...]
set -euo pipefail
TAG=${1:-rXX}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
if [ "$#" -gt 0 ]; then
  timeout -k 10 300 python -u tools/ab_libs.py "$@" enflow_amd/libenflow_hip.so > "$OUT/ab.txt" 2>&1
fi
timeout -k 10 300 python -u tools/strong_scaling_probe.py > "$OUT/strong.json" 2> "$OUT/strong.err"
timeout -k 10 300 python -u bench.py > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/bench_train.json" 2> "$OUT/train.err"
echo done
