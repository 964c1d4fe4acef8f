#!/bin/bash
# One GPU-box pass for a development step: the named test files first (verbose),
# then the whole GPU suite, then an interleaved A/B of the product library
# against enflow_amd/var/libenflow_base.so (the previous build) when present.
# Usage (via gpurun): bash tools/gpu_step.sh <tag> [test files...]
set -euo pipefail
TAG=${1:-rXX}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -v -s --timeout 200 --timeout-method thread > "$OUT/focus.log" 2>&1
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
if [ -f enflow_amd/var/libenflow_base.so ]; then
  timeout -k 10 300 python -u tools/ab_libs.py enflow_amd/var/libenflow_base.so enflow_amd/libenflow_hip.so > "$OUT/ab.txt" 2>&1
fi
echo done
