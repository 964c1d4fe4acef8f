#!/bin/bash
# Interleaved A/B of several library builds on the bench forward (one process).
# Usage (via gpurun): bash tools/gpu_ab.sh <tag> lib1.so lib2.so ...
set -euo pipefail
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u tools/ab_libs.py "$@" > "$OUT/ab_forward.txt" 2>&1
echo done
