#!/bin/bash
# Baseline timings of the current build: forward / train bench lines and the strong-scaling probe.
# Usage (via gpurun): bash tools/gpu_base.sh <tag>
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 300 python -u tools/strong_scaling_probe.py > "$OUT/strong_probe.json" 2> "$OUT/strong.err"
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/bench_train.json" 2> "$OUT/train.err"
echo done
