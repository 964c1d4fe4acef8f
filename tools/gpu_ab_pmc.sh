#!/bin/bash
# A/B of the forward against an older build (one process, interleaved), then PMC
# counters of the forward kernel and of the training kernels.
# Usage (via gpurun): bash tools/gpu_ab_pmc.sh <tag> <old.so>
set -euo pipefail
TAG=${1:-rXX}; OLD=${2:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -n "$OLD" ]; then
  timeout -k 10 300 python -u tools/ab_libs.py "$OLD" enflow_amd/libenflow_hip.so > "$OUT/ab_forward.txt" 2>&1
fi
timeout -k 10 900 python -u profiles/collect_pmc.py "$TAG" > "$OUT/pmc_forward.log" 2>&1
timeout -k 10 900 python -u profiles/collect_pmc.py "${TAG}_train" train lf_layer_bwd_kernel,outer_x3_kernel > "$OUT/pmc_train.log" 2>&1
echo done
