#!/bin/bash
# Kernel durations of the fused forward's instances at one batch size (rocprofv3
# kernel trace, one run per instance): 8-wave latency build vs cooperative build.
# Usage (via gpurun): bash tools/prof_instances.sh <tag> <mols>
set -euo pipefail
TAG=$1; MOLS=${2:-128}; LIB=${3:-}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for COOP in 0 1; do
  ENFLOW_LIB=${LIB:+$ROOT/$LIB} ENFLOW_AB_COOP=$COOP timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_coop$COOP" -o run -- \
    python3 "$ROOT/tools/ab_one_instance.py" "$MOLS" > "$OUT/one_coop$COOP.txt" 2> "$OUT/prof_coop$COOP.err"
done
echo done
