#!/bin/bash
# Cooperative instance diagnostics at one batch size: per library (ENFLOW_LIB)
# the cooperative build's step time (tools/ab_one_instance.py), plus the 8-wave one.
# Usage (via gpurun): bash tools/gpu_coop_diag.sh <tag> <mols> lib1.so [lib2.so ...]
set -euo pipefail
TAG=$1; MOLS=$2; shift 2
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
ENFLOW_AB_COOP=0 timeout -k 10 120 python -u tools/ab_one_instance.py "$MOLS" >> "$OUT/diag.txt" 2>&1
for LIB in "$@"; do
  echo "$LIB" >> "$OUT/diag.txt"
  ENFLOW_LIB="$ROOT/$LIB" ENFLOW_AB_COOP=1 timeout -k 10 120 python -u tools/ab_one_instance.py "$MOLS" >> "$OUT/diag.txt" 2>&1
done
echo done
