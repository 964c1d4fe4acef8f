#!/bin/bash
# Every bench mode (BASELINE configs 1-4) once on one GPU; JSON lines into gpurun_out/<tag>/.
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 200 python -u bench.py --mode generate --steps 20 --warmup 3 > "$OUT/bench_generate.json" 2> "$OUT/generate.err"
timeout -k 10 300 python -u bench.py --mode chain --steps 5 --warmup 2 > "$OUT/bench_chain.json" 2> "$OUT/chain.err"
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 > "$OUT/bench_train.json" 2> "$OUT/train.err"
echo done
