#!/bin/bash
# Training-path GPU pass: the gradient tests, then the train bench (overlapped and serial).
# Usage (via gpurun): bash tools/gpu_train_quick.sh <tag>
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_modules.py tests/test_gpu_large_systems.py tests/test_gpu_large.py tests/test_gpu_shapes.py tests/test_0_ddp_gpu.py -x -v -s --timeout 200 --timeout-method thread > "$OUT/gpu_train_tests.log" 2>&1
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/bench_train.json" 2> "$OUT/train.err"
ENFLOW_SERIAL_BWD=1 timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/bench_train_serial.json" 2> "$OUT/train_serial.err"
echo done
