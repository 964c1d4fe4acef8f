#!/bin/bash
# One GPU pass: the GPU test suite, smoke, forward / train bench lines, the strong-scaling probe.
# Usage (via gpurun): bash tools/gpu_round.sh <tag> [pytest-args...]
set -euo pipefail
TAG=${1:-rXX}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=20 -v -s --timeout 200 --timeout-method thread "$@" > "$OUT/gpu_tests.log" 2>&1 || rc=$?
echo "pytest rc=$rc"
# test failures (1) go on to the benches; a crash, fault or time limit stops here
if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 300 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/bench_train.json" 2> "$OUT/train.err"
timeout -k 10 300 python -u tools/strong_scaling_probe.py > "$OUT/strong_probe.json" 2> "$OUT/strong.err"
echo done
