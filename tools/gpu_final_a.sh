#!/bin/bash
# Round-end evidence, part 1 (tools/gpu_final.sh split to fit one gpurun call):
# GPU tests, smoke, every bench mode, rocprofv3 kernel stats of the forward and
# training benches.   Usage: bash tools/gpu_final_a.sh <tag>
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
if [ -z "${SKIP_TESTS:-}" ]; then   # SKIP_TESTS=1: the suite ran on this build in an earlier call
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
timeout -k 10 300 python -u bench.py > "$OUT/bench_forward.json" 2> "$OUT/forward.err"
timeout -k 10 200 python -u bench.py --mode generate > "$OUT/bench_generate.json" 2> "$OUT/generate.err"
timeout -k 10 300 python -u bench.py --mode chain > "$OUT/bench_chain.json" 2> "$OUT/chain.err"
timeout -k 10 300 python -u bench.py --mode train > "$OUT/bench_train.json" 2> "$OUT/train.err"
timeout -k 10 200 python -u bench.py --mode lj > "$OUT/bench_lj.json" 2> "$OUT/lj.err"
timeout -k 10 300 python -u bench.py --mode lj_train > "$OUT/bench_lj_train.json" 2> "$OUT/lj_train.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_fwd" -o run -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline > "$OUT/bench_forward_under_profiler.json" 2> "$OUT/prof_fwd.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_train" -o run -- \
  python3 "$ROOT/bench.py" --mode train --steps 5 --warmup 2 > "$OUT/bench_train_under_profiler.json" 2> "$OUT/prof_train.err"
echo done
