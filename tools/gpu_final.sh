#!/bin/bash
# Round-end evidence for one library build (run on the GPU box via gpurun):
# GPU tests, smoke, every bench mode, rocprofv3 kernel stats of the forward and
# training benches, PMC traffic of the flow kernel, then the forward bench again
# so its line carries the traffic of this exact build; the strong-scaling probe
# and PMC of the training kernels.
# Usage: bash tools/gpu_final.sh <tag>
set -euo pipefail
TAG=${1:-r02f}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
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
cd "$ROOT"
timeout -k 10 900 python -u profiles/collect_pmc.py "$TAG" > "$OUT/pmc.log" 2>&1
mkdir -p profiles/_box && cp "gpurun_out/${TAG}_pmc_traffic.json" profiles/_box/
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_forward_traffic.json" 2> "$OUT/forward_traffic.err"
rm -rf profiles/_box
timeout -k 10 300 python -u tools/strong_scaling_probe.py > "$OUT/strong_probe.json" 2> "$OUT/strong.err"
timeout -k 10 900 python -u profiles/collect_pmc.py "${TAG}_train" train lf_layer_bwd_kernel,outer_x3_kernel > "$OUT/pmc_train.log" 2>&1
echo done
