#!/bin/bash
# Round-end evidence, part 2: PMC traffic of the flow kernel and the forward line
# re-run with it (same build), the strong-scaling probe, PMC of the training kernels.
# Usage: bash tools/gpu_final_b.sh <tag>
set -euo pipefail
TAG=${1:-rXX}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 900 python -u profiles/collect_pmc.py "$TAG" > "$OUT/pmc.log" 2>&1
mkdir -p profiles/_box && cp "gpurun_out/${TAG}_pmc_traffic.json" profiles/_box/
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_forward_traffic.json" 2> "$OUT/forward_traffic.err"
rm -rf profiles/_box
timeout -k 10 300 python -u tools/strong_scaling_probe.py > "$OUT/strong_probe.json" 2> "$OUT/strong.err"
timeout -k 10 900 python -u profiles/collect_pmc.py "${TAG}_train" train lf_layer_bwd_kernel,outer_x3_kernel > "$OUT/pmc_train.log" 2>&1

# last: the strong-scaling probe (split instance included) under the profiler,
# with its exit status recorded (the round-4 exit-time SIGSEGV check)
cd /tmp && export TMPDIR=/tmp
rc=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_strong" -o run -- \
  python3 "$ROOT/tools/strong_scaling_probe.py" > "$OUT/strong_probe_under_profiler.json" 2> "$OUT/prof_strong.err" || rc=$?
echo "prof_strong exit status $rc" | tee "$OUT/prof_strong.status"
echo done
