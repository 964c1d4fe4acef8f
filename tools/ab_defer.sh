#!/bin/bash
# A/B of the deferred backward error check on the training step (bench.py --mode train),
# alternating sync (old) and deferred (new) runs; then the GPU suite.
set -euo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/defer
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
for i in 1 2; do
  timeout -k 10 200 python -u -c "import sys, runpy; sys.path.insert(0, '.'); import enflow_amd._lib as L; L.defer_err = L.raise_on_err; sys.argv = ['bench.py', '--mode', 'train', '--steps', '10', '--warmup', '3']; runpy.run_path('bench.py', run_name='__main__')" > "$OUT/sync_$i.json" 2> "$OUT/sync_$i.err"
  timeout -k 10 200 python -u bench.py --mode train --steps 10 --warmup 3 > "$OUT/defer_$i.json" 2> "$OUT/defer_$i.err"
done
echo done
