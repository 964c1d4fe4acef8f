set -e
mkdir -p gpurun_out/r02b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r02b/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 > gpurun_out/r02b/bench_train.json 2> gpurun_out/r02b/train.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02b/bench_forward.json 2> gpurun_out/r02b/forward.err
echo done
