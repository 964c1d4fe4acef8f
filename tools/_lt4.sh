set -e
mkdir -p gpurun_out/lt4
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_systems.py tests/test_gpu_modules.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/lt4/large.log 2>&1
timeout -k 10 300 python -u bench.py --mode lj_train --steps 5 --warmup 2 > gpurun_out/lt4/lj_train.json 2> gpurun_out/lt4/lj_train.err
echo done
