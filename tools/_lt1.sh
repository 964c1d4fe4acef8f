set -e
mkdir -p gpurun_out/lt1
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_systems.py tests/test_gpu_large.py -x -v -s --timeout 200 --timeout-method thread -k "training" > gpurun_out/lt1/large_train.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/lt1/pytest_gpu.log 2>&1
echo done
