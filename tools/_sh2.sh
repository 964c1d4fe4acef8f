set -e
mkdir -p gpurun_out/sh2
timeout -k 10 300 python -u -m pytest tests/test_gpu_shapes.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/sh2/shapes.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sh2/pytest_gpu.log 2>&1
echo done
