set -e
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r02c/pytest_gpu.log 2>&1
echo done
