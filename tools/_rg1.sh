set -e
mkdir -p gpurun_out/rg1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread -k "range_guard or floor" > gpurun_out/rg1/parity.log 2>&1
echo done
