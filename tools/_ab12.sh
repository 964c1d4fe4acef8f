set -e
mkdir -p gpurun_out/ab12
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/ab12/pytest_gpu.log 2>&1
timeout -k 10 400 python -u tools/ab_libs.py enflow_amd/var/libenflow_c460.so enflow_amd/libenflow_hip.so enflow_amd/var/libenflow_c460.so enflow_amd/libenflow_hip.so > gpurun_out/ab12/ab.txt 2>&1
echo done
