set -e
mkdir -p gpurun_out/ab8
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/ab8/pytest_gpu.log 2>&1
timeout -k 10 400 python -u tools/ab_libs.py enflow_amd/var/libenflow_pre_g0.so enflow_amd/libenflow_hip.so > gpurun_out/ab8/ab.txt 2>&1
echo done
