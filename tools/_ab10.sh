set -e
mkdir -p gpurun_out/ab10
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/ab10/pytest_gpu.log 2>&1
timeout -k 10 400 python -u tools/ab_libs.py enflow_amd/var/libenflow_pre_img.so enflow_amd/libenflow_hip.so > gpurun_out/ab10/ab.txt 2>&1
echo done
