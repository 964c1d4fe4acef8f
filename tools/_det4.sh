set -e
mkdir -p gpurun_out/det4
L=enflow_amd/libenflow_hip.so
timeout -k 10 200 env AB_LAYERS=2 python -u tools/det_check.py $L $L $L $L > gpurun_out/det4/L2.txt 2>&1
timeout -k 10 300 python -u tools/det_check.py $L $L $L $L $L > gpurun_out/det4/L8.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py tests/test_0_ddp_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/det4/train_tests.log 2>&1
echo done
