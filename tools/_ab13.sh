set -e
mkdir -p gpurun_out/ab13
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab13/train_tests.log 2>&1
timeout -k 10 200 env ENFLOW_LIB=$PWD/enflow_amd/var/libenflow_ox2oa.so python -u -m pytest tests/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab13/train_tests_ox2oa.log 2>&1
V=enflow_amd/var
timeout -k 10 500 python -u tools/ab_train.py $V/libenflow_t0.so $V/libenflow_ox2.so $V/libenflow_oa128.so $V/libenflow_ox2oa.so > gpurun_out/ab13/ab.txt 2>&1
echo done
