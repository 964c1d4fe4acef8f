set -e
mkdir -p gpurun_out/ab1
timeout -k 10 300 env ENFLOW_LIB=$PWD/enflow_amd/var/libenflow_B.so python -u -m pytest tests/test_gpu_parity.py -x -q -s --timeout 200 --timeout-method thread -k "forward or reverse or bench or ragged" > gpurun_out/ab1/parity_B.log 2>&1
timeout -k 10 300 python -u tools/ab_libs.py enflow_amd/var/libenflow_A.so enflow_amd/var/libenflow_B.so enflow_amd/var/libenflow_C.so enflow_amd/var/libenflow_D.so > gpurun_out/ab1/ab.txt 2>&1
echo done
