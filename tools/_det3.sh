set -e
mkdir -p gpurun_out/det3
L=enflow_amd/libenflow_hip.so
timeout -k 10 200 env AB_LAYERS=1 python -u tools/det_check.py $L $L $L $L > gpurun_out/det3/L1.txt 2>&1
timeout -k 10 200 env AB_LAYERS=2 python -u tools/det_check.py $L $L $L $L > gpurun_out/det3/L2.txt 2>&1
timeout -k 10 200 env AB_ATOMS=22 python -u tools/det_check.py $L $L $L $L > gpurun_out/det3/a22.txt 2>&1
echo done
