set -e
mkdir -p gpurun_out/det2
L=enflow_amd/libenflow_hip.so
timeout -k 10 300 env ENFLOW_SERIAL_BWD=1 python -u tools/det_check.py $L $L $L $L > gpurun_out/det2/serial.txt 2>&1
timeout -k 10 300 python -u tools/det_check.py $L $L $L $L > gpurun_out/det2/overlap.txt 2>&1
echo done
