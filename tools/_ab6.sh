set -e
mkdir -p gpurun_out/ab6
V=enflow_amd/var
timeout -k 10 200 python -u tools/stamps.py $V/libenflow_stamps2.so > gpurun_out/ab6/stamps.txt 2>&1
timeout -k 10 400 python -u tools/ab_libs.py enflow_amd/libenflow_hip.so $V/libenflow_w3.so > gpurun_out/ab6/ab.txt 2>&1
echo done
