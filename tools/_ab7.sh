set -e
mkdir -p gpurun_out/ab7
V=enflow_amd/var
timeout -k 10 400 python -u tools/ab_libs.py enflow_amd/libenflow_hip.so $V/libenflow_silu.so $V/libenflow_w3.so > gpurun_out/ab7/ab.txt 2>&1
echo done
