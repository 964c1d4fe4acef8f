set -e
mkdir -p gpurun_out/ab11
timeout -k 10 200 python -u tools/stamps.py enflow_amd/var/libenflow_stamps4.so > gpurun_out/ab11/stamps.txt 2>&1
echo done
