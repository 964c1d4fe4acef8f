set -e
mkdir -p gpurun_out/ab9
timeout -k 10 200 python -u tools/stamps.py enflow_amd/var/libenflow_stamps3.so > gpurun_out/ab9/stamps.txt 2>&1
echo done
