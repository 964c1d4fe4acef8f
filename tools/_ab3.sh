set -e
mkdir -p gpurun_out/ab3
V=enflow_amd/var
timeout -k 10 200 python -u tools/stamps.py $V/libenflow_stamps.so > gpurun_out/ab3/stamps.txt 2>&1
timeout -k 10 400 python -u tools/ab_libs.py $V/libenflow_B3.so $V/libenflow_sk3.so $V/libenflow_sk7.so $V/libenflow_sk14.so $V/libenflow_sk7b.so $V/libenflow_B3.so > gpurun_out/ab3/ab.txt 2>&1
echo done
