set -e
mkdir -p gpurun_out/det1
V=enflow_amd/var
timeout -k 10 300 python -u tools/det_check.py $V/libenflow_t0.so $V/libenflow_t0.so $V/libenflow_t0b.so $V/libenflow_ox2.so $V/libenflow_t0.so > gpurun_out/det1/det.txt 2>&1
echo done
