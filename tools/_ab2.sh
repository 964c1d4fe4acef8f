set -e
mkdir -p gpurun_out/ab2
V=enflow_amd/var
timeout -k 10 400 python -u tools/ab_libs.py $V/libenflow_B.so $V/libenflow_abl1.so $V/libenflow_abl2.so $V/libenflow_abl4.so $V/libenflow_abl8.so $V/libenflow_abl16.so $V/libenflow_abl30.so $V/libenflow_abl31.so > gpurun_out/ab2/ab.txt 2>&1
echo done
