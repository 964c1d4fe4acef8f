set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/gt_var.log 2>&1
timeout -k 10 300 python -u tools/ab_libs.py ab/wmax.so enflow_amd/libenflow_hip.so > gpurun_out/ab_fwd_var.log 2>&1
