set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/gt_det.log 2>&1
timeout -k 10 400 python -u tools/ab_train.py ab/wmax.so ab/det.so ab/det.so > gpurun_out/ab_train12.log 2>&1
