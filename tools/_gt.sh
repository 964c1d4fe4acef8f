set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/gt_red4.log 2>&1
timeout -k 10 400 python -u tools/ab_train.py ab/fold.so ab/red4.so > gpurun_out/ab_train10.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_red4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --mode train --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_red4.json 2>&1
