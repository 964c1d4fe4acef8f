"""Data-parallel training over the HIP backward (BASELINE configs[3]'s DP leg).

Two fresh child processes (this file sorts first, so the pytest process has
not initialised the GPU when they start) each wrap LFIntegrator in
DistributedDataParallel as the reference's driver does
(/root/reference/enflow/main.py:159) and run one step of its loop body
(main.py:217-222) on their shard of a global batch.  After DDP's all-reduce,
every rank's .grad must equal the mean of the single-process HIP gradients of
the two shards (normwise <= 1e-6: the all-reduce only reorders two fp32 adds),
and both ranks must hold identical gradients and identical parameters after
the optimizer step.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from _fixtures import rel_err

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TOL = 1e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ddp_two_ranks_average_the_hip_gradients(tmp_path):
    import torch
    if torch.cuda.device_count() < 1:          # does not initialise HIP on this image
        pytest.skip("no GPU")
    port = _free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "_ddp_worker.py"), str(r), "2", str(port),
                               str(tmp_path)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(2)]
    outs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(o)
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
    z = [np.load(os.path.join(tmp_path, f"rank{r}.npz")) for r in range(2)]
    n = int(z[0]["n"])
    worst = 0.0
    for i in range(n):
        want = (z[0][f"local0_{i}"] + z[0][f"local1_{i}"]) / 2
        for r in range(2):
            got = z[r][f"ddp_{i}"]
            err = rel_err(got, want)      # raises on NaN / inf
            worst = max(worst, err)
            assert err <= TOL, (i, r, err)
        np.testing.assert_array_equal(z[0][f"ddp_{i}"], z[1][f"ddp_{i}"])
        np.testing.assert_array_equal(z[0][f"after_{i}"], z[1][f"after_{i}"])
        # the single-process HIP gradients are deterministic: both ranks computed the same
        np.testing.assert_array_equal(z[0][f"local0_{i}"], z[1][f"local0_{i}"])
    print(f"DDP world 2: {n} parameter tensors, max normwise |ddp - mean(local)| = {worst:.2e} (bar {TOL:g})")
