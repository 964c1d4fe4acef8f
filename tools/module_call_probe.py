"""Where the host time of one inference module call goes.

``model(data)`` on the bench batch (configs[1]: 1024 x 22 atoms, 8 layers,
H = 128, f16x3) under torch.no_grad(), with perf_counter stamps at: call
entry, just before the kernel launch (forward_buffers entered), launch
returned, error-word read entered, error-word read returned, call return; the
kernel's own duration from the library's HIP-event timer.  Medians over
calls.

    python tools/module_call_probe.py [float32|float64] > profiles/rNN/module_call_probe.json
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    from enflow_amd.flow import dynamics
    dt = getattr(torch, sys.argv[1]) if len(sys.argv) > 1 else torch.float32
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    b = make_molecules(bench.MOLS_PER_GPU, bench.ATOMS, nf=bench.NF, seed=1000)
    d = Data.from_arrays(b, device=dev, dtype=dt)
    marks = {}
    fb, te = dynamics.LFIntegrator.forward_buffers, _lib.take_err

    def fb_w(self, *a, **k):
        marks.setdefault("launch_enter", time.perf_counter())
        r = fb(self, *a, **k)
        marks.setdefault("launch_return", time.perf_counter())
        return r

    def te_w(x):
        marks.setdefault("sync_enter", time.perf_counter())
        r = te(x)
        marks.setdefault("sync_return", time.perf_counter())
        return r

    dynamics.LFIntegrator.forward_buffers = fb_w
    _lib.take_err = te_w
    rows = []
    with torch.no_grad():
        for i in range(300):
            marks.clear()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            model(d._replace())
            t1 = time.perf_counter()
            if i >= 100:
                rows.append({"to_launch": marks["launch_enter"] - t0,
                             "launch_call": marks["launch_return"] - marks["launch_enter"],
                             "launch_to_sync": marks["sync_enter"] - marks["launch_return"],
                             "sync": marks["sync_return"] - marks["sync_enter"],
                             "after_sync": t1 - marks["sync_return"], "total": t1 - t0})
        with _lib.KernelTimer() as kt:
            for _ in range(50):
                model(d._replace())
    dynamics.LFIntegrator.forward_buffers, _lib.take_err = fb, te
    out = {k: float(np.median([r[k] for r in rows])) * 1e6 for k in rows[0]}
    out = {"dtype": str(dt), "median_us": out,
           "kernel_us": kt.ms_per_launch("lf_flow_kernel<fwd>") * 1e3,
           "note": "perf_counter stamps per call (median of 200 after 100 untimed); kernel_us from HIP events"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
