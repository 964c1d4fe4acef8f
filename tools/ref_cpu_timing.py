"""Time the REFERENCE implementation on this container's CPU cores (the
reference's own CPU path: float64 torch, enflow/flow/dynamics.py + nn/egcl.py
+ nn/argmax.py + flow/loss.py) on bounded samples of BASELINE configs[1]
(1024 x 22-atom molecules, 8 layers, H=128, forward) and configs[3] (64-atom
molecules, one training step: forward + Alchemical_NLL + loss.backward() +
Adam), and write the numbers to profiles/r02/r02_reference_cpu.json.

Build container only (the reference does not travel to the GPU boxes):

    PYTHONDONTWRITEBYTECODE=1 python tools/ref_cpu_timing.py

Data.edges is restated around the reference's own helpers exactly as the golden
generator does (tests/golden/make_golden.py RefData: enflow.data.base needs
rdkit, which is absent).  bench.py's cpu_baseline is the float64 numpy oracle
timed on the GPU box's host; this file is the reference itself, here.
"""
import importlib.util
import json
import os
import platform
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("make_golden", os.path.join(ROOT, "tests", "golden", "make_golden.py"))
G = importlib.util.module_from_spec(spec)
spec.loader.exec_module(G)           # puts /root/reference on sys.path, imports the reference's modules

import numpy as np  # noqa: E402
import torch  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def model(hid=128, nf=5, layers=8, seed=0):
    torch.manual_seed(seed)
    return G.LFIntegrator([G.EGCL(nf, nf, hid) for _ in range(layers)], G.ArgMax(nf, hid), dt=G.default_dt())


def batch(num, atoms, seed, radius=None):
    kw = {} if radius is None else {"radius": radius}
    b = G.make_molecules(num, atoms, nf=5, seed=seed, **kw)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = G.f32(b[k])
    return b


def time_forward(sample, reps):
    m = model()
    b = batch(sample, 22, 1)
    ts = []
    for r in range(reps + 1):
        d = G.ref_data(b)
        t0 = time.perf_counter()
        with torch.no_grad():
            m(d)
        ts.append(time.perf_counter() - t0)
    best = min(ts[1:])
    return {"sample": f"{sample} x 22-atom molecules, 8 layers, H=128, nf=5, float64 (BaseFlow casts)",
            "seconds_per_batch": best, "value": sample / best, "unit": "molecule-transforms/s"}


def time_train(sample, reps):
    m = model()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    nll = G.Alchemical_NLL(kBT=G.default_kBT(), softening=0.1)
    b = batch(sample, 64, 2, radius=4.0 * (64 / 22.0) ** (1.0 / 3.0))
    ts = []
    for r in range(reps + 1):
        d = G.ref_data(b)
        t0 = time.perf_counter()
        opt.zero_grad()
        out, ldj = m(d)
        loss = nll(out, ldj)
        loss.backward()
        opt.step()
        ts.append(time.perf_counter() - t0)
    best = min(ts[1:])
    return {"sample": f"{sample} x 64-atom molecules, 8 layers, H=128: forward + NLL + backward + Adam, float64",
            "seconds_per_step": best, "value": sample / best, "unit": "molecules/s"}


def main():
    threads = torch.get_num_threads()
    res = {
        "what": "reference implementation (bharath-raghavan/enflow, /root/reference) on CPU, float64 torch",
        "host": {"cpu": cpu_model(), "logical_cpus": os.cpu_count(),
                 "affinity": len(os.sched_getaffinity(0)), "torch_threads": threads,
                 "torch": torch.__version__},
        "configs[1]_forward": time_forward(64, 2),
        "configs[3]_train_step": time_train(8, 2),
    }
    out = os.path.join(ROOT, "profiles", "r02", "r02_reference_cpu.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
