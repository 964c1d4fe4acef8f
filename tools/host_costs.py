"""Host cost (us per call, GPU box) of the primitives a module call runs
before its launch: allocations, stream lookups, the noise-key draw, the
input checks, the ctypes launch argument build.  A development probe for
VERDICT r5 item 3 (tools/module_call_probe.py times the call itself)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def t(f, n=5000):
    for _ in range(50):
        f()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    b = make_molecules(bench.MOLS_PER_GPU, bench.ATOMS, nf=bench.NF, seed=1000)
    d = Data.from_arrays(b, device=dev)
    x = d.h
    out = {
        "empty_like": t(lambda: torch.empty_like(x)),
        "empty(1)": t(lambda: torch.empty(1, dtype=torch.float32, device=dev)),
        "current_stream": t(lambda: torch.cuda.current_stream(dev).cuda_stream),
        "randint_item": t(lambda: int(torch.randint(0, 2 ** 62, (1,)).item())),
        "device_eq": t(lambda: x.device == dev),
        "is_large": t(lambda: _lib.is_large(22)),
        "state": t(lambda: model._state(d)),
        "state_noout": t(lambda: model._state(d, outputs=False)),
        "infer_words": t(lambda: _lib.infer_words(dev, 1024)),
        "launch_cfg": t(lambda: model.launch_cfg(dev), 500),
        "params_key": t(lambda: model._params_key(dev), 500),
        "ptr": t(lambda: _lib.ptr(x)),
        "no_grad_enter_exit": t(lambda: torch.no_grad().__enter__()),
    }
    with torch.no_grad():
        out["needs_grad(no_grad)"] = t(model._needs_grad)
        out["module_call"] = t(lambda: model(d._replace()), 200)
    print(json.dumps({k: round(v, 2) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
