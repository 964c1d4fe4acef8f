"""Diagnostic: per-phase cycles of the ArgMax dequantisation kernel
(dequant_kernel, round 6) on the bench workload (1024 x 22 atoms, H = 128),
with in-kernel draws and with the caller's noise.  Uses the stamps library
(tools/stamps.py build; -DENFLOW_STAMPS, never the product).

    python tools/dq_stamps.py [MOLS] [lib.so]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "enflow_amd", "libenflow_hip_stamps.so")
PHASES = ["load + network.2 staging", "hidden layer", "barriers", "network outputs", "draws + u",
          "z + log_q", "copy-back + store"]


def main():
    mols = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    os.environ["ENFLOW_LIB"] = os.path.abspath(sys.argv[2]) if len(sys.argv) > 2 else SO
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import make_molecules
    L = _lib.lib()
    rd = L.enflow_read_dq_stamps
    rd.restype = ctypes.c_int
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    inp = bench.batch_tensors(make_molecules(mols, bench.ATOMS, nf=bench.NF, seed=1000), dev)
    work = {k: inp[k].clone() for k in ("h", "g", "pos", "vel")}
    ldj_mol = torch.empty(mols, device=dev)
    ldj = torch.empty(1, device=dev)
    err = torch.zeros(2, dtype=torch.int32, device=dev)
    buf = (ctypes.c_ulonglong * 8)()
    out = {}
    for draws in ("kernel", "caller"):
        noise = None if draws == "kernel" else torch.randn_like(inp["h"])
        for rep in range(3):
            torch.cuda.synchronize()
            rd(buf, 1)
            with _lib.KernelTimer() as kt:
                model.forward_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                                      inp["mol_ptr"], bench.ATOMS, noise, ldj_mol, ldj, err[:1], src=(
                                          inp["h"], inp["g"], inp["pos"], inp["vel"]), noise_key=(1234, 0))
                torch.cuda.synchronize()
            rd(buf, 1)
        tot = sum(buf[:7])
        out[draws] = {"cycles_per_wg": {p: round(buf[i] / mols) for i, p in enumerate(PHASES)},
                      "total_cycles_per_wg": round(tot / mols),
                      "dequant_kernel_ms": kt.ms_per_launch("dequant_kernel") if "dequant_kernel" in kt.stats else None}
        print(json.dumps({"draws": draws, **out[draws]}), flush=True)


if __name__ == "__main__":
    main()
