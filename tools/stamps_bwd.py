"""Diagnostic: per-phase cycle shares of lf_layer_bwd_kernel (training
backward), wave 0 of every workgroup, summed over the backward's layers.

Builds ab/stamps.so (-DENFLOW_STAMPS_BWD, never the product library:
`python -m enflow_amd.build ab/stamps.so ENFLOW_STAMPS_BWD`), runs one
training step of bench.py's train workload and prints each phase's cycles per
workgroup.  Usage (GPU box): python tools/stamps_bwd.py [lib.so]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PHASES = ["load", "leapfrog", "node", "pairs", "tile:setup+xin+gemm0", "tile:epi0", "tile:gemm1+epi1",
          "tile:gemm2+epi2+phi", "tile:gemm3", "tile:wait+epi3", "tile:gemm4", "tile:epi4", "tile:gemm5",
          "atomics+barrier", "writeback", "-", "tile:gemm3 scale(cv)", "tile:gemm3 chain", "tile:gemm1 chain",
          "tile:gemm2 chain"]


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "ab", "stamps.so")
    os.environ["ENFLOW_LIB"] = so
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator, Alchemical_NLL
    from enflow_amd.data import Data
    L = _lib.lib()
    L.enflow_read_stamps.restype = ctypes.c_int
    L.enflow_read_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda", 0)
    atoms = bench.TRAIN_ATOMS
    b = make_molecules(bench.MOLS_PER_GPU, atoms, nf=bench.NF, seed=2000, radius=4.0 * (atoms / 22.0) ** (1 / 3))
    torch.manual_seed(0)
    model = LFIntegrator([EGCL(bench.NF, bench.NF, bench.HID) for _ in range(bench.LAYERS)],
                         ArgMax(bench.NF, bench.HID), dt=default_dt()).to(dev)
    nll = Alchemical_NLL(kBT=default_kBT(), softening=0.1)
    base = Data.from_arrays(b, device=dev)
    noise = torch.randn_like(base.h)
    buf = (ctypes.c_ulonglong * 32)()
    for rep in range(3):
        model.zero_grad(set_to_none=True)
        out, ldj = model(base._replace(), noise=noise)
        loss = nll(out, ldj)
        torch.cuda.synchronize()
        L.enflow_read_stamps(buf, 1)
        loss.backward()
        torch.cuda.synchronize()
        L.enflow_read_stamps(buf, 1)
    tot = sum(buf)
    wgs = bench.MOLS_PER_GPU * bench.LAYERS
    for name, v in zip(PHASES, buf):
        if v:
            print(f"{name:24s} {100.0 * v / tot:6.2f} %   {v / wgs:12.0f} cycles/WG")


if __name__ == "__main__":
    main()
