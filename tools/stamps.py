"""Diagnostic: per-phase cycle shares of the fused flow kernel.

Builds libenflow_hip_stamps.so (-DENFLOW_STAMPS, never shipped as the product
library), runs the bench workload through it and prints the share of wave-0
cycles spent in each phase.  Usage (GPU box): python tools/stamps.py [MOLS]
(MOLS molecules of the bench's 22-atom workload, default 1024; the 4-wave
instance is forced, so e.g. 128 shows one molecule's latency chain per CU)
"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "enflow_amd", "libenflow_hip_stamps.so")
FS_PHASES = ["load", "dequant", "layer setup", "pairs:images+idmap", "pairs:counts+compact", "(after tiles)",
             "tail T1: node items + next weights", "tail T2: update + hand-off", "-", "  tiles:setup+decode0", "  A gemm0+act+split", "  barrier X",
             "  A gemm1", "  A act+split", "  barrier Y", "  tail", "  T1: G frags issued, h split",
             "  T1: G node_nn.0 chain", "  T1: G act + node_nn.2", "writeback"]
PHASES = ["load", "dequant", "pairs:counts+compact", "pairs:images+idmap", "edge_tiles(all)", "node", "update", "writeback",
          "  tiles:setup", "  gemm0", "  silu0", "  gemm1", "  silu1", "  segsum", "  gemm2+phi+force", "  tail-barrier"]


def main():
    global SO
    if len(sys.argv) > 1 and sys.argv[1].endswith(".so"):
        SO = os.path.abspath(sys.argv[1])
    if not os.path.exists(SO):          # build here (CPU container) and ship: the box only runs it
        sys.path.insert(0, ROOT)
        from enflow_amd.build import build
        build(force=False, out=SO, defines=["ENFLOW_STAMPS"])
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        return
    mols = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1024
    lat = "lat" in sys.argv[1:]         # the 8-wave latency instance instead of the 4-wave one
    fs = 2 if "fs2" in sys.argv[1:] else (1 if "fs1" in sys.argv[1:] else 0)   # the feature-split instance
    os.environ["ENFLOW_LIB"] = SO
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from enflow_amd import _lib
    L = _lib.lib()
    rd = L.enflow_read_stamps_fs if fs else (L.enflow_read_stamps_lat if lat else L.enflow_read_stamps)
    rd.restype = ctypes.c_int
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.enflow_set_latency_threshold(100000 if lat else 0)   # which instance is stamped
    L.enflow_set_split_threshold(100000 if fs == 2 else 0)
    L.enflow_set_fs_threshold(100000 if fs == 1 else 0)
    phases = FS_PHASES if fs else PHASES
    wgs = mols * (2 if fs == 2 else 1)
    dev = torch.device("cuda", 0)
    from enflow_amd.data.synthetic import make_molecules
    model = bench.build_model(dev, bench.LAYERS)
    inp = bench.batch_tensors(make_molecules(mols, bench.ATOMS, nf=bench.NF, seed=1000), dev)
    work = {k: inp[k].clone() for k in ("h", "g", "pos", "vel")}
    noise = torch.randn_like(inp["h"])
    ldj_mol = torch.empty(mols, device=dev)
    ldj = torch.empty(1, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    buf = (ctypes.c_ulonglong * 32)()
    for rep in range(3):
        for k in work:
            work[k].copy_(inp[k])
        torch.cuda.synchronize()
        rd(buf, 1)
        model.forward_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                              inp["mol_ptr"], bench.ATOMS, noise, ldj_mol, ldj, err)
        torch.cuda.synchronize()
        rd(buf, 1)
    tot = sum(buf)       # every stamp closes the interval since the previous one: disjoint
    for name, v in zip(phases, buf):
        print(f"{name:24s} {100.0 * v / tot:6.2f} %   {v / wgs:12.0f} cycles/WG  "
              f"{v / wgs / bench.LAYERS:10.0f} cycles/WG/layer")


if __name__ == "__main__":
    main()
