"""A/B several builds of libenflow_hip.so on the bench workload, interleaved
rounds in ONE process (cdna_hip_programming.md rule 24).

    python tools/ab_libs.py path/to/libA.so path/to/libB.so ...
    AB_MODE=chain python tools/ab_libs.py ...     # another bench.MODES workload (forward ones)
"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from enflow_amd import _lib
    libs = sys.argv[1:]
    dev = torch.device("cuda", 0)
    c = bench.MODES[os.environ.get("AB_MODE", "forward")]
    from enflow_amd.data.synthetic import make_molecules
    model = bench.build_model(dev, c["layers"])
    c = dict(c, mols=int(os.environ.get("AB_MOLS", c["mols"])))   # e.g. AB_MOLS=128: the latency instance
    inp = bench.batch_tensors(make_molecules(c["mols"], c["atoms"], nf=bench.NF, seed=1000, chain=c["chain"]), dev)
    model.gemm_precision = c["prec"]
    mols, atoms = c["mols"], c["atoms"]
    work = {k: inp[k].clone() for k in ("h", "g", "pos", "vel")}
    noise = torch.randn_like(inp["h"])
    ldj_mol = torch.empty(mols, device=dev)
    ldj = torch.empty(1, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    outs = {}

    def run(path, reps):
        _lib._libs.clear()
        _lib.LIB_PATH = path
        model._layers_key = None
        model.dequantize._packed_key = None
        ev = []
        for _ in range(reps):
            for k in work:
                work[k].copy_(inp[k])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            # the ABI-7 entry (in place, caller's noise): present in every build compared
            hid, nf, cw = model._geometry()
            _lib.check(_lib.lib().enflow_lf_forward_f32(
                mols, work["h"].shape[0], atoms, nf, hid, _lib.ptr(inp["mol_ptr"]), _lib.ptr(inp["r_cut"]),
                _lib.ptr(inp["box"]), _lib.ptr(work["h"]), _lib.ptr(work["g"]), _lib.ptr(work["pos"]),
                _lib.ptr(work["vel"]), _lib.ptr(model.packed_layers(dev)), len(model.networks), _lib.DEQUANT_ARGMAX,
                _lib.ptr(model.dequantize.packed(dev, hid)), _lib.ptr(noise), 0.0, float(model.dt), cw,
                _lib.ptr(ldj_mol), _lib.ptr(ldj), _lib.ptr(err), None, None, None, model._prec(),
                _lib.stream_ptr(dev)), "enflow_lf_forward_f32")
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()   # launches back to back: no idle gap lets the clocks drop
        outs[path] = (work["pos"].clone(), ldj.clone())
        return [a.elapsed_time(b) for a, b in ev]

    res = {p: [] for p in libs}
    for p in libs:
        run(p, 3)          # warm-up / pack
    for _ in range(int(os.environ.get("AB_PREWARM", "200")) // len(libs)):   # clocks up before the first timed round
        for p in libs:
            run(p, 1)
    for rnd in range(int(os.environ.get("AB_ROUNDS", "6"))):
        for p in libs:
            res[p] += run(p, 5)
    base = outs[libs[0]]
    for p in libs:
        same = torch.equal(outs[p][0], base[0])
        rel = float((outs[p][0] - base[0]).abs().max() / base[0].abs().max())
        print(f"{os.path.basename(p):40s} median {statistics.median(res[p]):.4f} ms  min {min(res[p]):.4f} ms"
              f"  mol/s {mols / statistics.median(res[p]) * 1e3:.0f}  bitwise-equal-to-first {same} "
              f"pos-rel-diff {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
