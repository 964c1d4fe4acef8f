"""Interleaved A/B of library builds on the bench forward (BASELINE configs[1]
molecules, H = 128, 8 layers, f16x3) at several batch sizes, each with the
instance the library picks by default (4-wave at 1024 molecules, the
feature-split instance at the 8- / 4-rank shards 128 / 256), in ONE process
(cdna_hip_programming.md rule 24): per round every library runs every size,
rounds repeated; medians and the outputs' difference to the first library.

    python tools/ab_flow.py libA.so libB.so [...]      (AB_MOLS=1024,128,256 AB_ROUNDS=7 AB_DIR=fwd|rev)
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rel(a, b):
    import torch
    return float(torch.linalg.norm((a - b).double()) / max(float(torch.linalg.norm(b.double())), 1e-30))


def main():
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import make_molecules
    libs = sys.argv[1:]
    sizes = [int(x) for x in os.environ.get("AB_MOLS", "1024,128,256").split(",")]
    rounds = int(os.environ.get("AB_ROUNDS", "7"))
    reverse = os.environ.get("AB_DIR", "fwd") == "rev"
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    model.gemm_precision = "f16x3"
    g = make_molecules(1024, bench.ATOMS, nf=bench.NF, seed=1000)
    inps = {m: bench.batch_tensors(bench.sub_batch(g, 0, m), dev) for m in sizes}
    times = {(lib, m): [] for lib in libs for m in sizes}
    outs = {}

    def use(spec):
        # "path" or "path:noahead" (the same library with enflow_set_dequant_ahead(0))
        path, _, opt = spec.partition(":")
        _lib._libs.clear()
        _lib._dq_ahead[0] = 0 if opt == "noahead" else None
        _lib.LIB_PATH = path
        model._layers_key = None
        model._train_key = None
        model.dequantize._packed_key = None
        model.__dict__.pop("_spec", None)

    for r in range(rounds):
        for lib in libs:
            use(lib)
            for m in sizes:
                run = bench.FlowRunner(model, inps[m], bench.ATOMS, reverse, dev, torch.Generator(dev).manual_seed(0))
                if reverse:   # every library inverts the first library's forward outputs
                    key = ("src", m)
                    if key not in outs:
                        outs[key] = {k: v.clone() for k, v in run.src.items()}
                    run.src = outs[key]
                if r == 0:   # the runner's first step: the same noise key in every library
                    run.step()
                    run.check()
                    outs[(lib, m)] = {k: run.work[k].clone() for k in ("h", "g", "pos", "vel")}
                el = bench.timed(run.step, 30, 10, None, dev)
                run.check()
                times[(lib, m)].append(el / 30 * 1e3)
    res = []
    for m in sizes:
        for lib in libs:
            t = times[(lib, m)]
            o, o0 = outs[(lib, m)], outs[(libs[0], m)]
            row = {"mols": m, "dir": "rev" if reverse else "fwd", "lib": os.path.basename(lib),
                   "median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
                   "vs_first": {k: rel(o[k], o0[k]) for k in o}}
            res.append(row)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
