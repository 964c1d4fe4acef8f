"""Interleaved timing of the two fused-kernel instances on one batch size:
the 4-wave throughput build vs the 8-wave latency build (threshold forced),
bench forward workload, AB_MOLS molecules (default 1024).

    python tools/ab_instance.py [MOLS ...]
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
    from enflow_amd.data.synthetic import make_molecules
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    for mols in [int(a) for a in sys.argv[1:]] or [1024]:
        g = make_molecules(mols, bench.ATOMS, nf=bench.NF, seed=1000)
        run = bench.FlowRunner(model, bench.batch_tensors(g, dev), bench.ATOMS, False, dev,
                               torch.Generator(dev).manual_seed(0))
        res = {"4-wave": [], "8-wave": []}
        for rnd in range(6):
            for name, thr in (("4-wave", 0), ("8-wave", 1 << 30)):
                _lib.set_latency_threshold(thr)
                el = bench.timed(run.step, 30, 10 if rnd else 40, None, dev)
                res[name].append(el / 30 * 1e3)
        _lib.set_latency_threshold(-1)
        for k, v in res.items():
            print(f"{mols:5d} molecules {k}: median {statistics.median(v):.4f} ms  min {min(v):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
