"""Interleaved timing of the fused-kernel instances per batch size: the
4-wave throughput build, the 8-wave latency build and the cooperative build
(two workgroups per molecule; instance forced through the latency threshold and
the cooperative limit), bench forward workload; outputs of the instances
compared with the 4-wave one (max relative position difference).

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
        modes = (("4-wave", 0, 0), ("8-wave", 1 << 30, 0), ("coop", 1 << 30, 1 << 30))
        res = {m[0]: [] for m in modes}
        outs = {}
        for rnd in range(6):
            for name, thr, coop in modes:
                _lib.set_latency_threshold(thr)
                _lib.set_coop_max(coop)
                el = bench.timed(run.step, 30, 10 if rnd else 40, None, dev)
                res[name].append(el / 30 * 1e3)
                if rnd == 0:   # one step with the same noise counters in every mode
                    run.calls = 999
                    run.step()
                    run.check()
                    outs[name] = torch.cat([run.work["h"].flatten(), run.work["pos"].flatten(), run.ldj_mol])
        _lib.set_latency_threshold(-1)
        _lib.set_coop_max(-1)
        for k, v in res.items():
            d = ""
            if outs.get(k) is not None and outs.get("4-wave") is not None:
                a, b = outs[k].double(), outs["4-wave"].double()
                d = f"  (h, pos, ldj) rel diff vs 4-wave {float((a - b).norm() / b.norm()):.2e}"
            print(f"{mols:5d} molecules {k}: median {statistics.median(v):.4f} ms  min {min(v):.4f} ms{d}", flush=True)


if __name__ == "__main__":
    main()
