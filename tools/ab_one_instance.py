"""One instance of the fused forward at one batch size (for a profiler run):
ENFLOW_AB_COOP=1 forces the cooperative build, 0 the 8-wave latency build.

    ENFLOW_AB_COOP=1 python tools/ab_one_instance.py 128
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import make_molecules
    dev = torch.device("cuda", 0)
    mols = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    model = bench.build_model(dev, bench.LAYERS)
    g = make_molecules(mols, bench.ATOMS, nf=bench.NF, seed=1000)
    run = bench.FlowRunner(model, bench.batch_tensors(g, dev), bench.ATOMS, False, dev,
                           torch.Generator(dev).manual_seed(0))
    _lib.set_latency_threshold(1 << 30)
    _lib.set_coop_max(1 << 30 if os.environ.get("ENFLOW_AB_COOP") == "1" else 0)
    el = bench.timed(run.step, 100, 50, None, dev)
    run.check()
    print(f"{mols} molecules coop={os.environ.get('ENFLOW_AB_COOP')}: {el / 100 * 1e3:.4f} ms per step")


if __name__ == "__main__":
    main()
