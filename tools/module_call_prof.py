"""Where the Python time of one inference module call goes: cProfile over
`model(data)` calls on the bench batch (1024 x 22, 8 layers, H = 128, f16x3)
under torch.no_grad(), top functions by own time.

    python tools/module_call_prof.py > profiles/rNN/module_call_prof.txt
"""
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    d = Data.from_arrays(make_molecules(bench.MOLS_PER_GPU, bench.ATOMS, nf=bench.NF, seed=1000), device=dev)
    with torch.no_grad():
        for _ in range(50):
            model(d._replace())
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(300):
            model(d._replace())
        pr.disable()
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(40)
    print(s.getvalue())
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("cumulative").print_stats(40)
    print(s.getvalue())


if __name__ == "__main__":
    main()
