"""Debug: per-molecule outputs and pair counts of the split instance (fs2) vs 4-wave at 128 molecules."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch, bench
from enflow_amd import _lib
from enflow_amd.data.synthetic import make_molecules
from fs_check import set_instance
dev = torch.device("cuda", 0)
model = bench.build_model(dev, int(os.environ.get("NL", bench.LAYERS)))
g = make_molecules(1024, bench.ATOMS, nf=bench.NF, seed=1000)
inp = bench.batch_tensors(bench.sub_batch(g, 0, 128), dev)
res = {}
for inst in ("4w", "fs1", "fs2"):
    set_instance(inst)
    run = bench.FlowRunner(model, inp, bench.ATOMS, False, dev, torch.Generator(dev).manual_seed(0))
    stats = torch.zeros(2, dtype=torch.int64, device=dev)
    run.forward_once(stats)
    run.check()
    res[inst] = ({k: run.work[k].clone() for k in ("h", "g", "pos", "vel")}, stats.tolist())
ptr = inp["mol_ptr"].cpu().tolist()
for inst in ("fs1", "fs2"):
    o, st = res[inst]
    o4, st4 = res["4w"]
    bad = []
    for m in range(128):
        a0, a1 = ptr[m], ptr[m + 1]
        e = max(float((o[k][a0:a1] - o4[k][a0:a1]).abs().max()) for k in o)
        if e > 1e-4:
            bad.append((m, e))
    print(inst, "stats", st, "4w stats", st4, "bad molecules", len(bad), bad[:8])
