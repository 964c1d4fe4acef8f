"""GPU check of the fused flow's instances on the bench workload (BASELINE
configs[1] molecules, H = 128, 8 layers, f16x3): the 4-wave and 8-wave
whole-tile instances and the feature-split instance with two workgroups per
molecule (fs2) or one (fs1), at strong-scaling batch sizes.  Prints each
instance's outputs against the 4-wave instance (normwise relative) and its
step time.   python tools/fs_check.py [mols ...]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

INSTANCES = {"4w": (0, 0, 0), "8w": (1 << 30, 0, 0), "fs2": (0, 1 << 30, 0), "fs1": (0, 0, 1 << 30)}


def set_instance(name):
    from enflow_amd import _lib
    lat, split, fs = INSTANCES[name]
    _lib.set_latency_threshold(lat)
    _lib.set_split_threshold(split)
    _lib.set_fs_threshold(fs)


def rel(a, b):
    import torch
    return float(torch.linalg.norm((a - b).double()) / max(float(torch.linalg.norm(b.double())), 1e-30))


def main():
    import torch
    import bench
    from enflow_amd.data.synthetic import make_molecules
    mols_list = [int(x) for x in sys.argv[1:]] or [128, 256, 64, 16]
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    model.gemm_precision = "f16x3"
    g = make_molecules(1024, bench.ATOMS, nf=bench.NF, seed=1000)
    out = []
    for mols in mols_list:
        inp = bench.batch_tensors(bench.sub_batch(g, 0, mols), dev)
        for reverse in (False, True):
            res = {}
            for name in INSTANCES:
                if name == "fs2" and 2 * mols > torch.cuda.get_device_properties(0).multi_processor_count:
                    continue
                set_instance(name)
                run = bench.FlowRunner(model, inp, bench.ATOMS, reverse, dev, torch.Generator(dev).manual_seed(0))
                if reverse:   # the same source for every instance: the 4-wave forward's outputs
                    if "src" not in res:
                        res["src"] = {k: v.clone() for k, v in run.src.items()}
                    run.src = res["src"]
                run.step()
                run.check()
                outs = {k: run.work[k].clone() for k in ("h", "g", "pos", "vel")}
                if not reverse:
                    outs["ldj"] = run.ldj.clone()
                el = bench.timed(run.step, 40, 20, None, dev)
                run.check()
                res[name] = (outs, el / 40 * 1e3)
            base = res["4w"][0]
            for name, v in res.items():
                if name == "src":
                    continue
                outs, ms = v
                row = {"mols": mols, "dir": "reverse" if reverse else "forward", "instance": name,
                       "ms_per_step": round(ms, 4),
                       "rel_vs_4w": {k: rel(outs[k], base[k]) for k in outs}}
                out.append(row)
                print(json.dumps(row), flush=True)
    set_instance("4w")
    from enflow_amd import _lib
    _lib.set_latency_threshold(-1)
    _lib.set_split_threshold(-1)
    _lib.set_fs_threshold(-1)


if __name__ == "__main__":
    main()
