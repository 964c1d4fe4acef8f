"""Per-rank time of the forward under strong scaling, measured on one GPU:
the 1024-molecule batch of BASELINE configs[1] split N ways is, on each rank,
a 1024/N-molecule forward with no data-path collective, so its step time IS
the N-rank strong-scaling time (max over ranks = the slowest shard).

Rows per rank count: the instance the library picks ("auto": the
feature-split instance with two workgroups per molecule for batches of at
most CUs/2 molecules, with one up to CUs; the 8-wave instance up to
enflow_latency_threshold(); else the 4-wave one) and each instance forced.

    python tools/strong_scaling_probe.py > profiles/r05/strong_scaling_probe.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    import torch
    import bench
    from enflow_amd.data.synthetic import make_molecules
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev, bench.LAYERS)
    model.gemm_precision = "f16x3"
    g = make_molecules(1024, bench.ATOMS, nf=bench.NF, seed=1000)
    out = {"workload": bench.workload_name("forward"), "rows": []}
    from enflow_amd import _lib
    from fs_check import set_instance
    L = _lib.lib()
    out["latency_threshold_auto"] = L.enflow_latency_threshold()
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out["split_threshold_auto"] = cus // 2
    t1 = None
    for n in (1, 2, 4, 8):
        m1 = 1024 // n
        auto = ("fs2" if m1 <= cus // 2 else "fs1" if m1 <= cus else
                "8w" if m1 <= out["latency_threshold_auto"] else "4w")
        for mode in ("auto", "4w", "8w", "fs2", "fs1"):
            if (mode == "fs2" and m1 > cus // 2) or (mode == "fs1" and m1 > cus):
                continue
            if mode == "auto":
                _lib.set_latency_threshold(-1)
                _lib.set_split_threshold(-1)
                _lib.set_fs_threshold(-1)
            else:
                set_instance(mode)
            run = bench.FlowRunner(model, bench.batch_tensors(bench.sub_batch(g, 0, m1), dev), bench.ATOMS, False,
                                   dev, torch.Generator(dev).manual_seed(0))
            el = bench.timed(run.step, 40, 30, None, dev)
            run.check()
            ms = el / 40 * 1e3
            if n == 1 and mode == "auto":
                t1 = ms
            out["rows"].append({"ranks": n, "kernel": mode, "auto_instance": auto, "molecules_per_rank": m1,
                                "ms_per_step": ms, "global_molecule_transforms_per_s": 1024 / (ms * 1e-3),
                                "strong_scaling_efficiency": t1 / (n * ms)})
            print(json.dumps(out["rows"][-1]), file=sys.stderr, flush=True)
    _lib.set_latency_threshold(-1)
    _lib.set_split_threshold(-1)
    _lib.set_fs_threshold(-1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
