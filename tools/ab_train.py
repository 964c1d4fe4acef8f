"""A/B several builds of libenflow_hip.so on the training step (bench.py
--mode train workload), interleaved rounds in ONE process; per lib the median
step time and the backward kernels' share (events around loss.backward()).

    python tools/ab_train.py path/to/libA.so path/to/libB.so ...
    python tools/ab_train.py lib.so lib.so@ENFLOW_SERIAL_BWD=1   # same build, a runtime knob set
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
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator, Alchemical_NLL
    from enflow_amd.data import Data
    libs = sys.argv[1:]
    dev = torch.device("cuda", 0)
    atoms = int(os.environ.get("AB_ATOMS", bench.TRAIN_ATOMS))
    radius = 4.0 * (atoms / 22.0) ** (1.0 / 3.0)
    b = make_molecules(bench.MOLS_PER_GPU, atoms, nf=bench.NF, seed=2000, radius=radius)
    torch.manual_seed(0)
    model = LFIntegrator([EGCL(bench.NF, bench.NF, bench.HID) for _ in range(bench.LAYERS)],
                         ArgMax(bench.NF, bench.HID), dt=default_dt()).to(dev)
    nll = Alchemical_NLL(kBT=default_kBT(), softening=0.1)
    base = Data.from_arrays(b, device=dev)
    noise = torch.randn_like(base.h)
    grads = {}

    def run(spec, reps):
        path, _, env = spec.partition("@")
        for kv in [e for e in env.split(",") if e]:
            k, _, v = kv.partition("=")
            os.environ[k] = v
        try:
            return _run(spec, path, reps)
        finally:
            for kv in [e for e in env.split(",") if e]:
                os.environ.pop(kv.partition("=")[0], None)

    def _run(spec, path, reps):
        if _lib.LIB_PATH != path or not _lib._libs:
            _lib._libs.clear()
            _lib.LIB_PATH = path
        for mod in model.modules():
            for attr in ("_packed_key", "_layers_key", "_train_key"):
                if hasattr(mod, attr):
                    setattr(mod, attr, None)
        ts = []
        for _ in range(reps):
            model.zero_grad(set_to_none=True)
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
            out, ldj = model(base._replace(), noise=noise)
            loss = nll(out, ldj)
            e1.record()
            loss.backward()
            e2.record()
            torch.cuda.synchronize()
            ts.append((e0.elapsed_time(e1), e1.elapsed_time(e2)))
        grads[spec] = [p.grad.clone() for p in model.parameters()]
        return ts

    res = {p: [] for p in libs}
    for p in libs:
        run(p, 2)
    for rnd in range(4):
        for p in libs:
            res[p] += run(p, 3)
    g0 = grads[libs[0]]
    for p in libs:
        fw = statistics.median(t[0] for t in res[p])
        bw = statistics.median(t[1] for t in res[p])
        rel = max(float((a - b).norm() / (b.norm() + 1e-30)) for a, b in zip(grads[p], g0))
        print(f"{os.path.basename(p):40s} fwd+nll {fw:7.3f} ms  backward {bw:7.3f} ms  "
              f"max grad rel diff vs first {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
