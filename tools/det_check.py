"""Training-step gradients across library copies / repeats in one process:
bitwise comparison per parameter (diagnostic)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import make_molecules, default_kBT, default_dt
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator, Alchemical_NLL
    from enflow_amd.data import Data
    dev = torch.device("cuda", 0)
    atoms = int(os.environ.get("AB_ATOMS", 64))
    mols = int(os.environ.get("AB_MOLS", 1024))
    b = make_molecules(mols, atoms, nf=5, seed=2000, radius=4.0 * (atoms / 22.0) ** (1.0 / 3.0))
    torch.manual_seed(0)
    nl = int(os.environ.get("AB_LAYERS", 8))
    model = LFIntegrator([EGCL(5, 5, 128) for _ in range(nl)], ArgMax(5, 128), dt=default_dt()).to(dev)
    nll = Alchemical_NLL(kBT=default_kBT(), softening=0.1)
    base = Data.from_arrays(b, device=dev)
    noise = torch.randn_like(base.h)
    names = [n for n, _ in model.named_parameters()] + ["input.pos", "input.vel"]

    def run(path):
        _lib._libs.clear()
        _lib.LIB_PATH = path
        for mod in model.modules():
            for attr in ("_packed_key", "_layers_key", "_train_key"):
                if hasattr(mod, attr):
                    setattr(mod, attr, None)
        model.zero_grad(set_to_none=True)
        d = base._replace()
        d.pos = d.pos.clone().requires_grad_(True)
        d.vel = d.vel.clone().requires_grad_(True)
        pos_in, vel_in = d.pos, d.vel
        out, ldj = model(d, noise=noise)
        loss = nll(out, ldj)
        loss.backward()
        torch.cuda.synchronize()
        _lib.check_pending()
        return float(loss), [p.grad.clone() for p in model.parameters()] + [pos_in.grad.clone(), vel_in.grad.clone()]

    runs = [(p, run(p)) for p in sys.argv[1:]]
    l0, g0 = runs[0][1]
    for p, (l, g) in runs:
        bad = [(n, float((a - b).norm() / (b.norm() + 1e-30))) for n, a, b in zip(names, g, g0) if not torch.equal(a, b)]
        bad.sort(key=lambda x: -x[1])
        print(os.path.basename(p), "loss", l, "==" if l == l0 else "!=", "params differing:", len(bad), bad[:5], flush=True)


if __name__ == "__main__":
    main()
