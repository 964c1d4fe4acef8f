"""Where the training gradients' error comes from.

For the reference training goldens (tests/golden: train_h128_L2,
train_h64_L2, train_h32_L3) and the bench-shape batch (12 x 22 atoms, H =
128, 8 layers, the float64 gradient oracle as the reference), prints the
worst normwise gradient error per parameter tensor of

  oracle32  the float64 gradient oracle re-run in float32 arithmetic on the CPU
            (same edges): what fp32 rounding alone does to these gradients
  hip_f32   the HIP path with gemm_precision='f32' (exact fp32 MFMA chains,
            ENFLOW_BWD_F32 backward)
  hip_f16x3 the HIP path at its default precision (f16x3)

    python tools/grad_precision.py          (GPU box; --cpu: the oracle32 column only)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def _worst(errs):
    k = max(errs, key=errs.get)
    return {"worst": errs[k], "tensor": k}


def _golden_case(name):
    from _fixtures import load, layer_params, dequant_params, state, n_layers
    inp, ref = load(name)
    layers = [layer_params(inp, i) for i in range(n_layers(inp))]
    ref_g = {f"p{i}.{k}": ref[f"grad_p{i}.{k}"] for i in range(n_layers(inp)) for k in layers[i]
             if f"grad_p{i}.{k}" in ref}
    ref_g.update({f"dq.{k}": ref[f"grad_dq.{k}"] for k in dequant_params(inp) if f"grad_dq.{k}" in ref})
    return dict(inp=inp, layers=layers, dq=dequant_params(inp), state=state(inp), eps=inp["eps"].astype(np.float64),
                dt=float(inp["dt"]), kBT=float(inp["kBT"]), soft=float(inp["softening"]), ref=ref_g)


def _bench_case():
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    b = make_molecules(12, [22] * 12, nf=5, seed=77, radius=4.0)
    torch.manual_seed(5)
    model = LFIntegrator([EGCL(5, 5, 128) for _ in range(8)], ArgMax(5, 128), dt=default_dt())
    st = {k: np.asarray(b[k], dtype=np.float32).astype(np.float64) for k in ("h", "g", "pos", "vel", "box", "r_cut")}
    st["mol_ptr"] = b["mol_ptr"]
    layers = [{k: v.detach().double().numpy() for k, v in n.named_parameters()} for n in model.networks]
    dq = {k: v.detach().double().numpy() for k, v in model.dequantize.named_parameters()}
    eps = np.random.default_rng(3).normal(size=b["h"].shape).astype(np.float32).astype(np.float64)
    _, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, st, eps, default_dt(), default_kBT(), 0.1)
    ref = {f"p{i}.{k}": v for i, g in enumerate(gl) for k, v in g.items()}
    ref.update({f"dq.{k}": v for k, v in gd.items()})
    return dict(model=model, layers=layers, dq=dq, state=st, eps=eps, dt=default_dt(), kBT=default_kBT(), soft=0.1,
                ref=ref)


def oracle32(c):
    from oracle import enflow_oracle_grad as OG
    from _fixtures import normwise
    _, _, gl, gd, _ = OG.train_loss_and_grads(c["layers"], c["dq"], c["state"], c["eps"], c["dt"], c["kBT"], c["soft"],
                                              dtype=torch.float32)
    got = {f"p{i}.{k}": v for i, g in enumerate(gl) for k, v in g.items()}
    got.update({f"dq.{k}": v for k, v in gd.items()})
    return _worst({k: normwise(got[k], c["ref"][k]) for k in c["ref"] if k in got})


def hip(c, prec):
    from _fixtures import normwise, flow_from_fixture
    from enflow_amd.flow import Alchemical_NLL
    from enflow_amd.data import Data
    if "inp" in c:
        model, data = flow_from_fixture(c["inp"], "cuda")
    else:
        model = c["model"].cuda()
        st = c["state"]
        f = lambda k: torch.tensor(st[k], dtype=torch.float32, device="cuda")  # noqa: E731
        data = Data(h=f("h"), g=f("g"), pos=f("pos"), vel=f("vel"), N=torch.tensor(np.diff(st["mol_ptr"])),
                    r_cut=f("r_cut"), box=f("box"), device="cuda")
    model.gemm_precision = prec
    model.zero_grad(set_to_none=True)
    out, ldj = model(data, noise=torch.tensor(c["eps"], dtype=torch.float32, device="cuda"))
    Alchemical_NLL(kBT=c["kBT"], softening=c["soft"])(out, ldj).backward()
    torch.cuda.synchronize()
    got = {f"p{i}.{k}": p.grad.double().cpu().numpy() for i, n in enumerate(model.networks)
           for k, p in n.named_parameters()}
    got.update({f"dq.{k}": p.grad.double().cpu().numpy() for k, p in model.dequantize.named_parameters()})
    model.gemm_precision = "f16x3"
    return _worst({k: normwise(got[k], c["ref"][k]) for k in c["ref"] if k in got})


def main():
    cpu = "--cpu" in sys.argv
    cases = {n: (lambda n=n: _golden_case(n)) for n in ("train_h128_L2", "train_h64_L2", "train_h32_L3")}
    cases["bench_22x12_h128_L8"] = _bench_case
    out = {}
    for name, mk in cases.items():
        c = mk()
        row = {"oracle32": oracle32(c)}
        if not cpu:
            row["hip_f32"] = hip(c, "f32")
            row["hip_f16x3"] = hip(c, "f16x3")
        out[name] = row
        print(name, json.dumps(row), flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
