"""GPU parity for act_fn other than SiLU (enflow/nn/egcl.py:11 and
enflow/nn/argmax.py:7 take the activation module as a constructor argument).

Goldens from the reference itself (tests/golden/make_golden.py act): one EGCL
forward per supported activation (ReLU, LeakyReLU, ELU, CELU, SELU, GELU erf /
tanh, Tanh, Sigmoid, Softplus, Mish, ReLU6, Identity), two flows (Tanh / GELU
layers with a Tanh / Sigmoid ArgMax), two training steps (Tanh; ELU layers with
attention / norm_diff / tanh flags and a Softplus ArgMax); the standalone
modules' backward against the gradient oracle.  Tolerances as
tests/test_gpu_parity.py / test_gpu_train.py."""
import numpy as np
import pytest
import torch

from oracle import enflow_oracle_grad as OG
from _fixtures import (load, flow_from_fixture, data_from_fixture, egcl_from_fixture, act_module, rel_err, normwise,
                       worst_of, assert_all_within)

# every test on both fused-kernel instances (conftest.kernel_instance: the
# 4-wave throughput build and the 8-wave latency build)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("kernel_instance")]
TOL = 1e-5
GRAD_TOL = 5e-5   # <= 2x the fp32 floor measured on these batches (tools/grad_precision.py, profiles/r05)
DEV = "cuda:0"
ACTS = ["relu", "leaky", "elu", "celu", "selu", "gelu", "gelutanh", "tanh", "sigmoid", "softplus", "mish",
        "relu6", "identity"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def fmt(errs):
    return "{" + ", ".join(f"{k}: {v:.2e}" for k, v in errs.items()) + "}"


@pytest.mark.parametrize("act", ACTS)
def test_egcl_activation_matches_reference(act):
    inp, out = load(f"egcl_act_{act}")
    nf, hid = inp["h"].shape[1], int(inp["p0.edge_nn.2.weight"].shape[0])
    net = egcl_from_fixture(inp, 0, nf, hid).to(DEV)
    assert net.variant_flags() & 8   # ENFLOW_EGCL_ACT: the variant-capable kernels run
    d = data_from_fixture(inp, DEV)
    with torch.no_grad():
        q, f, g = net(d.h, d.edges)
    errs = {"Q": rel_err(q.cpu().numpy(), out["Q"]), "F": rel_err(f.cpu().numpy(), out["F"]),
            "G": rel_err(g.cpu().numpy(), out["G"])}
    print(f"egcl act={act} vs reference golden:", fmt(errs))
    assert_all_within(errs, TOL)


@pytest.mark.parametrize("prec", ["f32", "f16x3"])
@pytest.mark.parametrize("name", ["lf_act_tanh_h64_L2", "lf_act_gelu_h128_L2"])
def test_flow_activation_forward_and_reverse(name, prec):
    from enflow_amd.flow import Alchemical_NLL
    inp, out = load(name)
    model, d = flow_from_fixture(inp, DEV)
    model.gemm_precision = prec
    with torch.no_grad():
        o, ldj = model(d, noise=torch.tensor(inp["eps"], device=DEV))
    errs = {k: rel_err(getattr(o, k).cpu().numpy(), out[k]) for k in ("h", "g", "pos", "vel")}
    errs["ldj"] = abs(float(ldj) - float(out["ldj"])) / abs(float(out["ldj"]))
    nll = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))(o, ldj)
    errs["nll"] = abs(float(nll) - float(out["nll"])) / abs(float(out["nll"]))
    print(f"{name} {prec} forward vs reference golden:", fmt(errs))
    assert_all_within(errs, TOL)
    d2 = data_from_fixture(inp, DEV)
    for k in ("h", "g", "pos", "vel"):
        setattr(d2, k, torch.tensor(out[k], dtype=torch.float32, device=DEV))
    with torch.no_grad():
        back = model.reverse(d2)
    np.testing.assert_array_equal(back.h.cpu().numpy(), out["rev_h"])
    gold = {k: rel_err(getattr(back, k).cpu().numpy(), out["rev_" + k]) for k in ("g", "pos", "vel")}
    print(f"{name} {prec} reverse vs golden:", fmt(gold))
    assert_all_within(gold, TOL)


@pytest.mark.parametrize("name", ["train_act_tanh_h32_L2", "train_act_elu_h64_L2"])
def test_training_with_activation_matches_reference(name):
    from enflow_amd.flow import Alchemical_NLL
    inp, ref = load(name)
    model, data = flow_from_fixture(inp, DEV)
    model.zero_grad(set_to_none=True)
    out, ldj = model(data, noise=torch.tensor(inp["eps"], device=DEV))
    loss = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))(out, ldj)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss.detach()) - ref["loss"]) <= 1e-5 * abs(ref["loss"]), (float(loss.detach()), ref["loss"])
    errs = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            errs[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_p{i}.{k}"])
    for k, p in model.dequantize.named_parameters():
        errs[f"dq.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_dq.{k}"])
    print(name, "max normwise grad err", f"{worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)


@pytest.mark.parametrize("act", ["gelu", "softplus", "leaky", "mish"])
def test_standalone_modules_backward_with_activation(act):
    """EGCL.forward and ArgMax.forward trained directly with a non-SiLU act_fn:
    every parameter gradient (and d h / d pos) vs the float64 autograd oracle."""
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    from oracle import enflow_oracle as O
    code = {"gelu": (6, 0, 0), "softplus": (10, 1.5, 20.0), "leaky": (2, 0.05, 0), "mish": (11, 0, 0)}[act]
    b = make_molecules(3, [22, 9, 15], nf=5, seed=40)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    torch.manual_seed(41)
    net = EGCL(5, 5, 64, act_fn=act_module(code)).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    h = d.h.clone().requires_grad_(True)
    pos = d.pos.clone().requires_grad_(True)
    d.pos = pos
    rng = np.random.default_rng(42)
    n = h.shape[0]
    wq, wf, wg = (torch.tensor(rng.normal(size=s), dtype=torch.float32, device=DEV) for s in ((n, 1), (n, 3), (n, 5)))
    q, f, g = net(h, d.edges)
    ((q * wq).sum() + (f * wf).sum() + (g * wg).sum()).backward()
    P = {k: torch.tensor(v.detach().cpu().double().numpy(), requires_grad=True) for k, v in net.named_parameters()}
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.float64))  # noqa: E731
    h64, p64 = t(b["h"]).requires_grad_(True), t(b["pos"]).requires_grad_(True)
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    rq, rf, rg = OG._egcl(P, h64, p64, torch.as_tensor(row), torch.as_tensor(col), t(eb), n, 1.0, act=code)
    ((rq * t(wq.cpu())).sum() + (rf * t(wf.cpu())).sum() + (rg * t(wg.cpu())).sum()).backward()
    errs = {k: normwise(p.grad.cpu().double().numpy(), P[k].grad.numpy()) for k, p in net.named_parameters()}
    errs["h"] = normwise(h.grad.cpu().double().numpy(), h64.grad.numpy())
    errs["pos"] = normwise(pos.grad.cpu().double().numpy(), p64.grad.numpy())
    # ArgMax with the same activation
    torch.manual_seed(43)
    am = ArgMax(5, 32, act_fn=act_module(code)).to(DEV)
    hh = torch.tensor(b["h"], dtype=torch.float32, device=DEV)
    eps = torch.randn(hh.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(44))
    z, lq = am(hh, noise=eps)
    wz = torch.tensor(rng.normal(size=tuple(hh.shape)), dtype=torch.float32, device=DEV)
    ((z * wz).sum() + 0.7 * lq).backward()
    D = {k: torch.tensor(v.detach().cpu().double().numpy(), requires_grad=True) for k, v in am.named_parameters()}
    rz, rlq = OG._argmax(D, t(b["h"]), t(eps.cpu()), code)
    ((rz * t(wz.cpu())).sum() + 0.7 * rlq).backward()
    errs.update({f"dq.{k}": normwise(p.grad.cpu().double().numpy(), D[k].grad.numpy())
                 for k, p in am.named_parameters()})
    print(f"standalone EGCL / ArgMax backward act={act}: max normwise err {worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)
