"""GPU parity for node_nf past 8: the 16-feature build (libenflow_hip_nf16.so,
the same sources with ENFLOW_NFMAX=16).  The reference takes node_nf from the
dataset (enflow/main.py:148-151: EGCL(node_nf, node_nf, hidden_nf),
ArgMax(node_nf, ...)), so any width is legal there.

Goldens from the reference itself (tests/golden/make_golden.py wide_nf):
flows at node_nf 12 / 16, an EGCL at 16, training steps at 12 / 15 / 16; the
large-system kernels (molecules past the fused image, and training past 64
atoms) against the CPU oracles.  Tolerances as tests/test_gpu_parity.py /
tests/test_gpu_train.py: outputs 1e-5 (max-abs relative per tensor),
gradients 1e-4 normwise per parameter tensor."""
import numpy as np
import pytest
import torch

from oracle import enflow_oracle as O
from _fixtures import (load, flow_from_fixture, data_from_fixture, egcl_from_fixture, layer_params, state, n_layers,
                       rel_err, normwise, worst_of, assert_all_within)

# every test on both fused-kernel instances (conftest.kernel_instance: the
# 4-wave throughput build and the 8-wave latency build)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("kernel_instance")]
TOL = 1e-5
GRAD_TOL = 5e-5   # <= 2x the fp32 floor measured on these batches (tools/grad_precision.py, profiles/r05)
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def fmt(errs):
    return "{" + ", ".join(f"{k}: {v:.2e}" for k, v in errs.items()) + "}"


def test_wide_features_load_the_16_feature_library():
    import os
    from enflow_amd import _lib
    L = _lib.lib(12)
    assert L.enflow_max_node_nf() == 16
    assert _lib.lib_path(12).endswith("libenflow_hip_nf16.so") and os.path.exists(_lib.lib_path(12))
    assert _lib.lib(5).enflow_max_node_nf() == 8
    with pytest.raises(NotImplementedError):
        _lib.lib_path(17)


@pytest.mark.parametrize("prec", ["f32", "f16x3"])
@pytest.mark.parametrize("name", ["lf_nf12_h64_L2", "lf_nf16_h32_L2"])
def test_wide_flow_forward_and_reverse_match_reference(name, prec):
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
    # reverse of the reference's forward output (generate direction)
    d2 = data_from_fixture(inp, DEV)
    for k in ("h", "g", "pos", "vel"):
        setattr(d2, k, torch.tensor(out[k], dtype=torch.float32, device=DEV))
    with torch.no_grad():
        back = model.reverse(d2)
    np.testing.assert_array_equal(back.h.cpu().numpy(), out["rev_h"])
    gold = {k: rel_err(getattr(back, k).cpu().numpy(), out["rev_" + k]) for k in ("g", "pos", "vel")}
    print(f"{name} {prec} reverse vs golden:", fmt(gold))
    assert_all_within(gold, TOL)


def test_wide_egcl_matches_reference():
    from enflow_amd.data import Data  # noqa: F401
    inp, out = load("egcl_nf16_h128")
    nf, hid = inp["h"].shape[1], int(inp["p0.edge_nn.2.weight"].shape[0])
    net = egcl_from_fixture(inp, 0, nf, hid).to(DEV)
    d = data_from_fixture(inp, DEV)
    with torch.no_grad():
        q, f, g = net(d.h, d.edges)
    errs = {"Q": rel_err(q.cpu().numpy(), out["Q"]), "F": rel_err(f.cpu().numpy(), out["F"]),
            "G": rel_err(g.cpu().numpy(), out["G"])}
    print("egcl_nf16_h128 vs reference golden:", fmt(errs))
    assert_all_within(errs, TOL)


@pytest.mark.parametrize("name", ["train_nf12_h32_L2", "train_nf15_h128_L2", "train_nf16_h64_L2"])
def test_wide_training_gradients_match_reference(name):
    """node_nf 12 / 15 / 16 training steps vs the reference's loss.backward()
    (nf 16: 2 nf + 1 = 33 edge_nn.0 inputs; the backward's radial row lies past
    the transposed GEMM's 32-row tile and is its own dot product)."""
    from enflow_amd.flow import Alchemical_NLL
    inp, ref = load(name)
    model, data = flow_from_fixture(inp, DEV)
    model.zero_grad(set_to_none=True)
    out, ldj = model(data, noise=torch.tensor(inp["eps"], device=DEV))
    loss = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))(out, ldj)
    loss.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - ref["loss"]) <= 1e-5 * abs(ref["loss"]), (float(loss), ref["loss"])
    errs = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            errs[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_p{i}.{k}"])
    for k, p in model.dequantize.named_parameters():
        errs[f"dq.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_dq.{k}"])
    print(name, "max normwise grad err", f"{worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)


def test_node_nf_16_standalone_egcl_backward_vs_oracle():
    """EGCL(16, 16, 128) alone with autograd (the one-layer tape and backward of
    the 16-feature library) vs the float64 gradient oracle's EGCL."""
    import torch
    from oracle import enflow_oracle_grad as OG
    inp, _ = load("egcl_nf16_h128")
    nf, hid = 16, 128
    net = egcl_from_fixture(inp, 0, nf, hid).to(DEV)
    d = data_from_fixture(inp, DEV)
    h = d.h.clone().requires_grad_(True)
    q, f, g = net(h, d.edges)
    (q.sum() + (f * f).sum() + (g * g).sum()).backward()
    p = {k: v.detach().double().cpu().requires_grad_(True) for k, v in net.named_parameters()}
    ht = torch.tensor(inp["h"], dtype=torch.float64, requires_grad=True)
    row, col, eb = O.batch_edges(inp["pos"].astype(np.float64), inp["box"].astype(np.float64),
                                 inp["r_cut"].astype(np.float64), inp["mol_ptr"])
    pos = torch.tensor(inp["pos"], dtype=torch.float64)
    qq, ff, gg = OG._egcl(p, ht, pos, torch.as_tensor(row), torch.as_tensor(col), torch.tensor(eb),
                          int(inp["mol_ptr"][-1]), 1.0)
    (qq.sum() + (ff * ff).sum() + (gg * gg).sum()).backward()
    errs = {k: normwise(v.grad.cpu().numpy(), p[k].grad.numpy()) for k, v in net.named_parameters()}
    errs["h"] = normwise(h.grad.cpu().numpy(), ht.grad.numpy())
    print("egcl nf16 backward vs gradient oracle:", f"{worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)


def _chains(sizes, seed, nf):
    from enflow_amd.data.synthetic import make_molecules
    b = make_molecules(len(sizes), sizes, nf=nf, seed=seed, chain=True)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    return b


def _model(hid, nf, n_layers, seed):
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data.synthetic import default_dt
    torch.manual_seed(seed)
    return LFIntegrator([EGCL(nf, nf, hid) for _ in range(n_layers)], ArgMax(nf, hid), dt=default_dt()).to(DEV)


@pytest.mark.parametrize("prec", ["f32", "f16x3"])
def test_wide_large_system_forward_vs_oracle(prec):
    """node_nf 12 on molecules past the fused LDS image (300 atoms: the
    layer-by-layer kernels) and the row-blocked fused instance (100 atoms)."""
    from enflow_amd.data import Data
    b = _chains([300, 100], 21, 12)
    model = _model(64, 12, 2, 22)
    model.gemm_precision = prec
    noise = torch.randn(b["h"].shape, device=DEV, generator=torch.Generator(DEV).manual_seed(23))
    with torch.no_grad():
        o, ldj = model(Data.from_arrays(b, device=DEV), noise=noise)
    layers = [{k: v.detach().cpu().double().numpy() for k, v in n.state_dict().items()} for n in model.networks]
    dq = {k: v.detach().cpu().double().numpy() for k, v in model.dequantize.state_dict().items()}
    ref, ref_ldj = O.lf_forward(layers, dq, b, noise.cpu().double().numpy(), model.dt)
    errs = {k: rel_err(getattr(o, k).cpu().numpy(), ref[k]) for k in ("h", "g", "pos", "vel")}
    errs["ldj"] = abs(float(ldj) - ref_ldj) / abs(ref_ldj)
    print(f"node_nf 12, 300 + 100 atoms, {prec}:", fmt(errs))
    assert_all_within(errs, TOL)


def test_wide_training_past_64_atoms_vs_oracle():
    """node_nf 12 through the large-system tape and backward ([90, 22] atoms)."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.data import Data
    from enflow_amd.flow import Alchemical_NLL
    b = _chains([90, 22], 24, 12)
    model = _model(32, 12, 2, 25)
    eps = np.random.default_rng(26).normal(size=b["h"].shape).astype(np.float32)
    model.zero_grad(set_to_none=True)
    o, ldj = model(Data.from_arrays(b, device=DEV), noise=torch.tensor(eps, device=DEV))
    loss = Alchemical_NLL(kBT=1.0, softening=0.1)(o, ldj)
    loss.backward()
    layers = [{k: v.detach().double().cpu().numpy() for k, v in n.named_parameters()} for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
    assert abs(float(loss) - rloss) <= 1e-5 * abs(rloss)
    errs = {f"p{i}.{k}": normwise(p.grad.cpu().double().numpy(), gl[i][k])
            for i, n in enumerate(model.networks) for k, p in n.named_parameters()}
    errs.update({f"dq.{k}": normwise(p.grad.cpu().double().numpy(), gd[k])
                 for k, p in model.dequantize.named_parameters()})
    print("node_nf 12, 90 + 22 atoms training: max normwise grad err", f"{worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)
