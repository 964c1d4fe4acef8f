"""Hidden widths past the compiled ones (the reference accepts any hidden_nf,
enflow/nn/egcl.py:11, enflow/nn/argmax.py:6): run zero-padded to the next of
32 / 64 / 128 (enflow_amd/nn/_pad.py, exact).  Outputs vs the float64 oracle
at 1e-5 normwise, gradients vs the gradient oracle at 1e-4 normwise (the bars
of tests/test_gpu_parity.py and tests/test_gpu_train.py); an ArgMax whose
hidden width differs from the EGCL layers' is padded to the flow's width."""
import numpy as np
import pytest
import torch

from oracle import enflow_oracle as O
from _fixtures import rel_err, normwise, worst_of, assert_all_within

# every test on both fused-kernel instances (conftest.kernel_instance: the
# 4-wave throughput build and the 8-wave latency build)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("kernel_instance")]
DEV = "cuda:0"


def _batch(sizes, seed):
    from enflow_amd.data.synthetic import make_molecules
    b = make_molecules(len(sizes), sizes, nf=5, seed=seed)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    return b


def _lp(net):
    p = {k: v.detach().double().cpu().numpy() for k, v in net.state_dict().items()}
    p["flags"] = (bool(net.attention), bool(net.norm_diff), bool(net.tanh))
    return p


@pytest.mark.parametrize("hid,variants", [(48, {}), (100, dict(attention=True, tanh=True)), (20, {})])
def test_egcl_padded_hidden_forward_and_grads(hid, variants):
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn import EGCL
    from enflow_amd.data import Data
    b = _batch([22, 9, 30], 71)
    b["h"] = np.random.default_rng(72).normal(size=b["h"].shape).astype(np.float32).astype(np.float64)
    torch.manual_seed(73)
    net = EGCL(5, 5, hid, **variants).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    d.h.requires_grad_(True)
    d.pos.requires_grad_(True)
    q, f, g = net(d.h, d.edges)
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    rq, rf, rg = O.egcl_forward(_lp(net), b["h"], row, col, O.coord_diff(b["pos"], row, col, eb))
    errs = {"Q": rel_err(q.detach().cpu().numpy(), rq), "F": rel_err(f.detach().cpu().numpy(), rf),
            "G": rel_err(g.detach().cpu().numpy(), rg)}
    rng = np.random.default_rng(74)
    n = b["h"].shape[0]
    wq, wf, wg = rng.normal(size=(n,)), rng.normal(size=(n, 3)), rng.normal(size=(n, 5))
    t32 = lambda a: torch.tensor(a, dtype=torch.float32, device=DEV)  # noqa: E731
    ((q.reshape(-1) * t32(wq)).sum() + (f * t32(wf)).sum() + (g * t32(wg)).sum()).backward()
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.float64))  # noqa: E731
    P = {k: t(v.detach().cpu().numpy()).requires_grad_(True) for k, v in net.named_parameters()}
    h64, p64 = t(b["h"]).requires_grad_(True), t(b["pos"]).requires_grad_(True)
    rq2, rf2, rg2 = OG._egcl(P, h64, p64, torch.as_tensor(row), torch.as_tensor(col), t(eb), n, 1.0,
                             _lp(net)["flags"])
    ((rq2.reshape(-1) * t(wq)).sum() + (rf2 * t(wf)).sum() + (rg2 * t(wg)).sum()).backward()
    gerr = {"h": normwise(d.h.grad.cpu().numpy(), h64.grad.numpy()),
            "pos": normwise(d.pos.grad.cpu().numpy(), p64.grad.numpy())}
    for k, p in net.named_parameters():
        assert p.grad.shape == p.shape
        gerr[k] = normwise(p.grad.cpu().numpy(), P[k].grad.numpy())
    print(f"EGCL hidden {hid}: outputs {worst_of(errs):.2e}, grads {worst_of(gerr):.2e}")
    assert_all_within(errs, 1e-5)
    assert_all_within(gerr, 1e-4)


def test_flow_padded_hidden_and_mismatched_argmax():
    """LFIntegrator with EGCL hidden 100 (kernel width 128) and ArgMax hidden 20:
    forward and reverse vs the oracle, one training step's gradients vs the
    gradient oracle."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator, Alchemical_NLL
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import default_dt
    b = _batch([22, 14, 40], 81)
    torch.manual_seed(82)
    model = LFIntegrator([EGCL(5, 5, 100) for _ in range(3)], ArgMax(5, 20), dt=default_dt()).to(DEV)
    eps = np.random.default_rng(83).normal(size=b["h"].shape).astype(np.float32)
    layers = [_lp(n) for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.state_dict().items()}
    with torch.no_grad():
        o, ldj = model(Data.from_arrays(b, device=DEV), noise=torch.tensor(eps, device=DEV))
    ref, ref_ldj = O.lf_forward(layers, dq, b, eps.astype(np.float64), model.dt)
    for k in ("h", "g", "pos", "vel"):
        assert rel_err(getattr(o, k).cpu().numpy(), ref[k]) < 1e-5, k
    assert abs(float(ldj) - ref_ldj) <= 1e-5 * abs(ref_ldj)
    model.zero_grad(set_to_none=True)
    o, ldj = model(Data.from_arrays(b, device=DEV), noise=torch.tensor(eps, device=DEV))
    loss = Alchemical_NLL(kBT=1.0, softening=0.1)(o, ldj)
    loss.backward()
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
    assert abs(float(loss) - rloss) <= 1e-5 * abs(rloss)
    errs = {f"p{i}.{k}": normwise(p.grad.cpu().numpy(), gl[i][k])
            for i, n in enumerate(model.networks) for k, p in n.named_parameters()}
    errs.update({f"dq.{k}": normwise(p.grad.cpu().numpy(), gd[k]) for k, p in model.dequantize.named_parameters()})
    print(f"flow hidden 100 / ArgMax 20: max normwise grad err {worst_of(errs):.2e}")
    assert_all_within(errs, 1e-4)


@pytest.mark.parametrize("fin,fout,hid", [(3, 5, 48), (6, 2, 64), (1, 8, 32)])
def test_egcl_input_output_widths(fin, fout, hid):
    """EGCL(input_nf != output_nf): run at the kernel width max(in, out) with
    zero-padded features; outputs and gradients (h, pos, every parameter) vs
    the float64 gradient oracle's EGCL, which takes any widths."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn import EGCL
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    b = make_molecules(3, [22, 9, 30], nf=fin, seed=91)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    b["h"] = np.random.default_rng(92).normal(size=b["h"].shape).astype(np.float32).astype(np.float64)
    torch.manual_seed(93)
    net = EGCL(fin, fout, hid).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    d.h.requires_grad_(True)
    d.pos.requires_grad_(True)
    q, f, g = net(d.h, d.edges)
    assert g.shape == (61, fout)
    n = 61
    rng = np.random.default_rng(94)
    wq, wf, wg = rng.normal(size=(n,)), rng.normal(size=(n, 3)), rng.normal(size=(n, fout))
    t32 = lambda a: torch.tensor(a, dtype=torch.float32, device=DEV)  # noqa: E731
    ((q.reshape(-1) * t32(wq)).sum() + (f * t32(wf)).sum() + (g * t32(wg)).sum()).backward()
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.float64))  # noqa: E731
    P = {k: t(v.detach().cpu().numpy()).requires_grad_(True) for k, v in net.named_parameters()}
    h64, p64 = t(b["h"]).requires_grad_(True), t(b["pos"]).requires_grad_(True)
    rq, rf, rg = OG._egcl(P, h64, p64, torch.as_tensor(row), torch.as_tensor(col), t(eb), n, 1.0)
    errs = {"Q": normwise(q.detach().cpu().numpy().reshape(-1), rq.detach().numpy().reshape(-1)),
            "F": normwise(f.detach().cpu().numpy(), rf.detach().numpy()),
            "G": normwise(g.detach().cpu().numpy(), rg.detach().numpy())}
    ((rq.reshape(-1) * t(wq)).sum() + (rf * t(wf)).sum() + (rg * t(wg)).sum()).backward()
    gerr = {"h": normwise(d.h.grad.cpu().numpy(), h64.grad.numpy()),
            "pos": normwise(d.pos.grad.cpu().numpy(), p64.grad.numpy())}
    for k, p in net.named_parameters():
        gerr[k] = normwise(p.grad.cpu().numpy(), P[k].grad.numpy())
    print(f"EGCL({fin}, {fout}, {hid}): outputs {worst_of(errs):.2e}, grads {worst_of(gerr):.2e}")
    assert_all_within(errs, 1e-5)
    assert_all_within(gerr, 1e-4)


def test_flow_training_node_nf_8():
    """node_nf = 8 (the compiled maximum): edge_nn.0's input [h_i, h_j, radial]
    is 17 wide, past the backward's 16-wide input rows (they widen to 32);
    training gradients vs the gradient oracle."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator, Alchemical_NLL
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules, default_dt
    b = make_molecules(3, [22, 14, 40], nf=8, seed=101)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    torch.manual_seed(102)
    model = LFIntegrator([EGCL(8, 8, 64) for _ in range(2)], ArgMax(8, 64), dt=default_dt()).to(DEV)
    eps = np.random.default_rng(103).normal(size=b["h"].shape).astype(np.float32)
    layers = [_lp(n) for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.state_dict().items()}
    model.zero_grad(set_to_none=True)
    o, ldj = model(Data.from_arrays(b, device=DEV), noise=torch.tensor(eps, device=DEV))
    loss = Alchemical_NLL(kBT=1.0, softening=0.1)(o, ldj)
    loss.backward()
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
    assert abs(float(loss) - rloss) <= 1e-5 * abs(rloss)
    errs = {f"p{i}.{k}": normwise(p.grad.cpu().numpy(), gl[i][k])
            for i, n in enumerate(model.networks) for k, p in n.named_parameters()}
    errs.update({f"dq.{k}": normwise(p.grad.cpu().numpy(), gd[k]) for k, p in model.dequantize.named_parameters()})
    print(f"flow nf 8: max normwise grad err {worst_of(errs):.2e}")
    assert_all_within(errs, 1e-4)
