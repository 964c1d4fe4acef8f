"""Standalone module autograd: EGCL.forward and ArgMax.forward are ordinary
autograd modules in the reference (/root/reference/enflow/nn/egcl.py:76-92,
/root/reference/enflow/nn/argmax.py:13-25).  Here their backward is the HIP
layer backward in EGCL mode (enflow_egcl_backward_f32) and the ArgMax
backward (enflow_argmax_backward_f32).  Gradients of every parameter (and of h
and the positions for EGCL) against the reference's own loss.backward()
(tests/golden/make_golden.py module_grads), GRAD_TOL normwise as the flow's
training tests."""
import numpy as np
import pytest
import torch

from _fixtures import load, egcl_from_fixture, data_from_fixture, ARGMAX_KEYS, normwise, worst_of, assert_all_within

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
GRAD_TOL = 5e-5   # <= 2x the fp32 floor measured on these batches (tools/grad_precision.py, profiles/r05)
LOSS_TOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("name", ["egcl_grad_h32", "egcl_grad_h128", "egcl_grad_h64_all"])
def test_egcl_backward_matches_reference(name):
    inp, ref = load(name)
    hid = int(inp["p0.edge_nn.2.weight"].shape[0])
    net = egcl_from_fixture(inp, 0, 5, hid).to(DEV)
    d = data_from_fixture(inp, DEV)
    d.h.requires_grad_(True)
    d.pos.requires_grad_(True)
    q, f, g = net(d.h, d.edges)
    t = lambda k: torch.tensor(inp[k], dtype=torch.float32, device=DEV)  # noqa: E731
    loss = (q * t("wq")).sum() + (f * t("wf")).sum() + (g * t("wg")).sum()
    loss.backward()
    assert abs(float(loss) - float(ref["loss"])) <= LOSS_TOL * abs(float(ref["loss"])) + 1e-6
    errs = {"h": normwise(d.h.grad.cpu().numpy(), ref["grad_h"]),
            "pos": normwise(d.pos.grad.cpu().numpy(), ref["grad_pos"])}
    for k, p in net.named_parameters():
        errs[k] = normwise(p.grad.cpu().numpy(), ref[f"grad_p0.{k}"])
    print(name, "max normwise grad err", f"{worst_of(errs):.2e}",
          {k: f"{v:.1e}" for k, v in errs.items() if v > 1e-6})
    assert_all_within(errs, GRAD_TOL)


def test_egcl_outputs_unchanged_by_autograd_path():
    """The grad-enabled forward returns the inference kernels' outputs exactly."""
    inp, _ = load("egcl_grad_h32")
    net = egcl_from_fixture(inp, 0, 5, 32).to(DEV)
    d = data_from_fixture(inp, DEV)
    q1, f1, g1 = net(d.h, d.edges)
    with torch.no_grad():
        q0, f0, g0 = net(d.h, d.edges)
    assert q1.requires_grad and torch.equal(q1.detach(), q0) and torch.equal(f1.detach(), f0)
    assert torch.equal(g1.detach(), g0)


def test_argmax_backward_matches_reference():
    from enflow_amd.nn import ArgMax
    inp, ref = load("argmax_grad_h32")
    am = ArgMax(5, 32)
    am.load_state_dict({k: torch.tensor(inp["dq." + k]) for k in ARGMAX_KEYS})
    am = am.to(DEV)
    h = torch.tensor(inp["h"], device=DEV)
    z, lq = am(h, noise=torch.tensor(inp["eps"], device=DEV), N=np.diff(inp["mol_ptr"]))
    loss = (z * torch.tensor(inp["wz"], device=DEV)).sum() + 0.7 * lq
    loss.backward()
    assert abs(float(loss) - float(ref["loss"])) <= LOSS_TOL * abs(float(ref["loss"]))
    errs = {k: normwise(p.grad.cpu().numpy(), ref[f"grad_dq.{k}"]) for k, p in am.named_parameters()}
    print("argmax max normwise grad err", f"{worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)


def test_egcl_training_loop_reduces_loss():
    """The reference's optimiser loop on a standalone EGCL: Adam steps lower a
    fixed quadratic loss of its outputs."""
    inp, _ = load("egcl_grad_h32")
    net = egcl_from_fixture(inp, 0, 5, 32).to(DEV)
    d = data_from_fixture(inp, DEV)
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    losses = []
    for _ in range(5):
        opt.zero_grad()
        q, f, g = net(d.h, d.edges)
        loss = (q ** 2).mean() + (g ** 2).mean()
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0], losses


@pytest.mark.parametrize("hid,variants", [(128, {}), (64, dict(attention=True, norm_diff=True, tanh=True))])
def test_egcl_backward_large_box_vs_oracle(hid, variants):
    """EGCL.forward on a 300-atom periodic box (past the fused backward's
    64-atom image: enflow_egcl_backward_large_f32) -- gradients of h, pos and
    every parameter vs the float64 gradient oracle's EGCL (pinned to the
    reference's loss.backward() goldens), 1e-4 normwise."""
    from oracle import enflow_oracle as O
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn import EGCL
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_lj_systems
    b = make_lj_systems([300], nf=5, seed=61)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    torch.manual_seed(62)
    net = EGCL(5, 5, hid, **variants).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    d.h.requires_grad_(True)
    d.pos.requires_grad_(True)
    q, f, g = net(d.h, d.edges)
    rng = np.random.default_rng(63)
    wq, wf, wg = rng.normal(size=(300,)), rng.normal(size=(300, 3)), rng.normal(size=(300, 5))
    t32 = lambda a: torch.tensor(a, dtype=torch.float32, device=DEV)  # noqa: E731
    loss = (q.reshape(-1) * t32(wq)).sum() + (f * t32(wf)).sum() + (g * t32(wg)).sum()
    loss.backward()
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.float64))  # noqa: E731
    P = {k: t(v.detach().cpu().numpy()).requires_grad_(True) for k, v in net.named_parameters()}
    h64, pos64 = t(b["h"]).requires_grad_(True), t(b["pos"]).requires_grad_(True)
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    rq, rf, rg = OG._egcl(P, h64, pos64, torch.as_tensor(row), torch.as_tensor(col), t(eb), 300,
                          float(net.coords_weight), (bool(net.attention), bool(net.norm_diff), bool(net.tanh)))
    rloss = (rq.reshape(-1) * t(wq)).sum() + (rf * t(wf)).sum() + (rg * t(wg)).sum()
    rloss.backward()
    assert abs(float(loss) - float(rloss)) <= LOSS_TOL * abs(float(rloss)) + 1e-6
    errs = {"h": normwise(d.h.grad.cpu().numpy(), h64.grad.numpy()),
            "pos": normwise(d.pos.grad.cpu().numpy(), pos64.grad.numpy())}
    for k, p in net.named_parameters():
        errs[k] = normwise(p.grad.cpu().numpy(), P[k].grad.numpy())
    print(f"EGCL 300-atom box H={hid} {sorted(variants)}: max normwise grad err {worst_of(errs):.2e}")
    assert_all_within(errs, GRAD_TOL)
