"""GPU parity for nn.PReLU as act_fn (enflow/nn/egcl.py:11 and
enflow/nn/argmax.py:7 take any activation module; PReLU is the parameterised
one torch ships with a default of one slope).

PReLU(a)(x) = max(0, x) + a * min(0, x) is LeakyReLU(a)(x) for every a, so the
kernels run it as ENFLOW_ACT_LEAKY_RELU with the module's slope (nn/_act.py).
Parity: the EGCL forward against the reference's own LeakyReLU golden
(egcl_act_leaky, tests/golden/make_golden.py act) with the slope set to the
golden's; flows, reverse and a training step bitwise equal to the same model
built with LeakyReLU (whose path the act goldens and the gradient oracle pin,
tests/test_gpu_act.py); a slope changed by an in-place update re-packs; a
trainable slope is refused on the differentiable paths."""
import numpy as np
import pytest
import torch
from torch import nn

from _fixtures import (load, data_from_fixture, layer_flags, rel_err, assert_all_within, EGCL_KEYS, ATT_KEYS,
                       ARGMAX_KEYS)

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("kernel_instance")]
TOL = 1e-5
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _flow(inp, act, dq_act):
    """LFIntegrator with the fixture's weights; act / dq_act: module factories."""
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    hid, nf, nl = int(inp["hid"]), inp["h"].shape[1], int(inp["n_layers"])
    nets = []
    for i in range(nl):
        att, nd, th = layer_flags(inp, i)
        net = EGCL(nf, nf, hid, attention=att, norm_diff=nd, tanh=th, act_fn=act())
        keys = EGCL_KEYS + (ATT_KEYS if att else ())
        net.load_state_dict({k: torch.tensor(inp[f"p{i}.{k}"]) for k in keys}, strict=False)
        nets.append(net)
    am = ArgMax(nf, hid, act_fn=dq_act())
    am.load_state_dict({k: torch.tensor(inp[f"dq.{k}"]) for k in ARGMAX_KEYS}, strict=False)
    model = LFIntegrator(nets, am, dt=float(inp["dt"])).to(DEV)
    for m in model.modules():
        if isinstance(m, nn.PReLU):
            m.weight.requires_grad_(False)
    return model


def _run(model, inp):
    d = data_from_fixture(inp, DEV)
    with torch.no_grad():
        o, ldj = model(d, noise=torch.tensor(inp["eps"], device=DEV))
        outs = {k: getattr(o, k).cpu().numpy().copy() for k in ("h", "g", "pos", "vel")}
        outs["ldj"] = np.array([float(ldj)])
        back = model.reverse(o)
        outs.update({"rev_" + k: getattr(back, k).cpu().numpy().copy() for k in ("h", "g", "pos", "vel")})
    return outs


def test_egcl_prelu_matches_reference_leaky_golden():
    from enflow_amd.nn import EGCL
    inp, out = load("egcl_act_leaky")
    nf, hid = inp["h"].shape[1], int(inp["p0.edge_nn.2.weight"].shape[0])
    slope = float(inp["p0.act"][1])
    net = EGCL(nf, nf, hid, act_fn=nn.PReLU(init=slope))
    net.load_state_dict({k: torch.tensor(inp[f"p0.{k}"]) for k in EGCL_KEYS}, strict=False)
    net = net.to(DEV)
    d = data_from_fixture(inp, DEV)
    with torch.no_grad():
        q, f, g = net(d.h, d.edges)
    errs = {"Q": rel_err(q.cpu().numpy(), out["Q"]), "F": rel_err(f.cpu().numpy(), out["F"]),
            "G": rel_err(g.cpu().numpy(), out["G"])}
    print("egcl PReLU(slope of the leaky golden) vs reference golden:", errs)
    assert_all_within(errs, TOL)


@pytest.mark.parametrize("name", ["lf_act_tanh_h64_L2", "lf_act_gelu_h128_L2"])
def test_flow_prelu_equals_leaky_and_repacks(name):
    inp, _ = load(name)
    a, b = 0.07, -0.3
    pre = _flow(inp, lambda: nn.PReLU(init=a), lambda: nn.PReLU(init=0.11))
    got = _run(pre, inp)
    want = _run(_flow(inp, lambda: nn.LeakyReLU(a), lambda: nn.LeakyReLU(0.11)), inp)
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    # an in-place slope update (what an optimizer step does) re-packs the layers
    with torch.no_grad():
        for m in pre.modules():
            if isinstance(m, nn.PReLU):
                m.weight.fill_(b)
    got = _run(pre, inp)
    want = _run(_flow(inp, lambda: nn.LeakyReLU(b), lambda: nn.LeakyReLU(b)), inp)
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    print(f"{name}: PReLU flow == LeakyReLU flow (forward, log|detJ|, reverse) at slopes {a} and {b}")


def test_training_with_frozen_prelu_equals_leaky():
    from enflow_amd.flow import Alchemical_NLL
    inp, _ = load("train_act_tanh_h32_L2")
    grads = []
    for act in (lambda: nn.PReLU(init=0.05), lambda: nn.LeakyReLU(0.05)):
        model = _flow(inp, act, act)
        model.zero_grad(set_to_none=True)
        d = data_from_fixture(inp, DEV)
        out, ldj = model(d, noise=torch.tensor(inp["eps"], device=DEV))
        loss = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))(out, ldj)
        loss.backward()
        g = {k: p.grad for k, p in model.named_parameters()}
        for m in model.modules():
            if isinstance(m, nn.PReLU):
                assert m.weight.grad is None
        grads.append({k: v.cpu().numpy() for k, v in g.items() if v is not None})
        grads[-1]["loss"] = np.array([float(loss.detach())])
    assert set(grads[0]) == set(grads[1])
    for k in grads[1]:
        np.testing.assert_array_equal(grads[0][k], grads[1][k], err_msg=k)
    print("frozen-PReLU training step == LeakyReLU training step:", len(grads[1]) - 1, "gradients, bitwise")


def test_trainable_prelu_is_refused():
    from enflow_amd.nn import EGCL, ArgMax
    inp, _ = load("train_act_tanh_h32_L2")
    model = _flow(inp, lambda: nn.PReLU(), nn.SiLU)
    model.networks[0].act_fn.weight.requires_grad_(True)
    d = data_from_fixture(inp, DEV)
    with pytest.raises(NotImplementedError, match="freeze"):
        model(d, noise=torch.tensor(inp["eps"], device=DEV))
    net = EGCL(5, 5, 32, act_fn=nn.PReLU()).to(DEV)
    with pytest.raises(NotImplementedError, match="freeze"):
        net(d.h, d.edges)
    am = ArgMax(5, 32, act_fn=nn.PReLU()).to(DEV)
    with pytest.raises(NotImplementedError, match="freeze"):
        am(d.h)
    with torch.no_grad():   # inference runs with the slope trainable
        net(d.h, d.edges)
        am(d.h)


@pytest.mark.parametrize("case", ["large_256_atoms", "nf12_library"])
def test_prelu_equals_leaky_on_the_other_paths(case):
    """The large-system kernels (> the fused kernels' 64-atom image) and the
    16-feature library take the same act code: EGCL forward and a 2-layer flow
    bitwise equal to the LeakyReLU-built modules."""
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    sizes, nf, chain = ([256, 40], 5, True) if case == "large_256_atoms" else ([22, 17, 30], 12, False)
    b = make_molecules(len(sizes), sizes, nf=nf, seed=7, chain=chain)
    res = []
    for act in (lambda: nn.PReLU(init=0.15), lambda: nn.LeakyReLU(0.15)):
        torch.manual_seed(8)
        nets = [EGCL(nf, nf, 64, act_fn=act()) for _ in range(2)]
        am = ArgMax(nf, 64, act_fn=act())
        model = LFIntegrator(nets, am, dt=0.05).to(DEV)
        d = Data.from_arrays(b, device=DEV)
        with torch.no_grad():
            q, f, g = model.networks[0](d.h, d.edges)
            eps = torch.randn(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(9))
            o, ldj = model(d, noise=eps)
        res.append([t.cpu().numpy().copy() for t in (q, f, g, o.h, o.g, o.pos, o.vel)] + [np.array([float(ldj)])])
    for i, (x, y) in enumerate(zip(*res)):
        np.testing.assert_array_equal(x, y, err_msg=str(i))
    print(f"{case}: PReLU == LeakyReLU (EGCL forward, flow forward, log|detJ|)")
