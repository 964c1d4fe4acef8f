"""GPU parity of the HIP training backward (enflow_lf_backward_f32 +
enflow_alchemical_nll_backward_f32) driven exactly like the reference's
training step (enflow/main.py:217-222):

    out, ldj = model(data); loss = nll(out, ldj); loss.backward(); optimizer.step()

Against golden gradients produced by the reference's own autograd
(tests/golden/make_golden.py train) and, at larger sizes, against the float64
gradient oracle (oracle/enflow_oracle_grad.py, pinned to the same goldens).

Tolerance: gradients are float32 end to end through up to 8 coupling layers
(the reference differentiates in float64); the bar is GRAD_TOL normwise per
parameter tensor, the loss itself 1e-5 relative (north_star).
"""
import os

import numpy as np
import pytest
import torch

from _fixtures import (load, flow_from_fixture, layer_params, dequant_params, state, n_layers, normwise, worst_of,
                       assert_all_within)

pytestmark = pytest.mark.gpu

GRAD_TOL = 5e-5   # <= 2x the fp32 floor measured on these batches (tools/grad_precision.py, profiles/r05)
LOSS_TOL = 1e-5


def _train_step(model, data, eps, kBT, softening):
    from enflow_amd.flow import Alchemical_NLL
    model.zero_grad(set_to_none=True)
    out, ldj = model(data, noise=eps)
    loss = Alchemical_NLL(kBT=kBT, softening=softening)(out, ldj)
    loss.backward()
    torch.cuda.synchronize()
    return loss, ldj


@pytest.mark.usefixtures("kernel_instance")   # the training forward of <= 32-atom batches: both instances
@pytest.mark.parametrize("name", ["train_h32_L3", "train_h128_L2", "train_h64_L2",
                                  "train_var_h64_L2", "train_var_h32_L3",    # var: EGCL(norm_diff, tanh)
                                  "train_att_h64_L2", "train_att_h32_L3"])   # att: + attention
def test_training_gradients_match_reference(name):
    inp, ref = load(name)
    model, data = flow_from_fixture(inp, "cuda")
    eps = torch.tensor(inp["eps"], device="cuda")
    loss, ldj = _train_step(model, data, eps, float(inp["kBT"]), float(inp["softening"]))
    assert loss.requires_grad is False or loss.grad_fn is not None
    assert abs(float(loss) - ref["loss"]) <= LOSS_TOL * abs(ref["loss"]), (float(loss), ref["loss"])
    worst = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            assert p.grad is not None, f"layer {i} {k} has no gradient"
            worst[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_p{i}.{k}"])
    for k, p in model.dequantize.named_parameters():
        worst[f"dq.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_dq.{k}"])
    bad = {k: v for k, v in worst.items() if not v <= GRAD_TOL}
    print(name, "max normwise grad err", worst_of(worst))
    assert not bad, bad


@pytest.mark.parametrize("sizes", [[22] * 12, [64, 33, 48]], ids=["22x12", "ragged33-64"])
def test_training_gradients_bench_shape_vs_oracle(sizes):
    """8 layers, hidden 128 (the bench's model): 22-atom molecules, and a
    ragged batch of 33..64-atom molecules (the training config's 64-atom
    kernels), on batches the float64 gradient oracle finishes in seconds."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    nf, hid, nl, M = 5, 128, 8, len(sizes)
    radius = 4.0 * (max(sizes) / 22.0) ** (1.0 / 3.0)
    b = make_molecules(M, sizes, nf=nf, seed=77, radius=radius)
    torch.manual_seed(5)
    model = LFIntegrator([EGCL(nf, nf, hid) for _ in range(nl)], ArgMax(nf, hid), dt=default_dt()).cuda()
    eps = np.random.default_rng(3).normal(size=b["h"].shape).astype(np.float32)
    f32 = lambda k: torch.tensor(b[k], dtype=torch.float32, device="cuda")  # noqa: E731
    data = Data(h=f32("h"), g=f32("g"), pos=f32("pos"), vel=f32("vel"), N=torch.tensor(np.diff(b["mol_ptr"])),
                r_cut=f32("r_cut"), box=f32("box"), device="cuda")
    kBT = default_kBT()
    loss, _ = _train_step(model, data, torch.tensor(eps, device="cuda"), kBT, 0.1)
    st = {k: np.asarray(b[k], dtype=np.float32).astype(np.float64) for k in ("h", "g", "pos", "vel", "box", "r_cut")}
    st["mol_ptr"] = b["mol_ptr"]
    layers = [{k: v.detach().double().cpu().numpy() for k, v in n.named_parameters()} for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, st, eps.astype(np.float64), default_dt(), kBT, 0.1)
    assert abs(float(loss) - rloss) <= LOSS_TOL * abs(rloss)
    errs = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            errs[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), gl[i][k])
    for k, p in model.dequantize.named_parameters():
        errs[f"dq.{k}"] = normwise(p.grad.cpu().numpy(), gd[k])
    print("bench-shape max normwise grad err", worst_of(errs))
    bad = {k: v for k, v in errs.items() if not v <= GRAD_TOL}
    assert not bad, bad


def test_reference_training_loop_runs_unchanged():
    """The reference's loop body (main.py:217-223) with torch.optim.Adam: the
    loss on a fixed batch goes down and the parameters move."""
    from enflow_amd.flow import Alchemical_NLL
    inp, _ = load("train_h32_L3")
    model, _ = flow_from_fixture(inp, "cuda")
    from _fixtures import data_from_fixture
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    nll = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))
    eps = torch.tensor(inp["eps"], device="cuda")
    before = [p.detach().clone() for p in model.parameters()]
    losses = []
    for _ in range(6):
        data = data_from_fixture(inp, "cuda")
        opt.zero_grad()
        out, ldj = model(data, noise=eps)
        loss = nll(out, ldj)
        loss.backward()
        opt.step()
        losses.append(float(loss))
    assert losses[-1] < losses[0], losses
    moved = sum(int(not torch.equal(a, p.detach())) for a, p in zip(before, model.parameters()))
    assert moved == len(before)


def test_inference_forward_unchanged_by_training_path():
    """With grad disabled the forward is the tape-less fused kernel and gives
    the same outputs as the differentiable forward."""
    inp, _ = load("train_h32_L3")
    model, data = flow_from_fixture(inp, "cuda")
    eps = torch.tensor(inp["eps"], device="cuda")
    with torch.no_grad():
        o1, l1 = model(data, noise=eps)
        o1 = {k: getattr(o1, k).clone() for k in ("h", "g", "pos", "vel")}
    from _fixtures import data_from_fixture
    o2, l2 = model(data_from_fixture(inp, "cuda"), noise=eps)
    assert l2.grad_fn is not None
    for k in o1:
        assert torch.equal(o1[k], getattr(o2, k).detach()), k
    assert float(l1) == float(l2)


def test_training_gradients_bitwise_reproducible():
    """Two identical training steps give bitwise-identical gradients: the layer
    backward sums d h / d pos per wave and then over the waves in a fixed
    order, the weight gradients are reduced over fixed row chunks in fp64."""
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    nf, hid, nl = 5, 128, 4
    sizes = [64, 40, 57, 22, 64, 33, 61, 48] * 4
    b = make_molecules(len(sizes), sizes, nf=nf, seed=11, radius=5.7)
    torch.manual_seed(9)
    model = LFIntegrator([EGCL(nf, nf, hid) for _ in range(nl)], ArgMax(nf, hid), dt=default_dt()).cuda()
    eps = torch.tensor(np.random.default_rng(4).normal(size=b["h"].shape).astype(np.float32), device="cuda")
    grads = []
    for lean in (False, False, True):
        # the third step with the minimum workspace (two rotating pair-row buffers
        # instead of three, enflow_lf_backward_workspace_size_min): same arithmetic
        if lean:
            os.environ["ENFLOW_BWD_MIN_WS"] = "1"
        try:
            data = Data.from_arrays(b, device="cuda")
            _train_step(model, data, eps, default_kBT(), 0.1)
        finally:
            os.environ.pop("ENFLOW_BWD_MIN_WS", None)
        grads.append([p.grad.clone() for p in model.parameters()])
    for g0, g1, g2 in zip(*grads):
        assert torch.equal(g0, g1)
        assert torch.equal(g0, g2)


def test_training_through_all_egcl_variants_vs_oracle():
    """Every constructor variant trains (lf_var_h64_L3: attention, norm_diff +
    tanh, all three): HIP gradients vs the gradient oracle (pinned to the
    reference's loss.backward() on train_att_* / train_var_*)."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.data.synthetic import default_kBT
    inp, _ = load("lf_var_h64_L3")
    model, data = flow_from_fixture(inp, "cuda")
    kBT = default_kBT()
    loss, _ = _train_step(model, data, torch.tensor(inp["eps"], device="cuda"), kBT, 0.1)
    nl = n_layers(inp)
    rloss, _, gl, gd, _ = OG.train_loss_and_grads([layer_params(inp, i) for i in range(nl)], dequant_params(inp),
                                                  state(inp), inp["eps"].astype(np.float64), float(inp["dt"]),
                                                  kBT, 0.1)
    assert abs(float(loss) - rloss) <= LOSS_TOL * abs(rloss)
    worst = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            worst[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), gl[i][k])
    print("variants max normwise grad err", worst_of(worst))
    assert_all_within(worst, GRAD_TOL)


def test_backward_error_word_is_deferred_then_checked():
    """The backward queues its device error word (pinned copy + event) instead
    of synchronising; the next forward check, or _lib.check_pending(), reads
    it.  A clean step leaves nothing pending afterwards and raises nothing; a
    forced error code queued the same way raises at the next check."""
    from enflow_amd import _lib
    inp, _ = load("train_h32_L3")
    model, data = flow_from_fixture(inp, "cuda")
    eps = torch.tensor(inp["eps"], device="cuda")
    _lib.check_pending()
    _train_step(model, data, eps, float(inp["kBT"]), float(inp["softening"]))
    assert len(_lib._pending) == 1
    _lib.check_pending()
    assert not _lib._pending
    _lib.defer_err(torch.full((1,), _lib.ERR_FEW_IMAGES, dtype=torch.int32, device="cuda"))
    with pytest.raises(IndexError):
        _lib.check_pending()
    assert not _lib._pending


def test_training_gradients_bitwise_reproducible_bench_scale():
    """The bench's training batch (1024 x 64-atom molecules), 2 layers, three
    steps: bitwise-identical gradients.  (Regression: the forward's tape copy
    of a layer's input state once raced the same layer's leapfrog update in
    the unblocked kernel -- a few atoms' taped positions were already updated
    -- which only showed at this scale.)"""
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    b = make_molecules(1024, 64, nf=5, seed=2000, radius=4.0 * (64 / 22.0) ** (1.0 / 3.0))
    torch.manual_seed(0)
    model = LFIntegrator([EGCL(5, 5, 128) for _ in range(2)], ArgMax(5, 128), dt=default_dt()).cuda()
    base = Data.from_arrays(b, device="cuda")
    eps = torch.randn_like(base.h)
    grads = []
    for _ in range(3):
        _train_step(model, base._replace(), eps, default_kBT(), 0.1)
        grads.append([p.grad.clone() for p in model.parameters()])
    for g in grads[1:]:
        for a, b_ in zip(grads[0], g):
            assert torch.equal(a, b_)


def test_inplace_parameter_change_between_forward_and_backward_raises():
    """The backward runs on the weights packed at forward time; a parameter
    changed in place in between makes it refuse (torch autograd reports a
    version mismatch in that case) instead of mixing old tape / new weights."""
    from enflow_amd.flow import Alchemical_NLL
    inp, _ = load("train_h32_L3")
    model, data = flow_from_fixture(inp, "cuda")
    out, ldj = model(data, noise=torch.tensor(inp["eps"], device="cuda"))
    loss = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))(out, ldj)
    with torch.no_grad():
        model.networks[1].edge_nn[0].weight.mul_(1.01)
    with pytest.raises(RuntimeError, match="modified in place"):
        loss.backward()


def test_configs3_training_step_1024x64_8_layers():
    """BASELINE configs[3] per GPU at its stated size: 1024 x 64-atom molecules,
    8 layers, H=128, one loss.backward().  The NLL is a sum over molecules
    divided by their number (enflow/flow/loss.py:21-25), so the full batch's
    gradient equals the molecule-weighted sum of the gradients of any partition
    into sub-batches (same noise).  Checked on the partition [4, 124, 7 x 128]:
    full vs weighted sum normwise <= SPLIT_TOL, and the 4-molecule sub-batch vs
    the float64 gradient oracle at GRAD_TOL (the oracle is pinned to the
    reference's loss.backward() by the train_* goldens)."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    SPLIT_TOL = 1e-5
    nf, hid, nl, M = 5, 128, 8, 1024
    b = make_molecules(M, 64, nf=nf, seed=3000, radius=4.0 * (64 / 22.0) ** (1.0 / 3.0))
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    torch.manual_seed(3001)
    model = LFIntegrator([EGCL(nf, nf, hid) for _ in range(nl)], ArgMax(nf, hid), dt=default_dt()).cuda()
    eps = np.random.default_rng(3002).normal(size=b["h"].shape).astype(np.float32)
    kBT = default_kBT()
    params = list(model.parameters())
    names = [f"p{i}.{k}" for i, n in enumerate(model.networks) for k, _ in n.named_parameters()] + \
            [f"dq.{k}" for k, _ in model.dequantize.named_parameters()]

    def step(lo, hi):
        a0, a1 = int(b["mol_ptr"][lo]), int(b["mol_ptr"][hi])
        sub = {k: b[k][a0:a1] for k in ("h", "g", "pos", "vel", "box")}
        sub["r_cut"] = b["r_cut"][lo:hi]
        sub["mol_ptr"] = b["mol_ptr"][lo:hi + 1] - b["mol_ptr"][lo]
        loss, _ = _train_step(model, Data.from_arrays(sub, device="cuda"),
                              torch.tensor(eps[a0:a1], device="cuda"), kBT, 0.1)
        return sub, float(loss), [p.grad.double().cpu().numpy() for p in params]

    _, loss_full, g_full = step(0, M)
    cuts = [0, 4, 128] + list(range(256, M + 1, 128))
    acc = [np.zeros_like(g) for g in g_full]
    loss_sum = 0.0
    sub4 = None
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        sub, loss, g = step(lo, hi)
        w = (hi - lo) / M
        loss_sum += w * loss
        for a, gk in zip(acc, g):
            a += w * gk
        if lo == 0:
            sub4, g4, loss4 = sub, g, loss
    split = {n: normwise(gf, a) for n, gf, a in zip(names, g_full, acc)}
    print(f"configs[3] 1024 x 64, 8 layers: full vs weighted sub-batch gradients worst {worst_of(split):.2e}; "
          f"loss {loss_full:.6e} vs {loss_sum:.6e}")
    assert abs(loss_full - loss_sum) <= 1e-5 * abs(loss_full)
    assert_all_within(split, SPLIT_TOL, "full vs sub-batch sum")
    layers = [{k: v.detach().double().cpu().numpy() for k, v in n.named_parameters()} for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, sub4, eps[:int(b["mol_ptr"][4])].astype(np.float64),
                                                  default_dt(), kBT, 0.1)
    assert abs(loss4 - rloss) <= LOSS_TOL * abs(rloss), (loss4, rloss)
    ref = [gl[i][k] for i, n in enumerate(model.networks) for k, _ in n.named_parameters()] + \
          [gd[k] for k, _ in model.dequantize.named_parameters()]
    oerr = {n: normwise(g, r) for n, g, r in zip(names, g4, ref)}
    print(f"configs[3] 4-molecule sub-batch vs gradient oracle worst {worst_of(oerr):.2e}")
    assert_all_within(oerr, GRAD_TOL, "sub-batch vs oracle")


@pytest.mark.parametrize("name", ["train_h128_L2", "train_h64_L2", "train_h32_L3"])
def test_f16x3_gradients_sit_at_the_fp32_floor(name):
    """the gradients' error vs the reference's
    float64 loss.backward() splits into what fp32 arithmetic alone gives (the
    HIP path with gemm_precision='f32': exact fp32 MFMA chains and the fp32
    backward) and what the f16x3 split adds on top.  Measured (profiles/r05,
    tools/grad_precision.py): train_h128_L2 f32 3.3e-5, f16x3 3.5e-5, and the
    float64 oracle re-run in float32 on the CPU 2.7-2.8e-5 -- the error is fp32
    conditioning (worst tensor coord_nn.0.bias behind the gain-0.001
    coord_nn.2), not the split.  Bar: f16x3 within 1.25x of f32 (+1e-6)."""
    inp, ref = load(name)
    errs = {}
    for prec in ("f32", "f16x3"):
        model, data = flow_from_fixture(inp, "cuda")
        model.gemm_precision = prec
        eps = torch.tensor(inp["eps"], device="cuda")
        _train_step(model, data, eps, float(inp["kBT"]), float(inp["softening"]))
        w = {}
        for i, net in enumerate(model.networks):
            for k, p in net.named_parameters():
                w[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_p{i}.{k}"])
        errs[prec] = worst_of(w)
    print(f"{name}: worst normwise grad err f32 {errs['f32']:.2e}, f16x3 {errs['f16x3']:.2e}")
    assert errs["f16x3"] <= 1.25 * errs["f32"] + 1e-6
    assert errs["f32"] <= GRAD_TOL
