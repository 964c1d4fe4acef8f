"""GPU parity for systems past the fused kernels' LDS image (> 256 atoms):
the layer-by-layer large-system kernels (enflow_amd/csrc/enflow_large.hip)
against the CPU oracle, on periodic Lennard-Jones boxes shaped like the
reference's LJ dataset (example/generate.yaml: one 2944-atom box, batch 1).

Oracle comparisons at 300-700 atoms (the float64 oracle builds the
reference's dense 27n x n distance matrix); at the example's 2944 atoms the
size-independent properties: forward -> reverse round trip and bitwise
determinism.  Tolerances as
tests/test_gpu_parity.py: 1e-5 normwise, neighbour lists exact."""
import collections

import numpy as np
import pytest
import torch

from oracle import enflow_oracle as O
from _fixtures import rel_err, normwise, worst_of, assert_all_within

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda:0"


def _boxes(sizes, seed, nf=5, **kw):
    from enflow_amd.data.synthetic import make_lj_systems
    b = make_lj_systems(sizes, nf=nf, seed=seed, **kw)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    return b


def _model(hid, nf, n_layers, seed, **egcl_kw):
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data.synthetic import default_dt
    torch.manual_seed(seed)
    nets = [EGCL(nf, nf, hid, **egcl_kw) for _ in range(n_layers)]
    return LFIntegrator(nets, ArgMax(nf, hid), dt=default_dt()).to(DEV)


def _np_params(module):
    return {k: v.detach().double().cpu().numpy() for k, v in module.state_dict().items()}


def _layer_params(net):
    p = _np_params(net)
    p["flags"] = (bool(net.attention), bool(net.norm_diff), bool(net.tanh))
    return p


def test_large_pairs_exact():
    """Data.edges of two LJ boxes (420 and 333 atoms): exact edge multiset."""
    from enflow_amd.data import Data
    b = _boxes([420, 333], 3)
    e = Data.from_arrays(b, device=DEV).edges
    got = collections.Counter(zip(e.row.cpu().tolist(), e.col.cpu().tolist()))
    row, col, _ = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    assert got == collections.Counter(zip(row.tolist(), col.tolist()))
    assert len(row) > 20000


@pytest.mark.parametrize("hid,variants", [(128, {}), (64, dict(attention=True, norm_diff=True, tanh=True))])
def test_large_egcl_vs_oracle(hid, variants):
    from enflow_amd.nn import EGCL
    from enflow_amd.data import Data
    b = _boxes([700], 4)
    torch.manual_seed(2)
    net = EGCL(5, 5, hid, **variants).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    with torch.no_grad():
        q, f, g = net(d.h, d.edges)
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    p = _layer_params(net)
    rq, rf, rg = O.egcl_forward(p, b["h"], row, col, O.coord_diff(b["pos"], row, col, eb))
    assert rel_err(q.cpu().numpy(), rq) < TOL
    assert rel_err(f.cpu().numpy(), rf) < TOL
    assert rel_err(g.cpu().numpy(), rg) < TOL


@pytest.mark.parametrize("prec", ["f32", "f16x3"])
def test_large_flow_vs_oracle(prec):
    """Ragged batch (a 300-atom box, a 5-atom molecule, a 520-atom box): the
    whole batch goes through the large-system kernels."""
    from enflow_amd.data import Data
    b = _boxes([300, 5, 520], 5)
    model = _model(128, 5, 3, 6)
    model.gemm_precision = prec
    d = Data.from_arrays(b, device=DEV)
    noise = torch.randn(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(7))
    with torch.no_grad():
        o, ldj = model(d, noise=noise)
    layers = [_layer_params(n) for n in model.networks]
    ref, ref_ldj = O.lf_forward(layers, _np_params(model.dequantize), b, noise.cpu().double().numpy(), model.dt)
    for k in ("h", "g", "pos", "vel"):
        assert rel_err(getattr(o, k).cpu().numpy(), ref[k]) < TOL, k
    assert abs(float(ldj) - ref_ldj) <= TOL * abs(ref_ldj)
    # reverse of the oracle's output vs the oracle's reverse
    st = {k: ref[k].astype(np.float32).astype(np.float64) for k in ("h", "g", "pos", "vel")}
    st.update(box=b["box"], r_cut=b["r_cut"], mol_ptr=b["mol_ptr"])
    with torch.no_grad():
        back = model.reverse(Data.from_arrays(st, device=DEV))
    rback = O.lf_reverse(layers, st, model.dt)
    np.testing.assert_array_equal(back.h.cpu().numpy(), rback["h"])
    errs = {k: rel_err(getattr(back, k).cpu().numpy(), rback[k]) for k in ("g", "pos", "vel")}
    print(f"large flow {prec} reverse vs oracle (same fp32 inputs):",
          {k: f"{v:.2e}" for k, v in errs.items()})
    assert_all_within(errs, TOL)


def test_large_flow_variants_vs_oracle():
    from enflow_amd.data import Data
    b = _boxes([400], 11)
    model = _model(64, 5, 2, 12, attention=True, norm_diff=True, tanh=True)
    d = Data.from_arrays(b, device=DEV)
    noise = torch.randn(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(13))
    with torch.no_grad():
        o, ldj = model(d, noise=noise)
    layers = [_layer_params(n) for n in model.networks]
    ref, ref_ldj = O.lf_forward(layers, _np_params(model.dequantize), b, noise.cpu().double().numpy(), model.dt)
    for k in ("h", "g", "pos", "vel"):
        assert rel_err(getattr(o, k).cpu().numpy(), ref[k]) < TOL, k
    assert abs(float(ldj) - ref_ldj) <= TOL * abs(ref_ldj)


def test_large_nll_vs_oracle():
    from enflow_amd.data import Data
    from enflow_amd.flow import Alchemical_NLL
    b = _boxes([600], 14)
    d = Data.from_arrays(b, device=DEV)
    ldj = torch.tensor(3.25, device=DEV)
    loss = Alchemical_NLL(kBT=1.0, softening=0.1)(d, ldj)
    ref = O.alchemical_nll(b, 3.25, 1.0, softening=0.1)
    assert abs(float(loss) - ref) <= 1e-5 * abs(ref)


def test_generate_example_box_2944():
    """example/generate.yaml's system: one 2944-atom LJ box, 8 layers, H=128.
    Forward -> reverse returns the input (one-hot h exactly, vel / g per
    atom), and two runs are bitwise identical."""
    from enflow_amd.data import Data
    b = _boxes([2944], 21, nf=5)
    # wrapped into the pbc range: the dataset's Center transform runs after
    # apply_pbc, and an atom outside [-L/2, L/2] comes back wrapped, which
    # re-labels the reference's id_mapping (the float64 oracle shows the same)
    b["pos"] = O.apply_pbc(b["pos"], b["box"]).astype(np.float32).astype(np.float64)
    onehot = np.eye(5)[np.random.default_rng(0).integers(0, 5, 2944)]
    b["h"] = onehot
    model = _model(128, 5, 8, 22)
    noise = torch.randn((2944, 5), device=DEV, generator=torch.Generator(DEV).manual_seed(23))
    outs = []
    for _ in range(2):
        with torch.no_grad():
            o, ldj = model(Data.from_arrays(b, device=DEV), noise=noise)
        outs.append((o.pos.clone(), o.h.clone(), o.vel.clone(), float(ldj)))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert outs[0][3] == outs[1][3] and np.isfinite(outs[0][3])
    with torch.no_grad():
        back = model.reverse(o)
    np.testing.assert_array_equal(back.h.cpu().numpy(), onehot)
    # in fp32 a pair within ~1e-6 of r_cut can fall on the other side of the
    # cut-off on the way back (~2 such pairs expected over 8 layers at 2944
    # atoms); the atoms they touch are allowed to miss, nobody else
    for k in ("vel", "g", "pos"):
        got, want = getattr(back, k).cpu().numpy(), b[k]
        bad = np.abs(got - want).max(axis=1) > 1e-4 * np.abs(want).max()
        assert bad.mean() < 0.01, (k, int(bad.sum()))


def test_example_box_2944_vs_oracle():
    """example/generate.yaml's 2944-atom LJ box, values: 2 layers at H=32 vs
    the float64 oracle (its neighbour search chunked over images), forward
    (h, g, pos, vel, log|detJ|) and the reverse of the HIP forward's float32
    output, 1e-5 normwise; the layer-0 neighbour list exactly."""
    from enflow_amd.data import Data
    b = _boxes([2944], 21, nf=5)
    b["pos"] = O.apply_pbc(b["pos"], b["box"]).astype(np.float32).astype(np.float64)
    b["h"] = np.eye(5)[np.random.default_rng(0).integers(0, 5, 2944)]
    model = _model(32, 5, 2, 31)
    noise = torch.randn((2944, 5), device=DEV, generator=torch.Generator(DEV).manual_seed(32))
    e = Data.from_arrays(b, device=DEV).edges
    row, col, _ = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    assert collections.Counter(zip(e.row.cpu().tolist(), e.col.cpu().tolist())) == \
        collections.Counter(zip(row.tolist(), col.tolist()))
    with torch.no_grad():
        o, ldj = model(Data.from_arrays(b, device=DEV), noise=noise)
    layers = [_layer_params(n) for n in model.networks]
    ref, ref_ldj = O.lf_forward(layers, _np_params(model.dequantize), b, noise.cpu().double().numpy(), model.dt)
    errs = {k: rel_err(getattr(o, k).cpu().numpy(), ref[k]) for k in ("h", "g", "pos", "vel")}
    errs["ldj"] = abs(float(ldj) - ref_ldj) / abs(ref_ldj)
    st = {k: getattr(o, k).cpu().double().numpy() for k in ("h", "g", "pos", "vel")}
    st.update(box=b["box"], r_cut=b["r_cut"], mol_ptr=b["mol_ptr"])
    with torch.no_grad():
        back = model.reverse(o)
    rback = O.lf_reverse(layers, st, model.dt)
    np.testing.assert_array_equal(back.h.cpu().numpy(), rback["h"])
    errs.update({"rev_" + k: rel_err(getattr(back, k).cpu().numpy(), rback[k]) for k in ("g", "pos", "vel")})
    print("2944-atom box, H=32, 2 layers vs oracle:", {k: f"{v:.2e}" for k, v in errs.items()})
    assert_all_within(errs, TOL)


def test_generate_example_box_2944_grad_enabled():
    """The reference's Main.generate calls self.model(out) outside no_grad
    (main.py:275): with autograd on, the 2944-atom box goes through the taped
    training forward and returns the inference kernels' state (fp32 round-off)."""
    from enflow_amd.data import Data
    b = _boxes([2944], 21, nf=5)
    b["pos"] = O.apply_pbc(b["pos"], b["box"]).astype(np.float32).astype(np.float64)
    b["h"] = np.eye(5)[np.random.default_rng(0).integers(0, 5, 2944)]
    model = _model(128, 5, 8, 22)
    noise = torch.randn((2944, 5), device=DEV, generator=torch.Generator(DEV).manual_seed(23))
    with torch.no_grad():
        ref, lref = model(Data.from_arrays(b, device=DEV), noise=noise)
    o, ldj = model(Data.from_arrays(b, device=DEV), noise=noise)
    assert ldj.requires_grad
    for k in ("h", "g", "pos", "vel"):
        got, want = getattr(o, k).detach().cpu().numpy(), getattr(ref, k).cpu().numpy()
        assert np.linalg.norm(got - want) <= 1e-5 * np.linalg.norm(want), k
    assert abs(float(ldj.detach()) - float(lref)) <= 1e-5 * abs(float(lref))


def _large_train_step(model, b, eps, kBT=1.0, softening=0.1):
    from enflow_amd.data import Data
    from enflow_amd.flow import Alchemical_NLL
    model.zero_grad(set_to_none=True)
    out, ldj = model(Data.from_arrays(b, device=DEV), noise=eps)
    loss = Alchemical_NLL(kBT=kBT, softening=softening)(out, ldj)
    loss.backward()
    torch.cuda.synchronize()
    return loss


@pytest.mark.parametrize("sizes,hid,nl,variants", [([300], 128, 2, {}), ([300, 5], 64, 3, {}),
                                                   ([320], 32, 2, dict(attention=True, norm_diff=True, tanh=True))],
                         ids=["box300_h128_L2", "box300+5_h64_L3", "box320_h32_L2_var"])
def test_large_training_gradients_vs_oracle(sizes, hid, nl, variants):
    """Training on periodic LJ boxes past the fused backward's 64-atom image
    (the reference trains its LJ boxes, enflow/data/lj.py:32-89, through
    enflow/main.py:212-223): loss.backward() through the large-system forward
    (tape) and backward (enflow_lf_backward_large_f32) vs the float64 gradient
    oracle (oracle/enflow_oracle_grad.py, pinned to the reference's
    loss.backward() goldens), 5e-5 normwise per parameter tensor."""
    from oracle import enflow_oracle_grad as OG
    b = _boxes(sizes, 41)
    model = _model(hid, 5, nl, 42, **variants)
    eps = np.random.default_rng(43).normal(size=b["h"].shape).astype(np.float32)
    loss = _large_train_step(model, b, torch.tensor(eps, device=DEV))
    layers = [_layer_params(n) for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
    assert abs(float(loss) - rloss) <= 1e-5 * abs(rloss), (float(loss), rloss)
    errs = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            assert p.grad is not None, (i, k)
            errs[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), gl[i][k])
    for k, p in model.dequantize.named_parameters():
        errs[f"dq.{k}"] = normwise(p.grad.cpu().numpy(), gd[k])
    worst = max(errs, key=lambda k: (not np.isfinite(errs[k]), errs[k]))
    print(f"large training {sizes} H={hid} L={nl}: max normwise grad err {errs[worst]:.2e} ({worst})")
    bad = {k: v for k, v in errs.items() if not v <= 5e-5}
    assert not bad, bad


def test_large_training_bitwise_reproducible_and_matches_inference():
    """Two identical large-system training steps: bitwise-identical gradients
    (column adjoints summed per column in a fixed order); the differentiable
    forward returns the inference forward's outputs exactly (both on the
    large-system kernels past 256 atoms)."""
    from enflow_amd.data import Data
    b = _boxes([420], 51)
    model = _model(64, 5, 2, 52)
    eps = torch.randn((420, 5), device=DEV, generator=torch.Generator(DEV).manual_seed(53))
    grads = []
    for _ in range(2):
        _large_train_step(model, b, eps)
        grads.append([p.grad.clone() for p in model.parameters()])
    for g0, g1 in zip(*grads):
        assert torch.equal(g0, g1)
    o, ldj = model(Data.from_arrays(b, device=DEV), noise=eps)
    with torch.no_grad():
        o2, ldj2 = model(Data.from_arrays(b, device=DEV), noise=eps)
    assert ldj.grad_fn is not None
    for k in ("h", "g", "pos", "vel"):
        assert torch.equal(getattr(o, k).detach(), getattr(o2, k)), k
    assert float(ldj) == float(ldj2)


def test_large_floor_dequant_vs_oracle():
    """Floor dequantisation (floor.py) on the large-system kernels: forward vs
    the oracle, reverse floors back to the input features."""
    from enflow_amd.nn import EGCL, Floor
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import default_dt
    b = _boxes([350], 31, nf=4)
    b["h"] = np.floor(np.abs(b["h"]) * 2.0)          # integer features, as Floor expects
    torch.manual_seed(32)
    model = LFIntegrator([EGCL(4, 4, 32) for _ in range(2)], Floor(), dt=default_dt()).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    u = torch.rand(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(33))
    with torch.no_grad():
        o, ldj = model(d, noise=u)
    layers = [_layer_params(n) for n in model.networks]
    ref, ref_ldj = O.lf_forward(layers, 1.0, b, u.cpu().double().numpy(), model.dt, dequant_kind="floor")
    for k in ("h", "g", "pos", "vel"):
        assert rel_err(getattr(o, k).cpu().numpy(), ref[k]) < TOL, k
    assert abs(float(ldj) - ref_ldj) <= TOL * abs(ref_ldj)
    with torch.no_grad():
        back = model.reverse(o.clone())
    from test_gpu_parity import floor_reverse_check
    st = {k: getattr(o, k).cpu().double().numpy() for k in ("h", "g", "pos", "vel")}
    st.update(box=b["box"], r_cut=b["r_cut"], mol_ptr=b["mol_ptr"])
    rc = O.lf_reverse(layers, st, model.dt, dequant_kind="none")
    n_ex = floor_reverse_check(back.h.cpu().numpy(), rc["h"], want_exact=b["h"])
    print(f"large floor reverse: exact except {n_ex} near-integer elements of {b['h'].size}")
    assert n_ex <= 4
