"""GPU parity for large molecules (BASELINE configs[4]: 256-atom chains):
the row-blocked kernels (pair lists, edge tiles and node phase per block of 32
rows, leapfrog update after the last block) against the CPU oracle.
Tolerances as tests/test_gpu_parity.py (1e-5 normwise, integer work exact)."""
import collections

import numpy as np
import pytest
import torch

from oracle import enflow_oracle as O
from _fixtures import rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda:0"
SIZES = [256, 131, 40, 256, 3]


def _batch(sizes, seed, nf=5):
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


def test_large_neighbour_pairs_exact():
    from enflow_amd.data import Data
    b = _batch(SIZES, 3)
    e = Data.from_arrays(b, device=DEV).edges
    got = collections.Counter(zip(e.row.cpu().tolist(), e.col.cpu().tolist()))
    row, col, _ = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    assert got == collections.Counter(zip(row.tolist(), col.tolist()))
    assert len(row) > 1000


def test_large_egcl_vs_oracle():
    from enflow_amd.nn import EGCL
    from enflow_amd.data import Data
    b = _batch(SIZES, 4)
    b["h"] = np.random.default_rng(1).normal(size=b["h"].shape).astype(np.float32).astype(np.float64)
    torch.manual_seed(2)
    net = EGCL(5, 5, 128).to(DEV)
    d = Data.from_arrays(b, device=DEV)
    with torch.no_grad():
        q, f, g = net(d.h, d.edges)
    p = {k: v.detach().double().cpu().numpy() for k, v in net.state_dict().items()}
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    rq, rf, rg = O.egcl_forward(p, b["h"], row, col, O.coord_diff(b["pos"], row, col, eb))
    assert rel_err(q.cpu().numpy(), rq) < TOL
    assert rel_err(f.cpu().numpy(), rf) < TOL
    assert rel_err(g.cpu().numpy(), rg) < TOL


@pytest.mark.parametrize("prec", ["f32", "f16x3"])
def test_large_flow_forward_and_roundtrip(prec):
    from enflow_amd.data import Data
    b = _batch(SIZES, 5)
    model = _model(128, 5, 3, 6)
    model.gemm_precision = prec
    d = Data.from_arrays(b, device=DEV)
    noise = torch.randn(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(7))
    with torch.no_grad():
        o, ldj = model(d, noise=noise)
    layers = [{k: v.detach().cpu().double().numpy() for k, v in n.state_dict().items()} for n in model.networks]
    dq = {k: v.detach().cpu().double().numpy() for k, v in model.dequantize.state_dict().items()}
    ref, ref_ldj = O.lf_forward(layers, dq, b, noise.cpu().double().numpy(), model.dt)
    for k in ("h", "g", "pos", "vel"):
        assert rel_err(getattr(o, k).cpu().numpy(), ref[k]) < TOL, k
    assert abs(float(ldj) - ref_ldj) <= TOL * abs(ref_ldj)
    st = {k: getattr(o, k).cpu().double().numpy() for k in ("h", "g", "pos", "vel")}
    st.update(box=b["box"], r_cut=b["r_cut"], mol_ptr=b["mol_ptr"])
    with torch.no_grad():
        back = model.reverse(o)
    np.testing.assert_array_equal(np.argmax(back.h.cpu().numpy(), 1), np.argmax(b["h"], 1))
    rback = O.lf_reverse(layers, st, model.dt)
    np.testing.assert_array_equal(back.h.cpu().numpy(), rback["h"])
    errs = {k: rel_err(getattr(back, k).cpu().numpy(), rback[k]) for k in ("g", "pos", "vel")}
    print(f"256-atom chains {prec} reverse vs oracle (same fp32 inputs):",
          {k: f"{v:.2e}" for k, v in errs.items()})
    assert all(v < TOL for v in errs.values()), errs
    assert rel_err(back.vel.cpu().numpy(), b["vel"]) < 1e-4      # round trip


def test_training_past_64_atoms_vs_oracle():
    """Molecules of 65..256 atoms (the row-blocked kernels' range at inference)
    train through the large-system tape and backward: gradients of a ragged
    [100, 22] batch vs the float64 gradient oracle, 1e-4 normwise."""
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.data import Data
    from enflow_amd.flow import Alchemical_NLL
    b = _batch([100, 22], 8)
    model = _model(64, 5, 2, 9)
    eps = np.random.default_rng(10).normal(size=b["h"].shape).astype(np.float32)
    model.zero_grad(set_to_none=True)
    o, ldj = model(Data.from_arrays(b, device=DEV), noise=torch.tensor(eps, device=DEV))
    loss = Alchemical_NLL(kBT=1.0, softening=0.1)(o, ldj)
    loss.backward()
    layers = [{k: v.detach().double().cpu().numpy() for k, v in n.named_parameters()} for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
    assert abs(float(loss) - rloss) <= 1e-5 * abs(rloss)
    nw = lambda a, r: float(np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-300))  # noqa: E731
    errs = {f"p{i}.{k}": nw(p.grad.cpu().double().numpy(), gl[i][k])
            for i, n in enumerate(model.networks) for k, p in n.named_parameters()}
    errs.update({f"dq.{k}": nw(p.grad.cpu().double().numpy(), gd[k]) for k, p in model.dequantize.named_parameters()})
    print("100+22-atom training: max normwise grad err", f"{max(errs.values()):.2e}")
    assert max(errs.values()) <= 1e-4, {k: v for k, v in errs.items() if v > 1e-4}
