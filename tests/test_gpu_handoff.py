"""The two-workgroup split instance's recovery path and its in-place rule.

ENFLOW_ERR_HANDOFF: a workgroup of the SPLIT = 2 instance
whose partner's hand-off never arrives gives up after a bounded wait and
flags the launch; the host re-runs that launch without the split instances
(ENFLOW_PREC_NO_SPLIT, a per-call flag).  enflow_set_handoff_spin_limit(0)
makes every wait give up without polling, so the path runs deterministically:
the word carries ERR_HANDOFF, the re-run lands on a whole-tile instance, and
the outputs equal the 4-wave instance's (1e-6) and the float64 oracle's
(1e-5) -- forward and reverse.

In place: both halves of a molecule read its whole state
at the start and write their own rows at the end, so an in-place launch with
no hand-off to order them (one layer) could read a partner's already updated
rows.  Since ABI 13 such launches take one workgroup per molecule; a
one-layer in-place forward on the split thresholds must equal the
out-of-place one.  Reference: enflow/flow/dynamics.py:10-37.
"""
import numpy as np
import pytest
import torch

from oracle import enflow_oracle as O
from _fixtures import rel_err, worst_of, assert_all_within

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def fmt(errs):
    return "{" + ", ".join(f"{k}: {v:.2e}" for k, v in errs.items()) + "}"


def _f32(b):
    out = dict(b)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        out[k] = b[k].astype(np.float32).astype(np.float64)
    return out


def _model(n_layers, seed):
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data.synthetic import default_dt
    torch.manual_seed(seed)
    return LFIntegrator([EGCL(5, 5, 128) for _ in range(n_layers)], ArgMax(5, 128), dt=default_dt()).to(DEV)


def _sub(b, m):
    a0, a1 = b["mol_ptr"][m], b["mol_ptr"][m + 1]
    sub = {k: b[k][a0:a1] for k in ("h", "g", "pos", "vel", "box")}
    sub["r_cut"] = b["r_cut"][m:m + 1]
    sub["mol_ptr"] = np.array([0, a1 - a0])
    return sub, a0, a1


class _Thresholds:
    """Set the instance thresholds (and the spin limit) for a block, restore after."""

    def __init__(self, lat=-1, split=-1, fs=-1, spin=None):
        self.want = (lat, split, fs, spin)

    def __enter__(self):
        from enflow_amd import _lib
        lat, split, fs, spin = self.want
        self.prev = (_lib.set_latency_threshold(lat), _lib.set_split_threshold(split), _lib.set_fs_threshold(fs),
                     _lib.set_handoff_spin_limit(-1 if spin is None else spin))
        return self

    def __exit__(self, *exc):
        from enflow_amd import _lib
        p = self.prev
        _lib.set_latency_threshold(-1 if p[0] is None else p[0])
        _lib.set_split_threshold(-1 if p[1] is None else p[1])
        _lib.set_fs_threshold(-1 if p[2] is None else p[2])
        _lib.set_handoff_spin_limit(-1 if p[3] is None else p[3])


def _needs_split_room(mols):
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if 2 * mols > cus:
        pytest.skip(f"{mols} molecules need {2 * mols} CUs for two workgroups per molecule ({cus})")


def test_forced_handoff_timeout_reruns_whole_tile():
    """128 molecules (the 8-rank shard of the stated batch), 8 layers, H = 128,
    f16x3: the split instance with every hand-off wait forced to give up."""
    from enflow_amd import _lib
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    mols = 128
    _needs_split_room(mols)
    b = _f32(make_molecules(mols, 22, nf=5, seed=71))
    model = _model(8, 72)
    d = Data.from_arrays(b, device=DEV)
    noise = torch.randn(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(73))
    with torch.no_grad(), _Thresholds(lat=0, split=0, fs=0):
        o4, l4 = model(d.clone(), noise=noise)                     # the 4-wave instance
        b4 = model.reverse(o4.clone())
    # the raw launch: its error word names the lost hand-off
    s = model._state(d.clone())
    M = s["mol_ptr"].numel() - 1
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    ldj_mol, ldj = torch.empty(M, device=DEV), torch.empty(1, device=DEV)
    with torch.no_grad(), _Thresholds(spin=0), _lib.KernelTimer() as t0:
        model.forward_buffers(s["h"], s["g"], s["pos"], s["vel"], s["box"], s["r_cut"], s["mol_ptr"], s["max_n"],
                              noise, ldj_mol, ldj, st[:1], src=s["src"], ticket=st[1:])
        torch.cuda.synchronize()
    raw = int(st[0].item())
    assert "lf_fs_kernel<fwd>" in t0.stats, sorted(t0.stats)
    assert raw & _lib.ERR_HANDOFF, raw
    # the module calls: re-run without the split instances, same outputs
    n0 = _lib.HANDOFF_RERUNS[0]
    with torch.no_grad(), _Thresholds(spin=0), _lib.KernelTimer() as t1:
        o, ldj_o = model(d.clone(), noise=noise)
        back = model.reverse(o.clone())
    reruns = _lib.HANDOFF_RERUNS[0] - n0
    names = sorted(t1.stats)
    assert reruns == 2, reruns
    for k in ("lf_fs_kernel<fwd>", "lf_fs_kernel<rev>"):
        assert t1.stats[k][1] == 1, names
    whole = [k for k in names if k.startswith("lf_flow_kernel<")]
    assert len(whole) == 2, names                                  # forward and reverse on a whole-tile instance
    vs4 = {k: rel_err(getattr(o, k).cpu().numpy(), getattr(o4, k).cpu().numpy()) for k in ("h", "g", "pos", "vel")}
    vs4["ldj"] = abs(float(ldj_o) - float(l4)) / abs(float(l4))
    vs4_r = {"rev_" + k: rel_err(getattr(back, k).cpu().numpy(), getattr(b4, k).cpu().numpy())
             for k in ("g", "pos", "vel")}
    assert torch.equal(back.h, b4.h)
    worst = {k: 0.0 for k in ("h", "g", "pos", "vel")}
    layers = [{k: v.detach().cpu().double().numpy() for k, v in n.state_dict().items()} for n in model.networks]
    dq = {k: v.detach().cpu().double().numpy() for k, v in model.dequantize.state_dict().items()}
    for m in sorted(set(list(range(0, mols, 16)) + [mols - 1])):
        sub, a0, a1 = _sub(b, m)
        ref, _ = O.lf_forward(layers, dq, sub, noise[a0:a1].cpu().double().numpy(), model.dt)
        for k in worst:
            worst[k] = worst_of([worst[k], rel_err(getattr(o, k)[a0:a1].cpu().numpy(), ref[k])])
    print(f"forced hand-off timeout, {mols} molecules: raw word {raw}, re-runs {reruns} on {whole}; vs 4-wave",
          fmt({**vs4, **vs4_r}), "forward vs oracle", fmt(worst))
    assert_all_within({**vs4, **vs4_r}, 1e-6)
    assert_all_within(worst, TOL)
    # the default spin limit: the split instance runs and nothing is re-run
    n1 = _lib.HANDOFF_RERUNS[0]
    with torch.no_grad(), _lib.KernelTimer() as t2:
        o2, _ = model(d.clone(), noise=noise)
    assert _lib.HANDOFF_RERUNS[0] == n1 and "lf_fs_kernel<fwd>" in t2.stats, sorted(t2.stats)
    assert_all_within({k: rel_err(getattr(o2, k).cpu().numpy(), getattr(o4, k).cpu().numpy())
                       for k in ("h", "g", "pos", "vel")}, 1e-6)


@pytest.mark.parametrize("n_layers", [1, 2])
def test_split_in_place_runs_one_workgroup_per_molecule(n_layers):
    """An in-place launch (h_in .. vel_in NULL) on the split thresholds: one
    workgroup per molecule (no torn reads), equal to the out-of-place launch
    and to the oracle."""
    from enflow_amd import _lib
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules
    mols = 64
    _needs_split_room(mols)
    b = _f32(make_molecules(mols, 22, nf=5, seed=81 + n_layers))
    model = _model(n_layers, 82)
    d = Data.from_arrays(b, device=DEV)
    noise = torch.randn(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(83))
    s = model._state(d)
    M = mols
    outs = {}
    with torch.no_grad(), _Thresholds(lat=0, split=1 << 30, fs=1 << 30):
        for mode in ("out", "in"):
            st = torch.zeros(2, dtype=torch.int32, device=DEV)
            ldj_mol, ldj = torch.empty(M, device=DEV), torch.empty(1, device=DEV)
            if mode == "out":
                w = {k: torch.empty_like(t) for k, t in zip(("h", "g", "pos", "vel"), s["src"])}
                src = s["src"]
            else:
                w = {k: t.clone() for k, t in zip(("h", "g", "pos", "vel"), s["src"])}
                src = None
            with _lib.KernelTimer() as t:
                model.forward_buffers(w["h"], w["g"], w["pos"], w["vel"], s["box"], s["r_cut"], s["mol_ptr"],
                                      s["max_n"], noise, ldj_mol, ldj, st[:1], src=src, ticket=st[1:])
                torch.cuda.synchronize()
            assert int(st[0].item()) == 0
            assert "lf_fs_kernel<fwd>" in t.stats, sorted(t.stats)
            outs[mode] = (w, float(ldj))
    w_out, l_out = outs["out"]
    w_in, l_in = outs["in"]
    vs = {k: rel_err(w_in[k].cpu().numpy(), w_out[k].cpu().numpy()) for k in w_out}
    vs["ldj"] = abs(l_in - l_out) / abs(l_out)
    layers = [{k: v.detach().cpu().double().numpy() for k, v in n.state_dict().items()} for n in model.networks]
    dq = {k: v.detach().cpu().double().numpy() for k, v in model.dequantize.state_dict().items()}
    ref, ref_ldj = O.lf_forward(layers, dq, b, noise.cpu().double().numpy(), model.dt)
    orc = {k: rel_err(w_in[k].cpu().numpy(), ref[k]) for k in ("h", "g", "pos", "vel")}
    orc["ldj"] = abs(l_in - ref_ldj) / abs(ref_ldj)
    print(f"split thresholds, {n_layers} layer(s): in place vs out of place", fmt(vs), "in place vs oracle", fmt(orc))
    assert_all_within(vs, 1e-6)
    assert_all_within(orc, TOL)
