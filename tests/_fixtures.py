"""Shared helpers for loading the golden fixtures in tests/golden/."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

EGCL_KEYS = (
    "edge_nn.0.weight", "edge_nn.0.bias", "edge_nn.2.weight", "edge_nn.2.bias",
    "node_nn.0.weight", "node_nn.0.bias", "node_nn.2.weight", "node_nn.2.bias",
    "coord_nn.0.weight", "coord_nn.0.bias", "coord_nn.2.weight",
    "vel_scaling_nn.0.weight", "vel_scaling_nn.0.bias",
    "vel_scaling_nn.2.weight", "vel_scaling_nn.2.bias",
)
ARGMAX_KEYS = ("network.0.weight", "network.0.bias", "network.2.weight", "network.2.bias")
ATT_KEYS = ("att_nn.0.weight", "att_nn.0.bias")


def layer_flags(inp, i):
    """(attention, norm_diff, tanh) of fixture layer i (defaults when absent)."""
    f = inp.get(f"p{i}.flags")
    return tuple(bool(x) for x in f) if f is not None else (False, False, False)


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    inp = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return inp, out


def act_module(code):
    """torch activation module of an act_fn code (kind, p0, p1) -- the
    ENFLOW_ACT_* numbering; None: nn.SiLU (the reference's default)."""
    from torch import nn
    if code is None:
        return nn.SiLU()
    k, p0, p1 = int(code[0]), float(code[1]), float(code[2])
    return [nn.SiLU, nn.ReLU, lambda: nn.LeakyReLU(p0), lambda: nn.ELU(p0), lambda: nn.CELU(p0), nn.SELU,
            nn.GELU, lambda: nn.GELU(approximate="tanh"), nn.Tanh, nn.Sigmoid, lambda: nn.Softplus(p0, p1),
            nn.Mish, lambda: nn.Hardtanh(p0, p1), nn.Identity][k]()


def layer_params(inp, i, dtype=np.float64):
    p = {k: inp[f"p{i}.{k}"].astype(dtype) for k in EGCL_KEYS}
    flags = layer_flags(inp, i)
    p["flags"] = flags
    if f"p{i}.act" in inp:
        p["act"] = tuple(float(x) for x in inp[f"p{i}.act"])
    if flags[0]:
        p.update({k: inp[f"p{i}.{k}"].astype(dtype) for k in ATT_KEYS})
    return p


def egcl_from_fixture(inp, i, nf, hid):
    """enflow_amd EGCL with fixture layer i's constructor flags and weights."""
    import torch
    from enflow_amd.nn import EGCL
    att, nd, th = layer_flags(inp, i)
    net = EGCL(nf, nf, hid, attention=att, norm_diff=nd, tanh=th, act_fn=act_module(inp.get(f"p{i}.act")))
    keys = EGCL_KEYS + (ATT_KEYS if att else ())
    net.load_state_dict({k: torch.tensor(inp[f"p{i}.{k}"]) for k in keys})
    return net


def dequant_params(inp, dtype=np.float64):
    p = {k: inp[f"dq.{k}"].astype(dtype) for k in ARGMAX_KEYS}
    if "dq.act" in inp:
        p["act"] = tuple(float(x) for x in inp["dq.act"])
    return p


def state(inp, dtype=np.float64):
    s = {k: inp[k].astype(dtype) for k in ("h", "g", "pos", "vel", "box")}
    s["r_cut"] = inp["r_cut"].astype(dtype)
    s["mol_ptr"] = inp["mol_ptr"].astype(np.int64)
    return s


def n_layers(inp):
    return int(inp["n_layers"])


class NonFiniteError(AssertionError):
    """A parity operand holds NaN / inf: the comparison is meaningless."""


def _finite_pair(a, b, allow_nonfinite):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if not allow_nonfinite:
        for name, x in (("result", a), ("reference", b)):
            if not np.all(np.isfinite(x)):
                bad = int(np.size(x) - np.count_nonzero(np.isfinite(x)))
                raise NonFiniteError(f"{name} holds {bad} non-finite of {np.size(x)} values")
    return a, b


def rel_err(a, b, allow_nonfinite=False):
    """max|a - b| / max|b| (per tensor).  Raises NonFiniteError when either
    side holds NaN / inf (NaN would otherwise compare False against any bar
    and vanish inside max()), unless the caller opts in."""
    a, b = _finite_pair(a, b, allow_nonfinite)
    if a.size == 0 and b.size == 0:
        return 0.0
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))


def normwise(a, b, allow_nonfinite=False):
    """||a - b||_2 / ||b||_2, same non-finite rule as rel_err."""
    a, b = _finite_pair(a, b, allow_nonfinite)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def scalar_rel(a, b):
    """|a - b| / |b| for two scalars; raises on non-finite."""
    a, b = float(a), float(b)
    if not (np.isfinite(a) and np.isfinite(b)):
        raise NonFiniteError(f"non-finite scalar: {a} vs {b}")
    return abs(a - b) / max(abs(b), 1e-300)


def worst_of(errs):
    """max over a dict / list of errors that is NaN-propagating."""
    vals = list(errs.values()) if isinstance(errs, dict) else list(errs)
    if any(not np.isfinite(v) for v in vals):
        return float("nan")
    return max(vals) if vals else 0.0


def assert_all_within(errs, tol, what=""):
    """Every error finite and <= tol.  NaN fails (it would slip through max())."""
    items = errs.items() if isinstance(errs, dict) else enumerate(errs)
    bad = {k: v for k, v in items if not (np.isfinite(v) and v <= tol)}
    assert not bad, f"{what} over {tol:g} or non-finite: {bad}"


def flow_from_fixture(inp, device="cuda"):
    """enflow_amd LFIntegrator + Data carrying exactly the fixture's weights/inputs."""
    import torch
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data

    hid, nf, nl = int(inp["hid"]), inp["h"].shape[1], int(inp["n_layers"])
    nets = [egcl_from_fixture(inp, i, nf, hid) for i in range(nl)]
    am = ArgMax(nf, hid, act_fn=act_module(inp.get("dq.act")))
    am.load_state_dict({k: torch.tensor(inp[f"dq.{k}"]) for k in ARGMAX_KEYS})
    model = LFIntegrator(nets, am, dt=float(inp["dt"])).to(device)
    return model, data_from_fixture(inp, device)


def data_from_fixture(inp, device="cuda"):
    import torch
    from enflow_amd.data import Data

    t = lambda k: torch.tensor(inp[k], dtype=torch.float32, device=device)  # noqa: E731
    N = torch.tensor(np.diff(inp["mol_ptr"]), dtype=torch.long)
    return Data(h=t("h"), g=t("g"), pos=t("pos"), vel=t("vel"), N=N, r_cut=t("r_cut"), box=t("box"),
                device=device)
