"""CPU oracle for the enflow coupling-flow hot path -- TEST INFRASTRUCTURE ONLY.

This module is a float64 numpy restatement of the reference algorithm
(bharath-raghavan/enflow @ 2025-07-11).  It exists to CHECK the HIP path:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The product path (``enflow_amd``) never
imports, links or calls anything under ``oracle/``.

Parity pinning: every function below is checked against golden vectors that
were produced by running the reference's own modules (``enflow.nn.egcl.EGCL``,
``enflow.nn.argmax.ArgMax``, ``enflow.flow.dynamics.LFIntegrator``,
``enflow.flow.loss.Alchemical_NLL`` and ``enflow.utils.helpers``) in the build
container; see ``tests/golden/make_golden.py`` and
``tests/test_oracle_golden.py``.  The reference's ``Data.edges`` property
(enflow/data/base.py:122-144) cannot be imported without rdkit, so the golden
generator restates its 10-line loop body around the reference's own
``get_periodic_images_within`` helper; the oracle's neighbour list is pinned
against that.

Layout conventions follow the reference: a batch is the concatenation of
molecules; ``mol_ptr`` (int, [M+1]) holds the CSR offsets derived from
``Data.N`` (enflow/data/base.py:34-50).
"""
import math

import numpy as np

LOG_2PI = math.log(2.0 * math.pi)


# --------------------------------------------------------------------------
# utils/helpers.py
# --------------------------------------------------------------------------
def log_gaussian(z):
    """enflow/utils/helpers.py:4-5 -- note: ONE log(2*pi) for the whole tensor."""
    return -0.5 * (float(np.sum(z * z)) + LOG_2PI)


def apply_pbc(x, box):
    """enflow/utils/helpers.py:7-8 (torch.round == round-half-to-even == np.round)."""
    return x - np.round(x / box) * box


def image_shifts(box):
    """The 27 shift vectors in the order of enflow/utils/helpers.py:17
    (c outermost over z, then b over y, a innermost over x; each in
    [-box, +box, 0])."""
    bx, by, bz = box
    return np.array([[a, b, c]
                     for c in (-bz, bz, 0.0)
                     for b in (-by, by, 0.0)
                     for a in (-bx, bx, 0.0)], dtype=np.float64)


def periodic_images_within(pos, box, r_cut):
    """enflow/utils/helpers.py:15-29: replicate positions to 27 images, keep the
    ones inside the ellipsoid with radii box + r_cut; return them with the
    image -> atom mapping."""
    n = pos.shape[0]
    imgs = np.concatenate([pos + s for s in image_shifts(box)], axis=0)
    radii = box + r_cut
    keep = np.sum((imgs / radii) ** 2, axis=1) <= 1.0
    id_mapping = np.tile(np.arange(n), 27)[keep]
    return imgs[keep], id_mapping


def silu(x):
    return x / (1.0 + np.exp(-x))


def activation(code):
    """The elementwise function of an act_fn code (kind, p0, p1) -- the
    ENFLOW_ACT_* numbering of include/enflow_hip.h; None = SiLU (the
    reference's default act_fn, enflow/nn/egcl.py:11).  float64, torch's
    definitions (torch.nn.{SiLU, ReLU, LeakyReLU, ELU, CELU, SELU, GELU, Tanh,
    Sigmoid, Softplus, Mish, Hardtanh, Identity})."""
    if code is None:
        return silu
    k, p0, p1 = int(code[0]), float(code[1]), float(code[2])
    if k == 0:
        return silu
    if k == 1:
        return lambda x: np.maximum(x, 0.0)
    if k == 2:
        return lambda x: np.where(x > 0, x, p0 * x)
    if k == 3:
        return lambda x: np.where(x > 0, x, p0 * np.expm1(np.minimum(x, 0.0)))
    if k == 4:
        return lambda x: np.where(x > 0, x, p0 * np.expm1(np.minimum(x, 0.0) / p0))
    if k == 5:
        a, s = 1.6732632423543772848170429916717, 1.0507009873554804934193349852946
        return lambda x: s * np.where(x > 0, x, a * np.expm1(np.minimum(x, 0.0)))
    if k == 6:
        from scipy.special import erf
        return lambda x: 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))
    if k == 7:
        c = math.sqrt(2.0 / math.pi)
        return lambda x: 0.5 * x * (1.0 + np.tanh(c * (x + 0.044715 * x ** 3)))
    if k == 8:
        return np.tanh
    if k == 9:
        return lambda x: 1.0 / (1.0 + np.exp(-x))
    if k == 10:
        return lambda x: np.where(x * p0 > p1, x, np.log1p(np.exp(np.minimum(p0 * x, p1))) / p0)
    if k == 11:
        return lambda x: x * np.tanh(softplus(x))
    if k == 12:
        return lambda x: np.clip(x, p0, p1)
    if k == 13:
        return lambda x: x
    raise ValueError(f"activation code {k}")


def softplus(x):
    """torch.nn.functional.softplus(beta=1, threshold=20)."""
    return np.where(x > 20.0, x, np.log1p(np.exp(np.minimum(x, 20.0))))


def logsigmoid(x):
    """torch.nn.functional.logsigmoid (stable form)."""
    return np.minimum(x, 0.0) - np.log1p(np.exp(-np.abs(x)))


def linear(x, w, b=None):
    y = x @ w.T
    return y if b is None else y + b


def segment_sum(data, seg, n):
    """enflow/utils/helpers.py:54-60 (unsorted_segment_sum)."""
    out = np.zeros((n, data.shape[1]), dtype=data.dtype)
    np.add.at(out, seg, data)
    return out


def segment_mean(data, seg, n):
    """enflow/utils/helpers.py:63-70 (unsorted_segment_mean, count clamped at 1)."""
    out = segment_sum(data, seg, n)
    cnt = np.zeros((n, data.shape[1]), dtype=data.dtype)
    np.add.at(cnt, seg, np.ones_like(data))
    return out / np.maximum(cnt, 1.0)


# --------------------------------------------------------------------------
# data/base.py: neighbour list
# --------------------------------------------------------------------------
def molecule_edges(pos, box, r_cut):
    """One molecule of Data.edges (enflow/data/base.py:129-143).

    Returns int64 [E, 2] (row, col) in the reference's order.  Reproduces the
    reference exactly, including that BOTH columns of the (image, atom) hit
    list are mapped through ``id_mapping`` (base.py:137), and the removal of
    self pairs by label (base.py:139).
    """
    imgs, id_mapping = periodic_images_within(pos, box, r_cut)
    # row-major hits (== torch.nonzero), in chunks of images so that large
    # boxes (example/generate.yaml: 2944 atoms, ~80 k images) fit in memory
    chunk = max(1, (1 << 24) // max(pos.shape[0], 1))
    parts = []
    for c0 in range(0, imgs.shape[0], chunk):
        d2 = np.sum((imgs[c0:c0 + chunk, None, :] - pos[None, :, :]) ** 2, axis=2)
        hit = np.argwhere(d2 < r_cut * r_cut)
        hit[:, 0] += c0
        parts.append(hit)
    ids = np.concatenate(parts) if parts else np.zeros((0, 2), dtype=np.int64)
    if ids.size and ids[:, 1].max() >= id_mapping.shape[0]:
        raise IndexError("reference would index id_mapping out of range "
                         "(fewer periodic images than atoms)")
    e = id_mapping[ids] if ids.size else np.zeros((0, 2), dtype=np.int64)
    return e[e[:, 0] != e[:, 1]]


def batch_edges(pos, box, r_cut, mol_ptr):
    """Data.edges over a batch: (row, col, edge_box) with per-molecule atom
    offsets; edge_box is each molecule's FIRST-atom box (base.py:130,140)."""
    rows, cols, boxes = [], [], []
    for m in range(len(mol_ptr) - 1):
        a0, a1 = int(mol_ptr[m]), int(mol_ptr[m + 1])
        mbox = box[a0]
        e = molecule_edges(pos[a0:a1], mbox, float(r_cut[m])) + a0
        rows.append(e[:, 0])
        cols.append(e[:, 1])
        boxes.append(np.repeat(mbox[None, :], e.shape[0], axis=0))
    row = np.concatenate(rows) if rows else np.zeros(0, np.int64)
    col = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    eb = np.concatenate(boxes) if boxes else np.zeros((0, 3))
    return row, col, eb


def coord_diff(pos, row, col, edge_box):
    """Edges.coord_diff (enflow/data/base.py:15-19): note the HALF-box
    minimum image used by the reference."""
    return apply_pbc(pos[row] - pos[col], edge_box * 0.5)


def pair_multiplicity(row, col, n_atoms):
    """Collapse an edge list to unique (row, col) pairs with multiplicities,
    sorted by (row, col) -- the form the HIP kernels build."""
    key = row.astype(np.int64) * n_atoms + col.astype(np.int64)
    uniq, cnt = np.unique(key, return_counts=True)
    return uniq // n_atoms, uniq % n_atoms, cnt


# --------------------------------------------------------------------------
# nn/egcl.py
# --------------------------------------------------------------------------
EGCL_PARAM_NAMES = (
    "edge_nn.0.weight", "edge_nn.0.bias", "edge_nn.2.weight", "edge_nn.2.bias",
    "node_nn.0.weight", "node_nn.0.bias", "node_nn.2.weight", "node_nn.2.bias",
    "coord_nn.0.weight", "coord_nn.0.bias", "coord_nn.2.weight",
    "vel_scaling_nn.0.weight", "vel_scaling_nn.0.bias",
    "vel_scaling_nn.2.weight", "vel_scaling_nn.2.bias",
)
ARGMAX_PARAM_NAMES = ("network.0.weight", "network.0.bias",
                      "network.2.weight", "network.2.bias")


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def egcl_forward(p, h, row, col, cdiff, coords_weight=1.0):
    """EGCL.forward (enflow/nn/egcl.py:76-92).  ``p`` maps EGCL_PARAM_NAMES to
    float64 arrays; the constructor variants come from optional keys:
    ``flags`` = (attention, norm_diff, tanh) and, with attention,
    ``att_nn.0.weight`` / ``att_nn.0.bias``.  Returns (Q [n,1], F [n,3], G [n,nf])."""
    attention, norm_diff, tanh = (bool(x) for x in p.get("flags", (0, 0, 0)))
    silu = activation(p.get("act"))   # act_fn (egcl.py:11); SiLU by default
    n = h.shape[0]
    radial = np.sum(cdiff ** 2, axis=1, keepdims=True)                 # egcl.py:79
    if norm_diff:                                                        # egcl.py:82-84
        cdiff = cdiff / (np.sqrt(radial) + 1.0)
    ein = np.concatenate([h[row], h[col], radial], axis=1)              # egcl.py:57
    e = silu(linear(silu(linear(ein, p["edge_nn.0.weight"], p["edge_nn.0.bias"])),
                    p["edge_nn.2.weight"], p["edge_nn.2.bias"]))         # egcl.py:20-24
    if attention:                                                        # egcl.py:60-62
        e = e * sigmoid(linear(e, p["att_nn.0.weight"], p["att_nn.0.bias"]))
    q = linear(silu(linear(h, p["vel_scaling_nn.0.weight"], p["vel_scaling_nn.0.bias"])),
               p["vel_scaling_nn.2.weight"], p["vel_scaling_nn.2.bias"])  # egcl.py:51-54
    phi = linear(silu(linear(e, p["coord_nn.0.weight"], p["coord_nn.0.bias"])),
                 p["coord_nn.2.weight"])                                  # egcl.py:35-42
    if tanh:                                                             # egcl.py:40-42
        phi = np.tanh(phi)
    trans = np.clip(cdiff * phi, -100.0, 100.0)                          # egcl.py:71-72
    f = segment_mean(trans, row, n) * coords_weight                      # egcl.py:73-74
    agg = segment_sum(e, row, n)                                          # egcl.py:65
    g = linear(silu(linear(np.concatenate([h, agg], axis=1),
                           p["node_nn.0.weight"], p["node_nn.0.bias"])),
               p["node_nn.2.weight"], p["node_nn.2.bias"])                # egcl.py:66-67
    return q, f, g


# --------------------------------------------------------------------------
# nn/argmax.py, nn/floor.py
# --------------------------------------------------------------------------
def argmax_forward(p, h, eps):
    """ArgMax.forward (enflow/nn/argmax.py:13-25) with the Gaussian draw
    ``torch.randn(h.size())`` supplied as ``eps``.  Returns (z, log_q)."""
    nf = h.shape[1]
    act = activation(p.get("act"))    # act_fn (argmax.py:7)
    net = linear(act(linear(h, p["network.0.weight"], p["network.0.bias"])),
                 p["network.2.weight"], p["network.2.bias"])
    log_scale, translate = net[:, :nf], net[:, nf:]
    u = translate + eps * np.exp(log_scale)
    log_q = log_gaussian(u) - float(np.sum(log_scale))
    t = np.sum(h * u, axis=-1, keepdims=True)
    z = h * u + (1.0 - h) * (t - softplus(t - u))
    ldj = (1.0 - h) * logsigmoid(t - u)
    return z, log_q - float(np.sum(ldj))


def argmax_reverse(z):
    """ArgMax.reverse (argmax.py:27-28): one-hot of the first maximum.  The
    reference calls helpers.one_hot without num_classes (helpers.py:43-52), so
    the width is max(index) + 1, not node_nf."""
    idx = np.argmax(z, axis=-1)
    out = np.zeros((z.shape[0], int(idx.max()) + 1 if idx.size else 0), dtype=z.dtype)
    out[np.arange(z.shape[0]), idx] = 1.0
    return out


def floor_forward(h, noise, dequant_scale=1.0):
    """Floor.forward (enflow/nn/floor.py:9-11) with the uniform draw supplied."""
    return h + dequant_scale * noise, 0.0


def floor_reverse(z):
    """Floor.reverse (floor.py:13)."""
    return np.floor(z)


# --------------------------------------------------------------------------
# flow/dynamics.py: LFIntegrator
# --------------------------------------------------------------------------
def _layer(p, h, pos, box, r_cut, mol_ptr, coords_weight):
    row, col, eb = batch_edges(pos, box, r_cut, mol_ptr)
    cd = coord_diff(pos, row, col, eb)
    return egcl_forward(p, h, row, col, cd, coords_weight)


def lf_forward(layers, dequant, state, noise, dt, coords_weight=1.0,
               dequant_kind="argmax"):
    """LFIntegrator.forward (enflow/flow/dynamics.py:10-24).

    ``state`` = dict(h, g, pos, vel, box, r_cut, mol_ptr) of float64 arrays.
    Returns (new_state, ldj)."""
    s = {k: np.array(v, copy=True) for k, v in state.items()}
    if dequant_kind == "argmax":
        s["h"], ldj = argmax_forward(dequant, s["h"], noise)
    else:
        s["h"], ldj = floor_forward(s["h"], noise, dequant)
    for p in layers:
        q, f, g = _layer(p, s["h"], s["pos"], s["box"], s["r_cut"], s["mol_ptr"],
                         coords_weight)
        s["vel"] = np.exp(q) * s["vel"] + f * dt
        s["g"] = s["g"] + g * dt
        s["pos"] = apply_pbc(s["pos"] + s["vel"] * dt, s["box"])
        s["h"] = s["h"] + s["g"] * dt
        ldj = ldj + float(np.sum(q))
    return s, ldj


def lf_reverse(layers, state, dt, coords_weight=1.0, dequant_kind="argmax"):
    """LFIntegrator.reverse (enflow/flow/dynamics.py:26-37)."""
    s = {k: np.array(v, copy=True) for k, v in state.items()}
    for p in reversed(layers):
        s["h"] = s["h"] - s["g"] * dt
        s["pos"] = apply_pbc(s["pos"] - s["vel"] * dt, s["box"])
        q, f, g = _layer(p, s["h"], s["pos"], s["box"], s["r_cut"], s["mol_ptr"],
                         coords_weight)
        s["g"] = s["g"] - g * dt
        s["vel"] = (s["vel"] - f * dt) / np.exp(q)
    if dequant_kind == "argmax":
        s["h"] = argmax_reverse(s["h"])
    elif dequant_kind == "floor":
        s["h"] = floor_reverse(s["h"])
    # dequant_kind "none": the continuous h before the dequantiser's reverse (test checks)
    return s


# --------------------------------------------------------------------------
# flow/loss.py: Alchemical_NLL
# --------------------------------------------------------------------------
def lj_potential(pos, mol_ptr, softening):
    """Alchemical_NLL._get_lj_potential (enflow/flow/loss.py:11-19): over each
    molecule, the strict upper triangle of squared distances, zero entries
    dropped, softened and summed as 4(r^-12 - r^-6)."""
    total = 0.0
    for m in range(len(mol_ptr) - 1):
        x = pos[int(mol_ptr[m]):int(mol_ptr[m + 1])]
        d2 = np.triu(np.sum((x[:, None, :] - x[None, :, :]) ** 2, axis=2))
        r2 = d2[d2 != 0] + softening
        r6 = r2 ** 3
        total += float(np.sum(4.0 * (1.0 / r6 ** 2 - 1.0 / r6)))
    return total


def alchemical_nll(state, ldj, kBT, softening=0.0, partition_func=10.0):
    """Alchemical_NLL.__call__ (enflow/flow/loss.py:21-24)."""
    mol_ptr = state["mol_ptr"]
    num_atoms = int(mol_ptr[-1])
    num_mols = len(mol_ptr) - 1
    H = lj_potential(state["pos"], mol_ptr, softening) + 0.5 * float(np.sum(state["vel"] ** 2))
    logZ = -num_atoms * (math.log(partition_func) - 1.5 * math.log(2 * math.pi / kBT))
    log_px = -H / kBT + logZ + ldj + log_gaussian(state["h"]) + log_gaussian(state["g"])
    return -log_px / num_mols
