"""CPU gradient oracle for the enflow training step -- TEST INFRASTRUCTURE ONLY.

Float64 torch restatement of the reference's training loss
(enflow/main.py:217-221: ``out, ldj = model(data); loss = nll(out, ldj);
loss.backward()``) so that parameter gradients of any batch can be checked.
Only ``tests/`` may import it; the product path (``enflow_amd``) never does.

The continuous part (EGCL, leapfrog, ArgMax, Alchemical_NLL) is restated with
torch ops so autograd yields the gradients; the neighbour lists are the
integer output of the numpy oracle (``enflow_oracle.batch_edges``), which
carry no gradient in the reference either (they index, the reference
differentiates through ``Edges.coord_diff`` only).

Parity pinning: tests/test_oracle_golden.py checks the loss and every
parameter gradient against golden vectors produced by running the reference's
own modules and ``loss.backward()`` (tests/golden/make_golden.py ``train``).
"""
import math

import numpy as np
import torch

from . import enflow_oracle as O

F = torch.nn.functional


def _silu(x):
    return x * torch.sigmoid(x)


def _activation(code):
    """torch form of enflow_oracle.activation (same numbering)."""
    if code is None:
        return _silu
    k, p0, p1 = int(code[0]), float(code[1]), float(code[2])
    table = {
        0: _silu, 1: F.relu, 2: lambda x: F.leaky_relu(x, p0), 3: lambda x: F.elu(x, p0),
        4: lambda x: F.celu(x, p0), 5: F.selu, 6: lambda x: F.gelu(x), 7: lambda x: F.gelu(x, approximate="tanh"),
        8: torch.tanh, 9: torch.sigmoid, 10: lambda x: F.softplus(x, p0, p1), 11: F.mish,
        12: lambda x: F.hardtanh(x, p0, p1), 13: lambda x: x,
    }
    return table[k]


def _pbc(x, box):
    """enflow/utils/helpers.py:7-8 (round has zero gradient)."""
    return x - torch.round(x / box) * box


def _egcl(p, h, pos, row, col, eb, n, cw, flags=(False, False, False), act=None):
    """EGCL.forward (enflow/nn/egcl.py:57-92); ``flags`` = the constructor's
    (attention, norm_diff, tanh)."""
    attention, norm_diff, tanh = (bool(x) for x in flags)
    _silu = _activation(act)                                                   # act_fn (egcl.py:11)
    cd = _pbc(pos[row] - pos[col], eb * 0.5)                                   # base.py:15-19
    radial = (cd ** 2).sum(1, keepdim=True)
    if norm_diff:                                                              # egcl.py:82-84
        cd = cd / (torch.sqrt(radial) + 1)
    x = torch.cat([h[row], h[col], radial], 1)
    e = _silu(F.linear(_silu(F.linear(x, p["edge_nn.0.weight"], p["edge_nn.0.bias"])),
                       p["edge_nn.2.weight"], p["edge_nn.2.bias"]))
    if attention:                                                              # egcl.py:60-62
        e = e * torch.sigmoid(F.linear(e, p["att_nn.0.weight"], p["att_nn.0.bias"]))
    q = F.linear(_silu(F.linear(h, p["vel_scaling_nn.0.weight"], p["vel_scaling_nn.0.bias"])),
                 p["vel_scaling_nn.2.weight"], p["vel_scaling_nn.2.bias"])
    phi = F.linear(_silu(F.linear(e, p["coord_nn.0.weight"], p["coord_nn.0.bias"])), p["coord_nn.2.weight"])
    if tanh:                                                                   # egcl.py:40-42
        phi = torch.tanh(phi)
    trans = torch.clamp(cd * phi, -100.0, 100.0)
    idx = row.unsqueeze(1).expand(-1, 3)
    fs = torch.zeros(n, 3, dtype=h.dtype).scatter_add(0, idx, trans)
    cnt = torch.zeros(n, 3, dtype=h.dtype).scatter_add(0, idx, torch.ones_like(trans))
    f = fs / cnt.clamp(min=1) * cw                                              # helpers.py:63-70
    agg = torch.zeros(n, e.shape[1], dtype=h.dtype).scatter_add(0, row.unsqueeze(1).expand(-1, e.shape[1]), e)
    g = F.linear(_silu(F.linear(torch.cat([h, agg], 1), p["node_nn.0.weight"], p["node_nn.0.bias"])),
                 p["node_nn.2.weight"], p["node_nn.2.bias"])
    return q, f, g


def _argmax(p, h, eps, act=None):
    """ArgMax.forward (enflow/nn/argmax.py:13-25)."""
    nf = h.shape[1]
    net = F.linear(_activation(act)(F.linear(h, p["network.0.weight"], p["network.0.bias"])),
                   p["network.2.weight"], p["network.2.bias"])
    ls, tr = net[:, :nf], net[:, nf:]
    u = tr + eps * ls.exp()
    log_q = -0.5 * ((u ** 2).sum() + math.log(2 * math.pi)) - ls.sum()
    t = (h * u).sum(-1, keepdim=True)
    z = h * u + (1 - h) * (t - F.softplus(t - u))
    return z, log_q - ((1 - h) * F.logsigmoid(t - u)).sum()


def _nll(h, g, pos, vel, ldj, mol_ptr, kBT, softening, partition_func):
    """Alchemical_NLL.__call__ (enflow/flow/loss.py:11-24)."""
    lj = 0.0
    for m in range(len(mol_ptr) - 1):
        x = pos[int(mol_ptr[m]):int(mol_ptr[m + 1])]
        d2 = torch.triu((x.unsqueeze(1) - x).pow(2).sum(2))
        r2 = d2[d2 != 0] + softening
        r6 = r2.pow(3)
        lj = lj + 4 * (1 / r6.pow(2) - 1 / r6).sum()
    Hn = lj + 0.5 * (vel ** 2).sum()
    num_atoms, num_mols = int(mol_ptr[-1]), len(mol_ptr) - 1
    logZ = -num_atoms * (math.log(partition_func) - 1.5 * math.log(2 * math.pi / kBT))
    lg = lambda z: -0.5 * ((z ** 2).sum() + math.log(2 * math.pi))  # noqa: E731
    return -(-Hn / kBT + logZ + ldj + lg(h) + lg(g)) / num_mols


def train_loss_and_grads(layers, dequant, state, eps, dt, kBT, softening, partition_func=10.0,
                         coords_weight=1.0, dequant_kind="argmax", dtype=torch.float64):
    """Loss of one training step and d loss / d parameter for every EGCL layer
    (list of dicts, EGCL_PARAM_NAMES) and the ArgMax dequantiser (dict).
    dequant_kind "floor" (enflow/nn/floor.py:15-16): h + dequant_scale * eps with
    eps the U[0, 1) draw, log|detJ| starts at 0; ``dequant`` is then the scale
    and the dequantiser gradient dict is empty.

    dtype: the arithmetic (default float64, the reference's; float32 measures
    what rounding alone does to the gradients -- the neighbour lists are then
    still built from float64 positions, so both runs see the same edges).

    Returns (loss, ldj, [layer grad dicts], dequant grad dict, output state)."""
    t = lambda a: torch.tensor(np.asarray(a, dtype=np.float64)).to(dtype)  # noqa: E731
    P = [{k: t(v).requires_grad_(True) for k, v in p.items() if k not in ("flags", "act")} for p in layers]
    floor = dequant_kind == "floor"
    D = {} if floor else {k: t(v).requires_grad_(True) for k, v in dequant.items() if k != "act"}
    mol_ptr = np.asarray(state["mol_ptr"], dtype=np.int64)
    n = int(mol_ptr[-1])
    box, r_cut = t(state["box"]), np.asarray(state["r_cut"], dtype=np.float64)
    if floor:
        h, ldj = t(state["h"]) + float(dequant) * t(eps), t(0.0)
    else:
        h, ldj = _argmax(D, t(state["h"]), t(eps), dequant.get("act"))
    g, pos, vel = t(state["g"]), t(state["pos"]), t(state["vel"])
    for p, lp in zip(P, layers):
        row, col, eb = O.batch_edges(pos.detach().double().numpy(), state["box"], r_cut, mol_ptr)
        row_t, col_t = torch.as_tensor(row, dtype=torch.long), torch.as_tensor(col, dtype=torch.long)
        q, f, gg = _egcl(p, h, pos, row_t, col_t, t(eb), n, coords_weight, lp.get("flags", (0, 0, 0)), lp.get("act"))
        vel = torch.exp(q) * vel + f * dt
        g = g + gg * dt
        pos = _pbc(pos + vel * dt, box)
        h = h + g * dt
        ldj = ldj + q.sum()
    loss = _nll(h, g, pos, vel, ldj, mol_ptr, kBT, softening, partition_func)
    loss.backward()
    gl = [{k: v.grad.double().numpy() for k, v in p.items()} for p in P]
    gd = {k: v.grad.double().numpy() for k, v in D.items()}
    out = {"h": h.detach().double().numpy(), "g": g.detach().double().numpy(), "pos": pos.detach().double().numpy(),
           "vel": vel.detach().double().numpy()}
    return float(loss), float(ldj), gl, gd, out
