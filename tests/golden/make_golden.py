"""Generate golden vectors by running the REFERENCE implementation.

Run in the build container only (the reference is not present on GPU boxes):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own modules from /root/reference
(enflow.nn.egcl.EGCL, enflow.nn.argmax.ArgMax, enflow.flow.dynamics.LFIntegrator,
enflow.flow.loss.Alchemical_NLL, enflow.utils.helpers) and runs them in
float64 on synthetic molecules.  ``enflow.data.base`` cannot be imported (its
import chain needs rdkit, which is absent), so ``RefData`` below restates the
batch container's edge / pbc / iteration behaviour (enflow/data/base.py:9-144)
around the reference's own ``get_periodic_images_within`` and ``apply_pbc``.

All inputs are float32-representable (weights come from torch's float32
nn.Linear init; positions etc. are rounded through float32) so the fp32 HIP
path sees bit-identical inputs.  Inputs are stored as float32, reference
outputs as float64, in one .npz per case.
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from enflow.nn.egcl import EGCL  # noqa: E402  (reference)
from enflow.nn.argmax import ArgMax  # noqa: E402  (reference)
from enflow.flow.dynamics import LFIntegrator  # noqa: E402  (reference)
from enflow.flow.loss import Alchemical_NLL  # noqa: E402  (reference)
from enflow.utils import helpers  # noqa: E402  (reference)

from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT  # noqa: E402


class RefEdges:
    """Restates enflow/data/base.py:9-19 (Edges)."""

    def __init__(self, edge_index, box, coord):
        self.box = box
        self.row, self.col = edge_index
        self.coord = coord

    @property
    def coord_diff(self):
        d = self.coord[self.row] - self.coord[self.col]
        return helpers.apply_pbc(d, self.box * 0.5)


class RefData:
    """Restates the parts of enflow/data/base.py:21-144 (Data) the flow uses."""

    def __init__(self, h, g, pos, vel, box, r_cut, N):
        self.h, self.g, self.pos, self.vel = h, g, pos, vel
        self.box, self.r_cut, self.N = box, r_cut, N

    def _mol(self, i):
        s = int(self.N[:i].sum())
        e = s + int(self.N[i])
        return RefData(self.h[s:e], self.g[s:e], self.pos[s:e], self.vel[s:e],
                       self.box[s:e], self.r_cut[i], self.N[i])

    def __iter__(self):
        return (self._mol(i) for i in range(len(self.N)))

    @property
    def num_atoms(self):
        return int(self.N.sum())

    @property
    def num_mols(self):
        return len(self.N)

    def pbc(self):
        self.pos = helpers.apply_pbc(self.pos, self.box)

    @property
    def edges(self):
        edge_index = torch.empty((2, 0), dtype=torch.long)
        boxes = []
        n_cnt = 0
        for mol in self:
            box = mol.box[0]
            imgs, id_mapping = helpers.get_periodic_images_within(mol.pos, box, mol.r_cut)
            r_sq = mol.r_cut * mol.r_cut
            d2 = (imgs.unsqueeze(1) - mol.pos).pow(2).sum(dim=2)
            ids = (d2 < r_sq).nonzero()
            e = id_mapping[ids] + n_cnt
            e = e[torch.nonzero(e[:, 0] - e[:, 1])].squeeze(1)
            boxes.append(box.repeat(e.shape[0], 1))
            edge_index = torch.cat((edge_index, e.T.long()), dim=1)
            n_cnt += int(mol.N)
        return RefEdges(edge_index, torch.cat(boxes), self.pos)


def f32(x):
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def to_t(x):
    return torch.tensor(x, dtype=torch.float64)


def batch_inputs(num_mols, n_atoms, nf, seed, box_ang=None, r_cut_ang=3.0, one_hot=True):
    b = make_molecules(num_mols, n_atoms, nf=nf, seed=seed, box_ang=box_ang, r_cut_ang=r_cut_ang)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = f32(b[k])
    if not one_hot:
        rng = np.random.default_rng(seed + 17)
        b["h"] = f32(rng.normal(size=b["h"].shape))
    return b


def ref_data(b):
    n = torch.tensor(np.diff(b["mol_ptr"]))
    return RefData(to_t(b["h"]), to_t(b["g"]), to_t(b["pos"]), to_t(b["vel"]),
                   to_t(b["box"]), to_t(b["r_cut"]), n)


def params_of(module, prefix):
    return {f"{prefix}{k}": v.detach().numpy().astype(np.float32)
            for k, v in module.state_dict().items()}


def save(name, inputs, outputs):
    out = {}
    for k, v in inputs.items():
        v = np.asarray(v)
        # act_fn codes keep their float64 parameters (the reference's module holds doubles)
        keep = k.endswith(".act")
        out["in_" + k] = v.astype(np.float32) if (v.dtype.kind == "f" and v.ndim > 0 and not keep) else v
    for k, v in outputs.items():
        out["out_" + k] = np.asarray(v, dtype=np.float64) if np.asarray(v).dtype.kind == "f" else np.asarray(v)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) // 1024} KiB)")


def case_edges():
    """Neighbour lists: default (extent) boxes, a large box, a small box."""
    for tag, kw in (("extent", {}), ("box20", {"box_ang": 20.0}), ("box5", {"box_ang": 5.0})):
        b = batch_inputs(6, [22, 9, 15, 3, 30, 22], 5, seed=11, **kw)
        d = ref_data(b)
        e = d.edges
        save(f"edges_{tag}", b, {"row": e.row.numpy(), "col": e.col.numpy(),
                                 "coord_diff": e.coord_diff.numpy()})


def act_fn_of(code):
    """torch activation module of an ENFLOW_ACT_* code (kind, p0, p1)."""
    from torch import nn
    k, p0, p1 = code
    return [nn.SiLU, nn.ReLU, lambda: nn.LeakyReLU(p0), lambda: nn.ELU(p0), lambda: nn.CELU(p0), nn.SELU,
            nn.GELU, lambda: nn.GELU(approximate="tanh"), nn.Tanh, nn.Sigmoid, lambda: nn.Softplus(p0, p1),
            nn.Mish, lambda: nn.Hardtanh(p0, p1), nn.Identity][k]()


def case_egcl(hid, seed, nf=5, name=None, act=None):
    torch.manual_seed(seed)
    net = (EGCL(nf, nf, hid) if act is None else EGCL(nf, nf, hid, act_fn=act_fn_of(act))).double()
    b = batch_inputs(4, [22, 9, 15, 3], nf, seed=seed, one_hot=False)
    d = ref_data(b)
    q, f, g = net(d.h, d.edges)
    inp = dict(b)
    inp.update(params_of(net, "p0."))
    if act is not None:
        inp["p0.act"] = np.array(act, dtype=np.float64)
    save(name or f"egcl_h{hid}", inp, {"Q": q.detach().numpy(), "F": f.detach().numpy(),
                                       "G": g.detach().numpy()})


def case_egcl_variant(hid, seed, flags, name):
    """EGCL with the constructor variants (attention, norm_diff, tanh)."""
    torch.manual_seed(seed)
    nf = 5
    att, nd, th = flags
    net = EGCL(nf, nf, hid, attention=att, norm_diff=nd, tanh=th).double()
    b = batch_inputs(4, [22, 9, 15, 3], nf, seed=seed, one_hot=False)
    d = ref_data(b)
    q, f, g = net(d.h, d.edges)
    inp = dict(b)
    inp.update(params_of(net, "p0."))
    inp["p0.flags"] = np.array(flags, dtype=np.int32)
    save(name, inp, {"Q": q.detach().numpy(), "F": f.detach().numpy(), "G": g.detach().numpy()})


def case_argmax(hid, seed):
    torch.manual_seed(seed)
    nf = 5
    am = ArgMax(nf, hid).double()
    b = batch_inputs(3, [22, 9, 15], nf, seed=seed)
    h = to_t(b["h"])
    torch.manual_seed(seed + 1)
    z, log_q = am(h)
    torch.manual_seed(seed + 1)
    eps = torch.randn(h.size())
    inp = {"h": b["h"], "mol_ptr": b["mol_ptr"], "eps": eps.numpy()}
    inp.update(params_of(am, "dq."))
    rev = am.reverse(z.detach())
    save(f"argmax_h{hid}", inp, {"z": z.detach().numpy(), "log_q": float(log_q),
                                 "reverse": rev.numpy()})


def case_flow(hid, n_layers, sizes, seed, name, flags=None, nf=5, act=None, dq_act=None):
    """``flags``: per layer (attention, norm_diff, tanh), default flags when None;
    ``act`` / ``dq_act``: act_fn codes of the EGCL layers / the ArgMax (None: SiLU)."""
    torch.manual_seed(seed)
    dt = default_dt()
    akw = {} if act is None else {"act_fn": act_fn_of(act)}
    if flags is None:
        nets = [EGCL(nf, nf, hid, **akw) for _ in range(n_layers)]
    else:
        nets = [EGCL(nf, nf, hid, attention=a, norm_diff=nd, tanh=th, **akw) for a, nd, th in flags]
    am = ArgMax(nf, hid) if dq_act is None else ArgMax(nf, hid, act_fn=act_fn_of(dq_act))
    model = LFIntegrator(nets, am, dt=dt)   # BaseFlow casts to float64
    b = batch_inputs(len(sizes), sizes, nf, seed=seed)
    d = ref_data(b)
    torch.manual_seed(seed + 1)
    eps = torch.randn(d.h.size())
    torch.manual_seed(seed + 1)
    with torch.no_grad():
        out, ldj = model(d)
    kBT = default_kBT()
    nll = Alchemical_NLL(kBT=kBT, softening=0.1)
    with torch.no_grad():
        loss = nll(out, ldj)
    fwd = {"h": out.h.numpy().copy(), "g": out.g.numpy().copy(), "pos": out.pos.numpy().copy(),
           "vel": out.vel.numpy().copy(), "ldj": float(ldj), "nll": float(loss)}
    # generate direction: reverse of the forward output (main.py:263-278)
    with torch.no_grad():
        back = model.reverse(out)
    rev = {"rev_h": back.h.numpy(), "rev_g": back.g.numpy(), "rev_pos": back.pos.numpy(),
           "rev_vel": back.vel.numpy()}
    inp = dict(b)
    inp["eps"] = eps.numpy()
    inp["dt"] = np.array(dt)
    inp["kBT"] = np.array(kBT)
    inp["softening"] = np.array(0.1)
    inp["n_layers"] = np.array(n_layers)
    inp["hid"] = np.array(hid)
    for i, net in enumerate(model.networks):
        inp.update(params_of(net, f"p{i}."))
        if flags is not None:
            inp[f"p{i}.flags"] = np.array(flags[i], dtype=np.int32)
        if act is not None:
            inp[f"p{i}.act"] = np.array(act, dtype=np.float64)
    inp.update(params_of(model.dequantize, "dq."))
    if dq_act is not None:
        inp["dq.act"] = np.array(dq_act, dtype=np.float64)
    fwd.update(rev)
    save(name, inp, fwd)


def case_train(hid, n_layers, sizes, seed, name, nf=5, flags=None, act=None, dq_act=None):
    """One training step of the reference (enflow/main.py:217-221):
    out, ldj = model(data); loss = nll(out, ldj); loss.backward() -- the
    parameter gradients of every EGCL layer and of the ArgMax dequantiser.
    ``flags``: per layer (attention, norm_diff, tanh), default flags when None."""
    torch.manual_seed(seed)
    dt = default_dt()
    akw = {} if act is None else {"act_fn": act_fn_of(act)}
    if flags is None:
        nets = [EGCL(nf, nf, hid, **akw) for _ in range(n_layers)]
    else:
        nets = [EGCL(nf, nf, hid, attention=a, norm_diff=nd, tanh=th, **akw) for a, nd, th in flags]
    am = ArgMax(nf, hid) if dq_act is None else ArgMax(nf, hid, act_fn=act_fn_of(dq_act))
    model = LFIntegrator(nets, am, dt=dt)   # BaseFlow casts to float64
    b = batch_inputs(len(sizes), sizes, nf, seed=seed)
    d = ref_data(b)
    torch.manual_seed(seed + 1)
    eps = torch.randn(d.h.size())
    torch.manual_seed(seed + 1)
    out, ldj = model(d)
    kBT = default_kBT()
    nll = Alchemical_NLL(kBT=kBT, softening=0.1)
    loss = nll(out, ldj)
    loss.backward()
    inp = dict(b)
    inp["eps"] = eps.numpy()
    inp["dt"] = np.array(dt)
    inp["kBT"] = np.array(kBT)
    inp["softening"] = np.array(0.1)
    inp["n_layers"] = np.array(n_layers)
    inp["hid"] = np.array(hid)
    res = {"loss": float(loss), "ldj": float(ldj)}
    for i, net in enumerate(model.networks):
        inp.update({f"p{i}.{k}": v.detach().numpy().astype(np.float32) for k, v in net.named_parameters()})
        res.update({f"grad_p{i}.{k}": v.grad.numpy() for k, v in net.named_parameters()})
        if flags is not None:
            inp[f"p{i}.flags"] = np.array(flags[i], dtype=np.int32)
        if act is not None:
            inp[f"p{i}.act"] = np.array(act, dtype=np.float64)
    inp.update({f"dq.{k}": v.detach().numpy().astype(np.float32)
                for k, v in model.dequantize.named_parameters()})
    if dq_act is not None:
        inp["dq.act"] = np.array(dq_act, dtype=np.float64)
    res.update({f"grad_dq.{k}": v.grad.numpy() for k, v in model.dequantize.named_parameters()})
    save(name, inp, res)


def case_few_images():
    """Fewer surviving periodic images than atoms (helpers.py:15-29 keeps only
    images inside the box + r_cut ellipsoid).  The reference's Data.edges
    (base.py:137) indexes id_mapping with the ATOM column q of every hit, so it
    raises IndexError iff some hit has q >= len(id_mapping); without such a hit
    it returns the (possibly empty) edge list.  Two single-molecule cases: one
    that raises, one that does not."""
    box = [3.0, 3.0, 3.0]
    far = [[40.0 + i, 40.0, 40.0] for i in range(9)]
    for tag, pos in (("raise", far + [[3.2, 0.1, 0.2]]), ("quiet", [[3.2, 0.1, 0.2]] + far)):
        n = len(pos)
        b = {"h": np.eye(5)[np.arange(n) % 5], "g": np.zeros((n, 5)), "pos": f32(pos), "vel": np.zeros((n, 3)),
             "box": f32(np.tile(box, (n, 1))), "r_cut": f32([1.0]), "mol_ptr": np.array([0, n])}
        d = ref_data(b)
        try:
            e = d.edges
            out = {"raised": 0, "row": e.row.numpy(), "col": e.col.numpy()}
        except IndexError:
            out = {"raised": 1, "row": np.zeros(0, np.int64), "col": np.zeros(0, np.int64)}
        save(f"edges_fewimg_{tag}", b, out)


def case_egcl_grad(hid, seed, flags, name):
    """A standalone EGCL.forward trained directly (the reference module is an
    ordinary autograd module, egcl.py:76-92): loss = sum(Q wq) + sum(F wf) +
    sum(G wg) with fixed random weights; gradients of every parameter, of h and
    of the positions (through Edges.coord_diff)."""
    torch.manual_seed(seed)
    nf = 5
    att, nd, th = flags
    net = EGCL(nf, nf, hid, attention=att, norm_diff=nd, tanh=th).double()
    b = batch_inputs(4, [22, 9, 15, 3], nf, seed=seed, one_hot=False)
    d = ref_data(b)
    rng = np.random.default_rng(seed + 5)
    n = d.h.shape[0]
    wq, wf, wg = (f32(rng.normal(size=s_)) for s_ in ((n, 1), (n, 3), (n, nf)))
    d.h.requires_grad_(True)
    d.pos.requires_grad_(True)
    q, f, g = net(d.h, d.edges)
    loss = (q * to_t(wq)).sum() + (f * to_t(wf)).sum() + (g * to_t(wg)).sum()
    loss.backward()
    inp = dict(b)
    inp.update(params_of(net, "p0."))
    inp["p0.flags"] = np.array(flags, dtype=np.int32)
    inp.update({"wq": wq, "wf": wf, "wg": wg})
    res = {"loss": float(loss), "grad_h": d.h.grad.numpy(), "grad_pos": d.pos.grad.numpy()}
    res.update({f"grad_p0.{k}": v.grad.numpy() for k, v in net.named_parameters()})
    save(name, inp, res)


def case_argmax_grad(hid, seed):
    """A standalone ArgMax.forward (argmax.py:13-25) trained directly: loss =
    sum(z wz) + 0.7 log_q; gradients of the network parameters."""
    torch.manual_seed(seed)
    nf = 5
    am = ArgMax(nf, hid).double()
    b = batch_inputs(3, [22, 9, 15], nf, seed=seed)
    h = to_t(b["h"])
    torch.manual_seed(seed + 1)
    z, log_q = am(h)
    torch.manual_seed(seed + 1)
    eps = torch.randn(h.size())
    wz = f32(np.random.default_rng(seed + 2).normal(size=tuple(h.shape)))
    loss = (z * to_t(wz)).sum() + 0.7 * log_q
    loss.backward()
    inp = {"h": b["h"], "mol_ptr": b["mol_ptr"], "eps": eps.numpy(), "wz": wz}
    inp.update(params_of(am, "dq."))
    res = {"loss": float(loss)}
    res.update({f"grad_dq.{k}": v.grad.numpy() for k, v in am.named_parameters()})
    save(f"argmax_grad_h{hid}", inp, res)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "module_grads":
        case_egcl_grad(32, 51, (False, False, False), "egcl_grad_h32")
        case_egcl_grad(128, 52, (False, False, False), "egcl_grad_h128")
        case_egcl_grad(64, 53, (True, True, True), "egcl_grad_h64_all")
        case_argmax_grad(32, 54)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "fewimg":
        case_few_images()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "train_variants":
        case_train(64, 2, [22, 40, 7], 41, "train_var_h64_L2", flags=[(False, True, True), (False, False, True)])
        case_train(32, 3, [22, 9, 15, 3], 42, "train_var_h32_L3",
                   flags=[(False, True, False), (False, True, True), (False, False, False)])
        case_train(64, 2, [22, 40, 7], 43, "train_att_h64_L2", flags=[(True, False, False), (True, True, True)])
        case_train(32, 3, [22, 9, 15, 3], 44, "train_att_h32_L3",
                   flags=[(True, False, False), (False, True, False), (True, False, True)])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "variants":
        case_egcl_variant(64, 31, (True, False, False), "egcl_h64_att")
        case_egcl_variant(32, 32, (False, True, True), "egcl_h32_nd_tanh")
        case_egcl_variant(128, 33, (True, True, True), "egcl_h128_all")
        case_flow(64, 3, [22, 9, 15, 3], 34, "lf_var_h64_L3",
                  flags=[(True, False, False), (False, True, True), (True, True, True)])
        case_flow(128, 2, [22, 22, 30], 35, "lf_var_h128_L2", flags=[(False, True, False), (True, False, True)])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "act":
        # act_fn other than SiLU (enflow/nn/egcl.py:11, enflow/nn/argmax.py:7); codes
        # (kind, p0, p1) as ENFLOW_ACT_*: every kind through one EGCL forward each
        codes = {"relu": (1, 0, 0), "leaky": (2, 0.05, 0), "elu": (3, 0.7, 0), "celu": (4, 1.3, 0),
                 "selu": (5, 0, 0), "gelu": (6, 0, 0), "gelutanh": (7, 0, 0), "tanh": (8, 0, 0),
                 "sigmoid": (9, 0, 0), "softplus": (10, 1.5, 20.0), "mish": (11, 0, 0), "relu6": (12, 0.0, 6.0),
                 "identity": (13, 0, 0)}
        for i, (tag, code) in enumerate(codes.items()):
            case_egcl(32, 70 + i, act=code, name=f"egcl_act_{tag}")
        case_flow(64, 2, [22, 9, 15], 90, "lf_act_tanh_h64_L2", act=(8, 0, 0), dq_act=(8, 0, 0))
        case_flow(128, 2, [22, 13], 91, "lf_act_gelu_h128_L2", act=(6, 0, 0), dq_act=(9, 0, 0))
        case_train(32, 2, [22, 9, 15], 92, "train_act_tanh_h32_L2", act=(8, 0, 0), dq_act=(8, 0, 0))
        case_train(64, 2, [22, 17], 93, "train_act_elu_h64_L2", act=(3, 0.7, 0), dq_act=(10, 1.5, 20.0),
                   flags=[(True, True, False), (False, False, True)])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "wide_nf":
        # node_nf past 8 (the dataset decides it: enflow/main.py:148-151): the
        # 16-feature build (libenflow_hip_nf16.so)
        case_flow(64, 2, [22, 9, 15], 61, "lf_nf12_h64_L2", nf=12)
        case_flow(32, 2, [22, 13], 62, "lf_nf16_h32_L2", nf=16)
        case_egcl(128, 63, nf=16, name="egcl_nf16_h128")
        case_train(32, 2, [22, 9, 15], 64, "train_nf12_h32_L2", nf=12)
        case_train(128, 2, [22, 17], 65, "train_nf15_h128_L2", nf=15)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "nf16_train":
        # node_nf 16 training (2 nf + 1 = 33 edge_nn.0 inputs: the radial row past
        # the transposed GEMM's 32-row tile)
        case_train(64, 2, [22, 17], 66, "train_nf16_h64_L2", nf=16)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "train":
        case_train(32, 3, [22, 9, 15, 3], 21, "train_h32_L3")
        case_train(128, 2, [22, 22], 22, "train_h128_L2")
        case_train(64, 2, [22, 40, 7], 23, "train_h64_L2")
        sys.exit(0)
    case_edges()
    case_egcl(32, 3)
    case_egcl(128, 4)
    case_argmax(32, 5)
    case_flow(32, 3, [22, 9, 15, 3], 7, "lf_h32_L3")
    case_flow(64, 2, [22, 22, 30], 8, "lf_h64_L2")
    case_flow(128, 2, [22, 22], 9, "lf_h128_L2")
