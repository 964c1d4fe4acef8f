"""EGCL message-passing block (mirrors enflow/nn/egcl.py:6-92).

Same constructor, same sub-module and parameter names (edge_nn, node_nn,
coord_nn, vel_scaling_nn) and the same initialisation order, so a reference
state_dict loads unchanged and a given torch seed yields the same weights.
``forward(h, edges)`` returns (Q [n, 1], F [n, 3], G [n, nf]) computed by
enflow_egcl_forward_f32: neighbour list, per-edge MLP chain on MFMA and the
segment reductions all run in one HIP kernel per molecule.
"""
import torch
from torch import nn

from .. import _lib
from ..data.base import Edges
from ._act import SILU, act_code, act_kind, check_trainable, supported as act_supported
from ._pad import EGCL_HDIMS, Geom, flat_padded, kernel_hidden
from ..utils.helpers import params_of


class EGCL(nn.Module):
    def __init__(self, input_nf, output_nf, hidden_nf, act_fn=nn.SiLU(), coords_weight=1.0,
                 attention=False, clamp=False, norm_diff=False, tanh=False):
        super().__init__()
        input_edge = input_nf * 2
        self.input_nf, self.output_nf, self.hidden_nf = input_nf, output_nf, hidden_nf
        self.coords_weight = coords_weight
        self.attention = attention
        self.norm_diff = norm_diff
        self.tanh = tanh
        # the reference never registers act_fn as a child of its own (egcl.py:11-55):
        # a parameterised activation's weights appear only inside the Sequentials
        # (PReLU: edge_nn.1.weight, after edge_nn.0.bias), so state_dict keys and
        # parameter order stay the reference's
        object.__setattr__(self, "act_fn", act_fn)
        edge_coords_nf = 1
        # construction order = reference order (egcl.py:12-55): same RNG stream
        self.edge_nn = nn.Sequential(nn.Linear(input_edge + edge_coords_nf, hidden_nf), act_fn,
                                     nn.Linear(hidden_nf, hidden_nf), act_fn)
        self.node_nn = nn.Sequential(nn.Linear(hidden_nf + input_nf, hidden_nf), act_fn,
                                     nn.Linear(hidden_nf, output_nf))
        layer = nn.Linear(hidden_nf, 1, bias=False)
        torch.nn.init.xavier_uniform_(layer.weight, gain=0.001)
        self.clamp = clamp
        coord_nn = [nn.Linear(hidden_nf, hidden_nf), act_fn, layer]
        if self.tanh:
            coord_nn.append(nn.Tanh())
            self.coords_range = nn.Parameter(torch.ones(1)) * 3
        self.coord_nn = nn.Sequential(*coord_nn)
        if self.attention:
            self.att_nn = nn.Sequential(nn.Linear(hidden_nf, 1), nn.Sigmoid())
        self.vel_scaling_nn = nn.Sequential(nn.Linear(input_nf, hidden_nf), act_fn,
                                            nn.Linear(hidden_nf, 1))
        self._packed = None
        self._packed_key = None

    # ------------------------------------------------------------------
    @property
    def kernel_hidden(self):
        """The compiled hidden width this layer runs at: hidden_nf, or the next
        of 32 / 64 / 128 with the extra units zero-padded (exact, nn/_pad.py)."""
        return kernel_hidden(self.hidden_nf)

    @property
    def kernel_nf(self):
        """The kernels' node-feature width: max(input_nf, output_nf), the
        narrower side zero-padded (exact, nn/_pad.py)."""
        return max(self.input_nf, self.output_nf)

    def pad_geom(self):
        return Geom(self.hidden_nf, self.kernel_hidden, self.input_nf, self.output_nf, self.kernel_nf)

    def hip_supported(self):
        """The HIP kernels implement every constructor flag of the reference
        (attention, norm_diff, tanh; ``clamp`` is stored and unused there too)
        with the activations of nn/_act.py (SiLU, ReLU, LeakyReLU, PReLU, ELU, CELU,
        SELU, GELU, Tanh, Sigmoid, Softplus, Mish, Hardtanh / ReLU6, Identity),
        input_nf and output_nf <= 16 and any hidden_nf
        <= 128 (hidden 32 / 64 / 128 and one feature width compiled, other
        shapes zero-padded)."""
        kh = self.kernel_hidden
        if not (act_supported(self.act_fn) and 1 <= min(self.input_nf, self.output_nf)
                and self.kernel_nf <= _lib.MAX_NODE_NF and kh is not None):
            return False
        L = _lib.lib(self.kernel_nf)
        return self.kernel_nf <= L.enflow_max_node_nf() and bool(L.enflow_supports_hidden(kh))

    def _check_supported(self):
        if not self.hip_supported():
            raise NotImplementedError(
                "enflow_amd EGCL kernels implement the torch activations of nn/_act.py, input_nf / output_nf <= 16 "
                "and hidden_nf <= 128")

    def variant_flags(self):
        """ENFLOW_EGCL_* flags of this layer's constructor variants (0 = defaults)."""
        return ((_lib.EGCL_ATTENTION if self.attention else 0) | (_lib.EGCL_NORM_DIFF if self.norm_diff else 0)
                | (_lib.EGCL_TANH if self.tanh else 0) | (_lib.EGCL_ACT if act_kind(self.act_fn) != SILU else 0))

    def act(self):
        """(kind, p0, p1) of act_fn (ENFLOW_ACT_*)."""
        return act_code(self.act_fn)

    def raw_named(self):
        """(name, parameter) in the default-flag named_parameters() order the C
        ABI expects (att_nn, present with attention=True, travels separately;
        act_fn's own parameters -- a PReLU slope, named edge_nn.1.weight as in the
        reference -- travel in the act code)."""
        own = self.act_param_ids()
        return [(k, p) for k, p in self.named_parameters() if not k.startswith("att_nn.") and id(p) not in own]

    def act_param_ids(self):
        """ids of act_fn's parameters (shared by every position of the block)."""
        return {id(p) for p in self.act_fn.parameters()}

    def raw_parameters(self):
        return [p for _, p in self.raw_named()]

    def kernel_raw(self, device):
        """The raw parameters as one flat fp32 vector at the kernel width."""
        return flat_padded(self.raw_named(), EGCL_HDIMS, self.pad_geom(), device)

    def _att_raw(self, device):
        """att_nn.0 weight [kernel width] + bias [1] (None without attention)."""
        if not self.attention:
            return None
        return flat_padded([(k, p) for k, p in self.named_parameters() if k.startswith("att_nn.")],
                           EGCL_HDIMS, self.pad_geom(), device)

    def _pack(self, raw, dst, device):
        L = _lib.lib(self.kernel_nf)
        att = self._att_raw(device)
        kind, p0, p1 = self.act()
        if kind == SILU:   # the ABI <= 9 entry (A/B tools load older builds too)
            _lib.check(L.enflow_pack_egcl_ex_f32(_lib.ptr(raw), self.kernel_hidden, self.kernel_nf,
                                                 self.variant_flags(), _lib.ptr(att), _lib.ptr(dst),
                                                 _lib.stream_ptr(device)), "enflow_pack_egcl_ex_f32")
            return
        _lib.check(L.enflow_pack_egcl_act_f32(_lib.ptr(raw), self.kernel_hidden, self.kernel_nf, self.variant_flags(),
                                              kind, p0, p1, _lib.ptr(att), _lib.ptr(dst), _lib.stream_ptr(device)),
                   "enflow_pack_egcl_act_f32")

    def packed(self, device):
        """MFMA-fragment packed fp32 weights on `device` (cached, re-packed when
        any parameter changes)."""
        key = (str(device),) + tuple((p.data_ptr(), p._version) for p in params_of(self))
        if self._packed is not None and self._packed_key == key:
            return self._packed
        L = _lib.lib(self.kernel_nf)
        raw = self.kernel_raw(device)
        size = L.enflow_egcl_packed_size(self.kernel_hidden, self.kernel_nf)
        out = torch.empty(size, dtype=torch.float32, device=device)
        self._pack(raw, out, device)
        self._packed, self._packed_key = out, key
        return out

    def pack_into(self, dst):
        """Pack into a slice of a caller-owned buffer (used by the fused flow)."""
        device = dst.device
        self._pack(self.kernel_raw(device), dst, device)

    # ------------------------------------------------------------------
    def _meta(self, edges, dev):
        return dict(mol_ptr=edges.mol_ptr, max_n=edges.max_mol_atoms, N=edges.N, num_mols=edges.num_mols,
                    box=edges.box.detach().to(device=dev, dtype=torch.float32).contiguous(),
                    r_cut=torch.as_tensor(edges.r_cut, device=dev).to(torch.float32).reshape(-1).contiguous())

    def _infer(self, h, pos, meta):
        """EGCL.forward on the HIP kernels: (Q [n, 1], F [n, 3], G [n, nf]) fp32."""
        L = _lib.lib(self.kernel_nf)
        dev = h.device
        n = h.shape[0]
        nf = self.kernel_nf
        hf = self.pad_h(h)
        pos = pos.to(torch.float32).contiguous()
        Q = torch.empty(n, dtype=torch.float32, device=dev)
        F = torch.empty((n, 3), dtype=torch.float32, device=dev)
        G = torch.empty((n, nf), dtype=torch.float32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        M, max_n = meta["num_mols"], meta["max_n"]
        if _lib.is_large(max_n):   # past the fused kernels' LDS image
            ws = _lib.large_workspace(M, n, max_n, nf, dev)
            prec = _lib.PREC_F32 | (_lib.EGCL_VARIANTS if self.variant_flags() else 0)
            _lib.check(L.enflow_egcl_forward_large_f32(
                M, n, max_n, nf, self.kernel_hidden, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(hf), _lib.ptr(pos), _lib.ptr(self.packed(dev)),
                float(self.coords_weight), _lib.ptr(Q), _lib.ptr(F), _lib.ptr(G), _lib.ptr(err), prec,
                _lib.ptr(ws), ws.numel(), _lib.stream_ptr(dev)), "enflow_egcl_forward_large_f32")
        else:
            _lib.check(L.enflow_egcl_forward_f32(M, n, max_n, nf, self.kernel_hidden, _lib.ptr(meta["mol_ptr"]),
                                                 _lib.ptr(meta["r_cut"]), _lib.ptr(meta["box"]), _lib.ptr(hf),
                                                 _lib.ptr(pos), _lib.ptr(self.packed(dev)),
                                                 float(self.coords_weight), _lib.ptr(Q), _lib.ptr(F), _lib.ptr(G),
                                                 _lib.ptr(err), _lib.stream_ptr(dev)), "enflow_egcl_forward_f32")
        _lib.raise_on_err(err)
        return Q.reshape(n, 1), F, G[:, :self.output_nf]

    def pad_h(self, h):
        """h [n][input_nf] -> fp32 [n][kernel_nf] (zero columns past input_nf)."""
        hf = h.to(torch.float32)
        if self.kernel_nf > self.input_nf:
            hf = torch.cat([hf, hf.new_zeros((hf.shape[0], self.kernel_nf - self.input_nf))], 1)
        return hf.contiguous()

    def forward(self, h, edges):
        """egcl.py:76-92.  Differentiable (w.r.t. the parameters, h and, through
        Edges.coord_diff, the positions) when autograd needs it: the backward is
        the HIP layer backward in EGCL mode (enflow_egcl_backward_f32)."""
        if not isinstance(edges, Edges):
            raise TypeError("EGCL.forward expects the Edges handle returned by Data.edges")
        self._check_supported()
        _lib.require_gpu(h)
        dev = h.device
        meta = self._meta(edges, dev)
        params = list(self.parameters())
        if torch.is_grad_enabled() and (h.requires_grad or edges.pos.requires_grad or
                                        any(p.requires_grad for p in params)):
            if self.kernel_nf > _lib.TRAIN_MAX_NODE_NF:
                raise NotImplementedError(f"enflow_amd differentiates EGCL up to node_nf {_lib.TRAIN_MAX_NODE_NF} "
                                          "(inference runs up to 16); call it under torch.no_grad()")
            check_trainable(self.act_fn, "EGCL.forward")
            from ..flow._train import _EGCLFunction
            q, f, g = _EGCLFunction.apply(self, meta, h, edges.pos, *params)
        else:
            q, f, g = self._infer(h.detach(), edges.pos.detach(), meta)
        return q.to(h.dtype), f.to(h.dtype), g.to(h.dtype)
