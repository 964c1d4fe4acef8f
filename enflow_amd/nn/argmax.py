"""ArgMax dequantiser (mirrors enflow/nn/argmax.py:5-28).

forward(h) -> (z, log_q) runs enflow_argmax_forward_f32 with a device-side
N(0, 1) draw (the reference's torch.randn(h.size()), argmax.py:16);
reverse(z) is the one-hot of the first maximum with the reference's width
(max index + 1).
"""
import torch
from torch import nn

from .. import _lib
from ..utils.helpers import one_hot, mol_ptr_from_counts, params_of
from ._act import SILU, act_code, act_kind, check_trainable
from ._pad import ARGMAX_HDIMS, Geom, flat_padded, kernel_hidden


class ArgMax(nn.Module):
    def __init__(self, node_nf, hidden_nf, act_fn=nn.SiLU()):
        super().__init__()
        self.node_nf, self.hidden_nf = node_nf, hidden_nf
        self.network = nn.Sequential(nn.Linear(node_nf, hidden_nf), act_fn,
                                     nn.Linear(hidden_nf, node_nf * 2))
        self._packed = None
        self._packed_key = None

    @property
    def kernel_hidden(self):
        """Compiled hidden width (hidden_nf zero-padded to 32 / 64 / 128, exact; nn/_pad.py)."""
        return kernel_hidden(self.hidden_nf)

    def kernel_raw(self, device, width=None):
        """network parameters as one flat fp32 vector padded to `width` (default
        kernel_hidden; the flow passes its layers' width)."""
        width = width or self.kernel_hidden
        if width is None or width < self.hidden_nf:
            raise NotImplementedError(f"ArgMax hidden_nf {self.hidden_nf} past the kernel width {width}")
        flat = flat_padded(self.kernel_named(), ARGMAX_HDIMS, self.pad_geom(width), device)
        # ABI 10: [act kind, p0, p1, 0] of network.1 after the parameters (argmax.py:7);
        # the device copy is cached (a host-to-device copy per call would stall the
        # stream once per training step)
        code = self.act()
        key = (str(device), code)
        trailer = getattr(self, "_act_trailer", None)
        if trailer is None or trailer[0] != key:
            t = torch.tensor([float(code[0]), code[1], code[2], 0.0], dtype=torch.float32, device=device)
            self._act_trailer = trailer = (key, t)
        return torch.cat([flat, trailer[1]])

    def kernel_named(self):
        """(name, parameter) of the two Linear layers (a PReLU slope, network.1,
        travels in the act code)."""
        return [(k, p) for k, p in self.named_parameters() if not k.startswith("network.1.")]

    def act(self):
        """(kind, p0, p1) of the network's activation (ENFLOW_ACT_*)."""
        return act_code(self.network[1])

    def generic_act(self):
        """True if the activation is not SiLU (the flow then runs its variant-capable kernels)."""
        return act_kind(self.network[1]) != SILU

    def pad_geom(self, width=None):
        nf = self.node_nf
        return Geom(self.hidden_nf, width or self.kernel_hidden, nf, nf, nf)

    def packed(self, device, width=None):
        width = width or self.kernel_hidden
        key = (str(device), width) + tuple((p.data_ptr(), p._version) for p in params_of(self))
        if self._packed is not None and self._packed_key == key:
            return self._packed
        L = _lib.lib(self.node_nf)
        raw = self.kernel_raw(device, width)
        out = torch.empty(L.enflow_argmax_packed_size(width, self.node_nf),
                          dtype=torch.float32, device=device)
        _lib.check(L.enflow_pack_argmax_f32(_lib.ptr(raw), width, self.node_nf, _lib.ptr(out),
                                            _lib.stream_ptr(device)), "enflow_pack_argmax_f32")
        self._packed, self._packed_key = out, key
        return out

    def _meta(self, n, N, dev, cap):
        """Molecule chunks of <= cap atoms (ArgMax is per atom; log_q is a sum)."""
        if N is None:
            N = torch.tensor([n])
        N = torch.as_tensor(N).reshape(-1)
        if N.numel() and int(N.max()) > cap:
            chunks = []
            for c in N.tolist():
                chunks += [cap] * (c // cap) + ([c % cap] if c % cap else [])
            N = torch.tensor(chunks)
        return dict(mol_ptr=mol_ptr_from_counts(N, device=dev), max_n=int(N.max()) if N.numel() else 0,
                    num_mols=N.numel())

    def _infer(self, h, eps, meta):
        L = _lib.lib(self.node_nf)
        dev = h.device
        n = h.shape[0]
        hf = h.to(torch.float32).contiguous()
        z = torch.empty_like(hf)
        lq_mol = torch.empty(max(meta["num_mols"], 1), dtype=torch.float32, device=dev)
        lq = torch.empty(1, dtype=torch.float32, device=dev)
        _lib.check(L.enflow_argmax_forward_f32(meta["num_mols"], n, meta["max_n"], self.node_nf, self.kernel_hidden,
                                               _lib.ptr(meta["mol_ptr"]), _lib.ptr(hf), _lib.ptr(self.packed(dev)),
                                               _lib.ptr(eps), _lib.ptr(z), _lib.ptr(lq_mol), _lib.ptr(lq),
                                               _lib.stream_ptr(dev)), "enflow_argmax_forward_f32")
        return z, lq.reshape(())

    def forward(self, h, noise=None, N=None):
        """argmax.py:13-25.  ``N``: atoms per molecule (defaults to one molecule
        holding every atom; log_q is a batch scalar either way).  ``noise``:
        optional N(0,1) draw of shape h.shape.  Differentiable w.r.t. the
        network parameters when autograd needs it (enflow_argmax_backward_f32);
        h is categorical data and receives no gradient."""
        _lib.require_gpu(h)
        dev = h.device
        eps = (torch.randn(h.shape, device=dev, dtype=torch.float32) if noise is None
               else noise.to(device=dev, dtype=torch.float32).contiguous())
        params = list(self.parameters())
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            check_trainable(self.network[1], "ArgMax.forward")
            from ..flow._train import _ArgMaxFunction
            meta = self._meta(h.shape[0], N, dev, _lib.TRAIN_MAX_ATOMS)
            z, lq = _ArgMaxFunction.apply(self, meta, h, eps, *params)
        else:
            z, lq = self._infer(h.detach(), eps, self._meta(h.shape[0], N, dev, _lib.lib().enflow_max_atoms()))
        return z.to(h.dtype), lq.to(h.dtype)

    def reverse(self, z):
        return one_hot(torch.argmax(z, dim=-1), dtype=z.dtype)
