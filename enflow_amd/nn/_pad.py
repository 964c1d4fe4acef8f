"""Shapes the kernels are not compiled for run zero-padded to compiled ones.

The reference accepts any ``hidden_nf`` and any ``input_nf`` / ``output_nf``
(enflow/nn/egcl.py:11, enflow/nn/argmax.py:6).  The kernels are compiled for
hidden widths 32 / 64 / 128 and one node-feature width ``nf`` (<= 16) for both
the input and the output features.  Other shapes are embedded in the next
compiled one with zero weights and biases, which is exact:

* a padded hidden unit has pre-activation 0 and zero outgoing weights, so
  whatever act_fn(0) is (SiLU(0) = 0, Sigmoid(0) = 0.5, Softplus(0) = log 2)
  it reaches no output, and its adjoint (zero outgoing weights) is 0;
* a padded input feature is a zero column of h with zero incoming weights;
* a padded output feature of node_nn.2 has zero weights and bias (G's extra
  columns are 0 and are sliced away).

So every output, and the gradient of every real parameter, equals the
unpadded network's.  Each parameter's real entries sit at fixed indices of the
padded tensor (`Geom` index maps): for edge_nn.0's input [h_i | h_j | radial]
and node_nn.0's input [h | messages] the blocks move to the padded offsets.
"""
import torch

KERNEL_HIDDEN = (32, 64, 128)

# per parameter and dim: None (kept), "H" hidden, "E" edge_nn.0 input
# [h_i (in) | h_j (in) | radial], "xH" node_nn.0 input [h (in) | messages (H)],
# "I" input features, "O" output features
EGCL_HDIMS = {
    "edge_nn.0.weight": ("H", "E"), "edge_nn.0.bias": ("H",),
    "edge_nn.2.weight": ("H", "H"), "edge_nn.2.bias": ("H",),
    "node_nn.0.weight": ("H", "xH"), "node_nn.0.bias": ("H",),
    "node_nn.2.weight": ("O", "H"), "node_nn.2.bias": ("O",),
    "coord_nn.0.weight": ("H", "H"), "coord_nn.0.bias": ("H",), "coord_nn.2.weight": (None, "H"),
    "vel_scaling_nn.0.weight": ("H", "I"), "vel_scaling_nn.0.bias": ("H",),
    "vel_scaling_nn.2.weight": (None, "H"), "vel_scaling_nn.2.bias": (None,),
    "att_nn.0.weight": (None, "H"), "att_nn.0.bias": (None,),
}
ARGMAX_HDIMS = {
    "network.0.weight": ("H", "I"), "network.0.bias": ("H",),
    "network.2.weight": (None, "H"), "network.2.bias": (None,),
}


def kernel_hidden(hidden_nf):
    """The compiled width a hidden_nf runs at (None past the largest)."""
    return next((k for k in KERNEL_HIDDEN if k >= hidden_nf), None)


class Geom:
    """Real (H, fin, fout) -> kernel (Hp, F) shape of one module."""

    def __init__(self, H, Hp, fin, fout, F):
        self.H, self.Hp, self.fin, self.fout, self.F = H, Hp, fin, fout, F

    @property
    def identity(self):
        return self.H == self.Hp and self.fin == self.F and self.fout == self.F

    def index(self, kind, size):
        """(padded size, indices of the real entries along this dim)."""
        a = torch.arange
        if kind is None:
            return size, a(size)
        if kind == "H":
            return self.Hp, a(self.H)
        if kind == "I":
            return self.F, a(self.fin)
        if kind == "O":
            return self.F, a(self.fout)
        if kind == "E":
            return 2 * self.F + 1, torch.cat([a(self.fin), self.F + a(self.fin), torch.tensor([2 * self.F])])
        if kind == "xH":
            return self.F + self.Hp, torch.cat([a(self.fin), self.F + a(self.H)])
        raise ValueError(kind)


_IDX_CACHE = {}


def _indices(spec, shape, g, device):
    """(padded sizes, index tuple on `device`); cached per shape, so a training
    step does no host-to-device index copies (they would stall the stream)."""
    key = (tuple(spec), tuple(shape), g.H, g.Hp, g.fin, g.fout, g.F, str(device))
    hit = _IDX_CACHE.get(key)
    if hit is not None:
        return hit
    dims = [g.index(k, d) for k, d in zip(spec, shape)]
    sizes = tuple(s for s, _ in dims)
    idx = [i.to(device) for _, i in dims]
    if len(idx) == 2:
        idx = (idx[0][:, None], idx[1][None, :])
    else:
        idx = (idx[0],)
    _IDX_CACHE[key] = (sizes, idx)
    return sizes, idx


def pad(t, spec, g):
    """t (real parameter) -> zero-padded tensor of the kernel shape."""
    if g.identity:
        return t
    sizes, idx = _indices(spec, t.shape, g, t.device)
    out = torch.zeros(sizes, dtype=t.dtype, device=t.device)
    out[idx] = t
    return out


def flat_padded(named, table, g, device):
    """Concatenated flat fp32 padded parameters, in the given (name, param) order."""
    return torch.cat([pad(p.detach().to(device=device, dtype=torch.float32), table[k], g).reshape(-1)
                      for k, p in named])


def unpad_grads(flat, named, table, g):
    """Split a flat gradient in the padded layout of `named` into the real
    parameters' shapes (their entries of each padded tensor).  Returns
    ({name: grad}, floats consumed)."""
    out, off = {}, 0
    for k, p in named:
        if g.identity:
            sizes, idx = tuple(p.shape), None
        else:
            sizes, idx = _indices(table[k], p.shape, g, flat.device)
        n = 1
        for d in sizes:
            n *= d
        gp = flat[off:off + n].view(sizes)
        out[k] = gp if idx is None else gp[idx]
        off += n
    return out, off
