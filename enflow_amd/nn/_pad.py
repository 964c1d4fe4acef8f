"""Hidden widths the kernels are not compiled for run zero-padded to the next
compiled width (32, 64, 128).

The reference accepts any ``hidden_nf`` (enflow/nn/egcl.py:11,
enflow/nn/argmax.py:6).  Padding every hidden dimension with zero weights and
zero biases is exact: a padded hidden unit has pre-activation 0, SiLU(0) = 0,
and its outgoing weights are 0, so every output (and every gradient of a real
parameter) equals the unpadded network's.  The real parameters occupy the
leading block of each padded tensor: for node_nn.0.weight the columns are
[h (nf) | messages (H)], so the messages' padding is appended at the tail too.
"""
import torch

KERNEL_HIDDEN = (32, 64, 128)

# per parameter: the dims that have the hidden width ("H") or end with it ("xH")
EGCL_HDIMS = {
    "edge_nn.0.weight": ("H", None), "edge_nn.0.bias": ("H",),
    "edge_nn.2.weight": ("H", "H"), "edge_nn.2.bias": ("H",),
    "node_nn.0.weight": ("H", "xH"), "node_nn.0.bias": ("H",),
    "node_nn.2.weight": (None, "H"), "node_nn.2.bias": (None,),
    "coord_nn.0.weight": ("H", "H"), "coord_nn.0.bias": ("H",), "coord_nn.2.weight": (None, "H"),
    "vel_scaling_nn.0.weight": ("H", None), "vel_scaling_nn.0.bias": ("H",),
    "vel_scaling_nn.2.weight": (None, "H"), "vel_scaling_nn.2.bias": (None,),
    "att_nn.0.weight": (None, "H"), "att_nn.0.bias": (None,),
}
ARGMAX_HDIMS = {
    "network.0.weight": ("H", None), "network.0.bias": ("H",),
    "network.2.weight": (None, "H"), "network.2.bias": (None,),
}


def kernel_hidden(hidden_nf):
    """The compiled width a hidden_nf runs at (None past the largest)."""
    return next((k for k in KERNEL_HIDDEN if k >= hidden_nf), None)


def padded_shape(spec, shape, H, Hp):
    return tuple(Hp if s == "H" else (d - H + Hp if s == "xH" else d) for s, d in zip(spec, shape))


def pad(t, spec, H, Hp):
    """t (real parameter) -> zero-padded fp32 tensor of the kernel width."""
    if H == Hp:
        return t
    out = torch.zeros(padded_shape(spec, t.shape, H, Hp), dtype=t.dtype, device=t.device)
    out[tuple(slice(0, d) for d in t.shape)] = t
    return out


def flat_padded(named, table, H, Hp, device):
    """Concatenated flat fp32 padded parameters, in the given (name, param) order."""
    return torch.cat([pad(p.detach().to(device=device, dtype=torch.float32), table[k], H, Hp).reshape(-1)
                      for k, p in named])


def unpad_grads(flat, named, table, H, Hp):
    """Split a flat gradient in the padded layout of `named` into the real
    parameters' shapes (the leading block of each padded tensor)."""
    out, off = {}, 0
    for k, p in named:
        ps = padded_shape(table[k], p.shape, H, Hp)
        n = 1
        for d in ps:
            n *= d
        g = flat[off:off + n].view(ps)
        out[k] = g[tuple(slice(0, d) for d in p.shape)]
        off += n
    return out, off
