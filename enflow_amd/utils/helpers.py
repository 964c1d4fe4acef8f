"""Small tensor helpers mirroring enflow/utils/helpers.py.

These are the element-wise / bookkeeping helpers of the reference's public
API.  The hot path (edges, EGCL, flow, loss) never calls them: it runs inside
the HIP kernels of libenflow_hip.so.
"""
import math

import torch


def log_gaussian(z):
    """enflow/utils/helpers.py:4-5 (one log(2 pi) for the whole tensor)."""
    return -0.5 * ((z ** 2).sum() + math.log(2 * math.pi))


def apply_pbc(pos, box):
    """enflow/utils/helpers.py:7-8."""
    return pos - (pos / box).round() * box


def get_box_len(pos):
    """enflow/utils/helpers.py:10-13."""
    return (pos.max(dim=0)[0] - pos.min(dim=0)[0]).round()


def one_hot(index, num_classes=None, dtype=None):
    """enflow/utils/helpers.py:43-52 (width = max + 1 when num_classes is None)."""
    if index.dim() != 1:
        raise ValueError("'index' tensor needs to be one-dimensional")
    if num_classes is None:
        num_classes = int(index.max()) + 1
    out = torch.zeros((index.size(0), num_classes), dtype=dtype, device=index.device)
    return out.scatter_(1, index.unsqueeze(1), 1)


def mol_ptr_from_counts(N, device=None):
    """CSR atom offsets (int32, [M+1]) from per-molecule atom counts Data.N.
    Host counts (the reference's Data.N) are summed on the host into pinned
    memory and copied asynchronously: one queued copy instead of a synchronous
    pageable copy and three small kernels (~25 us of every module call on a
    fresh batch, profiles/r06/r06n_module_call_cprofile.txt)."""
    N = torch.as_tensor(N)
    if N.ndim == 0:
        N = N.reshape(1)
    dev = torch.device(device) if device is not None else N.device
    if N.device.type == "cpu":
        host = torch.empty(N.numel() + 1, dtype=torch.int32, pin_memory=dev.type == "cuda")
        host[0] = 0
        torch.cumsum(N, 0, dtype=torch.int32, out=host[1:])
        return host if dev.type == "cpu" else host.to(dev, non_blocking=True)
    ptr = torch.zeros(N.numel() + 1, dtype=torch.int32, device=dev)
    ptr[1:] = torch.cumsum(N.to(dev), 0).to(torch.int32)
    return ptr


def params_of(module):
    """The parameters of `module`, each once (the set module.parameters()
    yields), by a direct walk of the _modules / _parameters dicts: ~4x faster
    than named_parameters()'s prefixed generators, which the packed-weight
    cache keys used to run on every launch (8 EGCL layers: ~300 -> ~75 us
    with the versions)."""
    out, seen_p, seen_m, stack = [], set(), set(), [module]
    while stack:
        m = stack.pop()
        if m is None or id(m) in seen_m:
            continue
        seen_m.add(id(m))
        for p in m._parameters.values():
            if p is not None and id(p) not in seen_p:
                seen_p.add(id(p))
                out.append(p)
        stack.extend(m._modules.values())
    return out


def batch_meta(data, device):
    """(mol_ptr int32 [M+1] on device, max atoms per molecule) for any batch
    object with the reference's fields -- enflow_amd.data.Data caches them,
    the reference's own enflow.data.base.Data only has N."""
    ptr = getattr(data, "mol_ptr", None)
    if ptr is None or ptr.device != device:
        ptr = mol_ptr_from_counts(data.N, device=device)
    mx = getattr(data, "max_mol_atoms", None)
    if mx is None:
        N = torch.as_tensor(data.N)
        mx = int(N.max()) if N.numel() else 0
    return ptr, mx
