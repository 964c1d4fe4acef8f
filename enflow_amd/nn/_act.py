"""act_fn of EGCL / ArgMax as the kernels' activation codes.

The reference takes the activation module as a constructor argument
(enflow/nn/egcl.py:11 ``act_fn=nn.SiLU()``, enflow/nn/argmax.py:7) and uses
the same instance at every position of the block's MLPs.  The kernels know
the elementwise torch activations below (ENFLOW_ACT_* in include/enflow_hip.h,
forward and derivative in flow_device.h act_f / act_d); a layer whose act_fn
is not SiLU is packed with its code and runs the variant-capable kernels.

nn.PReLU (one learnable slope, the torch default num_parameters=1) runs as
LeakyReLU with the module's current slope: max(0, x) + a * min(0, x) is
LeakyReLU(a) for every a, and the slope is read when the layer is packed (the
packed-weight caches key on every parameter's version, so an optimizer step on
it re-packs).  The HIP backward has no slope gradient: training with the slope
trainable is refused (check_trainable); a frozen slope trains.
"""
from torch import nn

SILU, RELU, LEAKY_RELU, ELU, CELU, SELU, GELU, GELU_TANH, TANH, SIGMOID, SOFTPLUS, MISH, HARDTANH, IDENTITY = range(14)


def act_kind(m):
    """The ENFLOW_ACT_* kind alone (no parameter read: no device sync for PReLU)."""
    if isinstance(m, nn.PReLU):
        _check_prelu(m)
        return LEAKY_RELU
    return act_code(m)[0]


def _check_prelu(m):
    if m.weight.numel() != 1:
        raise NotImplementedError(f"enflow_amd kernels implement PReLU with one slope (num_parameters=1), "
                                  f"got {m.weight.numel()}")


def check_trainable(m, where):
    """Refuse a differentiable call while act_fn has trainable parameters (the
    HIP backward differentiates the Linear layers, not the activation)."""
    if any(p.requires_grad for p in m.parameters()):
        raise NotImplementedError(
            f"{where}: the HIP backward has no gradient for the parameters of act_fn {type(m).__name__}; "
            "freeze them (requires_grad_(False)) to train the rest, or run under torch.no_grad()")


def act_code(m):
    """(kind, p0, p1) of an activation module; NotImplementedError otherwise."""
    if isinstance(m, nn.PReLU):
        _check_prelu(m)
        return LEAKY_RELU, float(m.weight.detach().reshape(())), 0.0
    if isinstance(m, nn.SiLU):
        return SILU, 0.0, 0.0
    if isinstance(m, nn.ReLU):
        return RELU, 0.0, 0.0
    if isinstance(m, nn.LeakyReLU):
        return LEAKY_RELU, float(m.negative_slope), 0.0
    if isinstance(m, nn.ELU):
        return ELU, float(m.alpha), 0.0
    if isinstance(m, nn.CELU):
        return CELU, float(m.alpha), 0.0
    if isinstance(m, nn.SELU):
        return SELU, 0.0, 0.0
    if isinstance(m, nn.GELU):
        if m.approximate == "tanh":
            return GELU_TANH, 0.0, 0.0
        return GELU, 0.0, 0.0
    if isinstance(m, nn.Tanh):
        return TANH, 0.0, 0.0
    if isinstance(m, nn.Sigmoid):
        return SIGMOID, 0.0, 0.0
    if isinstance(m, nn.Softplus):
        return SOFTPLUS, float(m.beta), float(m.threshold)
    if isinstance(m, nn.Mish):
        return MISH, 0.0, 0.0
    if isinstance(m, nn.Hardtanh):          # ReLU6 is Hardtanh(0, 6)
        return HARDTANH, float(m.min_val), float(m.max_val)
    if isinstance(m, nn.Identity):
        return IDENTITY, 0.0, 0.0
    raise NotImplementedError(f"enflow_amd kernels do not implement the activation {type(m).__name__}")


def supported(m):
    try:
        act_kind(m)
        return True
    except NotImplementedError:
        return False
