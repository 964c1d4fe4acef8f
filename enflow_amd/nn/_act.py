"""act_fn of EGCL / ArgMax as the kernels' activation codes.

The reference takes the activation module as a constructor argument
(enflow/nn/egcl.py:11 ``act_fn=nn.SiLU()``, enflow/nn/argmax.py:7) and uses
the same instance at every position of the block's MLPs.  The kernels know
the elementwise torch activations below (ENFLOW_ACT_* in include/enflow_hip.h,
forward and derivative in flow_device.h act_f / act_d); a layer whose act_fn
is not SiLU is packed with its code and runs the variant-capable kernels.
"""
from torch import nn

SILU, RELU, LEAKY_RELU, ELU, CELU, SELU, GELU, GELU_TANH, TANH, SIGMOID, SOFTPLUS, MISH, HARDTANH, IDENTITY = range(14)


def act_code(m):
    """(kind, p0, p1) of an activation module; NotImplementedError otherwise."""
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
        act_code(m)
        return True
    except NotImplementedError:
        return False
