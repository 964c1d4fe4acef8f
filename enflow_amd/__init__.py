"""enflow_amd: MI355X-native (gfx950) implementation of the enflow coupling-flow
hot path -- LFIntegrator forward/reverse + log|detJ| driven by EGCL message
passing -- behind the reference's nn.Module surface.

Kernels: enflow_amd/csrc/enflow_flow.hip -> libenflow_hip.so (C ABI in
include/enflow_hip.h), bound with ctypes in enflow_amd/_lib.py.
"""
__version__ = "0.1.0"
