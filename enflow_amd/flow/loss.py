"""Alchemical negative log-likelihood (mirrors enflow/flow/loss.py:5-24).

__call__(out, ldj) -> 0-d tensor, computed by enflow_alchemical_nll_f32: one
workgroup per molecule sums the softened LJ energy over i < j pairs (zero
distances dropped, loss.py:14-18), sum vel^2, h^2, g^2; a fixed-order double
reduction forms the reference's scalar.  When its inputs carry autograd
history the loss is differentiable (backward: enflow_alchemical_nll_backward_f32).
"""
import torch

from .. import _lib
from ..utils.helpers import batch_meta


class Alchemical_NLL:
    def __init__(self, kBT, partition_func=10, softening=0):
        self.kBT = kBT
        self.z_lj = partition_func
        self.softening = softening

    def __call__(self, out, ldj):
        _lib.require_gpu(out.pos)
        if torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad
                                           for t in (out.h, out.g, out.pos, out.vel, ldj)):
            return self._differentiable(out, ldj)
        L = _lib.lib(out.h.shape[1])
        dev = out.pos.device
        f = lambda t: t.detach().to(device=dev, dtype=torch.float32).contiguous()  # noqa: E731
        h, g, pos, vel = f(out.h), f(out.g), f(out.pos), f(out.vel)
        ptr, max_n = batch_meta(out, dev)
        M = ptr.numel() - 1
        ldj_t = torch.as_tensor(ldj, device=dev).to(torch.float32).reshape(1).contiguous()
        nll_mol = torch.empty((max(M, 1), 4), dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        _lib.check(L.enflow_alchemical_nll_f32(M, h.shape[0], max_n, h.shape[1], _lib.ptr(ptr),
                                               _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos), _lib.ptr(vel),
                                               _lib.ptr(ldj_t), float(self.kBT), float(self.softening),
                                               float(self.z_lj), _lib.ptr(nll_mol), _lib.ptr(loss),
                                               _lib.stream_ptr(dev)), "enflow_alchemical_nll_f32")
        return loss.reshape(()).to(out.h.dtype)

    def _differentiable(self, out, ldj):
        """Same value, with a grad_fn whose backward is enflow_alchemical_nll_backward_f32."""
        from ._train import _NLLFunction
        dev = out.pos.device
        ptr, max_n = batch_meta(out, dev)
        f = lambda t: t.to(device=dev, dtype=torch.float32)  # noqa: E731
        ldj_t = torch.as_tensor(ldj, device=dev)
        loss = _NLLFunction.apply(self, {"mol_ptr": ptr, "max_n": max_n}, f(out.h), f(out.g), f(out.pos),
                                  f(out.vel), ldj_t.to(torch.float32).reshape(()))
        return loss.to(out.h.dtype)
