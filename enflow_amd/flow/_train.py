"""Autograd glue of the HIP training path.

``LFIntegrator.forward`` (enflow/flow/dynamics.py:10-24) and
``Alchemical_NLL.__call__`` (enflow/flow/loss.py:21-24) become
``torch.autograd.Function`` s whose backward passes call the C ABI
(enflow_alchemical_nll_backward_f32, enflow_lf_backward_f32).  Parameters
enter the flow function as inputs, so ``loss.backward()`` fills every
``p.grad`` exactly like the reference's autograd, and DDP / optimisers / LR
schedulers work on them unchanged (enflow/main.py:212-223).
"""
import os

import torch

from .. import _lib
from ..nn.argmax import ArgMax
from ..nn._pad import ARGMAX_HDIMS, EGCL_HDIMS, unpad_grads


def pair_row_bound(N):
    """Upper bound of the backward's pair rows: sum of n(n-1) rounded up to 32."""
    N = torch.as_tensor(N).reshape(-1).to(torch.int64)
    return int((((N * (N - 1)) + 31) // 32 * 32).sum())


class _FlowFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flow, meta, h, g, pos, vel, *params):
        hid, nf, cw = flow._geometry()
        kind = flow._dequant_kind()
        dev = h.device
        L = _lib.lib(nf)
        n_layers = len(flow.networks)
        A = h.shape[0]
        M = meta["mol_ptr"].numel() - 1
        # out of place: the kernel reads the inputs and writes fresh outputs (the
        # input h is kept for the dequantiser's backward as is, no copy)
        src = tuple(t.detach().contiguous() for t in (h, g, pos, vel))
        h_in = src[0]
        hw, gw, pw, vw = (torch.empty_like(t) for t in src)
        tape = torch.empty(max(L.enflow_lf_tape_size_for(A, nf, hid, n_layers, meta["max_n"]), 1),
                           dtype=torch.float32, device=dev)
        # fused: unique pairs [n_layers][M]; large: the backward's pair rows per layer
        counts = torch.zeros(max(n_layers * (1 if meta["large"] else M), 1), dtype=torch.int32, device=dev)
        ldj_mol = torch.empty(max(M, 1), dtype=torch.float32, device=dev)
        ldj = torch.empty(1, dtype=torch.float32, device=dev)
        st = torch.zeros(2, dtype=torch.int32, device=dev)   # error word, ldj reduction ticket
        err = st[:1]
        prec = flow._prec()
        if (prec & 0xff) == _lib.PREC_BF16:
            # the tape feeds the fp32-accurate backward: record it from an fp32-accurate forward
            prec = (prec & ~0xff) | _lib.PREC_F16X3
            if not _warned_bf16:
                _warned_bf16.append(True)
                import warnings
                warnings.warn("enflow_amd: gemm_precision='bf16' is a generate-path setting; the training "
                              "forward runs f16x3", RuntimeWarning, stacklevel=2)
        # both packed sections of every layer first (training_layers: after an
        # optimiser step, two launches per section for the whole flow, ABI 13), so
        # the forward launch reuses the forward section (packed_layers' cache); the
        # buffers and the parameter versions they were packed from go with this
        # graph: the backward uses exactly these and refuses in-place changes since
        ctx.train_bufs = flow.training_layers(dev)
        ctx.train_key = flow._params_key(dev)
        flow.forward_buffers(hw, gw, pw, vw, meta["box"], meta["r_cut"], meta["mol_ptr"], meta["max_n"],
                             meta["noise"], ldj_mol, ldj, err, tape=tape, pair_counts=counts, prec=prec,
                             src=src, ticket=st[1:])
        # an fp32-GEMM forward's tape gets the fp32-GEMM backward (ENFLOW_BWD_F32)
        ctx.bwd_f32 = (prec & 0xff) == _lib.PREC_F32
        # the dequantiser's flat parameters behind the forward kernel, ahead of the
        # error check's sync
        ctx.dq_raw = None
        if kind == _lib.DEQUANT_ARGMAX:
            ctx.dq_raw = flow.dequantize.kernel_raw(dev, hid)
        if meta["check_errors"]:
            if getattr(flow, "defer_error_check", False):
                # no host sync: the word is read at the start of this graph's
                # backward (before anything consumes the outputs' gradients) or
                # at the next check; an ENFLOW_ERR_RANGE then raises (the outputs
                # were consumed already, so the step cannot be re-run); an
                # ENFLOW_ERR_SMALL alone (an operand entirely below 2^-7: ~1e-5
                # relative, not an overflow) warns
                _lib.defer_err(err, small_warns=True)
            else:
                _lib.check_pending()        # an older deferred word is not this launch's
                e = _lib.take_err(err)
                if e and not e & ~_lib.ERR_RERUN and (prec & 0xff) != _lib.PREC_F32:
                    # a split-precision operand left its range (an fp16 overflow, or an
                    # operand entirely below 2^-7): the step's forward again with fp32
                    # GEMMs, same inputs and draws, and the fp32 backward on its tape
                    prec = (prec & ~0xff) | _lib.PREC_F32
                    counts.zero_()
                    flow.forward_buffers(hw, gw, pw, vw, meta["box"], meta["r_cut"], meta["mol_ptr"],
                                         meta["max_n"], meta["noise"], ldj_mol, ldj, err, tape=tape,
                                         pair_counts=counts, prec=prec, src=src, ticket=st[1:])
                    ctx.bwd_f32 = True
                    _lib.FP32_RERUNS[0] += 1
                    e = _lib.take_err(err)
                _lib.raise_code(e)          # the reference raises inside forward
        ctx.flow, ctx.meta, ctx.kind = flow, meta, kind
        ctx.n_params = len(params)
        ctx.save_for_backward(h_in, tape, counts)
        return hw, gw, pw, vw, ldj.reshape(())

    @staticmethod
    def backward(ctx, gh, gg, gpos, gvel, gldj):
        flow, meta, kind = ctx.flow, ctx.meta, ctx.kind
        h_in, tape, counts = ctx.saved_tensors
        hid, nf, cw = flow._geometry()
        dev = h_in.device
        L = _lib.lib(nf)
        A = h_in.shape[0]
        M = meta["mol_ptr"].numel() - 1
        n_layers = len(flow.networks)

        def adj(t, shape):
            if t is None:
                return torch.zeros(shape, dtype=torch.float32, device=dev)
            return t.detach().to(dtype=torch.float32).contiguous().clone()

        ah, ag = adj(gh, (A, nf)), adj(gg, (A, nf))
        apos, avel = adj(gpos, (A, 3)), adj(gvel, (A, 3))
        aldj = adj(gldj, ()).reshape(1)
        if flow._params_key(dev) != ctx.train_key:
            raise RuntimeError("enflow_amd: a parameter of the flow was modified in place between forward "
                               "and backward (autograd would report a version mismatch here)")
        fwd, bwd, raw = ctx.train_bufs
        grad_layers = torch.empty_like(raw)
        dq_raw, grad_dq = None, None
        if kind == _lib.DEQUANT_ARGMAX:
            dq_raw = ctx.dq_raw
            grad_dq = torch.empty_like(dq_raw)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        kindv = kind | (_lib.EGCL_VARIANTS if flow._has_variants() else 0) | (_lib.BWD_F32 if ctx.bwd_f32 else 0)
        if meta["large"]:
            # the forward counted each layer's pair rows on the device: size the
            # workspace by their maximum (one small read; large systems only)
            prb = int(counts[:max(n_layers, 1)].max().item()) if n_layers else 0
            wsb = L.enflow_lf_backward_large_workspace_size(M, A, meta["max_n"], nf, hid, prb)
            if wsb < 0:
                raise _lib.HipPathError("enflow_lf_backward_large_workspace_size rejected the batch")
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            _lib.check(L.enflow_lf_backward_large_f32(
                M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(tape), _lib.ptr(fwd), _lib.ptr(bwd), _lib.ptr(raw), n_layers,
                kindv, _lib.ptr(dq_raw), _lib.ptr(h_in), _lib.ptr(meta["noise"]), float(flow.dt), cw,
                _lib.ptr(ah), _lib.ptr(ag), _lib.ptr(apos), _lib.ptr(avel), _lib.ptr(aldj),
                _lib.ptr(grad_layers), _lib.ptr(grad_dq), _lib.ptr(ws), wsb, prb, _lib.ptr(err),
                _lib.stream_ptr(dev)), "enflow_lf_backward_large_f32")
        else:
            prb = meta["pair_row_bound"]
            wsb = L.enflow_lf_backward_workspace_size(M, A, nf, hid, n_layers, prb)
            if os.environ.get("ENFLOW_BWD_MIN_WS") == "1":     # memory-lean: two rotating buffers
                wsb = L.enflow_lf_backward_workspace_size_min(M, A, nf, hid, n_layers, prb)
            if wsb < 0:
                raise _lib.HipPathError("enflow_lf_backward_workspace_size rejected the batch")
            try:
                ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            except torch.cuda.OutOfMemoryError:
                # three rotating pair-row buffers do not fit: two (the layer chain
                # then waits for the weight-gradient pass two layers up); the failed
                # request's cached blocks are released first
                torch.cuda.empty_cache()
                wsb = L.enflow_lf_backward_workspace_size_min(M, A, nf, hid, n_layers, prb)
                try:
                    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
                except torch.cuda.OutOfMemoryError as exc:
                    raise torch.cuda.OutOfMemoryError(
                        f"enflow_amd backward workspace ({wsb / 2**30:.2f} GiB with two rotating pair-row "
                        "buffers, the ENFLOW_BWD_MIN_WS=1 size) does not fit: train on a smaller batch") from exc
            _lib.check(L.enflow_lf_backward_f32(
                M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(tape), _lib.ptr(counts), _lib.ptr(fwd), _lib.ptr(bwd),
                _lib.ptr(raw), n_layers, kindv, _lib.ptr(dq_raw), _lib.ptr(h_in), _lib.ptr(meta["noise"]),
                float(flow.dt), cw, _lib.ptr(ah), _lib.ptr(ag), _lib.ptr(apos), _lib.ptr(avel), _lib.ptr(aldj),
                _lib.ptr(grad_layers), _lib.ptr(grad_dq), _lib.ptr(ws), wsb, prb, _lib.ptr(err),
                _lib.stream_ptr(dev)), "enflow_lf_backward_f32")
        if meta["check_errors"]:
            # the forward's deferred word (the reference's IndexError), read once the
            # backward is queued behind it, so the device never drains while the host
            # prepares the backward; raised before any gradient is returned (the
            # backward kernels validate their own geometry and only compute on a
            # failed batch's state).  The backward's own word is read at the next check.
            _lib.check_pending()
            _lib.defer_err(err)
        # split the flat gradients into the parameters' shapes (inputs order)
        grads = []
        rstride = grad_layers.numel() // max(len(flow.networks), 1)
        for li, net in enumerate(flow.networks):
            grads += layer_grads(net, grad_layers[li * rstride:(li + 1) * rstride])
        if kind == _lib.DEQUANT_ARGMAX:
            am = flow.dequantize
            grads += argmax_grads(am, grad_dq, am.pad_geom(hid))
        # d h of the data only exists without a learned dequantiser (z = h + noise)
        gh_in = ah if kind != _lib.DEQUANT_ARGMAX else None
        return (None, None, gh_in, ag, apos, avel) + tuple(grads)


_warned_bf16 = []


def flow_forward_train(flow, data, noise, check_errors):
    """Differentiable LFIntegrator.forward (HIP forward with tape)."""
    flow._check_trainable()
    s = flow._state(data)
    dev = s["dev"]
    kind = flow._dequant_kind()
    if noise is None:
        if kind == _lib.DEQUANT_ARGMAX:
            noise = torch.randn(s["h"].shape, device=dev, dtype=torch.float32)
        elif kind == _lib.DEQUANT_FLOOR:
            noise = torch.rand(s["h"].shape, device=dev, dtype=torch.float32)
    else:
        noise = noise.to(device=dev, dtype=torch.float32).contiguous()
    large = s["max_n"] > _lib.TRAIN_MAX_ATOMS   # past the fused backward: large-system training kernels
    meta = dict(box=s["box"], r_cut=s["r_cut"], mol_ptr=s["mol_ptr"], max_n=s["max_n"], noise=noise,
                check_errors=check_errors, large=large,
                pair_row_bound=0 if large else pair_row_bound(data.N))
    params = [p for n in flow.networks for _, p in n.named_parameters()]
    if isinstance(flow.dequantize, ArgMax):
        params += list(flow.dequantize.parameters())

    def inp(t):
        return t.to(device=dev, dtype=torch.float32)

    h, g, pos, vel, ldj = _FlowFunction.apply(flow, meta, inp(data.h), inp(data.g), inp(data.pos),
                                              inp(data.vel), *params)
    dt = data.h.dtype
    data.h, data.g = h.to(dt), g.to(dt)
    data.pos, data.vel = pos.to(data.pos.dtype), vel.to(data.vel.dtype)
    return data, ldj.to(dt)


class _NLLFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, nll, meta, h, g, pos, vel, ldj):
        L = _lib.lib(h.shape[1])
        dev = h.device
        M = meta["mol_ptr"].numel() - 1
        nll_mol = torch.empty((max(M, 1), 4), dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        ldj_t = ldj.detach().reshape(1).contiguous()
        hc, gc, pc, vc = (t.detach().contiguous() for t in (h, g, pos, vel))
        _lib.check(L.enflow_alchemical_nll_f32(M, h.shape[0], meta["max_n"], h.shape[1],
                                               _lib.ptr(meta["mol_ptr"]), _lib.ptr(hc), _lib.ptr(gc),
                                               _lib.ptr(pc), _lib.ptr(vc), _lib.ptr(ldj_t), float(nll.kBT),
                                               float(nll.softening), float(nll.z_lj), _lib.ptr(nll_mol),
                                               _lib.ptr(loss), _lib.stream_ptr(dev)), "enflow_alchemical_nll_f32")
        ctx.nll, ctx.meta = nll, meta
        ctx.save_for_backward(hc, gc, pc, vc)
        return loss.reshape(())

    @staticmethod
    def backward(ctx, gloss):
        h, g, pos, vel = ctx.saved_tensors
        nll, meta = ctx.nll, ctx.meta
        L = _lib.lib(h.shape[1])
        dev = h.device
        M = meta["mol_ptr"].numel() - 1
        ah, ag = torch.empty_like(h), torch.empty_like(g)
        apos, avel = torch.empty_like(pos), torch.empty_like(vel)
        aldj = torch.empty(1, dtype=torch.float32, device=dev)
        gl = gloss.detach().to(torch.float32).reshape(1).contiguous()
        _lib.check(L.enflow_alchemical_nll_backward_f32(
            M, h.shape[0], meta["max_n"], h.shape[1], _lib.ptr(meta["mol_ptr"]), _lib.ptr(h), _lib.ptr(g),
            _lib.ptr(pos), _lib.ptr(vel), float(nll.kBT), float(nll.softening), _lib.ptr(gl), _lib.ptr(ah),
            _lib.ptr(ag), _lib.ptr(apos), _lib.ptr(avel), _lib.ptr(aldj), _lib.stream_ptr(dev)),
            "enflow_alchemical_nll_backward_f32")
        return None, None, ah, ag, apos, avel, aldj.reshape(())


# ---------------------------------------------------------------------------
# standalone modules: EGCL.forward (enflow/nn/egcl.py:76-92) and ArgMax.forward
# (enflow/nn/argmax.py:13-25) as autograd Functions over the HIP backward
# ---------------------------------------------------------------------------
def layer_grads(net, flat):
    """Split one layer's flat gradient (layers_raw layout at the kernel width:
    default-flag parameters in named order, then att_nn.0 weight / bias in the
    width + 1 slots) into the module's parameters, in named_parameters() order
    (the real block of each zero-padded tensor, nn/_pad.py)."""
    geom = net.pad_geom()
    g, off = unpad_grads(flat, net.raw_named(), EGCL_HDIMS, geom)
    att = [(k, p) for k, p in net.named_parameters() if k.startswith("att_nn.")]
    if att:
        ga, _ = unpad_grads(flat[off:], att, EGCL_HDIMS, geom)
        g.update(ga)
    # act_fn's own parameters (a frozen PReLU slope) get no gradient
    own = net.act_param_ids()
    return [None if id(p) in own else g[name].contiguous().to(p.dtype)
            for name, p in net.named_parameters()]


def argmax_grads(am, flat, geom):
    """ArgMax's flat gradient split into its parameters, named_parameters() order
    (None for a frozen PReLU slope, network.1)."""
    gd, _ = unpad_grads(flat, am.kernel_named(), ARGMAX_HDIMS, geom)
    return [None if k.startswith("network.1.") else gd[k].contiguous().to(p.dtype)
            for k, p in am.named_parameters()]


class _EGCLFunction(torch.autograd.Function):
    """EGCL.forward with the HIP backward: outputs from enflow_egcl_forward_f32;
    the backward regenerates the one-layer tape (message sums, pair counts) with
    enflow_lf_forward_f32 and runs enflow_egcl_backward_f32."""

    @staticmethod
    def forward(ctx, net, meta, h, pos, *params):
        q, f, g = net._infer(h.detach(), pos.detach(), meta)
        ctx.net, ctx.meta = net, meta
        ctx.save_for_backward(net.pad_h(h.detach()), pos.detach().to(torch.float32).contiguous())
        return q, f, g

    @staticmethod
    def backward(ctx, gq, gf, gg):
        net, meta = ctx.net, ctx.meta
        h, pos = ctx.saved_tensors
        large = meta["max_n"] > _lib.TRAIN_MAX_ATOMS
        L = _lib.lib(net.kernel_nf)
        dev = h.device
        A, nf, hid = h.shape[0], net.kernel_nf, net.kernel_hidden
        M = meta["mol_ptr"].numel() - 1
        st = _lib.stream_ptr(dev)
        prec = _lib.PREC_F16X3 | (_lib.EGCL_VARIANTS if net.variant_flags() else 0)
        # the one-layer tape: layer-input state, message sums, Q; pair counts
        hw, pw = h.clone(), pos.clone()
        gw = torch.zeros_like(h)
        vw = torch.zeros_like(pos)
        tape = torch.empty(max(L.enflow_lf_tape_size_for(A, nf, hid, 1, meta["max_n"]), 1), dtype=torch.float32,
                           device=dev)
        counts = torch.zeros(max(M, 1), dtype=torch.int32, device=dev)
        ldj_mol = torch.empty(max(M, 1), dtype=torch.float32, device=dev)
        ldj = torch.empty(1, dtype=torch.float32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        fwd = net.packed(dev)
        if large:   # the large-system forward records the tape and the backward's pair rows
            lws = _lib.large_workspace(M, A, meta["max_n"], nf, dev)
            _lib.check(L.enflow_lf_forward_large_f32(
                M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(hw), _lib.ptr(gw), _lib.ptr(pw), _lib.ptr(vw), _lib.ptr(fwd), 1,
                _lib.DEQUANT_NONE, None, None, 0.0, 0.0, float(net.coords_weight), _lib.ptr(ldj_mol), _lib.ptr(ldj),
                _lib.ptr(err), prec, _lib.ptr(tape), _lib.ptr(counts), _lib.ptr(lws), lws.numel(), st),
                "enflow_lf_forward_large_f32 (EGCL tape)")
        else:
            _lib.check(L.enflow_lf_forward_f32(
                M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(hw), _lib.ptr(gw), _lib.ptr(pw), _lib.ptr(vw), _lib.ptr(fwd), 1,
                _lib.DEQUANT_NONE, None, None, 0.0, 0.0, float(net.coords_weight), _lib.ptr(ldj_mol), _lib.ptr(ldj),
                _lib.ptr(err), None, _lib.ptr(tape), _lib.ptr(counts), prec, st), "enflow_lf_forward_f32 (EGCL tape)")
        bwd_flags = net.variant_flags()
        e = _lib.take_err(err)
        if e and not e & ~_lib.ERR_RERUN:
            # the f16x3 tape lost its range (overflow, or an operand entirely below
            # 2^-7): the tape again with fp32 GEMMs, and the fp32 backward on it
            prec = (prec & ~0xff) | _lib.PREC_F32
            bwd_flags |= _lib.BWD_F32
            hw.copy_(h), pw.copy_(pos), gw.zero_(), vw.zero_(), counts.zero_()
            _lib.FP32_RERUNS[0] += 1
            if large:
                _lib.check(L.enflow_lf_forward_large_f32(
                    M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                    _lib.ptr(meta["box"]), _lib.ptr(hw), _lib.ptr(gw), _lib.ptr(pw), _lib.ptr(vw), _lib.ptr(fwd), 1,
                    _lib.DEQUANT_NONE, None, None, 0.0, 0.0, float(net.coords_weight), _lib.ptr(ldj_mol),
                    _lib.ptr(ldj), _lib.ptr(err), prec, _lib.ptr(tape), _lib.ptr(counts), _lib.ptr(lws), lws.numel(),
                    st), "enflow_lf_forward_large_f32 (EGCL tape, fp32)")
            else:
                _lib.check(L.enflow_lf_forward_f32(
                    M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                    _lib.ptr(meta["box"]), _lib.ptr(hw), _lib.ptr(gw), _lib.ptr(pw), _lib.ptr(vw), _lib.ptr(fwd), 1,
                    _lib.DEQUANT_NONE, None, None, 0.0, 0.0, float(net.coords_weight), _lib.ptr(ldj_mol),
                    _lib.ptr(ldj), _lib.ptr(err), None, _lib.ptr(tape), _lib.ptr(counts), prec, st),
                    "enflow_lf_forward_f32 (EGCL tape, fp32)")
            e = _lib.take_err(err)
        _lib.raise_code(e)
        raw = torch.cat([net.kernel_raw(dev), net._att_raw(dev) if net.attention else torch.zeros(hid + 1, device=dev)])
        bwd = torch.empty(max(L.enflow_egcl_bwd_packed_size(hid, nf), 1), dtype=torch.float32, device=dev)
        _lib.check(L.enflow_pack_egcl_bwd_f32(_lib.ptr(raw), hid, nf, _lib.ptr(bwd), st), "enflow_pack_egcl_bwd_f32")
        if large:
            prb = int(counts[0].item())
            wsb = L.enflow_egcl_backward_large_workspace_size(M, A, meta["max_n"], nf, hid, prb)
        else:
            prb = pair_row_bound(meta["N"])
            wsb = L.enflow_egcl_backward_workspace_size(M, A, nf, hid, prb)
        if wsb < 0:
            raise _lib.HipPathError("enflow_egcl_backward_workspace_size rejected the batch")
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)

        def adj(t, shape):
            if t is None:
                return torch.zeros(shape, dtype=torch.float32, device=dev)
            return t.detach().to(dtype=torch.float32).reshape(shape).contiguous()

        aq, af = adj(gq, (A,)), adj(gf, (A, 3))
        ag = torch.zeros((A, nf), dtype=torch.float32, device=dev)   # G's padded columns: no adjoint
        if gg is not None:
            ag[:, :net.output_nf] = gg.detach().to(torch.float32).reshape(A, net.output_nf)
        dh = torch.empty((A, nf), dtype=torch.float32, device=dev)
        dpos = torch.empty((A, 3), dtype=torch.float32, device=dev)
        grad = torch.empty_like(raw)
        if large:
            _lib.check(L.enflow_egcl_backward_large_f32(
                M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(tape), _lib.ptr(fwd), _lib.ptr(bwd), _lib.ptr(raw),
                bwd_flags, float(net.coords_weight), _lib.ptr(aq), _lib.ptr(af), _lib.ptr(ag),
                _lib.ptr(dh), _lib.ptr(dpos), _lib.ptr(grad), _lib.ptr(ws), wsb, prb, _lib.ptr(err), st),
                "enflow_egcl_backward_large_f32")
        else:
            _lib.check(L.enflow_egcl_backward_f32(
                M, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(meta["r_cut"]),
                _lib.ptr(meta["box"]), _lib.ptr(tape), _lib.ptr(counts), _lib.ptr(fwd), _lib.ptr(bwd),
                _lib.ptr(raw), bwd_flags, float(net.coords_weight), _lib.ptr(aq), _lib.ptr(af),
                _lib.ptr(ag), _lib.ptr(dh), _lib.ptr(dpos), _lib.ptr(grad), _lib.ptr(ws), wsb, prb, _lib.ptr(err),
                st), "enflow_egcl_backward_f32")
        _lib.raise_on_err(err)
        return (None, None, dh[:, :net.input_nf], dpos) + tuple(layer_grads(net, grad))


class _ArgMaxFunction(torch.autograd.Function):
    """ArgMax.forward with the HIP backward (enflow_argmax_backward_f32)."""

    @staticmethod
    def forward(ctx, am, meta, h, noise, *params):
        z, lq = am._infer(h.detach(), noise, meta)
        ctx.am, ctx.meta = am, meta
        ctx.save_for_backward(h.detach().to(torch.float32).contiguous(), noise)
        return z, lq

    @staticmethod
    def backward(ctx, gz, glq):
        am, meta = ctx.am, ctx.meta
        h, noise = ctx.saved_tensors
        L = _lib.lib(am.node_nf)
        dev = h.device
        A, nf, hid = h.shape[0], am.node_nf, am.kernel_hidden
        raw = am.kernel_raw(dev)
        az = (torch.zeros_like(h) if gz is None else gz.detach().to(torch.float32).contiguous())
        alq = (torch.zeros(1, device=dev) if glq is None else glq.detach().to(torch.float32).reshape(1).contiguous())
        grad = torch.empty_like(raw)
        wsb = L.enflow_argmax_backward_workspace_size(A, nf, hid)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        _lib.check(L.enflow_argmax_backward_f32(
            meta["mol_ptr"].numel() - 1, A, meta["max_n"], nf, hid, _lib.ptr(meta["mol_ptr"]), _lib.ptr(h),
            _lib.ptr(raw), _lib.ptr(noise), _lib.ptr(az), _lib.ptr(alq), _lib.ptr(grad), _lib.ptr(ws), wsb,
            _lib.stream_ptr(dev)), "enflow_argmax_backward_f32")
        grads = argmax_grads(am, grad, am.pad_geom())
        # h is the categorical data (one-hot, argmax.py:13): no gradient is returned for it
        return (None, None, None, None) + tuple(grads)
