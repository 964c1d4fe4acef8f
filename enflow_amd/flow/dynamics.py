"""Leapfrog coupling flow (mirrors enflow/flow/dynamics.py:4-37).

``LFIntegrator.forward(data) -> (data, ldj)`` and ``reverse(data) -> data``
run the whole flow -- dequantisation, every layer's periodic neighbour list,
EGCL and leapfrog update, and the log|detJ| sum -- as ONE HIP kernel launch
(enflow_lf_forward_f32 / enflow_lf_reverse_f32): one workgroup per molecule,
molecule state resident in LDS across layers.  Systems larger than that LDS
image (> enflow_max_atoms() atoms, e.g. the reference's 2944-atom LJ box in
example/generate.yaml) run layer by layer through the large-system kernels
(enflow_lf_forward_large_f32 / enflow_lf_reverse_large_f32).  Like the reference, ``data`` is
updated (its tensors rebound) and returned.

VVIntegrator (dynamics.py:39-86) is not provided: in the reference it cannot
run (it reads ``self.n_iter``, which BaseFlow never sets, and treats the
dequantiser's (z, ldj) tuple as a tensor), see DESIGN.md.
"""
import warnings

import torch

from .. import _lib
from ..nn._act import check_trainable
from ..nn.argmax import ArgMax
from ..nn.egcl import EGCL
from ..nn.floor import Floor
from ..utils.helpers import batch_meta, params_of
from .base import BaseFlow


class LFIntegrator(BaseFlow):
    """``gemm_precision`` selects how the two H x H edge GEMMs run on the
    matrix cores: "f32" (exact fp32 MFMA), "f16x3" (fp32 operands split into
    fp16 hi+lo, three products, fp32 accumulation; default) or "bf16"
    (reduced-precision generate path, BASELINE configs[2])."""
    gemm_precision = "f16x3"
    # training forward: False (default) reads the kernel's error word before
    # returning, so a bad batch raises inside forward like the reference
    # (enflow/data/base.py:137); True queues it and raises at the start of
    # loss.backward() instead (no host sync between forward and backward)
    defer_error_check = False

    def _prec(self):
        try:
            p = _lib.PRECISIONS[self.gemm_precision]
        except KeyError:
            raise ValueError(f"gemm_precision must be one of {sorted(_lib.PRECISIONS)}") from None
        if self._has_variants():
            p |= _lib.EGCL_VARIANTS      # attention / norm_diff / tanh / act_fn layers: variant-capable kernels
        return p

    def make_networks(self, network):
        return [network for _ in range(self.n_iter)]

    # ------------------------------------------------------------------
    def _geometry(self):
        nets = list(self.networks)
        if not nets:
            return None, None, 1.0
        if not all(isinstance(n, EGCL) for n in nets):
            raise NotImplementedError("LFIntegrator on the HIP path needs enflow_amd.nn.EGCL networks")
        h0, f0 = nets[0].hidden_nf, nets[0].input_nf
        for n in nets:
            n._check_supported()
            if n.input_nf != n.output_nf:   # dynamics.py:17-18 adds G to g
                raise NotImplementedError("LFIntegrator needs EGCL layers with input_nf == output_nf")
            if (n.hidden_nf, n.input_nf) != (h0, f0) or n.coords_weight != nets[0].coords_weight:
                raise NotImplementedError("all EGCL layers must share hidden_nf, node_nf and coords_weight")
        # the kernels' hidden width (hidden_nf, or zero-padded to the next compiled one)
        return nets[0].kernel_hidden, f0, float(nets[0].coords_weight)

    def _dequant_kind(self):
        d = self.dequantize
        if isinstance(d, ArgMax):
            return _lib.DEQUANT_ARGMAX
        if isinstance(d, Floor):
            return _lib.DEQUANT_FLOOR
        if d is None:
            return _lib.DEQUANT_NONE
        raise NotImplementedError(f"unsupported dequantiser {type(d).__name__}")

    def _params_key(self, device):
        return (str(device),) + tuple((p.data_ptr(), p._version) for n in self.networks for p in params_of(n))

    def launch_cfg(self, device):
        """The module's half of a fused inference launch -- geometry,
        dequantiser, precision word, packed weights -- computed the full way
        (every layer checked, every parameter's version compared by
        packed_layers), so it reflects the module as it is now."""
        hid, nf, cw = self._geometry()
        kind = self._dequant_kind()
        prec = self._prec()
        layers = self.packed_layers(device)
        dq = self.dequantize.packed(device, hid) if kind == _lib.DEQUANT_ARGMAX else None
        scale = float(getattr(self.dequantize, "dequant_scale", 1.0)) if kind == _lib.DEQUANT_FLOOR else 0.0
        return _LaunchCfg(str(device), hid, nf, cw, kind, prec, layers, dq, scale, len(self.networks), float(self.dt))

    def packed_layers(self, device):
        """All layers packed back to back (cached; re-packed on any parameter change)."""
        key = self._params_key(device)
        if getattr(self, "_layers_key", None) == key:
            return self._layers_buf
        hid, nf, _ = self._geometry()
        L = _lib.lib(nf)
        stride = L.enflow_egcl_packed_size(hid, nf)
        buf = torch.empty(max(stride * len(self.networks), 1), dtype=torch.float32, device=device)
        for i, n in enumerate(self.networks):
            n.pack_into(buf[i * stride:(i + 1) * stride])
        self._layers_buf, self._layers_key = buf, key
        return buf

    def training_layers(self, device):
        """(forward-packed, backward-packed, raw) layer buffers for the HIP backward."""
        key = self._params_key(device)
        if getattr(self, "_train_key", None) == key:
            return self._train_bufs
        hid, nf, _ = self._geometry()
        L = _lib.lib(nf)
        self._check_trainable()
        # per layer: the default-flag raw parameters, then att_nn.0 (weight, bias) or
        # H + 1 zeros (enflow_lf_backward_f32's layers_raw stride)
        # (one flat cat launch; the zero pad is allocated once per device)
        zkey = (str(device), hid)
        if getattr(self, "_zpad_key", None) != zkey:
            self._zpad = torch.zeros(hid + 1, dtype=torch.float32, device=device)
            self._zpad_key = zkey
        zpad = self._zpad
        pieces = []
        for n in self.networks:
            pieces.append(n.kernel_raw(device))
            pieces.append(n._att_raw(device) if n.attention else zpad)
        raw = torch.cat(pieces)
        stride = L.enflow_egcl_bwd_packed_size(hid, nf)
        n_l = len(self.networks)
        rstride = raw.numel() // max(n_l, 1)
        bwd = torch.empty(max(stride * n_l, 1), dtype=torch.float32, device=device)
        st = _lib.stream_ptr(device)
        if n_l and hasattr(L, "enflow_pack_egcl_layers_f32") and not any(n.variant_flags() for n in self.networks):
            # default-flag SiLU layers (the training loop's repack after every
            # optimiser step): both sections of every layer in two launches each
            # (ABI 13) instead of two per layer and section; the forward section is
            # packed_layers' buffer, from the same raw parameters
            fstride = L.enflow_egcl_packed_size(hid, nf)
            fwd = torch.empty(max(fstride * n_l, 1), dtype=torch.float32, device=device)
            _lib.check(L.enflow_pack_egcl_layers_f32(_lib.ptr(raw), rstride, n_l, hid, nf, _lib.ptr(fwd), st),
                       "enflow_pack_egcl_layers_f32")
            _lib.check(L.enflow_pack_egcl_bwd_layers_f32(_lib.ptr(raw), rstride, n_l, hid, nf, _lib.ptr(bwd), st),
                       "enflow_pack_egcl_bwd_layers_f32")
            self._layers_buf, self._layers_key = fwd, key
        else:
            for i in range(n_l):
                _lib.check(L.enflow_pack_egcl_bwd_f32(_lib.ptr(raw[i * rstride:]), hid, nf,
                                                      _lib.ptr(bwd[i * stride:]), st), "enflow_pack_egcl_bwd_f32")
        self._train_bufs = (self.packed_layers(device), bwd, raw)
        self._train_key = key
        return self._train_bufs

    def _has_variants(self):
        """Layers with constructor variants or a non-SiLU act_fn, or an ArgMax
        dequantiser with a non-SiLU activation: the variant-capable kernels."""
        return (any(isinstance(n, EGCL) and n.variant_flags() for n in self.networks)
                or (isinstance(self.dequantize, ArgMax) and self.dequantize.generic_act()))

    def _check_trainable(self):
        """The HIP backward covers every EGCL constructor variant (attention,
        norm_diff, tanh); non-EGCL networks are refused (by _geometry), and
        node_nf 16 (the backward holds 2 node_nf + 1 <= 32 edge inputs)."""
        _, nf, _ = self._geometry()
        if nf is not None and nf > _lib.TRAIN_MAX_NODE_NF:
            raise NotImplementedError(f"enflow_amd trains node_nf <= {_lib.TRAIN_MAX_NODE_NF} (got {nf}); "
                                      "inference runs up to 16")
        for n in self.networks:
            check_trainable(n.act_fn, "LFIntegrator training")
        if isinstance(self.dequantize, ArgMax):
            check_trainable(self.dequantize.network[1], "LFIntegrator training (ArgMax)")

    def _needs_grad(self):
        return torch.is_grad_enabled() and any(p.requires_grad for p in params_of(self))

    def _warn_grad(self):
        if self._needs_grad():
            warnings.warn("enflow_amd LFIntegrator.reverse is not differentiable (the reference "
                          "only trains through forward); outputs are detached",
                          RuntimeWarning, stacklevel=3)

    # ------------------------------------------------------------------
    def forward_buffers(self, h, g, pos, vel, box, r_cut, mol_ptr, max_mol_atoms, noise,
                        ldj_mol, ldj_total, err, pair_stats=None, tape=None, pair_counts=None, prec=None,
                        src=None, noise_key=(0, 0), ticket=None, mol_err=None, mol_list=None, cfg=None):
        """Fused forward on preallocated fp32 device buffers (no host sync, no
        allocation): the entry point the benchmark times.  ``src`` = (h, g,
        pos, vel) inputs read by the kernel (None: h, g, pos, vel are updated
        in place); ``noise`` None draws the dequantiser's noise in the kernel
        (Philox keyed by ``noise_key`` = (seed, offset)); ``ticket`` (uint32
        device word, zero) reduces log|detJ| in the same launch
        (enflow_lf_forward_io_f32).  ``mol_err`` (int32 [M], zeroed) receives
        each molecule's error bits and ``mol_list`` (int32 device tensor) runs
        only those molecules, in place (enflow_lf_forward_io2_f32, ABI 12).
        ``cfg``: a launch_cfg() to use (default: computed now).
        Molecules past the fused kernel's LDS image (> enflow_max_atoms()) go
        through the layer-by-layer large-system kernels
        (enflow_lf_forward_large_f32; needs a workspace, allocated once per
        shape; no per-molecule words there)."""
        c = self.launch_cfg(h.device) if cfg is None else cfg
        hid, nf, cw, kind = c.hid, c.nf, c.cw, c.kind
        dev = h.device
        prec = c.prec if prec is None else prec
        L = _lib.lib(nf)
        # training past the fused backward's molecule size records its tape on the
        # large-system path (pair_counts then holds the per-layer pair rows)
        if _lib.is_large(max_mol_atoms) or (tape is not None and max_mol_atoms > _lib.TRAIN_MAX_ATOMS):
            if src is not None:      # the layer-by-layer path updates its state in place
                for o, i in zip((h, g, pos, vel), src):
                    if o.data_ptr() != i.data_ptr():
                        o.copy_(i)
            if noise is None and kind != _lib.DEQUANT_NONE:
                noise = _host_noise(kind, h.shape, dev)
            ws = _lib.large_workspace(mol_ptr.numel() - 1, h.shape[0], max_mol_atoms, nf, dev)
            _lib.check(L.enflow_lf_forward_large_f32(
                mol_ptr.numel() - 1, h.shape[0], max_mol_atoms, nf, hid,
                _lib.ptr(mol_ptr), _lib.ptr(r_cut), _lib.ptr(box), _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos),
                _lib.ptr(vel), _lib.ptr(c.layers), c.n_layers, kind, _lib.ptr(c.dq),
                _lib.ptr(noise), c.scale, c.dt, cw, _lib.ptr(ldj_mol), _lib.ptr(ldj_total),
                _lib.ptr(err), prec & ~_lib.PREC_NO_SPLIT, _lib.ptr(tape),
                _lib.ptr(pair_counts if tape is not None else None),
                _lib.ptr(ws), ws.numel(), _lib.stream_ptr(dev)),
                "enflow_lf_forward_large_f32")
            return
        si = (None,) * 4 if src is None else tuple(_lib.ptr(t) for t in src)
        args = (mol_ptr.numel() - 1, h.shape[0], max_mol_atoms, nf, hid,
                _lib.ptr(mol_ptr), _lib.ptr(r_cut), _lib.ptr(box), *si, _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos),
                _lib.ptr(vel), _lib.ptr(c.layers), c.n_layers, kind, _lib.ptr(c.dq),
                _lib.ptr(noise), int(noise_key[0]) & 0xFFFFFFFFFFFFFFFF, int(noise_key[1]) & 0xFFFFFFFFFFFFFFFF,
                c.scale, c.dt, cw, _lib.ptr(ldj_mol), _lib.ptr(ldj_total), _lib.ptr(ticket),
                _lib.ptr(err), _lib.ptr(pair_stats), _lib.ptr(tape), _lib.ptr(pair_counts), prec)
        if mol_err is None and mol_list is None:
            _lib.check(L.enflow_lf_forward_io_f32(*args, _lib.stream_ptr(dev)), "enflow_lf_forward_io_f32")
        else:
            _lib.check(L.enflow_lf_forward_io2_f32(
                *args, _lib.ptr(mol_err), _lib.ptr(mol_list), 0 if mol_list is None else mol_list.numel(),
                _lib.stream_ptr(dev)), "enflow_lf_forward_io2_f32")

    def reverse_buffers(self, h, g, pos, vel, box, r_cut, mol_ptr, max_mol_atoms, argmax_idx, max_idx, err,
                        src=None, prec=None, mol_err=None, mol_list=None, cfg=None):
        """Fused reverse on preallocated fp32 device buffers (no host sync, no
        allocation); ``src`` = (h, g, pos, vel) inputs (None: in place); with
        ArgMax, argmax_idx / max_idx receive the dequantiser's indices
        (enflow_one_hot_f32 materialises the one-hot)."""
        c = self.launch_cfg(h.device) if cfg is None else cfg
        hid, nf, cw, kind = c.hid, c.nf, c.cw, c.kind
        L = _lib.lib(nf)
        prec = c.prec if prec is None else prec
        if _lib.is_large(max_mol_atoms):
            if src is not None:
                for o, i in zip((h, g, pos, vel), src):
                    if o.data_ptr() != i.data_ptr():
                        o.copy_(i)
            ws = _lib.large_workspace(mol_ptr.numel() - 1, h.shape[0], max_mol_atoms, nf, h.device)
            _lib.check(L.enflow_lf_reverse_large_f32(
                mol_ptr.numel() - 1, h.shape[0], max_mol_atoms, nf, hid, _lib.ptr(mol_ptr), _lib.ptr(r_cut),
                _lib.ptr(box), _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos), _lib.ptr(vel),
                _lib.ptr(c.layers), c.n_layers, kind, c.dt, cw,
                _lib.ptr(argmax_idx), _lib.ptr(max_idx), _lib.ptr(err), prec & ~_lib.PREC_NO_SPLIT, _lib.ptr(ws),
                ws.numel(), _lib.stream_ptr(h.device)), "enflow_lf_reverse_large_f32")
            return
        si = (None,) * 4 if src is None else tuple(_lib.ptr(t) for t in src)
        args = (mol_ptr.numel() - 1, h.shape[0], max_mol_atoms, nf, hid, _lib.ptr(mol_ptr), _lib.ptr(r_cut),
                _lib.ptr(box), *si, _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos), _lib.ptr(vel),
                _lib.ptr(c.layers), c.n_layers, kind, c.dt, cw,
                _lib.ptr(argmax_idx), _lib.ptr(max_idx), _lib.ptr(err), prec)
        if mol_err is None and mol_list is None:
            _lib.check(L.enflow_lf_reverse_io_f32(*args, _lib.stream_ptr(h.device)), "enflow_lf_reverse_io_f32")
        else:
            _lib.check(L.enflow_lf_reverse_io2_f32(
                *args, _lib.ptr(mol_err), _lib.ptr(mol_list), 0 if mol_list is None else mol_list.numel(),
                _lib.stream_ptr(h.device)), "enflow_lf_reverse_io2_f32")

    def _state(self, data, outputs=True):
        """Kernel inputs (fp32, contiguous, on the device: the data's own
        tensors when they already are) and fresh output buffers."""
        _lib.require_gpu(data.pos)
        dev = data.pos.device
        ptr, max_n = batch_meta(data, dev)
        src = tuple(_as_f32(t, dev) for t in (data.h, data.g, data.pos, data.vel))
        rc = data.r_cut
        rc = (rc if isinstance(rc, torch.Tensor) and rc.device == dev and rc.dtype == torch.float32 and rc.dim() == 1
              else torch.as_tensor(rc, device=dev).to(torch.float32).reshape(-1).contiguous())
        s = dict(src=src, box=_as_f32(data.box, dev), r_cut=rc, mol_ptr=ptr, max_n=max_n, dev=dev)
        if outputs:
            s["h"], s["g"], s["pos"], s["vel"] = (torch.empty_like(t) for t in src)
        return s

    def _spec_cfg(self, dev, nf_data):
        """(cfg, fresh): the previous call's launch_cfg for this device, used
        speculatively and checked after the launch (fresh None), or -- first
        call, or data whose feature width it does not match -- a fresh one."""
        spec = self.__dict__.get("_spec")
        if spec is None:
            spec = self.__dict__["_spec"] = {}
        c = spec.get(str(dev))
        if c is not None and c.nf == nf_data:
            return c, None
        c = self.launch_cfg(dev)
        if c.nf != nf_data:
            raise ValueError(f"data has {nf_data} node features, the flow's layers {c.nf}")
        return c, c

    def _confirm_cfg(self, dev, cfg, fresh):
        """After a speculative launch: the launch_cfg of the module as it is now
        (the full check, while the kernel runs), remembered for the next call;
        None if the launch used it, else the new cfg to launch again with."""
        if fresh is None:
            fresh = self.launch_cfg(dev)
        self._spec[str(dev)] = fresh
        return None if fresh.same(cfg) else fresh

    def forward(self, data, noise=None, check_errors=True):
        """dynamics.py:10-24.  ``noise`` optionally supplies the dequantiser's
        draw (N(0,1) for ArgMax, U[0,1) for Floor), shape h.shape.

        With autograd enabled and trainable parameters the outputs carry a
        grad_fn whose backward is the HIP backward (enflow_lf_backward_f32;
        batches with molecules past 64 atoms: enflow_lf_backward_large_f32),
        so the reference's ``loss.backward()`` / optimiser loop runs unchanged.

        Inference is one launch with the host's work around it kept off the
        device's path: the previous call's launch_cfg is used speculatively
        and the module is checked (layers, parameter versions: launch_cfg)
        while the kernel runs -- a changed module launches again before
        anything is returned -- and the per-molecule error words, log|detJ|
        partials and status words are cached per (device, stream) and stay
        zero between calls."""
        if self._needs_grad():
            from ._train import flow_forward_train
            return flow_forward_train(self, data, noise, check_errors)
        s = self._state(data)
        dev = s["dev"]
        cfg, fresh = self._spec_cfg(dev, s["src"][0].shape[1])
        key = (0, 0)
        if noise is None:
            # the dequantiser's draws are made in the kernel (N(0,1) / U[0,1),
            # argmax.py:16 / floor.py), keyed from torch's generator so that
            # torch.manual_seed makes runs reproducible
            key = (int(torch.randint(0, 2 ** 62, (1,)).item()), 0)
        else:
            noise = noise.to(device=dev, dtype=torch.float32).contiguous()
        large = _lib.is_large(s["max_n"])
        if noise is None and large and cfg.kind != _lib.DEQUANT_NONE:
            # the large-system path takes its draws from the caller: draw once here so
            # that a range re-run (below) sees the same noise
            noise = _host_noise(cfg.kind, s["h"].shape, dev)
        M = s["mol_ptr"].numel() - 1
        ldj = torch.empty(1, dtype=torch.float32, device=dev)
        w = _lib.infer_words(dev, M)
        st = w.status if check_errors else torch.zeros(2, dtype=torch.int32, device=dev)
        if check_errors:
            _lib.check_pending()     # an older deferred error is not this launch's
        # per-molecule error words (fused path): a split-precision flag names its molecules
        mol_err = w.mol_err if check_errors and not large else None
        prec, mol_list = None, None

        def launch(c, prec=None, mol_list=None):
            self.forward_buffers(s["h"], s["g"], s["pos"], s["vel"], s["box"], s["r_cut"], s["mol_ptr"],
                                 s["max_n"], noise, w.ldj_mol, ldj, st[:1], src=s["src"], noise_key=key,
                                 ticket=st[1:] if mol_list is None else None, prec=prec, mol_err=mol_err,
                                 mol_list=mol_list, cfg=c)

        launch(cfg)
        redo = self._confirm_cfg(dev, cfg, fresh)
        if redo is not None:      # the module changed since the last call: the launch again on its current state
            st[:1].zero_()
            if mol_err is not None:
                mol_err.zero_()
            cfg = redo
            launch(cfg)
        prec = cfg.prec
        dt, pdt = data.h.dtype, data.pos.dtype

        def outputs():      # in the data's dtypes, queued behind the launch (no-ops for fp32 data)
            return (_as_dtype(s["h"], dt), _as_dtype(s["g"], dt), _as_dtype(s["pos"], pdt),
                    _as_dtype(s["vel"], data.vel.dtype), _as_dtype(ldj.reshape(()), dt))

        outs = outputs()    # a float64 caller's conversions run while the host waits for the word
        reran = False
        while check_errors:
            e = _lib.take_err(st[:1])
            if e & _lib.ERR_HANDOFF and not e & ~(_lib.ERR_HANDOFF | _lib.ERR_RERUN):
                # the two-workgroup instance lost a partner: this launch again without
                # the split instances (a per-call flag; the thresholds stay as they are)
                _lib.HANDOFF_RERUNS[0] += 1
                prec |= _lib.PREC_NO_SPLIT
                if mol_err is not None:
                    mol_err.zero_()
                launch(cfg, prec)
                reran = True
                e = _lib.take_err(st[:1])
            if _retry_fp32(e, prec):
                # a split-precision operand left its range (or was entirely small): the
                # same molecules with fp32 GEMMs (same noise elements, same inputs) give
                # the reference's result -- only the flagged molecules when the words
                # name few of them, else the whole launch
                prec = _fp32_prec(prec)
                _lib.FP32_RERUNS[0] += 1
                mol_list = None
                if mol_err is not None:
                    flagged = torch.nonzero(mol_err[:M] & _lib.ERR_RERUN).flatten().to(torch.int32)
                    if 0 < flagged.numel() <= max(1, M // 4):
                        mol_list = flagged.contiguous()
                        _lib.FP32_MOL_RERUNS[0] += mol_list.numel()
                    mol_err.zero_()
                launch(cfg, prec, mol_list)
                reran = True
                e = _lib.take_err(st[:1])
            if e and mol_err is not None:
                mol_err.zero_()      # the cached words stay zero between calls
            _lib.raise_code(e)
            break
        if reran:
            outs = outputs()
        data.h, data.g, data.pos, data.vel, ldj_out = outs
        return data, ldj_out

    def reverse(self, data, check_errors=True):
        """dynamics.py:26-37 (ends with dequantize.reverse).  The same
        speculative launch_cfg and cached words as forward; the error word and
        the ArgMax index maximum come back in one read."""
        self._warn_grad()
        s = self._state(data)
        dev = s["dev"]
        cfg, fresh = self._spec_cfg(dev, s["src"][0].shape[1])
        kind = cfg.kind
        n = s["h"].shape[0]
        M = s["mol_ptr"].numel() - 1
        large = _lib.is_large(s["max_n"])
        w = _lib.infer_words(dev, M, n)
        rw = w.rev if check_errors else torch.zeros(2, dtype=torch.int32, device=dev)   # error word, index maximum
        err, mx = rw[:1], rw[1:]
        if check_errors:
            _lib.check_pending()
        mol_err = w.mol_err if check_errors and not large else None

        def launch(c, prec=None, mol_list=None):
            self.reverse_buffers(s["h"], s["g"], s["pos"], s["vel"], s["box"], s["r_cut"], s["mol_ptr"],
                                 s["max_n"], w.idx, mx, err, src=s["src"], prec=prec, mol_err=mol_err,
                                 mol_list=mol_list, cfg=c)

        launch(cfg)
        redo = self._confirm_cfg(dev, cfg, fresh)
        if redo is not None:
            rw.zero_()
            if mol_err is not None:
                mol_err.zero_()
            cfg = redo
            kind = cfg.kind
            launch(cfg)
        prec, mol_list = cfg.prec, None
        words = [int(x) for x in rw.tolist()] if check_errors else [0, 0]
        while check_errors:
            e = words[0]
            if e & _lib.ERR_HANDOFF and not e & ~(_lib.ERR_HANDOFF | _lib.ERR_RERUN):
                _lib.HANDOFF_RERUNS[0] += 1
                prec |= _lib.PREC_NO_SPLIT
                rw.zero_()
                if mol_err is not None:
                    mol_err.zero_()
                launch(cfg, prec)
                words = [int(x) for x in rw.tolist()]
                e = words[0]
            if _retry_fp32(e, prec):     # as in forward: re-run the flagged molecules (or all) with fp32 GEMMs
                prec = _fp32_prec(prec)
                _lib.FP32_RERUNS[0] += 1
                if mol_err is not None:
                    flagged = torch.nonzero(mol_err[:M] & _lib.ERR_RERUN).flatten().to(torch.int32)
                    if 0 < flagged.numel() <= max(1, M // 4):
                        mol_list = flagged.contiguous()
                        _lib.FP32_MOL_RERUNS[0] += mol_list.numel()
                    mol_err.zero_()
                err.zero_()
                if mol_list is None:
                    mx.zero_()
                launch(cfg, prec, mol_list)
                words = [int(x) for x in rw.tolist()]
                e = words[0]
            if e and mol_err is not None:
                mol_err.zero_()
            if any(words):
                rw.zero_()           # the cached words stay zero between calls
            _lib.raise_code(e)
            break
        dt = data.h.dtype
        if kind == _lib.DEQUANT_ARGMAX:
            if mol_list is not None:
                # the first launch's batch maximum saw the flagged molecules' f16x3 argmax
                width = int(w.idx[:n].max().item()) + 1 if n > 0 else 1
            else:
                width = (words[1] if check_errors else int(mx.item())) + 1
            oh = torch.empty((n, width), dtype=torch.float32, device=dev)
            _lib.check(_lib.lib(cfg.nf).enflow_one_hot_f32(_lib.ptr(w.idx), n, width, _lib.ptr(oh),
                                                           _lib.stream_ptr(dev)), "enflow_one_hot_f32")
            data.h = _as_dtype(oh, dt)
        else:
            data.h = _as_dtype(s["h"], dt)
        data.g = _as_dtype(s["g"], dt)
        data.pos, data.vel = _as_dtype(s["pos"], data.pos.dtype), _as_dtype(s["vel"], data.vel.dtype)
        return data


class _LaunchCfg:
    """LFIntegrator.launch_cfg(): what a fused launch takes from the module."""
    __slots__ = ("dev", "hid", "nf", "cw", "kind", "prec", "layers", "dq", "scale", "n_layers", "dt")

    def __init__(self, dev, hid, nf, cw, kind, prec, layers, dq, scale, n_layers, dt):
        self.dev, self.hid, self.nf, self.cw, self.kind, self.prec = dev, hid, nf, cw, kind, prec
        self.layers, self.dq, self.scale, self.n_layers, self.dt = layers, dq, scale, n_layers, dt

    def same(self, o):
        """Equal scalars and the very same packed buffers (a re-pack allocates
        a new buffer, so a changed parameter never compares equal)."""
        return (self.layers is o.layers and self.dq is o.dq and
                (self.dev, self.hid, self.nf, self.cw, self.kind, self.prec, self.scale, self.n_layers, self.dt) ==
                (o.dev, o.hid, o.nf, o.cw, o.kind, o.prec, o.scale, o.n_layers, o.dt))


def _as_f32(t, dev):
    """t as a contiguous fp32 tensor on dev (t itself when it already is)."""
    if t.device == dev and t.dtype == torch.float32 and t.is_contiguous():
        return t.detach() if t.requires_grad else t
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def _as_dtype(t, dt):
    return t if t.dtype == dt else t.to(dt)


def _retry_fp32(e, prec):
    """The launch's own word says only ENFLOW_ERR_RANGE / ENFLOW_ERR_SMALL and
    the GEMMs were not fp32 yet: re-run with fp32 GEMMs (any other bit is raised
    as is)."""
    return e != 0 and not e & ~_lib.ERR_RERUN and (prec & 0xff) != _lib.PREC_F32


def _fp32_prec(prec):
    """The same kernel selection with fp32 edge GEMMs (variant / no-split bits kept)."""
    return (prec & ~0xff) | _lib.PREC_F32


def _host_noise(kind, shape, dev):
    """Draws for the large-system path (it takes the caller's noise)."""
    if kind == _lib.DEQUANT_ARGMAX:
        return torch.randn(shape, device=dev, dtype=torch.float32)
    return torch.rand(shape, device=dev, dtype=torch.float32)
