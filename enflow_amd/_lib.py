"""ctypes binding of the C ABI in include/enflow_hip.h (libenflow_hip.so).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc, gfx950).
There is deliberately no fallback: if the shared object is missing or cannot
be loaded every operator raises.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ENFLOW_LIB") or os.path.join(_HERE, "libenflow_hip.so")
# the same sources built with -DENFLOW_NFMAX=16: node_nf 9..16 (inference and training)
LIB_NF16_PATH = os.environ.get("ENFLOW_LIB_NF16") or os.path.join(_HERE, "libenflow_hip_nf16.so")
BASE_NFMAX = 8
MAX_NODE_NF = 16
# training takes every node_nf of the libraries (nf 16: the radial row of the
# backward's transposed edge_nn.0 GEMM, past its 32-row tile, is a separate dot)
TRAIN_MAX_NODE_NF = 16

ERR_TOO_MANY_ATOMS = 1
ERR_FEW_IMAGES = 2
ERR_TOO_MANY_FEATURES = 4
ERR_RANGE = 8
ERR_SMALL = 16      # ABI 12: f16x3 operand entirely small (precision, not overflow)
ERR_HANDOFF = 32    # ABI 12: a two-workgroup latency launch lost its partner (re-run without the split)
ERR_RERUN = ERR_RANGE | ERR_SMALL   # bits an fp32-GEMM re-run of the flagged molecules resolves
DEQUANT_NONE, DEQUANT_ARGMAX, DEQUANT_FLOOR = 0, 1, 2
PREC_F32, PREC_F16X3, PREC_BF16 = 0, 1, 2
PRECISIONS = {"f32": PREC_F32, "f16x3": PREC_F16X3, "bf16": PREC_BF16}
PREC_NO_SPLIT = 0x400   # ABI 13, ENFLOW_PREC_NO_SPLIT: OR into gemm_precision, this launch skips the split instances
EGCL_ATTENTION, EGCL_NORM_DIFF, EGCL_TANH, EGCL_ACT = 1, 2, 4, 8   # ENFLOW_EGCL_* (include/enflow_hip.h)
EGCL_VARIANTS = 0x100                                  # OR into gemm_precision
BWD_F32 = 0x200                                        # ENFLOW_BWD_F32: OR into the backward's dequant_kind

_i, _i64, _f, _p = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
_u64 = ctypes.c_uint64

# name -> (restype, argtypes); mirrors include/enflow_hip.h one to one
SIGNATURES = {
    "enflow_abi_version": (_i, []),
    "enflow_set_latency_threshold": (_i, [_i]),
    "enflow_latency_threshold": (_i, []),
    "enflow_set_split_threshold": (_i, [_i]),
    "enflow_set_fs_threshold": (_i, [_i]),
    "enflow_set_handoff_spin_limit": (_i, [_i]),
    "enflow_set_dequant_ahead": (_i, [_i]),
    "enflow_max_atoms": (_i, []),
    "enflow_max_node_nf": (_i, []),
    "enflow_supports_hidden": (_i, [_i]),
    "enflow_egcl_packed_size": (_i64, [_i, _i]),
    "enflow_argmax_packed_size": (_i64, [_i, _i]),
    "enflow_pack_egcl_f32": (_i, [_p, _i, _i, _p, _p]),
    "enflow_pack_egcl_ex_f32": (_i, [_p, _i, _i, _i, _p, _p, _p]),
    "enflow_pack_egcl_act_f32": (_i, [_p, _i, _i, _i, _i, _f, _f, _p, _p, _p]),
    "enflow_pack_argmax_f32": (_i, [_p, _i, _i, _p, _p]),
    "enflow_lf_forward_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                   _i, _p, _p, _f, _f, _f, _p, _p, _p, _p, _p, _p, _i, _p]),
    "enflow_lf_reverse_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                   _i, _f, _f, _p, _p, _p, _i, _p]),
    "enflow_lf_forward_io_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                      _i, _p, _p, _u64, _u64, _f, _f, _f, _p, _p, _p, _p, _p, _p, _p, _i, _p]),
    "enflow_lf_reverse_io_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                      _i, _f, _f, _p, _p, _p, _i, _p]),
    "enflow_lf_forward_io2_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                       _i, _p, _p, _u64, _u64, _f, _f, _f, _p, _p, _p, _p, _p, _p, _p, _i,
                                       _p, _p, _i, _p]),
    "enflow_lf_reverse_io2_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                       _i, _f, _f, _p, _p, _p, _i, _p, _p, _i, _p]),
    "enflow_lf_large_workspace_size": (_i64, [_i, _i, _i, _i]),
    "enflow_lf_forward_large_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                         _i, _p, _p, _f, _f, _f, _p, _p, _p, _i, _p, _p, _p, _i64, _p]),
    "enflow_lf_reverse_large_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                         _i, _f, _f, _p, _p, _p, _i, _p, _i64, _p]),
    "enflow_egcl_forward_large_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _f,
                                           _p, _p, _p, _p, _i, _p, _i64, _p]),
    "enflow_neighbour_pairs_large_f32": (_i, [_i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "enflow_one_hot_f32": (_i, [_p, _i, _i, _p, _p]),
    "enflow_egcl_forward_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _f,
                                     _p, _p, _p, _p, _p]),
    "enflow_argmax_forward_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p]),
    "enflow_neighbour_pairs_f32": (_i, [_i, _i, _i, _p, _p, _p, _p, _i, _p, _p, _p, _p]),
    "enflow_alchemical_nll_f32": (_i, [_i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _f, _f, _f,
                                       _p, _p, _p]),
    "enflow_lf_tape_size": (_i64, [_i, _i, _i, _i]),
    "enflow_lf_tape_size_for": (_i64, [_i, _i, _i, _i, _i]),
    "enflow_egcl_bwd_packed_size": (_i64, [_i, _i]),
    "enflow_pack_egcl_bwd_f32": (_i, [_p, _i, _i, _p, _p]),
    "enflow_pack_egcl_layers_f32": (_i, [_p, _i64, _i, _i, _i, _p, _p]),
    "enflow_pack_egcl_bwd_layers_f32": (_i, [_p, _i64, _i, _i, _i, _p, _p]),
    "enflow_lf_backward_workspace_size": (_i64, [_i, _i, _i, _i, _i, _i64]),
    "enflow_lf_backward_workspace_size_min": (_i64, [_i, _i, _i, _i, _i, _i64]),
    "enflow_alchemical_nll_backward_f32": (_i, [_i, _i, _i, _i, _p, _p, _p, _p, _p, _f, _f, _p,
                                                _p, _p, _p, _p, _p, _p]),
    "enflow_lf_backward_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i,
                                    _i, _p, _p, _p, _f, _f, _p, _p, _p, _p, _p, _p, _p,
                                    _p, _i64, _i64, _p, _p]),
    "enflow_lf_backward_large_workspace_size": (_i64, [_i, _i, _i, _i, _i, _i64]),
    "enflow_lf_backward_large_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _i,
                                          _i, _p, _p, _p, _f, _f, _p, _p, _p, _p, _p, _p, _p,
                                          _p, _i64, _i64, _p, _p]),
    "enflow_egcl_backward_workspace_size": (_i64, [_i, _i, _i, _i, _i64]),
    "enflow_egcl_backward_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i, _f, _p, _p, _p,
                                      _p, _p, _p, _p, _i64, _i64, _p, _p]),
    "enflow_egcl_backward_large_workspace_size": (_i64, [_i, _i, _i, _i, _i, _i64]),
    "enflow_egcl_backward_large_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _i, _f, _p, _p,
                                            _p, _p, _p, _p, _p, _i64, _i64, _p, _p]),
    "enflow_argmax_backward_workspace_size": (_i64, [_i, _i, _i]),
    "enflow_argmax_backward_f32": (_i, [_i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i64, _p]),
    "enflow_timing_enable": (_i, [_i]),
    "enflow_timing_collect": (_i, []),
    "enflow_timing_entry": (_i, [_i, ctypes.c_char_p, _i, ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_int64)]),
    "enflow_timing_reset": (_i, []),
}

_libs = {}


class HipPathError(RuntimeError):
    pass


class RangeError(FloatingPointError):
    """ENFLOW_ERR_RANGE: a split-precision (f16x3 / bf16) GEMM operand left the
    fp16 / bf16 range.  Inference calls catch it and re-run the same launch
    with fp32 GEMMs; the training path raises it."""


def lib_path(nf=None):
    """The library whose kernels hold `nf` node features: libenflow_hip.so up
    to 8, libenflow_hip_nf16.so for 9..16."""
    if nf is None or int(nf) <= BASE_NFMAX:
        return LIB_PATH
    if int(nf) <= MAX_NODE_NF:
        return LIB_NF16_PATH
    raise NotImplementedError(f"enflow_amd kernels are built for node_nf <= {MAX_NODE_NF} (got {nf})")


def lib(nf=None):
    """Load (once) and return the ctypes handle of the library for `nf` node
    features (default: the 8-feature build); raise if it is unavailable."""
    path = lib_path(nf)
    handle = _libs.get(path)
    if handle is None:
        if not os.path.exists(path):
            raise HipPathError(
                f"{path} is missing: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950)")
        handle = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(handle, name):    # an older build (A/B tools): calling it raises
                continue
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if _lat_threshold[0] is not None and hasattr(handle, "enflow_set_latency_threshold"):
            handle.enflow_set_latency_threshold(_lat_threshold[0])
        if _split_threshold[0] is not None and hasattr(handle, "enflow_set_split_threshold"):
            handle.enflow_set_split_threshold(_split_threshold[0])
        if _fs_threshold[0] is not None and hasattr(handle, "enflow_set_fs_threshold"):
            handle.enflow_set_fs_threshold(_fs_threshold[0])
        if _spin_limit[0] is not None and hasattr(handle, "enflow_set_handoff_spin_limit"):
            handle.enflow_set_handoff_spin_limit(_spin_limit[0])
        if _dq_ahead[0] is not None and hasattr(handle, "enflow_set_dequant_ahead"):
            handle.enflow_set_dequant_ahead(_dq_ahead[0])
        _libs[path] = handle
    return handle


_lat_threshold = [None]


def set_latency_threshold(max_mols):
    """Route fused <= 32-atom launches of at most `max_mols` molecules to the
    8-wave latency instance (-1: the device's CU count, the default; 0: never).
    The C setting is per library (enflow_set_latency_threshold): this applies
    it to every loaded library and to any loaded later.  Returns the previous
    setting (None: never set from Python)."""
    prev = _lat_threshold[0]
    _lat_threshold[0] = int(max_mols)
    for h in _libs.values():
        if hasattr(h, "enflow_set_latency_threshold"):
            h.enflow_set_latency_threshold(int(max_mols))
    return prev


_split_threshold = [None]
_fs_threshold = [None]
_spin_limit = [None]
_dq_ahead = [None]


def set_dequant_ahead(on):
    """ArgMax dequantisation of <= 64-atom forward launches as its own kernel
    ahead of the flow kernel (True, the default) or fused into it (False, A/B).
    Every loaded library and any loaded later; returns the previous setting."""
    prev = _dq_ahead[0]
    _dq_ahead[0] = 1 if on else 0
    for h in _libs.values():
        if hasattr(h, "enflow_set_dequant_ahead"):
            h.enflow_set_dequant_ahead(_dq_ahead[0])
    return prev


def set_handoff_spin_limit(polls):
    """Polls a workgroup of the two-workgroup split instance makes for one
    partner granule before it gives up with ENFLOW_ERR_HANDOFF (-1: the
    default 2^20; 0: give up without polling -- forces the host's re-run, for
    tests).  Every loaded library and any loaded later; returns the previous
    setting (None: never set from Python)."""
    prev = _spin_limit[0]
    _spin_limit[0] = int(polls)
    for h in _libs.values():
        if hasattr(h, "enflow_set_handoff_spin_limit"):
            h.enflow_set_handoff_spin_limit(int(polls))
    return prev


def set_split_threshold(max_mols):
    """Route fused <= 32-atom H = 128 f16x3 inference launches of at most
    `max_mols` molecules (and at most half the device's CUs) to the
    feature-split instance with two workgroups per molecule
    (enflow_split.hip; -1: CUs / 2, the default; 0: never).  Per library, like
    set_latency_threshold.  Returns the previous setting (None: never set)."""
    prev = _split_threshold[0]
    _split_threshold[0] = int(max_mols)
    for h in _libs.values():
        if hasattr(h, "enflow_set_split_threshold"):
            h.enflow_set_split_threshold(int(max_mols))
    return prev


def set_fs_threshold(max_mols):
    """Route such launches of at most `max_mols` molecules that do not take
    the two-workgroup split to the feature-split instance with one workgroup
    per molecule (-1: the device's CU count, the default; 0: never).  Returns
    the previous setting."""
    prev = _fs_threshold[0]
    _fs_threshold[0] = int(max_mols)
    for h in _libs.values():
        if hasattr(h, "enflow_set_fs_threshold"):
            h.enflow_set_fs_threshold(int(max_mols))
    return prev


def ptr(t):
    """Device pointer of a tensor (None -> NULL), as the int the c_void_p argtypes take."""
    return None if t is None else t.data_ptr()


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def check(rc, what):
    if rc != 0:
        raise HipPathError(f"{what} failed with code {rc}")


def require_gpu(t):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise HipPathError("the enflow_amd HIP path needs tensors on a ROCm GPU "
                           "(there is no CPU fallback)")


# the fused training backward keeps whole-molecule pair lists in LDS up to this
# size; batches with larger molecules train through the large-system kernels
# (enflow_lf_forward_large_f32 with a tape, enflow_lf_backward_large_f32)
TRAIN_MAX_ATOMS = 64
_large_ws = {}


def is_large(max_mol_atoms):
    """True if the batch goes through the layer-by-layer large-system kernels:
    its largest molecule exceeds the fused kernels' LDS image, or the
    ENFLOW_LARGE_MIN_ATOMS threshold (A/B runs)."""
    thr = os.environ.get("ENFLOW_LARGE_MIN_ATOMS")
    limit = lib().enflow_max_atoms() + 1 if not thr else int(thr)
    return int(max_mol_atoms) >= limit


def large_workspace(num_mols, num_atoms, max_mol_atoms, nf, device):
    """Device workspace of the large-system kernels (uint8, cached per device;
    grown on demand, never shrunk)."""
    need = lib(nf).enflow_lf_large_workspace_size(num_mols, num_atoms, int(max_mol_atoms), nf)
    if need < 0:
        raise HipPathError("enflow_lf_large_workspace_size: bad arguments")
    key = str(device)
    ws = _large_ws.get(key)
    if ws is None or ws.numel() < need:
        ws = torch.empty(max(need, 1), dtype=torch.uint8, device=device)
        _large_ws[key] = ws
    return ws


class KernelTimer:
    """Per-kernel HIP-event timing of this library's launches (enflow_timing_*):

        with KernelTimer() as t:
            ...launches...
        t.ms_per_launch("lf_flow_kernel<fwd>")

    Each launch is bracketed by an event pair on its own stream; exit waits for
    the events and snapshots {name: (total_ms, launches)}."""

    def __enter__(self):
        L = lib()
        L.enflow_timing_reset()
        L.enflow_timing_enable(1)
        self.stats = {}
        return self

    def __exit__(self, *exc):
        L = lib()
        L.enflow_timing_enable(0)
        n = L.enflow_timing_collect()
        buf = ctypes.create_string_buffer(128)
        ms, cnt = ctypes.c_double(), ctypes.c_int64()
        for i in range(n):
            if L.enflow_timing_entry(i, buf, 128, ctypes.byref(ms), ctypes.byref(cnt)) == 0 and cnt.value:
                self.stats[buf.value.decode()] = (ms.value, int(cnt.value))
        L.enflow_timing_reset()
        return False

    def ms_per_launch(self, name):
        tot, cnt = self.stats.get(name, (0.0, 0))
        return tot / cnt if cnt else None


_pending = []
# launches re-run with fp32 GEMMs after an ENFLOW_ERR_RANGE / _SMALL (inference and training; tests read
# it); FP32_MOL_RERUNS: molecules of the inference re-runs that ran only the flagged molecules
FP32_RERUNS = [0]
FP32_MOL_RERUNS = [0]
# inference launches re-run without the split instances after an ENFLOW_ERR_HANDOFF (tests read it)
HANDOFF_RERUNS = [0]
# deferred-check training steps whose word held ENFLOW_ERR_SMALL alone (warned, not re-run): a caller
# that needs every step at fp32 accuracy reads it, or sets STRICT_SMALL[0] = True to raise instead
DEFERRED_SMALL_STEPS = [0]
STRICT_SMALL = [False]


def defer_err(err_flag, small_warns=False):
    """Queue a device error word for a later check instead of synchronising now:
    a non-blocking copy into pinned host memory plus an event.  The training
    backward uses this so the host-side tail of the step (gradient views, the
    optimiser's launches) overlaps the backward kernels; the word is read by the
    next raise_on_err / check_pending (normally the next step's forward check),
    by which time the event has long completed."""
    host = torch.empty(1, dtype=torch.int32, pin_memory=True)
    host.copy_(err_flag, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(err_flag.device))
    _pending.append((ev, host, small_warns))


def check_pending():
    """Raise for any deferred error word (waits only for the queued events)."""
    while _pending:
        ev, host, small_warns = _pending.pop(0)
        ev.synchronize()
        e = int(host.item())
        if small_warns and e == ERR_SMALL and not STRICT_SMALL[0]:
            DEFERRED_SMALL_STEPS[0] += 1
            import warnings
            warnings.warn("enflow_amd: a deferred-check training step ran an f16x3 GEMM whose operand was "
                          "entirely below 2^-7 (gradients ~1e-5 relative instead of fp32 accuracy); set "
                          "gemm_precision='f32' or defer_error_check=False for the fp32 re-run",
                          RuntimeWarning, stacklevel=2)
            continue
        _raise_code(e)


def take_err(err_flag):
    """Read (synchronises) and zero a non-zero device error word; returns the
    code without raising and without touching queued (deferred) words."""
    e = int(err_flag.item())
    if e:
        err_flag.zero_()
    return e


def raise_code(e):
    """Raise for an error code read by take_err (no-op for 0)."""
    _raise_code(e)


def raise_on_err(err_flag, reset=False):
    """Read the device error word (synchronises) and raise like the reference;
    reset: zero a non-zero word (a cached status_word stays reusable).  The
    word is read and reset BEFORE any queued (deferred) error is raised, so a
    stale bit never outlives this call; the first error found is raised."""
    e = int(err_flag.item())
    if e and reset:
        err_flag.zero_()
    check_pending()      # an older queued error is raised first
    _raise_code(e)


_status = {}


def status_word(device):
    """int32[2] device words per (device, stream), zero between calls: [0] the
    error word (read synchronously and re-zeroed by raise_on_err(reset=True)),
    [1] the in-launch log|detJ| reduction ticket (the kernel resets it).  Saves
    a fill launch per inference call."""
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    st = _status.get(key)
    if st is None:
        st = torch.zeros(2, dtype=torch.int32, device=device)
        _status[key] = st
    return st


class _InferWords:
    """Per-(device, stream) buffers of the inference module calls, zero
    between calls (the kernels OR bits into them; a call that finds any set
    zeroes them before it returns): the status word pair (error word, log|detJ|
    ticket), the reverse's (error word, ArgMax index maximum), per-molecule
    error words, and the scratch the caller never sees (per-molecule log|detJ|,
    the reverse's ArgMax indices).  Grown on demand, never shrunk."""
    __slots__ = ("status", "rev", "mol_err", "ldj_mol", "idx", "cap_m", "cap_a")


def infer_words(device, num_mols, num_atoms=0):
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    w = _words.get(key)
    if w is None:
        w = _InferWords()
        w.status = status_word(device)
        w.rev = torch.zeros(2, dtype=torch.int32, device=device)
        w.cap_m = w.cap_a = -1
        _words[key] = w
    if num_mols > w.cap_m:
        cap = max(num_mols, 1)
        w.mol_err = torch.zeros(cap, dtype=torch.int32, device=device)
        w.ldj_mol = torch.empty(cap, dtype=torch.float32, device=device)
        w.cap_m = cap
    if num_atoms > w.cap_a:
        cap = max(num_atoms, 1)
        w.idx = torch.empty(cap, dtype=torch.int32, device=device)
        w.cap_a = cap
    return w


_words = {}


def _raise_code(e):
    if e & ERR_FEW_IMAGES:
        raise IndexError("fewer periodic images than atoms in a molecule: the reference "
                         "indexes id_mapping out of range here (enflow/data/base.py:137)")
    if e & ERR_TOO_MANY_ATOMS:
        raise HipPathError(f"molecule larger than {lib().enflow_max_atoms()} atoms")
    if e & ERR_TOO_MANY_FEATURES:
        raise HipPathError(f"node_nf larger than the kernels' feature width (at most {MAX_NODE_NF})")
    if e & ERR_HANDOFF:
        raise HipPathError("a two-workgroup latency launch timed out waiting for its partner workgroup "
                           "(not co-resident on the device); run with enflow_amd._lib.set_split_threshold(0)")
    if e & ERR_SMALL and not e & ERR_RANGE:
        raise RangeError("an f16x3 GEMM operand of a molecule was entirely below 2^-7 in magnitude (its "
                         "fp16 split loses fp32 accuracy there); run with gemm_precision='f32'")
    if e & ERR_RANGE:
        raise RangeError("a split-precision (f16x3 / bf16) GEMM operand left the range its split "
                         "represents at fp32 accuracy (an fp16 / bf16 overflow, or a layer whose "
                         "operand is entirely below 2^-7 in f16x3); run with gemm_precision='f32'")
