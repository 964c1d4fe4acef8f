"""f16x3 at small operand magnitudes and the fp32 re-run on ENFLOW_ERR_SMALL.

The f16x3 split x = hi + lo keeps fp32 accuracy only while lo = x - hi is a
normal fp16 (|x| >~ 2^-3); the weights carry a power-of-two scale, the
activation operands do not.  The kernels record per molecule and layer
whether every GEMM operand kind (edge_nn.0 / edge_nn.2 / coord_nn.0 / node
inputs) reached 2^-7 somewhere (flow_device.h, BIGK_*); one that never did
flags ENFLOW_ERR_SMALL (ABI 12; ENFLOW_ERR_RANGE before), and the host re-runs
with fp32 GEMMs -- only the flagged molecules when they are few (per-molecule
error words, enflow_lf_forward_io2_f32),
inference (dynamics.py) and, since ABI 11, training: the step's forward
again in fp32 and the fp32-GEMM backward (ENFLOW_BWD_F32) on its tape.

Batches: features / messages near 1e-2, 1e-3, 1e-4 (h and g of the batch and
one layer's edge_nn.0 / edge_nn.2 scaled down; the float64 reference stays
finite).  Bars: 1e-5 normwise per tensor (north_star) for the outputs,
GRAD_TOL for gradients, as everywhere else.  Reference: enflow/nn/egcl.py:57-69
(the edge MLP), enflow/flow/dynamics.py:10-37, enflow/main.py:217-222.
"""
import numpy as np
import pytest
import torch

from oracle import enflow_oracle as O
from _fixtures import rel_err, scalar_rel, normwise, assert_all_within, worst_of

pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("kernel_instance")]
DEV = "cuda:0"
TOL = 1e-5
GRAD_TOL = 5e-5   # <= 2x the fp32 floor measured on these batches (tools/grad_precision.py, profiles/r05)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def fmt(errs):
    return "{" + ", ".join(f"{k}: {v:.2e}" for k, v in errs.items()) + "}"


def _f32(b):
    out = dict(b)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        out[k] = np.asarray(b[k], dtype=np.float32).astype(np.float64)
    return out


def _layers(model):
    out = []
    for n in model.networks:
        p = {k: v.detach().cpu().double().numpy() for k, v in n.state_dict().items()}
        p["flags"] = (bool(n.attention), bool(n.norm_diff), bool(n.tanh))
        out.append(p)
    return out


def _small_model_and_batch(scale, where, hid=64):
    """6 x 22-atom molecules, Floor(dequant_scale=scale) so the dequantised h is
    ~scale, g ~scale; `where` = "edge0": layer 1's edge_nn.0 (weight and bias)
    scaled by `scale` (its edge_nn.2 input act(edge_nn.0 ..) ~scale), "msg":
    layer 1's edge_nn.2 scaled (the messages, coord_nn.0's input and the node
    aggregates ~scale)."""
    from enflow_amd.nn import EGCL, Floor
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data.synthetic import make_molecules, default_dt
    b = _f32(make_molecules(6, 22, nf=5, seed=41))
    rng = np.random.default_rng(42)
    b["h"] = _f32({**b, "h": np.floor(rng.uniform(0, 3, size=b["h"].shape)) * scale})["h"]
    b["g"] = _f32({**b, "g": b["g"] * scale})["g"]
    torch.manual_seed(43)
    nets = [EGCL(5, 5, hid) for _ in range(3)]
    with torch.no_grad():
        lin = nets[1].edge_nn[0] if where == "edge0" else nets[1].edge_nn[2]
        lin.weight.mul_(scale)
        lin.bias.mul_(scale)
    model = LFIntegrator(nets, Floor(dequant_scale=scale), dt=default_dt()).to(DEV)
    return model, b


def _oracle_fwd(model, b, u):
    return O.lf_forward(_layers(model), float(model.dequantize.dequant_scale), b, u.cpu().double().numpy(),
                        model.dt, dequant_kind="floor")


def _raw_launch_flagged(model, b, u):
    """The f16x3 launch without the host's retry: (its error word, its outputs)."""
    from enflow_amd import _lib
    from enflow_amd.data import Data
    model.gemm_precision = "f16x3"
    s = model._state(Data.from_arrays(b, device=DEV))
    M = s["mol_ptr"].numel() - 1
    ldj_mol, ldj = torch.empty(M, device=DEV), torch.empty(1, device=DEV)
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    with torch.no_grad():
        model.forward_buffers(s["h"], s["g"], s["pos"], s["vel"], s["box"], s["r_cut"], s["mol_ptr"], s["max_n"],
                              u, ldj_mol, ldj, st[:1], src=s["src"], ticket=st[1:])
    return int(st[0].item()), {k: s[k].cpu().numpy() for k in ("h", "g", "pos", "vel")}


@pytest.mark.parametrize("where", ["edge0", "msg"])
@pytest.mark.parametrize("scale", [1e-1, 3e-2, 1e-2, 1e-3, 1e-4])
def test_f16x3_small_operands_forward_reverse(scale, where, kernel_instance):
    """Forward and reverse at the default f16x3 precision vs the float64 oracle
    (1e-5).  At 1e-3 / 1e-4 every value of one operand kind is below 2^-7: the
    raw launch must flag ENFLOW_ERR_SMALL and the module call re-runs in fp32.
    Near the threshold (1e-2 .. 1e-1 scales the largest values sit around
    2^-7 .. 2^-3) a launch may or may not flag; one that does not must itself
    meet the bar (the raw f16x3 outputs vs the oracle)."""
    from enflow_amd import _lib
    from enflow_amd.data import Data
    model, b = _small_model_and_batch(scale, where)
    u = torch.rand(b["h"].shape, device=DEV, generator=torch.Generator(DEV).manual_seed(44))
    ref, ref_ldj = _oracle_fwd(model, b, u)
    code, raw = _raw_launch_flagged(model, b, u)
    raw_errs = {k: rel_err(raw[k], ref[k], allow_nonfinite=True) for k in raw}
    n0 = _lib.FP32_RERUNS[0]
    with torch.no_grad():
        o, ldj = model(Data.from_arrays(b, device=DEV), noise=u)
    reran = _lib.FP32_RERUNS[0] - n0
    errs = {k: rel_err(getattr(o, k).cpu().numpy(), ref[k]) for k in ("h", "g", "pos", "vel")}
    errs["ldj"] = scalar_rel(ldj, ref_ldj)
    # the reverse of the same float32 outputs vs the oracle's reverse
    st = {k: getattr(o, k).cpu().double().numpy() for k in ("h", "g", "pos", "vel")}
    st.update(box=b["box"], r_cut=b["r_cut"], mol_ptr=b["mol_ptr"])
    n1 = _lib.FP32_RERUNS[0]
    with torch.no_grad():
        back = model.reverse(o)
    rev_reran = _lib.FP32_RERUNS[0] - n1
    rref = O.lf_reverse(_layers(model), st, model.dt, dequant_kind="none")
    rerr = {"rev_" + k: rel_err(getattr(back, k).cpu().numpy(), rref[k]) for k in ("g", "pos", "vel")}
    print(f"[{kernel_instance}] small operands {where} x{scale:g}: raw f16x3 flag={code} "
          f"(raw outputs {fmt(raw_errs)}), forward re-run={reran}, reverse re-run={rev_reran}:", fmt({**errs, **rerr}))
    if scale <= 1e-3:
        assert code == _lib.ERR_SMALL, "an operand entirely below 2^-7 was not flagged (ENFLOW_ERR_SMALL)"
        assert reran == 1 and rev_reran == 1
    if code == 0:
        assert_all_within(raw_errs, TOL, "unflagged raw f16x3 launch")
        assert reran == 0
    assert_all_within(errs, TOL, "forward")
    assert_all_within(rerr, TOL, "reverse")


def _grad_check(model, b, u, kBT, softening, dequant_kind):
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.flow import Alchemical_NLL
    from enflow_amd.data import Data
    model.zero_grad(set_to_none=True)
    out, ldj = model(Data.from_arrays(b, device=DEV), noise=u)
    loss = Alchemical_NLL(kBT=kBT, softening=softening)(out, ldj)
    loss.backward()
    torch.cuda.synchronize()
    layers = _layers(model)
    dq = float(model.dequantize.dequant_scale) if dequant_kind == "floor" else \
        {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, u.cpu().double().numpy(), model.dt, kBT, softening,
                                                  dequant_kind=dequant_kind)
    errs = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            errs[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), gl[i][k])
    return float(loss), rloss, errs


@pytest.mark.parametrize("scale", [1e-3, 1e-4])
def test_training_step_small_operands_reruns_fp32(scale, kernel_instance):
    """One training step (forward, Alchemical_NLL, loss.backward()) on the small
    batch: the f16x3 training forward flags, is re-run with fp32 GEMMs, and the
    fp32-GEMM backward runs on its tape; loss and gradients vs the float64
    gradient oracle."""
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import default_kBT
    model, b = _small_model_and_batch(scale, "edge0")
    u = torch.rand(b["h"].shape, device=DEV, generator=torch.Generator(DEV).manual_seed(45))
    n0 = _lib.FP32_RERUNS[0]
    loss, rloss, errs = _grad_check(model, b, u, default_kBT(), 0.1, "floor")
    print(f"[{kernel_instance}] training x{scale:g}: re-runs {_lib.FP32_RERUNS[0] - n0}, loss {loss:.6e} vs "
          f"{rloss:.6e}, worst normwise grad err {worst_of(errs):.2e}")
    assert _lib.FP32_RERUNS[0] - n0 == 1
    assert abs(loss - rloss) <= TOL * abs(rloss)
    assert_all_within(errs, GRAD_TOL, "gradients vs oracle")


def _range_train_model_and_batch():
    """tests/test_gpu_parity.py's range-guard batch at 3e4 (features past the
    fp16 range in the node MLP's message sums; a tanh layer) as a training
    step -- without that test's coord_nn.2 x300, which drives |coord_diff * phi|
    across the +-100 clamp on a fifth of the pairs: there the gradient is
    discontinuous and pairs within fp32 rounding of the clamp edge make any
    fp32 gradient differ from the float64 one by ~2e-4 (measured, r04b)."""
    from enflow_amd.nn import EGCL, Floor
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data.synthetic import make_molecules, default_dt
    b = _f32(make_molecules(4, 22, nf=4, seed=13))
    b["h"] = np.floor(np.random.default_rng(14).uniform(0, 3e4, size=b["h"].shape)).astype(np.float32).astype(np.float64)
    torch.manual_seed(15)
    nets = [EGCL(4, 4, 64), EGCL(4, 4, 64, tanh=True)]
    with torch.no_grad():
        for n in nets:
            n.vel_scaling_nn[2].weight.zero_()
            n.vel_scaling_nn[2].bias.fill_(0.01)
    return LFIntegrator(nets, Floor(), dt=default_dt()).to(DEV), b


def test_training_step_on_fp16_overflow_reruns_fp32(kernel_instance):
    """the range-guard batch under loss.backward() trains
    (fp32 re-run of the step) instead of raising RangeError: loss and
    gradients vs the float64 oracle, and bitwise the gradients of the same
    step run with gemm_precision='f32' from the start (the re-run IS that
    step: fp32 forward, ENFLOW_BWD_F32 backward)."""
    from enflow_amd import _lib
    from enflow_amd.data.synthetic import default_kBT
    model, b = _range_train_model_and_batch()
    u = torch.rand(b["h"].shape, device=DEV, generator=torch.Generator(DEV).manual_seed(16))
    n0 = _lib.FP32_RERUNS[0]
    loss, rloss, errs = _grad_check(model, b, u, default_kBT(), 0.1, "floor")
    reruns = _lib.FP32_RERUNS[0] - n0
    g_rerun = [p.grad.clone() for p in model.parameters()]
    model.gemm_precision = "f32"
    loss32, _, _ = _grad_check(model, b, u, default_kBT(), 0.1, "floor")
    same = all(torch.equal(a, p.grad) for a, p in zip(g_rerun, model.parameters()))
    print(f"[{kernel_instance}] range-guard training step: re-runs {reruns}, loss {loss:.6e} vs "
          f"{rloss:.6e}, worst normwise grad err {worst_of(errs):.2e}, bitwise = explicit f32 step: {same}")
    assert reruns == 1
    assert loss == loss32 and same
    assert abs(loss - rloss) <= TOL * abs(rloss)
    assert_all_within(errs, GRAD_TOL, "gradients vs oracle")


def test_fp32_precision_trains_with_the_fp32_backward():
    """gemm_precision='f32' in training: fp32 forward and the ENFLOW_BWD_F32
    backward (no f16x3 anywhere), gradients vs the oracle on a golden batch."""
    from _fixtures import load, flow_from_fixture, layer_params, dequant_params, state, n_layers
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.flow import Alchemical_NLL
    inp, ref = load("train_h32_L3")
    model, data = flow_from_fixture(inp, DEV)
    model.gemm_precision = "f32"
    out, ldj = model(data, noise=torch.tensor(inp["eps"], device=DEV))
    loss = Alchemical_NLL(kBT=float(inp["kBT"]), softening=float(inp["softening"]))(out, ldj)
    loss.backward()
    worst = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            worst[f"p{i}.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_p{i}.{k}"])
    for k, p in model.dequantize.named_parameters():
        worst[f"dq.{k}"] = normwise(p.grad.cpu().numpy(), ref[f"grad_dq.{k}"])
    print("f32 training vs reference golden: loss", float(loss), ref["loss"], "worst grad", worst_of(worst))
    assert abs(float(loss) - float(ref["loss"])) <= TOL * abs(float(ref["loss"]))
    assert_all_within(worst, GRAD_TOL)


def test_deferred_training_check_small_warns_overflow_raises():
    """defer_error_check=True (no host sync in the forward) cannot re-run a step
    whose outputs were already consumed.  ADVICE r4: an operand entirely below
    2^-7 (ENFLOW_ERR_SMALL, a precision loss of ~1e-5 relative) warns at
    backward; a real fp16 overflow (ENFLOW_ERR_RANGE) raises RangeError there."""
    from enflow_amd import _lib
    from enflow_amd.flow import Alchemical_NLL
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import default_kBT
    _lib.check_pending()
    model, b = _small_model_and_batch(1e-4, "edge0")
    model.defer_error_check = True
    u = torch.rand(b["h"].shape, device=DEV)
    n0 = _lib.DEFERRED_SMALL_STEPS[0]
    out, ldj = model(Data.from_arrays(b, device=DEV), noise=u)
    loss = Alchemical_NLL(kBT=default_kBT(), softening=0.1)(out, ldj)
    with pytest.warns(RuntimeWarning, match="below 2\\^-7"):
        loss.backward()
        _lib.check_pending()
    assert not _lib._pending
    assert _lib.DEFERRED_SMALL_STEPS[0] == n0 + 1           # the warned step is counted
    # STRICT_SMALL: the same step raises instead of warning
    _lib.STRICT_SMALL[0] = True
    try:
        out, ldj = model(Data.from_arrays(b, device=DEV), noise=u)
        loss = Alchemical_NLL(kBT=default_kBT(), softening=0.1)(out, ldj)
        with pytest.raises(_lib.RangeError):
            loss.backward()
            _lib.check_pending()
    finally:
        _lib.STRICT_SMALL[0] = False
    _lib.check_pending()
    assert not _lib._pending
    model, b = _range_train_model_and_batch()
    model.defer_error_check = True
    u = torch.rand(b["h"].shape, device=DEV)
    out, ldj = model(Data.from_arrays(b, device=DEV), noise=u)
    loss = Alchemical_NLL(kBT=default_kBT(), softening=0.1)(out, ldj)
    with pytest.raises(_lib.RangeError):
        loss.backward()
    _lib.check_pending()
    assert not _lib._pending


def test_one_small_molecule_reruns_only_itself():
    """a BASELINE configs[1]-shaped batch (1024 x 22 atoms,
    H = 128, 8 layers, f16x3) in which ONE molecule's GEMM0 operands are all
    ~1e-4 (features and geometry scaled down: the same neighbour list at 1e-3
    of the size).  The kernel names that molecule in its per-molecule error
    word (ENFLOW_ERR_SMALL); the host re-runs only it with fp32 GEMMs (in place,
    same noise elements) and reduces log|detJ| over the batch.  Sampled
    molecules including the small one match the float64 oracle at 1e-5, and
    the module call's time is printed beside the clean batch's."""
    import time
    from enflow_amd import _lib
    from enflow_amd.nn import EGCL, Floor
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules, default_dt
    k = 517
    base = _f32(make_molecules(1024, 22, nf=5, seed=61))
    rng = np.random.default_rng(62)
    base["h"] = _f32({**base, "h": np.floor(rng.uniform(0, 3, size=base["h"].shape))})["h"]
    small = {kk: (v.copy() if isinstance(v, np.ndarray) else v) for kk, v in base.items()}
    a0, a1 = int(base["mol_ptr"][k]), int(base["mol_ptr"][k + 1])
    for key, f in (("h", 1e-4), ("g", 1e-4), ("pos", 1e-3), ("vel", 1e-3), ("box", 1e-3)):
        small[key][a0:a1] = small[key][a0:a1] * f
    small["r_cut"][k] = small["r_cut"][k] * 1e-3
    small = _f32(small)
    torch.manual_seed(63)
    model = LFIntegrator([EGCL(5, 5, 128) for _ in range(8)], Floor(dequant_scale=1e-4), dt=default_dt()).to(DEV)
    u = torch.rand(base["h"].shape, device=DEV, generator=torch.Generator(DEV).manual_seed(64))

    def run(b, reps=1):
        d = Data.from_arrays(b, device=DEV)
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            with torch.no_grad():
                o, ldj = model(d.clone(), noise=u)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return o, ldj, float(np.median(ts)) * 1e3

    run(base, 3)
    n0, m0 = _lib.FP32_RERUNS[0], _lib.FP32_MOL_RERUNS[0]
    o, ldj, _ = run(small)
    reruns, mol_reruns = _lib.FP32_RERUNS[0] - n0, _lib.FP32_MOL_RERUNS[0] - m0
    _, _, t_clean = run(base, 9)
    _, _, t_small = run(small, 9)
    model.gemm_precision = "f32"     # what the whole-batch fp32 re-run (ABI <= 11) cost on top of the clean call
    _, _, t_f32 = run(base, 5)
    model.gemm_precision = "f16x3"
    ref, ref_ldj = _oracle_fwd(model, small, u)
    worst = {kk: 0.0 for kk in ("h", "g", "pos", "vel")}
    for m in sorted(set(list(range(0, 1024, 64)) + [k, 1023])):
        b0, b1 = int(small["mol_ptr"][m]), int(small["mol_ptr"][m + 1])
        for kk in worst:
            worst[kk] = worst_of([worst[kk], rel_err(getattr(o, kk)[b0:b1].cpu().numpy(), ref[kk][b0:b1])])
    err_k = {kk: rel_err(getattr(o, kk)[a0:a1].cpu().numpy(), ref[kk][a0:a1]) for kk in worst}
    ldj_err = scalar_rel(ldj, ref_ldj)
    print(f"one small molecule in 1024: re-runs {reruns} ({mol_reruns} molecule), sampled vs oracle {fmt(worst)}, "
          f"the small molecule {fmt(err_k)}, ldj {ldj_err:.2e}; module call {t_small:.3f} ms vs clean batch "
          f"{t_clean:.3f} ms ({t_small / t_clean:.2f}x; a whole-batch fp32 re-run would add {t_f32:.3f} ms: "
          f"{(t_clean + t_f32) / t_clean:.2f}x)")
    assert reruns == 1 and mol_reruns == 1
    # the timing is printed evidence only (a wall-clock assert on a shared
    # box fails on load, not on a wrong re-run); what the per-molecule re-run costs
    # and why it stays above the 1.2x asked is in DESIGN.md (round 6, item 6)
    assert_all_within(worst, TOL, "sampled molecules")
    assert_all_within(err_k, TOL, "the small molecule")
    assert ldj_err < TOL
