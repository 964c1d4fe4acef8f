"""CPU-only checks of the host side: the C ABI library loads and exports
every symbol include/enflow_hip.h declares; argument validation works
without launching anything; host helpers behave like the reference."""
import os
import re

import numpy as np
import pytest
import torch

from enflow_amd import _lib
from enflow_amd.data.synthetic import make_molecules
from enflow_amd.utils.helpers import mol_ptr_from_counts, one_hot, apply_pbc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "enflow_hip.h")


def header_symbols():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(enflow_\w+)\s*\(", txt)))


@pytest.mark.parametrize("nf", [None, 16], ids=["libenflow_hip", "libenflow_hip_nf16"])
def test_library_exports_every_header_symbol(nf):
    L = _lib.lib(nf)
    syms = header_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"


def test_node_feature_library_selection():
    """node_nf <= 8: libenflow_hip.so; 9..16: libenflow_hip_nf16.so (the same
    sources with ENFLOW_NFMAX=16); wider is refused."""
    assert _lib.lib_path(5) == _lib.lib_path(None) == _lib.LIB_PATH
    assert _lib.lib_path(8) == _lib.LIB_PATH and _lib.lib_path(9) == _lib.LIB_NF16_PATH
    L16 = _lib.lib(16)
    assert L16.enflow_abi_version() == 13 and L16.enflow_max_node_nf() == 16
    assert L16.enflow_egcl_packed_size(128, 16) > 0 and L16.enflow_egcl_packed_size(128, 17) == -1
    # training: every node_nf of the build (nf 16's radial row past the transposed
    # edge_nn.0 GEMM's 32-row tile is a dot product of its own), not past it
    assert L16.enflow_lf_backward_workspace_size(4, 88, 15, 128, 2, 4 * 480) > 0
    assert L16.enflow_lf_backward_workspace_size(4, 88, 16, 128, 2, 4 * 480) > 0
    assert L16.enflow_lf_backward_workspace_size(4, 88, 17, 128, 2, 4 * 480) == -1
    assert _lib.TRAIN_MAX_NODE_NF == 16
    with pytest.raises(NotImplementedError):
        _lib.lib_path(17)


def test_abi_queries():
    L = _lib.lib()
    assert L.enflow_abi_version() == 13
    assert L.enflow_max_atoms() == 256
    assert L.enflow_max_node_nf() == 8
    for h in (32, 64, 128):
        assert L.enflow_supports_hidden(h) == 1
        assert L.enflow_egcl_packed_size(h, 5) > 2 * h * h
        assert L.enflow_egcl_packed_size(h, 5) % 64 == 0
    assert L.enflow_supports_hidden(96) == 0
    assert L.enflow_egcl_packed_size(96, 5) == -1
    assert L.enflow_egcl_packed_size(128, 9) == -1


def test_argument_errors_launch_nothing():
    L = _lib.lib()
    # too-large molecule, bad hidden width, bad nf: rejected before any launch
    args = [1, 300, 300, 5, 128] + [None] * 8 + [1, 1, None, None, 0.0, 0.1, 1.0] + [None] * 6 + [1, None]
    assert L.enflow_lf_forward_f32(*args) == -3
    args[2], args[4] = 20, 96
    assert L.enflow_lf_forward_f32(*args) == -5
    args[3], args[4] = 9, 128
    assert L.enflow_lf_forward_f32(*args) == -4
    args[3] = 5
    args[-2] = 7    # unknown GEMM precision
    assert L.enflow_lf_forward_f32(*args) == -1
    # the out-of-place entry (ABI 8): same checks, and NULL outputs / ldj / error word are rejected
    io = [1, 300, 300, 5, 128] + [None] * 12 + [1, 1, None, None, 0, 0, 0.0, 0.1, 1.0] + [None] * 7 + [1, None]
    assert L.enflow_lf_forward_io_f32(*io) == -3
    io[2] = 20
    assert L.enflow_lf_forward_io_f32(*io) == -1
    rev = [1, 300, 300, 5, 128] + [None] * 12 + [1, 0, 0.1, 1.0, None, None, None, 1, None]
    assert L.enflow_lf_reverse_io_f32(*rev) == -3
    rev[2] = 20
    assert L.enflow_lf_reverse_io_f32(*rev) == -1


def test_backward_sizes_and_argument_errors():
    L = _lib.lib()
    A, M, nf, H, nl = 22 * 4, 4, 5, 128, 8
    # per layer and atom: h | message sums, g, pos, vel, Q, the pair-word slab (63) and the row's edge count
    assert L.enflow_lf_tape_size(A, nf, H, nl) == nl * A * (nf + H + nf + 3 + 3 + 1 + 63 + 1)
    # the pair-word section only for the 33..64-atom instance that writes it
    base = nl * A * (nf + H + nf + 3 + 3 + 1)
    assert L.enflow_lf_tape_size_for(A, nf, H, nl, 22) == base
    assert L.enflow_lf_tape_size_for(A, nf, H, nl, 32) == base
    assert L.enflow_lf_tape_size_for(A, nf, H, nl, 33) == L.enflow_lf_tape_size(A, nf, H, nl)
    assert L.enflow_lf_tape_size_for(A, nf, H, nl, 64) == L.enflow_lf_tape_size(A, nf, H, nl)
    assert L.enflow_lf_tape_size_for(A, nf, H, nl, 65) == base
    assert L.enflow_lf_tape_size_for(A, nf, H, nl, -1) == -1
    assert L.enflow_egcl_bwd_packed_size(H, nf) >= 2 * H * H
    assert L.enflow_egcl_bwd_packed_size(96, nf) == -1
    assert L.enflow_lf_backward_workspace_size(M, A, nf, H, nl, 4 * 480) > 4 * 480 * 5 * H * 4
    # three rotating pair-row buffers for chains of >= 3 layers, two at the minimum
    assert L.enflow_lf_backward_workspace_size_min(M, A, nf, H, nl, 4 * 480) < \
        L.enflow_lf_backward_workspace_size(M, A, nf, H, nl, 4 * 480)
    assert L.enflow_lf_backward_workspace_size_min(M, A, nf, H, 2, 4 * 480) == \
        L.enflow_lf_backward_workspace_size(M, A, nf, H, 2, 4 * 480)
    assert L.enflow_lf_backward_workspace_size(M, A, nf, H, nl, -1) == -1
    # missing tape / buffers: rejected before any launch
    args = [M, A, 22, nf, H] + [None] * 8 + [nl, 1, None, None, None, 0.1, 1.0] + [None] * 7 + \
        [None, 0, 480 * 4, None, None]
    assert L.enflow_lf_backward_f32(*args) == -1
    args[2] = 100
    assert L.enflow_lf_backward_f32(*args) == -1


def test_synthetic_batch_layout():
    b = make_molecules(5, [22, 3, 9, 22, 1], nf=5, seed=1)
    assert b["mol_ptr"].tolist() == [0, 22, 25, 34, 56, 57]
    assert b["h"].shape == (57, 5) and np.all(b["h"].sum(1) == 1)
    # box of the first molecule reused for all (BaseDataset caches self.box)
    assert np.all(b["box"] == b["box"][0])
    for m in range(5):
        x = b["pos"][b["mol_ptr"][m]:b["mol_ptr"][m + 1]]
        assert np.allclose(x.mean(0), 0, atol=1e-12)


def test_mol_ptr_and_helpers():
    ptr = mol_ptr_from_counts(torch.tensor([3, 0, 2]))
    assert ptr.tolist() == [0, 3, 3, 5] and ptr.dtype == torch.int32
    oh = one_hot(torch.tensor([0, 2, 1]))
    assert oh.shape == (3, 3)
    oh = one_hot(torch.tensor([0, 1, 1]))
    assert oh.shape == (3, 2)          # reference width = max + 1
    x = torch.tensor([[0.6, -0.6, 1.5]])
    assert torch.allclose(apply_pbc(x, torch.tensor([[1.0, 1.0, 1.0]])), torch.tensor([[-0.4, 0.4, -0.5]]))


def test_hip_path_refuses_cpu_tensors():
    from enflow_amd.nn import EGCL
    from enflow_amd.data import Data
    net = EGCL(5, 5, 32)
    d = Data.from_arrays(make_molecules(1, 22, seed=0), device="cpu")
    with pytest.raises(_lib.HipPathError):
        net(d.h, d.edges)


def test_module_surface_matches_reference_names():
    """state_dict keys equal the reference's so its checkpoints load as-is."""
    from enflow_amd.nn import EGCL, ArgMax
    from _fixtures import EGCL_KEYS, ARGMAX_KEYS
    assert tuple(EGCL(5, 5, 32).state_dict().keys()) == EGCL_KEYS
    assert tuple(ArgMax(5, 32).state_dict().keys()) == ARGMAX_KEYS


def test_same_seed_same_init_as_reference():
    """Construction order mirrors egcl.py, so a seed gives the reference's weights."""
    from _fixtures import load, EGCL_KEYS
    from enflow_amd.nn import EGCL
    inp, _ = load("egcl_h32")
    torch.manual_seed(3)                       # make_golden.case_egcl(32, 3)
    net = EGCL(5, 5, 32)
    for k in EGCL_KEYS:
        np.testing.assert_array_equal(net.state_dict()[k].numpy(), inp["p0." + k])


def test_kernel_timer_without_launches():
    """enflow_timing_*: enabling, collecting and reading back with nothing
    launched (CPU-only: no events are recorded)."""
    with _lib.KernelTimer() as t:
        pass
    assert t.stats == {}
    assert t.ms_per_launch("lf_flow_kernel<fwd>") is None
    L = _lib.lib()
    assert L.enflow_timing_entry(10 ** 6, None, 0, None, None) == -1


def test_bench_flop_accounting():
    """bench.py's roofline: f16x3 issues 3 products per MFMA FLOP, bf16 one for
    the two H x H edge GEMMs; frac = issued FLOPs / pipe peak."""
    import bench
    alg, iss = bench.flop_counts(1000, 100, 8, 128, 5, "f16x3")
    parts = bench.gemm_parts(128, 5)
    valu = 1000 * parts["pair"]["coord_nn.2"] + 800 * parts["atom_layer"]["vel_scaling_nn.2"] + \
        100 * parts["atom"]["argmax.network"]
    assert iss == 3 * (alg - valu)
    alg_b, iss_b = bench.flop_counts(1000, 100, 8, 128, 5, "bf16")
    assert alg_b == alg and iss_b == iss - 2 * 1000 * 2 * (2 * 128 * 128)
    r = bench.roofline_mfma(alg, iss, 1.0, "f16x3", "k")
    assert abs(r["frac"] - iss / 1e-3 / 1e12 / 2500.0) < 1e-12
    assert abs(r["frac"] - r["matrix_pipe"]["frac"]) < 1e-12
    assert bench.flops_per_launch(1000, 100, 8, 128, 5) == alg


def test_hidden_padding_is_exact_on_cpu():
    """Hidden widths the kernels are not compiled for run zero-padded
    (enflow_amd/nn/_pad.py): the float64 EGCL restatement on the padded
    parameters gives the unpadded outputs, and pad -> unpad_grads returns every
    real parameter (CPU-only check of the padding layout)."""
    import numpy as np
    from oracle import enflow_oracle as O
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn._pad import EGCL_HDIMS, Geom, pad, kernel_hidden, unpad_grads
    from enflow_amd.nn import EGCL
    from enflow_amd.data.synthetic import make_molecules
    torch.manual_seed(3)
    net = EGCL(5, 5, 48, attention=True, norm_diff=True, tanh=True).double()
    H, Hp = 48, kernel_hidden(48)
    assert Hp == 64 and kernel_hidden(100) == 128 and kernel_hidden(129) is None
    b = make_molecules(3, [12, 7, 9], nf=5, seed=4)
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    args = (torch.tensor(b["h"]), torch.tensor(b["pos"]), torch.as_tensor(row), torch.as_tensor(col),
            torch.tensor(eb), 28, 1.0, (True, True, True))
    real = {k: p.detach() for k, p in net.named_parameters()}
    g = Geom(H, Hp, 5, 5, 5)
    padded = {k: pad(p, EGCL_HDIMS[k], g) for k, p in real.items()}
    for a, c in zip(OG._egcl(real, *args), OG._egcl(padded, *args)):
        np.testing.assert_allclose(a.numpy(), c.numpy(), rtol=1e-13, atol=1e-15)
    named = list(net.named_parameters())
    flat = torch.cat([padded[k].reshape(-1) for k, _ in named])
    back, off = unpad_grads(flat, named, EGCL_HDIMS, g)
    assert off == flat.numel()
    for k, p in named:
        assert torch.equal(back[k], real[k]), k


@pytest.mark.parametrize("fin,fout", [(3, 5), (6, 2)])
def test_feature_padding_is_exact_on_cpu(fin, fout):
    """EGCL(input_nf != output_nf) runs at the kernel width max(in, out):
    zero input columns / zero output rows (enflow_amd/nn/_pad.py).  The float64
    restatement on the padded parameters and padded h gives the real outputs."""
    import numpy as np
    from oracle import enflow_oracle as O
    from oracle import enflow_oracle_grad as OG
    from enflow_amd.nn._pad import EGCL_HDIMS, pad
    from enflow_amd.nn import EGCL
    from enflow_amd.data.synthetic import make_molecules
    torch.manual_seed(5)
    net = EGCL(fin, fout, 40).double()
    g = net.pad_geom()
    assert (g.Hp, g.F) == (64, max(fin, fout))
    b = make_molecules(2, [11, 8], nf=fin, seed=6)
    row, col, eb = O.batch_edges(b["pos"], b["box"], b["r_cut"], b["mol_ptr"])
    h = torch.tensor(np.random.default_rng(7).normal(size=(19, fin)))
    hp = torch.cat([h, h.new_zeros((19, g.F - fin))], 1)
    common = (torch.tensor(b["pos"]), torch.as_tensor(row), torch.as_tensor(col), torch.tensor(eb), 19, 1.0)
    real = {k: p.detach() for k, p in net.named_parameters()}
    padded = {k: pad(p, EGCL_HDIMS[k], g) for k, p in real.items()}
    q, f, gg = OG._egcl(real, h, *common)
    qp, fp, ggp = OG._egcl(padded, hp, *common)
    np.testing.assert_allclose(q.numpy(), qp.numpy(), rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(f.numpy(), fp.numpy(), rtol=1e-13, atol=1e-15)
    np.testing.assert_allclose(gg.numpy(), ggp[:, :fout].numpy(), rtol=1e-13, atol=1e-15)
    assert float(ggp[:, fout:].abs().max()) == 0.0 if g.F > fout else True


def test_activation_codes_and_variant_flags():
    """act_fn -> ENFLOW_ACT_* codes (include/enflow_hip.h); a non-SiLU act_fn
    marks the layer ENFLOW_EGCL_ACT (variant-capable kernels), the ArgMax raw
    vector carries the [kind, p0, p1, 0] trailer (ABI 10)."""
    from torch import nn
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.nn._act import act_code
    assert act_code(nn.SiLU()) == (0, 0.0, 0.0)
    assert act_code(nn.LeakyReLU(0.2))[:2] == (2, 0.2)
    assert act_code(nn.ReLU6()) == (12, 0.0, 6.0)
    assert act_code(nn.GELU(approximate="tanh"))[0] == 7
    assert act_code(nn.Softplus(2.0, 10.0)) == (10, 2.0, 10.0)
    assert act_code(nn.PReLU(init=0.125)) == (2, 0.125, 0.0)   # LeakyReLU with the module's slope
    with pytest.raises(NotImplementedError):
        act_code(nn.PReLU(num_parameters=3))
    with pytest.raises(NotImplementedError):
        act_code(nn.Hardswish())
    assert EGCL(5, 5, 32).variant_flags() == 0
    assert EGCL(5, 5, 32, act_fn=nn.Tanh()).variant_flags() == _lib.EGCL_ACT
    assert EGCL(5, 5, 32, act_fn=nn.Tanh()).hip_supported() in (True, False)   # needs only the library
    assert not EGCL(5, 5, 32, act_fn=nn.Hardswish()).hip_supported()
    assert not EGCL(5, 5, 32, act_fn=nn.PReLU(3)).hip_supported()
    am = ArgMax(5, 32, act_fn=nn.ELU(0.5))
    raw = am.kernel_raw("cpu")
    assert raw.numel() == sum(p.numel() for p in am.parameters()) + 4
    assert raw[-4:].tolist() == [3.0, 0.5, 0.0, 0.0]
    assert am.generic_act() and not ArgMax(5, 32).generic_act()


def test_prelu_slope_travels_in_the_act_code():
    """PReLU (one slope): the slope is not a kernel weight (raw vectors as the
    SiLU layer's), it is the act code's p0; its gradient slot is None and a
    trainable slope is refused on the differentiable paths."""
    from torch import nn
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.nn._act import check_trainable
    from enflow_amd.flow._train import layer_grads, argmax_grads
    torch.manual_seed(0)
    ref = EGCL(5, 5, 32)
    torch.manual_seed(0)
    act = nn.PReLU(init=0.2)
    net = EGCL(5, 5, 32, act_fn=act)
    names = [k for k, _ in net.named_parameters()]
    # the reference's order (egcl.py:11-55): the shared slope first appears as edge_nn.1.weight
    assert names[:4] == ["edge_nn.0.weight", "edge_nn.0.bias", "edge_nn.1.weight", "edge_nn.2.weight"]
    assert [k for k, _ in net.raw_named()] == [k for k, _ in ref.raw_named()]
    assert torch.equal(net.kernel_raw("cpu"), ref.kernel_raw("cpu"))   # same init stream, slope excluded
    assert net.act() == (2, pytest.approx(0.2), 0.0) and net.variant_flags() == _lib.EGCL_ACT
    with torch.no_grad():
        act.weight.fill_(-0.5)
    assert net.act()[1] == -0.5
    flat = torch.arange(ref.kernel_raw("cpu").numel() + 33, dtype=torch.float32)
    gl = layer_grads(net, flat)
    assert gl[2] is None and all(torch.equal(a, b) for a, b in zip(gl[:2] + gl[3:], layer_grads(ref, flat)))
    am = ArgMax(5, 32, act_fn=nn.PReLU(init=0.3))
    raw = am.kernel_raw("cpu")
    assert raw.numel() == sum(p.numel() for p in am.parameters()) - 1 + 4
    assert raw[-4:].tolist() == [2.0, pytest.approx(0.3), 0.0, 0.0]
    ga = argmax_grads(am, raw[:-4], am.pad_geom())
    assert [g is None for g in ga] == [k.startswith("network.1.") for k, _ in am.named_parameters()]
    with pytest.raises(NotImplementedError, match="freeze"):
        check_trainable(act, "test")
    act.weight.requires_grad_(False)
    check_trainable(act, "test")


def test_asm_hazard_scan_gate_on_synthetic_assembly(tmp_path):
    """tools/asm_hazard_scan.py (the build gate of enflow_amd/build.py): an MFMA
    result read inside an asm block too early, and an asm-written VGPR read as
    an MFMA operand 1 state later, are flagged; the padded forms are not."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("asm_hazard_scan", os.path.join(ROOT, "tools", "asm_hazard_scan.py"))
    scan = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(scan)

    def hits(body):
        p = tmp_path / "k.s"
        p.write_text("_Z1kv:\n" + "\n".join("\t" + ln for ln in body) + "\n")
        return [h[1] for h in scan.scan(str(p))]

    mfma = "v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], v[0:15]"
    read = [";;#ASMSTART", "v_exp_f32 v30, v3", ";;#ASMEND"]
    assert hits([mfma] + read) == ["mfma-result read in asm"]
    assert hits([mfma, "s_nop 7", "s_nop 3"] + read) == []                   # 12 states
    f32 = "v_mfma_f32_32x32x2_f32 v[0:15], v16, v17, v[0:15]"
    assert hits([f32, "s_nop 7", "s_nop 3"] + read) == ["mfma-result read in asm"]   # 16-pass: 18 states
    write = [";;#ASMSTART", "v_fma_mixlo_f16 v23, v40, 1.0, -v6 op_sel_hi:[0,0,1]", ";;#ASMEND"]
    assert hits(write + ["v_add_f32 v50, v51, v52", mfma]) == ["asm write read by mfma"]
    assert hits(write[:2] + ["s_nop 1", ";;#ASMEND", mfma]) == []


def test_product_build_refuses_diagnostic_switches():
    from enflow_amd import build
    with pytest.raises(ValueError):
        build.build(out=build.OUT, defines=("ENFLOW_STAMPS",))


def test_code_sha_ignores_the_build_path(tmp_path):
    """roofline.traffic is keyed on the hash of the gfx950 code objects' .text
    (bench.code_sha), which a rebuild of the same sources at another path keeps
    (the whole-.so hash does not: hipcc's path-derived __hip_cuid_* symbols)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    a = bench.code_sha()
    assert len(a) == 16 and a == bench.code_sha()
    assert bench.code_sha(_lib.LIB_NF16_PATH) != a     # another build: other code


def test_committed_pmc_traffic_for_the_built_library():
    """Report whether a committed PMC summary covers this build's device code
    (bench.py then carries roofline.traffic).  Evidence, not correctness: a
    kernel edit legitimately leaves no summary until the next GPU profile, so
    a miss skips instead of failing."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    traffic, src = bench.load_traffic(bench.workload_name("forward"), bench.lib_sha(), bench.code_sha())
    if traffic is None:
        pytest.skip(f"no profiles/**/*pmc_traffic.json for code {bench.code_sha()} yet")
    assert traffic > 0
    print("traffic", traffic, "from", src)


def test_prelu_state_dict_is_the_reference_layout():
    """A PReLU EGCL's state_dict has the reference's keys (the slope under every
    Sequential position that holds it, no act_fn.* key of its own), so a
    reference checkpoint loads with strict=True and the optimiser's parameter
    order is the reference's (enflow/nn/egcl.py:11-55 registers act_fn only
    inside edge_nn / node_nn / coord_nn / vel_scaling_nn)."""
    from torch import nn
    from enflow_amd.nn import EGCL
    torch.manual_seed(0)
    net = EGCL(5, 5, 32, act_fn=nn.PReLU(init=0.3))
    sd = net.state_dict()
    slope_keys = ["edge_nn.1.weight", "edge_nn.3.weight", "node_nn.1.weight", "coord_nn.1.weight",
                  "vel_scaling_nn.1.weight"]
    ref_keys = (["edge_nn.0.weight", "edge_nn.0.bias", "edge_nn.1.weight", "edge_nn.2.weight", "edge_nn.2.bias",
                 "edge_nn.3.weight", "node_nn.0.weight", "node_nn.0.bias", "node_nn.1.weight", "node_nn.2.weight",
                 "node_nn.2.bias", "coord_nn.0.weight", "coord_nn.0.bias", "coord_nn.1.weight", "coord_nn.2.weight",
                 "vel_scaling_nn.0.weight", "vel_scaling_nn.0.bias", "vel_scaling_nn.1.weight",
                 "vel_scaling_nn.2.weight", "vel_scaling_nn.2.bias"])
    assert list(sd) == ref_keys
    ref_sd = {k: (torch.full_like(v, -0.7) if k in slope_keys else v.clone() + 0.01) for k, v in sd.items()}
    torch.manual_seed(1)
    other = EGCL(5, 5, 32, act_fn=nn.PReLU())
    other.load_state_dict(ref_sd, strict=True)
    assert float(other.act_fn.weight) == pytest.approx(-0.7) and other.act()[1] == pytest.approx(-0.7)
    assert torch.equal(other.edge_nn[0].weight, ref_sd["edge_nn.0.weight"])
    # one parameter object per tensor, in the reference's first-occurrence order
    assert [k for k, _ in other.named_parameters()][2] == "edge_nn.1.weight"
    assert len(list(other.parameters())) == len(ref_keys) - 4
