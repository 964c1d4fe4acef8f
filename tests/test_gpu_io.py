"""ABI 8: the self-contained forward (enflow_lf_forward_io_f32) -- out of place,
the dequantiser's draws made in the kernel, log|detJ| reduced in the same
launch -- against the ABI-7 call sequence it replaces (in-place buffers, the
caller's noise, a separate reduction launch), and the in-kernel Philox draws
against a numpy restatement of the generator (test-side checker only)."""
import numpy as np
import pytest
import torch

from _fixtures import load, flow_from_fixture, rel_err, assert_all_within

# every test on both fused-kernel instances (conftest.kernel_instance: the
# 4-wave throughput build and the 8-wave latency build)
pytestmark = [pytest.mark.gpu, pytest.mark.usefixtures("kernel_instance")]
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# ---------------------------------------------------------------------------
# Philox4x32-10 (Salmon et al., SC'11), as NoiseSrc in enflow_amd/csrc/flow_device.h
# ---------------------------------------------------------------------------
def philox_bits(seed, offset, n):
    M32 = np.uint64(0xFFFFFFFF)
    e = np.arange(n, dtype=np.uint64)
    c0, c1 = e & M32, e >> np.uint64(32)
    c2 = np.full(n, offset & 0xFFFFFFFF, np.uint64)
    c3 = np.full(n, (offset >> 32) & 0xFFFFFFFF, np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0, k1 = (k0 + 0x9E3779B9) & 0xFFFFFFFF, (k1 + 0xBB67AE85) & 0xFFFFFFFF
        p0 = c0 * np.uint64(0xD2511F53)
        p1 = c2 * np.uint64(0xCD9E8D57)
        hi0, lo0 = p0 >> np.uint64(32), p0 & M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & M32
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
    return c0, c1


def philox_normal(seed, offset, n):
    x, y = philox_bits(seed, offset, n)
    u1 = ((x >> np.uint64(8)) + np.uint64(1)).astype(np.float64) * 2.0 ** -24
    u2 = (y >> np.uint64(8)).astype(np.float64) * 2.0 ** -24
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def philox_uniform(seed, offset, n):
    x, _ = philox_bits(seed, offset, n)
    return (x >> np.uint64(8)).astype(np.float64) * 2.0 ** -24


def _floor_draws(seed, offset, A, nf):
    """h + 1.0 * U through a zero-layer Floor flow: the kernel's uniforms."""
    from enflow_amd import _lib
    L = _lib.lib()
    h = torch.zeros((A, nf), dtype=torch.float32, device=DEV)
    g = torch.zeros_like(h)
    pos = torch.zeros((A, 3), dtype=torch.float32, device=DEV)
    vel = torch.zeros_like(pos)
    box = torch.full((A, 3), 10.0, dtype=torch.float32, device=DEV)
    mols = A // 8
    ptr = torch.arange(0, A + 1, 8, dtype=torch.int32, device=DEV)
    rc = torch.ones(mols, dtype=torch.float32, device=DEV)
    layers = torch.zeros(16, dtype=torch.float32, device=DEV)
    out = [torch.empty_like(t) for t in (h, g, pos, vel)]
    ldj_mol = torch.empty(mols, dtype=torch.float32, device=DEV)
    ldj = torch.empty(1, dtype=torch.float32, device=DEV)
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    _lib.check(L.enflow_lf_forward_io_f32(
        mols, A, 8, nf, 32, _lib.ptr(ptr), _lib.ptr(rc), _lib.ptr(box), _lib.ptr(h), _lib.ptr(g), _lib.ptr(pos),
        _lib.ptr(vel), *(_lib.ptr(t) for t in out), _lib.ptr(layers), 0, _lib.DEQUANT_FLOOR, None, None,
        seed, offset, 1.0, 0.1, 1.0, _lib.ptr(ldj_mol), _lib.ptr(ldj), _lib.ptr(st[1:]), _lib.ptr(st[:1]),
        None, None, None, _lib.PREC_F16X3, _lib.stream_ptr(DEV)), "enflow_lf_forward_io_f32")
    torch.cuda.synchronize()
    assert int(st[0]) == 0 and int(st[1]) == 0          # no error; ticket reset
    assert float(ldj) == 0.0
    return out[0].cpu().numpy().reshape(-1)


@pytest.mark.parametrize("seed,offset", [(0, 0), (12345, 0), (2 ** 40 + 7, 3 * 2 ** 33 + 11)])
def test_in_kernel_uniforms_are_philox(seed, offset):
    A, nf = 4096, 5
    got = _floor_draws(seed, offset, A, nf)
    want = philox_uniform(seed, offset, A * nf)
    assert np.array_equal(got.astype(np.float64), want)     # exact: 24-bit uniforms
    print(f"uniforms: mean {got.mean():.4f}, var {got.var():.4f} (1/12 = {1 / 12:.4f})")
    assert abs(got.mean() - 0.5) < 0.01 and abs(got.var() - 1 / 12) < 0.01


def test_in_kernel_uniforms_differ_by_offset_and_seed():
    a = _floor_draws(1, 0, 1024, 5)
    b = _floor_draws(1, 5120, 1024, 5)
    c = _floor_draws(2, 0, 1024, 5)
    assert not np.array_equal(a, b) and not np.array_equal(a, c)


def _bench_like(mols=256, atoms=22, layers=3, hid=128, seed=0):
    from enflow_amd.data.synthetic import make_molecules, default_dt
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.utils.helpers import mol_ptr_from_counts
    torch.manual_seed(seed)
    model = LFIntegrator([EGCL(5, 5, hid) for _ in range(layers)], ArgMax(5, hid), dt=default_dt()).to(DEV)
    b = make_molecules(mols, atoms, nf=5, seed=77)
    f = lambda k: torch.tensor(b[k], dtype=torch.float32, device=DEV).contiguous()  # noqa: E731
    inp = {k: f(k) for k in ("h", "g", "pos", "vel", "box", "r_cut")}
    inp["mol_ptr"] = mol_ptr_from_counts(torch.tensor(np.diff(b["mol_ptr"])), device=DEV)
    return model, inp


def _run(model, inp, atoms, noise, key=(0, 0), io=True, ticket=True):
    mols = inp["mol_ptr"].numel() - 1
    out = {k: (torch.empty_like(inp[k]) if io else inp[k].clone()) for k in ("h", "g", "pos", "vel")}
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    ldj_mol = torch.empty(mols, dtype=torch.float32, device=DEV)
    ldj = torch.empty(1, dtype=torch.float32, device=DEV)
    with torch.no_grad():
        model.forward_buffers(out["h"], out["g"], out["pos"], out["vel"], inp["box"], inp["r_cut"],
                              inp["mol_ptr"], atoms, noise, ldj_mol, ldj, st[:1],
                              src=(inp["h"], inp["g"], inp["pos"], inp["vel"]) if io else None,
                              noise_key=key, ticket=st[1:] if ticket else None)
    torch.cuda.synchronize()
    assert int(st[0]) == 0 and int(st[1]) == 0
    return {k: v.cpu().numpy() for k, v in out.items()}, float(ldj), ldj_mol.cpu().numpy()


def test_io_forward_bitwise_equals_in_place_and_separate_reduction():
    model, inp = _bench_like()
    before = {k: v.clone() for k, v in inp.items()}
    noise = torch.randn(inp["h"].shape, device=DEV, generator=torch.Generator(DEV).manual_seed(3))
    a, la, ma = _run(model, inp, 22, noise, io=True, ticket=True)
    b, lb, mb = _run(model, inp, 22, noise, io=False, ticket=False)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(ma, mb)
    assert la == lb                            # the in-launch reduction is the separate kernel's, bitwise
    for k, v in inp.items():                   # inputs untouched
        assert torch.equal(v, before[k]), k
    # the ticket resets: repeated launches on one ticket keep reducing
    st = torch.zeros(2, dtype=torch.int32, device=DEV)
    ldj = torch.empty(1, dtype=torch.float32, device=DEV)
    ldj_mol = torch.empty(inp["mol_ptr"].numel() - 1, dtype=torch.float32, device=DEV)
    outs = {k: torch.empty_like(inp[k]) for k in ("h", "g", "pos", "vel")}
    with torch.no_grad():
        for _ in range(5):
            ldj.fill_(float("nan"))
            model.forward_buffers(outs["h"], outs["g"], outs["pos"], outs["vel"], inp["box"], inp["r_cut"],
                                  inp["mol_ptr"], 22, noise, ldj_mol, ldj, st[:1],
                                  src=(inp["h"], inp["g"], inp["pos"], inp["vel"]), ticket=st[1:])
            torch.cuda.synchronize()
            assert float(ldj) == la and int(st[1]) == 0


def test_in_kernel_normals_match_explicit_philox_noise():
    model, inp = _bench_like(mols=64)
    key = (987654321, 1 << 20)
    n = inp["h"].numel()
    explicit = torch.tensor(philox_normal(key[0], key[1], n).reshape(inp["h"].shape), dtype=torch.float32,
                            device=DEV)
    a, la, _ = _run(model, inp, 22, None, key=key)
    b, lb, _ = _run(model, inp, 22, explicit)
    errs = {k: rel_err(a[k], b[k]) for k in a}
    errs["ldj"] = abs(la - lb) / abs(lb)
    print("in-kernel vs explicit Philox normals:", errs)
    assert_all_within(errs, 1e-6)
    z = philox_normal(1, 0, 1 << 16)
    assert abs(z.mean()) < 0.02 and abs(z.var() - 1) < 0.02


def test_product_forward_reproducible_under_manual_seed_and_matches_oracle():
    """LFIntegrator.forward without noise: draws in the kernel, keyed from
    torch's generator (torch.manual_seed reproduces a run); with the fixture's
    noise it is the reference's forward (goldens), inputs left untouched."""
    inp, out = load("lf_h32_L3")
    model, data = flow_from_fixture(inp, DEV)
    h0 = data.h.clone()
    outs = []
    for _ in range(2):
        torch.manual_seed(11)
        d = flow_from_fixture(inp, DEV)[1]
        with torch.no_grad():
            o, ldj = model(d)
        outs.append((o.h.cpu().numpy(), float(ldj)))
    assert np.array_equal(outs[0][0], outs[1][0]) and outs[0][1] == outs[1][1]
    src_h = data.h
    with torch.no_grad():
        o, ldj = model(data, noise=torch.tensor(inp["eps"], device=DEV))
    assert torch.equal(src_h, h0)                  # the caller's input tensor is not written
    assert rel_err(o.h.cpu().numpy(), out["h"]) < 1e-5
    assert abs(float(ldj) - float(out["ldj"])) <= 1e-5 * abs(float(out["ldj"]))


def test_product_floor_forward_draws_in_kernel_and_round_trips():
    """LFIntegrator(..., Floor()).forward without noise: the U[0,1) draws are
    made in the kernel; they lie in [0, 1) (h_out - h_in before the layers is
    not observable, so check the dequantised state through a zero-layer-like
    round trip: reverse floors back to the integer data, floor.py)."""
    from enflow_amd.nn import EGCL, Floor
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    from enflow_amd.data.synthetic import make_molecules, default_dt
    b = make_molecules(8, 22, nf=4, seed=5)
    b["h"] = np.floor(np.abs(b["h"]) * 3.0).astype(np.float32)       # integer-valued features
    torch.manual_seed(2)
    model = LFIntegrator([EGCL(4, 4, 32) for _ in range(2)], Floor(), dt=default_dt()).to(DEV)
    outs = []
    for _ in range(2):
        torch.manual_seed(9)
        d = Data.from_arrays({k: (v.astype(np.float32) if k != "mol_ptr" else v) for k, v in b.items()}, device=DEV)
        with torch.no_grad():
            o, ldj = model(d)
        outs.append(o.h.cpu().numpy().copy())
    assert np.array_equal(outs[0], outs[1])                         # keyed from torch's generator
    with torch.no_grad():
        back = model.reverse(o)
    h0 = b["h"].astype(np.float64)
    got = back.h.cpu().numpy().astype(np.float64)
    frac_ok = np.mean(got == h0)
    print(f"floor round trip with in-kernel draws: {frac_ok:.4f} of elements exact")
    assert frac_ok > 0.999
