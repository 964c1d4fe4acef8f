"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import enflow_oracle as O
from _fixtures import load, layer_params, dequant_params, state, n_layers, rel_err


@pytest.mark.parametrize("tag", ["extent", "box20", "box5"])
def test_edges_match_reference(tag):
    inp, out = load(f"edges_{tag}")
    row, col, eb = O.batch_edges(inp["pos"].astype(np.float64), inp["box"].astype(np.float64),
                                 inp["r_cut"].astype(np.float64), inp["mol_ptr"])
    np.testing.assert_array_equal(row, out["row"])
    np.testing.assert_array_equal(col, out["col"])
    cd = O.coord_diff(inp["pos"].astype(np.float64), row, col, eb)
    np.testing.assert_allclose(cd, out["coord_diff"], rtol=0, atol=1e-14)


def test_edges_quirk_is_exercised():
    """The reference maps the atom column through id_mapping (base.py:137);
    the fixtures must contain molecules where that mapping is not the
    identity, or the quirk is untested."""
    inp, _ = load("edges_extent")
    pos, box = inp["pos"].astype(np.float64), inp["box"].astype(np.float64)
    ptr = inp["mol_ptr"]
    non_identity = 0
    for m in range(len(ptr) - 1):
        a0, a1 = ptr[m], ptr[m + 1]
        _, idmap = O.periodic_images_within(pos[a0:a1], box[a0], float(inp["r_cut"][m]))
        non_identity += int(np.any(idmap[:a1 - a0] != np.arange(a1 - a0)))
    assert non_identity > 0


ACTS = ["relu", "leaky", "elu", "celu", "selu", "gelu", "gelutanh", "tanh", "sigmoid", "softplus", "mish",
        "relu6", "identity"]


@pytest.mark.parametrize("name", ["egcl_h32", "egcl_h128", "egcl_h64_att", "egcl_h32_nd_tanh", "egcl_h128_all",
                                  "egcl_nf16_h128"] + [f"egcl_act_{a}" for a in ACTS])
def test_egcl_matches_reference(name):
    """Default flags and the constructor variants (attention, norm_diff, tanh)."""
    inp, out = load(name)
    s = state(inp)
    row, col, eb = O.batch_edges(s["pos"], s["box"], s["r_cut"], s["mol_ptr"])
    cd = O.coord_diff(s["pos"], row, col, eb)
    q, f, g = O.egcl_forward(layer_params(inp, 0), s["h"], row, col, cd)
    assert rel_err(q, out["Q"]) < 1e-12
    assert rel_err(f, out["F"]) < 1e-12
    assert rel_err(g, out["G"]) < 1e-12


def test_argmax_matches_reference():
    inp, out = load("argmax_h32")
    z, log_q = O.argmax_forward(dequant_params(inp), inp["h"].astype(np.float64),
                                inp["eps"].astype(np.float64))
    assert rel_err(z, out["z"]) < 1e-12
    assert abs(log_q - float(out["log_q"])) <= 1e-10 * abs(float(out["log_q"]))
    np.testing.assert_array_equal(O.argmax_reverse(z), out["reverse"])


@pytest.mark.parametrize("name", ["lf_h32_L3", "lf_h64_L2", "lf_h128_L2", "lf_var_h64_L3", "lf_var_h128_L2",
                                  "lf_nf12_h64_L2", "lf_nf16_h32_L2", "lf_act_tanh_h64_L2", "lf_act_gelu_h128_L2"])
def test_lf_flow_matches_reference(name):
    inp, out = load(name)
    layers = [layer_params(inp, i) for i in range(n_layers(inp))]
    s, ldj = O.lf_forward(layers, dequant_params(inp), state(inp), inp["eps"].astype(np.float64),
                          float(inp["dt"]))
    for k in ("h", "g", "pos", "vel"):
        assert rel_err(s[k], out[k]) < 1e-10, k
    assert abs(ldj - float(out["ldj"])) <= 1e-10 * abs(float(out["ldj"]))
    nll = O.alchemical_nll(s, ldj, float(inp["kBT"]), float(inp["softening"]))
    assert abs(nll - float(out["nll"])) <= 1e-10 * abs(float(out["nll"]))
    back = O.lf_reverse(layers, s, float(inp["dt"]))
    for k in ("g", "pos", "vel"):
        assert rel_err(back[k], out["rev_" + k]) < 1e-8, k
    np.testing.assert_array_equal(back["h"], out["rev_h"])


def test_multiplicity_roundtrip():
    inp, out = load("edges_box5")
    n = int(inp["mol_ptr"][-1])
    pi, pj, pc = O.pair_multiplicity(out["row"], out["col"], n)
    assert int(pc.sum()) == len(out["row"])
    assert np.all(pc >= 1)


TRAIN_CASES = ["train_h32_L3", "train_h128_L2", "train_h64_L2", "train_var_h64_L2", "train_var_h32_L3",
               "train_att_h64_L2", "train_att_h32_L3", "train_nf12_h32_L2", "train_nf15_h128_L2", "train_nf16_h64_L2",
               "train_act_tanh_h32_L2", "train_act_elu_h64_L2"]


@pytest.mark.parametrize("name", TRAIN_CASES)
def test_gradient_oracle_matches_reference_backward(name):
    """The gradient oracle (torch float64 restatement) reproduces the reference's
    loss.backward() on every parameter (enflow/main.py:219-221)."""
    from oracle import enflow_oracle_grad as OG
    inp, out = load(name)
    nl = n_layers(inp)
    loss, ldj, gl, gd, _ = OG.train_loss_and_grads(
        [layer_params(inp, i) for i in range(nl)], dequant_params(inp), state(inp),
        inp["eps"].astype(np.float64), float(inp["dt"]), float(inp["kBT"]), float(inp["softening"]))
    assert abs(loss - out["loss"]) <= 1e-12 * abs(out["loss"])
    assert abs(ldj - out["ldj"]) <= 1e-12 * abs(out["ldj"])
    for i in range(nl):
        for k, v in gl[i].items():
            np.testing.assert_allclose(v, out[f"grad_p{i}.{k}"], rtol=1e-9, atol=1e-12 * np.abs(out[f"grad_p{i}.{k}"]).max())
    for k, v in gd.items():
        np.testing.assert_allclose(v, out[f"grad_dq.{k}"], rtol=1e-9, atol=1e-12 * np.abs(out[f"grad_dq.{k}"]).max())


@pytest.mark.parametrize("tag", ["raise", "quiet"])
def test_oracle_few_images_matches_reference(tag):
    """The reference raises IndexError only for a hit on an atom column past
    id_mapping (base.py:137), not merely for fewer images than atoms."""
    inp, out = load(f"edges_fewimg_{tag}")
    pos, box = inp["pos"].astype(np.float64), inp["box"].astype(np.float64)
    rc = float(inp["r_cut"][0])
    if int(out["raised"]):
        with pytest.raises(IndexError):
            O.molecule_edges(pos, box[0], rc)
    else:
        e = O.molecule_edges(pos, box[0], rc)
        assert e.shape[0] == out["row"].shape[0]
