"""Shared helpers for loading the golden fixtures in tests/golden/."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

EGCL_KEYS = (
    "edge_nn.0.weight", "edge_nn.0.bias", "edge_nn.2.weight", "edge_nn.2.bias",
    "node_nn.0.weight", "node_nn.0.bias", "node_nn.2.weight", "node_nn.2.bias",
    "coord_nn.0.weight", "coord_nn.0.bias", "coord_nn.2.weight",
    "vel_scaling_nn.0.weight", "vel_scaling_nn.0.bias",
    "vel_scaling_nn.2.weight", "vel_scaling_nn.2.bias",
)
ARGMAX_KEYS = ("network.0.weight", "network.0.bias", "network.2.weight", "network.2.bias")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    inp = {k[3:]: z[k] for k in z.files if k.startswith("in_")}
    out = {k[4:]: z[k] for k in z.files if k.startswith("out_")}
    return inp, out


def layer_params(inp, i, dtype=np.float64):
    return {k: inp[f"p{i}.{k}"].astype(dtype) for k in EGCL_KEYS}


def dequant_params(inp, dtype=np.float64):
    return {k: inp[f"dq.{k}"].astype(dtype) for k in ARGMAX_KEYS}


def state(inp, dtype=np.float64):
    s = {k: inp[k].astype(dtype) for k in ("h", "g", "pos", "vel", "box")}
    s["r_cut"] = inp["r_cut"].astype(dtype)
    s["mol_ptr"] = inp["mol_ptr"].astype(np.int64)
    return s


def n_layers(inp):
    return int(inp["n_layers"])


def rel_err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))
