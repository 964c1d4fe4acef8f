"""Debug: large H=32 training gradients -- run-to-run and serial vs overlapped."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_large_systems as T  # noqa: E402
from oracle import enflow_oracle_grad as OG  # noqa: E402

sizes, hid, nl = [320], 32, 1
b = T._boxes(sizes, 41)
eps = np.random.default_rng(43).normal(size=b["h"].shape).astype(np.float32)
ref = None
for rep in range(3):
    model = T._model(hid, 5, nl, 42)
    T._large_train_step(model, b, torch.tensor(eps, device="cuda"))
    g = {k: p.grad.cpu().numpy().copy() for k, p in model.networks[0].named_parameters()}
    if ref is None:
        layers = [T._layer_params(n) for n in model.networks]
        dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
        _, _, gl, _, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
        ref = gl[0]
    w = g["coord_nn.0.weight"]
    err = T._normwise(w, ref["coord_nn.0.weight"])
    diff = np.abs(w - ref["coord_nn.0.weight"])
    rows = np.where(diff.max(1) > 1e-3 * np.abs(ref["coord_nn.0.weight"]).max())[0]
    cols = np.where(diff.max(0) > 1e-3 * np.abs(ref["coord_nn.0.weight"]).max())[0]
    print(os.environ.get("ENFLOW_SERIAL_BWD"), rep, "coord_nn.0.weight err", f"{err:.3e}", "bad rows", rows.tolist()[:40],
          "bad cols", cols.tolist()[:40], "bias err", f"{T._normwise(g['coord_nn.0.bias'], ref['coord_nn.0.bias']):.2e}",
          "wc2 err", f"{T._normwise(g['coord_nn.2.weight'], ref['coord_nn.2.weight']):.2e}", flush=True)
