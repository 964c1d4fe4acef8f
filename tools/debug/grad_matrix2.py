"""Debug: fused vs large training gradients at H=32 (errors per tensor)."""
import os
import sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_large_systems as T  # noqa: E402
from oracle import enflow_oracle_grad as OG  # noqa: E402


def large(sizes, hid, nl, var, force_large=False):
    b = T._boxes(sizes, 41)
    model = T._model(hid, 5, nl, 42, **var)
    eps = np.random.default_rng(43).normal(size=b["h"].shape).astype(np.float32)
    loss = T._large_train_step(model, b, torch.tensor(eps, device="cuda"))
    layers = [T._layer_params(n) for n in model.networks]
    dq = {k: v.detach().double().cpu().numpy() for k, v in model.dequantize.named_parameters()}
    rloss, _, gl, gd, _ = OG.train_loss_and_grads(layers, dq, b, eps.astype(np.float64), model.dt, 1.0, 0.1)
    errs = {}
    for i, net in enumerate(model.networks):
        for k, p in net.named_parameters():
            errs[f"p{i}.{k}"] = T._normwise(p.grad.cpu().numpy(), gl[i][k])
    bad = {k: f"{v:.1e}" for k, v in errs.items() if v > 1e-5}
    print(sizes, hid, nl, var, "large" if force_large else "", "loss", float(loss), rloss, "bad:", bad, flush=True)


for args in [([60, 50, 40, 30], 32, 2, {}), ([320], 32, 1, {}), ([320], 64, 2, {}), ([320], 32, 2, {})]:
    large(*args)
large([70, 30], 32, 2, {}, True)
large([70, 30], 64, 2, {}, True)
large([70, 30], 128, 2, {}, True)
