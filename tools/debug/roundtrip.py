"""Diagnostic: forward->reverse round-trip error per GEMM precision (Floor dequant, nf=4, H=32)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np, torch
from enflow_amd.nn import EGCL, Floor
from enflow_amd.flow import LFIntegrator
from enflow_amd.data import Data
from enflow_amd.data.synthetic import make_molecules, default_dt
DEV = "cuda:0"
b = make_molecules(4, 22, nf=4, seed=3)
for k in ("h", "g", "pos", "vel", "box", "r_cut"):
    b[k] = b[k].astype(np.float32).astype(np.float64)
for prec in ("f32", "f16x3", "bf16"):
    for hid, nl in ((32, 2), (128, 2)):
        torch.manual_seed(1)
        model = LFIntegrator([EGCL(4, 4, hid) for _ in range(nl)], Floor(), dt=default_dt()).to(DEV)
        model.gemm_precision = prec
        d = Data.from_arrays(b, device=DEV)
        u = torch.rand(d.h.shape, device=DEV, generator=torch.Generator(DEV).manual_seed(0))
        with torch.no_grad():
            o, ldj = model(d, noise=u)
            z = o.h.clone()
            model.dequantize = None
            back = model.reverse(o)
        hz = (torch.tensor(b["h"], device=DEV, dtype=torch.float32) + u)
        err = {k: float((getattr(back, k) - torch.tensor(b[k], device=DEV, dtype=torch.float32)).abs().max())
               for k in ("g", "vel")}
        err["h(pre-floor)"] = float((back.h - hz).abs().max())
        frac = float((torch.floor(back.h) == torch.tensor(b["h"], device=DEV)).float().mean())
        print(prec, hid, "max abs round-trip err", err, "floor match", frac, "max|z|", float(z.abs().max()))
