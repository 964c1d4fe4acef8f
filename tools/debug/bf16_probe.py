"""Debug probe: the lf_h64_L2 golden forward in each precision, with the
latency (8-wave) and the 4-wave instance, for the library in ENFLOW_LIB."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402
from _fixtures import load, flow_from_fixture, rel_err  # noqa: E402
from enflow_amd import _lib  # noqa: E402

for name in sys.argv[1:] or ["lf_h64_L2"]:
    inp, out = load(name)
    for thr in (256, 0):
        _lib.lib().enflow_set_latency_threshold(thr)
        for prec in ("f32", "f16x3", "bf16"):
            model, d = flow_from_fixture(inp, "cuda:0")
            model.gemm_precision = prec
            with torch.no_grad():
                o, ldj = model(d, noise=torch.tensor(inp["eps"], device="cuda:0"))
            errs = {k: rel_err(getattr(o, k).cpu().numpy(), out[k]) for k in ("h", "g", "pos", "vel")}
            print(os.path.basename(_lib.LIB_PATH), name, "thr", thr, prec, {k: f"{v:.2e}" for k, v in errs.items()},
                  flush=True)
