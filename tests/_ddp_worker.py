"""One rank of the 2-process data-parallel training check (tests/test_0_ddp_gpu.py).

Both ranks run on cuda:0 under the gloo backend with CUDA tensors (RCCL does
not allow two ranks on one device).  Each rank wraps LFIntegrator in DDP
exactly as the reference's training driver does (enflow/main.py:159) and runs
its loop body (main.py:217-222: forward, Alchemical_NLL, loss.backward(),
optimizer.step()) on its shard of a global batch (the reference's
DistributedSampler, main.py:141-145).  It then recomputes, single-process and
without DDP, the HIP gradients of BOTH shards with a fresh copy of the same
initial weights, and saves everything for the parent to compare.

usage: python _ddp_worker.py RANK WORLD PORT OUTDIR
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

NF, HID, LAYERS, MOLS = 5, 64, 3, 12


def make_model(dev):
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data.synthetic import default_dt
    torch.manual_seed(0)
    return LFIntegrator([EGCL(NF, NF, HID) for _ in range(LAYERS)], ArgMax(NF, HID), dt=default_dt()).to(dev)


def shard(b, noise, m0, m1, dev):
    from enflow_amd.data import Data
    p = b["mol_ptr"]
    a0, a1 = int(p[m0]), int(p[m1])
    sub = {k: b[k][a0:a1] for k in ("h", "g", "pos", "vel", "box")}
    sub["r_cut"] = b["r_cut"][m0:m1]
    sub["mol_ptr"] = p[m0:m1 + 1] - a0
    return Data.from_arrays(sub, device=dev), torch.tensor(noise[a0:a1], device=dev)


def grads_of(model):
    return [p.grad.detach().cpu().double().numpy().copy() for p in model.parameters()]


def main():
    rank, world, port, outdir = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    from enflow_amd.data.synthetic import make_molecules, default_kBT
    from enflow_amd.distributed import shard_range
    from enflow_amd.flow import Alchemical_NLL
    from enflow_amd import _lib
    from torch.nn.parallel import DistributedDataParallel as DDP

    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    sizes = [22, 9, 30, 22, 15, 22, 40, 3, 22, 17, 22, 28]
    b = make_molecules(MOLS, sizes, nf=NF, seed=77)
    for k in ("h", "g", "pos", "vel", "box", "r_cut"):
        b[k] = b[k].astype(np.float32).astype(np.float64)
    noise = np.random.default_rng(5).normal(size=b["h"].shape).astype(np.float32)
    nll = Alchemical_NLL(kBT=default_kBT(), softening=0.1)
    ranges = [shard_range(MOLS, r, world) for r in range(world)]

    # --- DDP step (main.py:159, 217-222)
    model = make_model(dev)
    net = DDP(model, device_ids=[0])
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    data, eps = shard(b, noise, *ranges[rank], dev)
    opt.zero_grad()
    out, ldj = net(data, noise=eps)
    loss = nll(out, ldj)
    loss.backward()
    _lib.check_pending()
    ddp_grads = grads_of(model)
    opt.step()
    torch.cuda.synchronize()
    params_after = [p.detach().cpu().double().numpy().copy() for p in model.parameters()]

    # --- single-process HIP gradients of every shard (no DDP, same initial weights)
    ref = make_model(dev)
    local = []
    for r in range(world):
        for p in ref.parameters():
            p.grad = None
        d, e = shard(b, noise, *ranges[r], dev)
        o, l = ref(d, noise=e)
        nll(o, l).backward()
        _lib.check_pending()
        local.append(grads_of(ref))
    torch.cuda.synchronize()
    res = {"loss": float(loss.detach())}
    for i, g in enumerate(ddp_grads):
        res[f"ddp_{i}"] = g
        res[f"after_{i}"] = params_after[i]
        for r in range(world):
            res[f"local{r}_{i}"] = local[r][i]
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), n=len(ddp_grads), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
