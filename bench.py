"""Benchmark: enflow LFIntegrator forward + log|detJ| on MI355X.

Workload (BASELINE.json configs[1]): per GPU a batch of 1024 synthetic
22-atom molecules, 8 EGCL coupling layers, hidden_nf 128, node_nf 5,
float32, ArgMax dequantisation, periodic neighbour lists rebuilt every layer.
One step = one fused forward over the batch (ArgMax noise drawn on device,
inputs copied into the work buffers, ONE flow kernel + one reduce kernel),
inputs already resident in HBM.

Multi-GPU: one process per GPU (torch.distributed.run), molecules sharded
across ranks (weak scaling: 1024 per GPU), no collective in the data path;
barrier + synchronize around the timed region and the MAX time over ranks.

Also reported (rank 0): the roofline of the flow kernel (algorithmic FLOPs
from the kernel's own pair counters / its event-timed duration vs the f32
MFMA peak) and the CPU oracle timed on a bounded sample (cpu_baseline).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "molecule-transforms/sec (fwd+log|detJ|), batch 1024×22 atoms, 1/2/4/8 GPU"
PEAK_F32_MFMA_TFLOPS = 157.3      # MI355X_MICROARCH.md: dense f32 MFMA (= f32 vector) peak
PEAK_F16_MFMA_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense BF16/F16 MFMA peak (spec, no sparsity)
PRODUCTS = {"f32": 1, "f16x3": 3, "bf16": 1}   # MFMA products per fp32-equivalent GEMM FLOP


def matrix_pipe(achieved, prec):
    """What the matrix cores actually issue: f16x3 runs every fp32 GEMM FLOP as
    3 split-fp16 products on the F16 pipe; bf16 as one BF16 product; f32 on the
    F32 pipe.  Reported next to the fp32-equivalent roofline so neither hides
    the other (upper bound: ignores the K padding of edge_nn.0 / node items)."""
    if prec == "f32":
        return {"dtype": "f32", "issued_tflops": achieved, "peak": PEAK_F32_MFMA_TFLOPS,
                "frac": achieved / PEAK_F32_MFMA_TFLOPS}
    issued = achieved * PRODUCTS[prec]
    return {"dtype": "f16" if prec == "f16x3" else "bf16", "products_per_flop": PRODUCTS[prec],
            "issued_tflops": issued, "peak": PEAK_F16_MFMA_TFLOPS, "frac": issued / PEAK_F16_MFMA_TFLOPS}
MOLS_PER_GPU, ATOMS, LAYERS, HID, NF = 1024, 22, 8, 128, 5


def flops_per_launch(pairs, atoms, layers, hid, nf):
    """Algorithmic FLOPs of one forward launch.  Per unique neighbour pair:
    edge_nn.0 (2nf+1 -> H), edge_nn.2 (H -> H), coord_nn.0 (H -> H),
    coord_nn.2 (H -> 1); per atom and layer: vel_scaling_nn, node_nn; per
    atom once: ArgMax.network.  Multiply-add = 2 FLOPs; activations excluded."""
    per_pair = 2 * hid * (2 * nf + 1) + 4 * hid * hid + 2 * hid
    per_atom_layer = (2 * hid * nf + 2 * hid) + (2 * hid * (hid + nf) + 2 * hid * nf)
    per_atom_dq = 2 * hid * nf + 2 * hid * 2 * nf
    return pairs * per_pair + atoms * layers * per_atom_layer + atoms * per_atom_dq


# per-mode workload (BASELINE.json configs): molecules/GPU, atoms, layers,
# direction, GEMM precision, chain geometry, metric
MODES = {
    "forward": dict(mols=MOLS_PER_GPU, atoms=ATOMS, layers=LAYERS, reverse=False, prec="f16x3", chain=False,
                    metric=METRIC, unit="molecule-transforms/s"),
    "generate": dict(mols=1024, atoms=22, layers=8, reverse=True, prec="bf16", chain=False,
                     metric="molecule-generations/sec (reverse/generate path, bf16), batch 1024×22 atoms",
                     unit="molecule-generations/s"),
    "chain": dict(mols=512, atoms=256, layers=16, reverse=False, prec="f16x3", chain=True,
                  metric="molecule-transforms/sec (fwd+log|detJ|), 512×256-atom chains, 16 layers",
                  unit="molecule-transforms/s"),
}


def build_workload(rank, device, mols=MOLS_PER_GPU, atoms=ATOMS, layers=LAYERS, chain=False):
    from enflow_amd.data.synthetic import make_molecules, default_dt
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.utils.helpers import mol_ptr_from_counts
    b = make_molecules(mols, atoms, nf=NF, seed=1000 + rank, chain=chain)
    torch.manual_seed(0)                    # same (random-init) weights on every rank
    model = LFIntegrator([EGCL(NF, NF, HID) for _ in range(layers)], ArgMax(NF, HID),
                         dt=default_dt()).to(device)
    f = lambda k: torch.tensor(b[k], dtype=torch.float32, device=device).contiguous()  # noqa: E731
    inp = {k: f(k) for k in ("h", "g", "pos", "vel", "box", "r_cut")}
    inp["mol_ptr"] = mol_ptr_from_counts(torch.tensor(np.diff(b["mol_ptr"])), device=device)
    return b, model, inp


def cpu_baseline(sample_mols=1536):
    """The CPU oracle (numpy float64 port of the reference path) on a bounded
    sample of the same workload, scaled to molecule-transforms/s."""
    from oracle import enflow_oracle as O
    from enflow_amd.data.synthetic import make_molecules, default_dt
    from enflow_amd.nn import EGCL, ArgMax
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:  # pragma: no cover
        threads = 1
    torch.manual_seed(0)
    nets = [EGCL(NF, NF, HID) for _ in range(LAYERS)]
    am = ArgMax(NF, HID)
    layers = [{k: v.double().numpy() for k, v in n.state_dict().items()} for n in nets]
    dq = {k: v.double().numpy() for k, v in am.state_dict().items()}
    b = make_molecules(sample_mols, ATOMS, nf=NF, seed=4242)
    eps = np.random.default_rng(0).normal(size=b["h"].shape)
    t0 = time.perf_counter()
    O.lf_forward(layers, dq, b, eps, default_dt())
    dt = time.perf_counter() - t0
    return {"value": sample_mols / dt, "unit": "molecule-transforms/s", "cores": int(threads),
            "kind": "port",
            "sample": f"{sample_mols} molecules x {ATOMS} atoms, {LAYERS} layers, hidden {HID}, "
                      f"numpy float64 oracle (oracle/enflow_oracle.py), {dt:.1f} s"}


def load_traffic():
    """HBM bytes per flow-kernel launch from the committed rocprofv3 PMC
    summary (profiles/*pmc_traffic.json, written by profiles/collect_pmc.py),
    if it was collected for this workload."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")), reverse=True):
        try:
            with open(path) as fh:
                d = json.load(fh)
            if d.get("workload") == workload_name():
                return d.get("hbm_bytes_per_launch")
        except Exception:
            continue
    return None


def workload_name(mode="forward"):
    c = MODES[mode]
    kind = "reverse" if c["reverse"] else "forward"
    geo = "chain" if c["chain"] else ""
    return f"lf_{kind}_{c['mols']}x{c['atoms']}{geo}_L{c['layers']}_H{HID}_nf{NF}_f32"


TRAIN_METRIC = "molecule-train-steps/sec (fwd+NLL+bwd+Adam, RCCL grad all-reduce), batch 1024×64 atoms per GPU"
TRAIN_ATOMS = 64


def train_flops(pairs, atoms, layers, hid, nf):
    """Algorithmic FLOPs of one training step's flow part: the forward
    (flops_per_launch) plus, per unique pair, the recomputed edge chain, its
    adjoint GEMMs (coord_nn.0^T, edge_nn.2^T, edge_nn.0^T) and the three
    weight-gradient outer products; per atom-layer the node MLP recompute,
    adjoint and weight gradients."""
    fwd_pair = 2 * hid * (2 * nf + 1) + 4 * hid * hid + 2 * hid
    bwd_pair = fwd_pair + (4 * hid * hid + 2 * hid * (2 * nf + 1)) + (4 * hid * hid + 2 * hid * (2 * nf + 2) + 2 * hid)
    node = (2 * hid * nf + 2 * hid) + (2 * hid * (hid + nf) + 2 * hid * nf)
    return (flops_per_launch(pairs, atoms, layers, hid, nf) + pairs * bwd_pair +
            atoms * layers * 3 * node)


def run_train(args, world, rank, local, device, dist):
    """Config 3: a full training step (the reference's loop body,
    enflow/main.py:217-223) per GPU on 1024 synthetic 64-atom molecules."""
    from enflow_amd.data.synthetic import make_molecules, default_dt, default_kBT
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator, Alchemical_NLL
    from enflow_amd.data import Data
    atoms = args.atoms or TRAIN_ATOMS
    radius = 4.0 * (atoms / 22.0) ** (1.0 / 3.0)
    b = make_molecules(MOLS_PER_GPU, atoms, nf=NF, seed=2000 + rank, radius=radius)
    torch.manual_seed(0)
    model = LFIntegrator([EGCL(NF, NF, HID) for _ in range(LAYERS)], ArgMax(NF, HID), dt=default_dt()).to(device)
    net = model
    if dist:
        from torch.nn.parallel import DistributedDataParallel as DDP
        net = DDP(model, device_ids=[local])      # main.py:159; backend nccl = RCCL
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    nll = Alchemical_NLL(kBT=default_kBT(), softening=0.1)
    base = Data.from_arrays(b, device=device)
    noise = torch.empty_like(base.h)
    gen = torch.Generator(device).manual_seed(rank)

    def step():
        opt.zero_grad(set_to_none=True)
        torch.randn(noise.shape, generator=gen, out=noise)
        out, ldj = net(base._replace(), noise=noise)
        loss = nll(out, ldj)
        loss.backward()
        opt.step()
        return loss

    # pair statistics for the algorithmic FLOPs (one counted inference forward)
    stats = torch.zeros(2, dtype=torch.int64, device=device)
    with torch.no_grad():
        ptr = base.mol_ptr
        w = {k: getattr(base, k).clone() for k in ("h", "g", "pos", "vel")}
        ldj_mol = torch.empty(MOLS_PER_GPU, dtype=torch.float32, device=device)
        ldj = torch.empty(1, dtype=torch.float32, device=device)
        err = torch.zeros(1, dtype=torch.int32, device=device)
        model.forward_buffers(w["h"], w["g"], w["pos"], w["vel"], base.box, base.r_cut, ptr, atoms,
                              torch.randn_like(w["h"]), ldj_mol, ldj, err, stats)
    torch.cuda.synchronize()
    if int(err.item()) != 0:
        raise RuntimeError(f"flow kernel error flag {int(err.item())}")
    pairs = int(stats[0].item())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    from enflow_amd.distributed import max_over_ranks
    elapsed = max_over_ranks(time.perf_counter() - t0, device)
    if rank == 0:
        n_atoms = MOLS_PER_GPU * atoms
        flops = train_flops(pairs, n_atoms, LAYERS, HID, NF)
        ms = elapsed / args.steps * 1e3
        line = {
            "metric": TRAIN_METRIC, "value": MOLS_PER_GPU * world * args.steps / elapsed,
            "unit": "molecules/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": f"synthetic (random-walk {atoms}-atom molecules, random-init weights)",
            "config": {"workload": f"lf_train_{MOLS_PER_GPU}x{atoms}_L{LAYERS}_H{HID}_nf{NF}_f32",
                       "molecules_per_gpu": MOLS_PER_GPU, "atoms_per_molecule": atoms,
                       "coupling_layers": LAYERS, "hidden_nf": HID, "node_nf": NF,
                       "global_batch": MOLS_PER_GPU * world,
                       "parallelism": f"molecule-sharded x{world}, DDP grad all-reduce" if world > 1
                       else "single GPU", "unique_pairs_per_layer_pass": pairs},
            "step_tflops": flops / (ms * 1e-3) / 1e12, "flops_per_step": flops,
            "final_loss": float(loss),
        }
        print(json.dumps(line), flush=True)


LJ_METRIC = "LJ-box generations/sec (reverse/generate path, example/generate.yaml: 2944-atom periodic box)"


def run_lj(args, world, rank, device, dist):
    """The reference's example/generate.yaml system: one periodic 2944-atom
    Lennard-Jones box per GPU (batch 1), 8 coupling layers, hidden 128,
    generated by LFIntegrator.reverse (main.py:263-278) through the
    layer-by-layer large-system kernels (enflow_amd/csrc/enflow_large.hip).
    Not a BASELINE.json config: reported for the large-system path."""
    from enflow_amd.data.synthetic import make_lj_systems, default_dt
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    from enflow_amd.data import Data
    from enflow_amd.utils.helpers import mol_ptr_from_counts
    from enflow_amd import _lib as L_
    n = args.atoms or 2944
    b = make_lj_systems([n], seed=3000 + rank, nf=NF)
    b["pos"] = b["pos"] - np.round(b["pos"] / b["box"]) * b["box"]
    torch.manual_seed(0)
    model = LFIntegrator([EGCL(NF, NF, HID) for _ in range(LAYERS)], ArgMax(NF, HID), dt=default_dt()).to(device)
    f = lambda k: torch.tensor(b[k], dtype=torch.float32, device=device).contiguous()  # noqa: E731
    inp = {k: f(k) for k in ("h", "g", "pos", "vel", "box", "r_cut")}
    inp["mol_ptr"] = mol_ptr_from_counts(torch.tensor(np.diff(b["mol_ptr"])), device=device)
    work = {k: inp[k].clone() for k in ("h", "g", "pos", "vel")}
    ldj_mol = torch.empty(1, dtype=torch.float32, device=device)
    ldj = torch.empty(1, dtype=torch.float32, device=device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    idx = torch.empty(n, dtype=torch.int32, device=device)
    mx = torch.zeros(1, dtype=torch.int32, device=device)
    model.forward_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                          inp["mol_ptr"], n, torch.randn_like(work["h"]), ldj_mol, ldj, err)
    gsrc = {k: work[k].clone() for k in work}
    e = Data.from_arrays({**b, "pos": gsrc["pos"].double().cpu().numpy()}, device=device).edges
    pairs = int(e._materialise()[0].numel()) * LAYERS          # unique pairs of the first layer x layers

    def step():
        for k in work:
            work[k].copy_(gsrc[k])
        model.reverse_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                              inp["mol_ptr"], n, idx, mx, err)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if int(err.item()) != 0:
        raise RuntimeError(f"flow kernel error flag {int(err.item())}")
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    from enflow_amd.distributed import max_over_ranks
    elapsed = max_over_ranks(time.perf_counter() - t0, device)
    stream = torch.cuda.current_stream(device)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for e0, e1 in evs:
        for k in work:
            work[k].copy_(gsrc[k])
        e0.record(stream)
        model.reverse_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                              inp["mol_ptr"], n, idx, mx, err)
        e1.record(stream)
    torch.cuda.synchronize()
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))
    if rank == 0:
        flops = flops_per_launch(pairs, n, LAYERS, HID, NF) - n * (2 * HID * NF + 2 * HID * 2 * NF)
        achieved = flops / (kern_ms * 1e-3) / 1e12
        line = {
            "metric": LJ_METRIC, "value": world * args.steps / elapsed, "unit": "box-generations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic ({n}-atom LJ box, density 0.8, r_cut 2.5 sigma, random-init weights)",
            "config": {"workload": f"lf_reverse_1x{n}lj_L{LAYERS}_H{HID}_nf{NF}_f32", "atoms": n,
                       "coupling_layers": LAYERS, "hidden_nf": HID, "node_nf": NF,
                       "parallelism": f"independent boxes x{world}", "unique_pairs_per_launch": pairs},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / PEAK_F32_MFMA_TFLOPS, "traffic": None,
                         "kernel": "enflow_lf_reverse_large_f32 (per layer: images, id_mapping, pairs, "
                                   "lg_layer_kernel<128,1,false>)",
                         "kernel_ms": kern_ms, "flops_per_launch": flops, "gemm_precision": model.gemm_precision,
                         "matrix_pipe": matrix_pipe(achieved, model.gemm_precision)},
            "cpu_baseline": None,
        }
        print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1536)
    ap.add_argument("--mode", choices=("forward", "generate", "chain", "train", "lj"), default="forward",
                    help="forward: the headline metric (configs[1]); generate: configs[2] (bf16 reverse); "
                         "chain: configs[4] (256-atom chains, 16 layers); train: configs[3] per GPU; "
                         "lj: example/generate.yaml's 2944-atom LJ box (large-system kernels)")
    ap.add_argument("--atoms", type=int, default=None,
                    help="train mode: atoms per molecule (default 64); lj mode: atoms per box (default 2944)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    if args.mode in ("train", "lj"):
        if args.mode == "train":
            run_train(args, world, rank, local, device, dist)
        else:
            run_lj(args, world, rank, device, dist)
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return

    c = MODES[args.mode]
    mols, atoms, layers = c["mols"], c["atoms"], c["layers"]
    b, model, inp = build_workload(rank, device, mols, atoms, layers, c["chain"])
    model.gemm_precision = c["prec"]
    n_atoms = inp["h"].shape[0]
    work = {k: torch.empty_like(inp[k]) for k in ("h", "g", "pos", "vel")}
    noise = torch.empty_like(inp["h"])
    ldj_mol = torch.empty(mols, dtype=torch.float32, device=device)
    ldj = torch.empty(1, dtype=torch.float32, device=device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    stats = torch.zeros(2, dtype=torch.int64, device=device)
    idx = torch.empty(n_atoms, dtype=torch.int32, device=device)
    mx = torch.zeros(1, dtype=torch.int32, device=device)
    onehot = torch.empty((n_atoms, NF), dtype=torch.float32, device=device)
    model.packed_layers(device)
    model.dequantize.packed(device)
    gen = torch.Generator(device).manual_seed(rank)
    from enflow_amd import _lib as L_
    Lh = L_.lib()

    def fwd(st=None):
        for k in work:
            work[k].copy_(inp[k])
        torch.randn(noise.shape, generator=gen, out=noise)
        model.forward_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                              inp["mol_ptr"], atoms, noise, ldj_mol, ldj, err, st)

    # one counted forward: pair statistics for the roofline's algorithmic FLOPs
    fwd(stats)
    torch.cuda.synchronize()
    pairs, edges = (int(x) for x in stats.tolist())
    if int(err.item()) != 0:
        raise RuntimeError(f"flow kernel error flag {int(err.item())}")
    if c["reverse"]:
        # generate direction: invert a forward output (main.py:263-278)
        gsrc = {k: work[k].clone() for k in work}

        def step():
            for k in work:
                work[k].copy_(gsrc[k])
            model.reverse_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                                  inp["mol_ptr"], atoms, idx, mx, err)
            L_.check(Lh.enflow_one_hot_f32(L_.ptr(idx), n_atoms, NF, L_.ptr(onehot), L_.stream_ptr(device)),
                     "one_hot")
    else:
        step = fwd

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    from enflow_amd.distributed import max_over_ranks
    elapsed = max_over_ranks(elapsed, device)

    # kernel-only timing with HIP events on the launch stream (torch's current stream)
    stream = torch.cuda.current_stream(device)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    for e0, e1 in evs:
        for k in work:
            work[k].copy_(gsrc[k] if c["reverse"] else inp[k])
        if c["reverse"]:
            e0.record(stream)
            model.reverse_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                                  inp["mol_ptr"], atoms, idx, mx, err)
            e1.record(stream)
        else:
            torch.randn(noise.shape, generator=gen, out=noise)
            e0.record(stream)
            model.forward_buffers(work["h"], work["g"], work["pos"], work["vel"], inp["box"], inp["r_cut"],
                                  inp["mol_ptr"], atoms, noise, ldj_mol, ldj, err)
            e1.record(stream)
    torch.cuda.synchronize()
    kern_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs]))

    if rank == 0:
        prec_id = L_.PRECISIONS[model.gemm_precision]
        total_mols = mols * world * args.steps
        flops = flops_per_launch(pairs, n_atoms, layers, HID, NF)
        if c["reverse"]:
            flops -= n_atoms * (2 * HID * NF + 2 * HID * 2 * NF)     # no ArgMax network in reverse
        achieved = flops / (kern_ms * 1e-3) / 1e12
        nmax = 32 if atoms <= 32 else (64 if atoms <= 64 else 256)
        line = {
            "metric": c["metric"],
            "value": total_mols / elapsed,
            "unit": c["unit"],
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if c["prec"] == "bf16" else "f32",
            "data": f"synthetic (random-walk {atoms}-atom {'chains' if c['chain'] else 'molecules'}, "
                    f"random-init weights)",
            "config": {"workload": workload_name(args.mode), "molecules_per_gpu": mols,
                       "atoms_per_molecule": atoms, "coupling_layers": layers, "hidden_nf": HID,
                       "node_nf": NF, "global_batch": mols * world,
                       "parallelism": f"molecule-sharded x{world}",
                       "unique_pairs_per_launch": pairs, "reference_edges_per_launch": edges},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": PEAK_F32_MFMA_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / PEAK_F32_MFMA_TFLOPS,
                         "traffic": load_traffic() if args.mode == "forward" else None,
                         "kernel": f"lf_flow_kernel<128,{nmax},{str(c['reverse']).lower()},{prec_id}>",
                         "kernel_ms": kern_ms, "flops_per_launch": flops,
                         "gemm_precision": model.gemm_precision,
                         "matrix_pipe": matrix_pipe(achieved, model.gemm_precision),
                         "note": "achieved = fp32-equivalent algorithmic FLOPs / event-timed launch; peak = dense "
                                 "f32 MFMA (the arithmetic the path delivers). f16x3 runs the GEMMs as 3 "
                                 "split-fp16 products on the f16 MFMA pipe: matrix_pipe is that pipe's "
                                 "issued rate vs its dense peak (see DESIGN.md)"},
            "cpu_baseline": None,
        }
        if world == 1 and not args.no_cpu_baseline and args.mode == "forward":
            line["cpu_baseline"] = cpu_baseline(args.cpu_sample)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
