"""Benchmark: enflow LFIntegrator forward + log|detJ| on MI355X.

Workload (BASELINE.json configs[1]): per GPU a batch of 1024 synthetic
22-atom molecules, 8 EGCL coupling layers, hidden_nf 128, node_nf 5,
float32, ArgMax dequantisation, periodic neighbour lists rebuilt every layer.
One step = one fused forward over the batch (ArgMax noise drawn on device,
inputs copied into the work buffers, ONE flow kernel + one reduce kernel),
inputs already resident in HBM.

Multi-GPU: one process per GPU, molecules sharded across ranks with no
collective in the data path.  `--gpus N` launches the N ranks itself (a
`torch.distributed.run` child, started before this process touches the GPU)
unless WORLD_SIZE is already set by an external launcher.  `value` is weak
scaling (1024 molecules per GPU); `strong_scaling` re-times the same flow with
a fixed global batch of 1024 molecules split over the ranks.  Barrier +
synchronize around every timed region, MAX time over ranks.

Also reported (rank 0): the roofline of the flow kernel -- algorithmic FLOPs
from the kernel's own pair counters over its per-launch duration, measured
with HIP events bracketing exactly that kernel on its launch stream
(enflow_timing_*), against the peak of the matrix pipe the GEMMs issue on --
and the CPU oracle timed on a bounded sample over the host's cores
(cpu_baseline), run in a child process before the GPU is initialised.
"""
import argparse
import hashlib
import struct
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "molecule-transforms/sec (fwd+log|detJ|), batch 1024×22 atoms, 1/2/4/8 GPU"
# MI355X_MICROARCH.md: dense peaks (no sparsity)
PEAK_TFLOPS = {"f32": 157.3, "f16": 2500.0, "bf16": 2500.0}
MOLS_PER_GPU, ATOMS, LAYERS, HID, NF = 1024, 22, 8, 128, 5
BOX_CPU_SHARE = 16          # host CPUs a one-GPU box grants this job


# ---------------------------------------------------------------------------
# FLOP accounting
# ---------------------------------------------------------------------------
def gemm_parts(hid, nf):
    """Algorithmic FLOPs (multiply-add = 2) of each GEMM / dot of the flow,
    with where it runs: per unique pair edge_nn.0 (2nf+1 -> H), edge_nn.2,
    coord_nn.0 (H -> H) on MFMA, coord_nn.2 (H -> 1) on VALU; per atom and
    layer vel_scaling_nn.0, node_nn.0, node_nn.2 on MFMA, vel_scaling_nn.2 on
    VALU; per atom once ArgMax.network (VALU)."""
    return {
        "pair": {"edge_nn.0": 2 * hid * (2 * nf + 1), "edge_nn.2": 2 * hid * hid,
                 "coord_nn.0": 2 * hid * hid, "coord_nn.2": 2 * hid},
        "atom_layer": {"vel_scaling_nn.0": 2 * hid * nf, "vel_scaling_nn.2": 2 * hid,
                       "node_nn.0": 2 * hid * (hid + nf), "node_nn.2": 2 * hid * nf},
        "atom": {"argmax.network": 2 * hid * nf + 2 * hid * 2 * nf},
    }


VALU_PARTS = {"coord_nn.2", "vel_scaling_nn.2", "argmax.network"}


def products(prec, part):
    """MFMA products issued per algorithmic FLOP of `part` (0 = VALU).
    f16x3: x = hi + lo in fp16, hi*hi + hi*lo + lo*hi on the F16 pipe.  bf16
    (generate config): the two H x H edge GEMMs are one bf16 product, edge_nn.0
    and the node phase stay f16x3.  f32: one product on the F32 pipe."""
    if part in VALU_PARTS:
        return 0
    if prec == "bf16" and part in ("edge_nn.2", "coord_nn.0"):
        return 1
    return 3 if prec in ("f16x3", "bf16") else 1


def flop_counts(pairs, atoms, layers, hid, nf, prec, argmax=True):
    """(algorithmic FLOPs, issued matrix-pipe FLOPs) of one launch."""
    parts = gemm_parts(hid, nf)
    units = {"pair": pairs, "atom_layer": atoms * layers, "atom": atoms if argmax else 0}
    alg = issued = 0
    for kind, d in parts.items():
        for name, f in d.items():
            alg += units[kind] * f
            issued += units[kind] * f * products(prec, name)
    return alg, issued


def flops_per_launch(pairs, atoms, layers, hid, nf):
    return flop_counts(pairs, atoms, layers, hid, nf, "f32")[0]


def pipe_of(prec):
    return "f32" if prec == "f32" else ("f16" if prec == "f16x3" else "bf16")


def roofline_mfma(alg, issued, kern_ms, prec, kernel, traffic=None, extra=None):
    """Roofline object: achieved = algorithmic FLOPs / per-launch duration;
    peak = the issuing pipe's dense peak scaled by algorithmic/issued FLOPs (so
    frac = issued FLOP rate / pipe peak exactly)."""
    pipe = pipe_of(prec)
    t = kern_ms * 1e-3
    achieved = alg / t / 1e12
    eff_peak = PEAK_TFLOPS[pipe] * alg / issued
    r = {"bound": "mfma", "achieved": achieved, "peak": eff_peak, "unit": "TFLOP/s",
         "frac": achieved / eff_peak, "traffic": traffic, "kernel": kernel, "kernel_ms": kern_ms,
         "flops_per_launch": alg, "gemm_precision": prec,
         "matrix_pipe": {"pipe": pipe, "issued_flops_per_launch": issued,
                         "issued_tflops": issued / t / 1e12, "pipe_peak_tflops": PEAK_TFLOPS[pipe],
                         "frac": issued / t / 1e12 / PEAK_TFLOPS[pipe]},
         "fp32_equivalent": {"tflops": achieved, "vs_f32_peak": achieved / PEAK_TFLOPS["f32"]},
         "note": ("achieved = algorithmic FLOPs (pair counters x per-pair FLOPs) / HIP-event duration of "
                  "the kernel; peak = dense peak of the pipe the GEMMs issue on (MI355X_MICROARCH.md) x "
                  "algorithmic / issued FLOPs, so frac = issued matrix FLOPs / pipe peak")}
    if extra:
        r.update(extra)
    return r


# ---------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------
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


def workload_name(mode="forward"):
    c = MODES[mode]
    kind = "reverse" if c["reverse"] else "forward"
    geo = "chain" if c["chain"] else ""
    return f"lf_{kind}_{c['mols']}x{c['atoms']}{geo}_L{c['layers']}_H{HID}_nf{NF}_f32"


def lib_sha():
    from enflow_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as fh:
        for blk in iter(lambda: fh.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def _elf_sections(d, base=0):
    """{name: (offset, size)} of an ELF64 image at d[base:]."""
    shoff = struct.unpack_from("<Q", d, base + 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", d, base + 0x3A)
    raw = []
    for i in range(shnum):
        name, _typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", d, base + shoff + i * shentsize)
        raw.append((name, off, size))
    stroff = base + raw[shstrndx][1]
    out = {}
    for name, off, size in raw:
        e = d.index(b"\0", stroff + name)
        out[d[stroff + name:e].decode()] = (base + off, size)
    return out


def code_sha(path=None):
    """Hash of the device code the library runs: the .text of every gfx950 code
    object in its .hip_fatbin (offload bundles in order).  Unlike a hash of the
    whole .so it does not move with the build directory (hipcc's path-derived
    __hip_cuid_* symbols live outside .text), so a rebuild of the same sources
    anywhere keeps roofline.traffic's PMC summary."""
    from enflow_amd import _lib
    with open(path or _lib.LIB_PATH, "rb") as fh:
        d = fh.read()
    off, size = _elf_sections(d)[".hip_fatbin"]
    fat = d[off:off + size]
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    h = hashlib.sha256()
    pos = fat.find(magic)
    while pos >= 0:
        n = struct.unpack_from("<Q", fat, pos + len(magic))[0]
        q = pos + len(magic) + 8
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple and esize > 0:
                t_off, t_size = _elf_sections(fat, pos + eoff)[".text"]
                h.update(fat[t_off:t_off + t_size])
        pos = fat.find(magic, q)
    return h.hexdigest()[:16]


def load_traffic(workload, sha, code=None):
    """HBM bytes per flow-kernel launch from a committed rocprofv3 PMC summary
    (profiles/*pmc_traffic.json, written by profiles/collect_pmc.py) -- only if
    it was collected for this workload AND this exact library build."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc_traffic.json"), recursive=True),
                       reverse=True):
        try:
            with open(path) as fh:
                d = json.load(fh)
        except Exception:
            continue
        if d.get("workload") != workload:
            continue
        if (code is not None and d.get("code_sha") == code) or d.get("lib_sha") == sha:
            return d.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def build_model(device, layers, seed=0):
    from enflow_amd.data.synthetic import default_dt
    from enflow_amd.nn import EGCL, ArgMax
    from enflow_amd.flow import LFIntegrator
    torch.manual_seed(seed)                  # same (random-init) weights on every rank
    return LFIntegrator([EGCL(NF, NF, HID) for _ in range(layers)], ArgMax(NF, HID),
                        dt=default_dt()).to(device)


def batch_tensors(b, device):
    from enflow_amd.utils.helpers import mol_ptr_from_counts
    f = lambda k: torch.tensor(b[k], dtype=torch.float32, device=device).contiguous()  # noqa: E731
    inp = {k: f(k) for k in ("h", "g", "pos", "vel", "box", "r_cut")}
    inp["mol_ptr"] = mol_ptr_from_counts(torch.tensor(np.diff(b["mol_ptr"])), device=device)
    return inp


def sub_batch(b, m0, m1):
    p = b["mol_ptr"]
    a0, a1 = int(p[m0]), int(p[m1])
    out = {k: b[k][a0:a1] for k in ("h", "g", "pos", "vel", "box")}
    out["r_cut"] = b["r_cut"][m0:m1]
    out["mol_ptr"] = p[m0:m1 + 1] - a0
    return out


class FlowRunner:
    """Preallocated buffers + one step of the fused flow on a batch."""

    def __init__(self, model, inp, atoms, reverse, device, gen):
        self.model, self.inp, self.atoms, self.reverse = model, inp, atoms, reverse
        self.dev, self.gen = device, gen
        n_atoms = inp["h"].shape[0]
        mols = inp["mol_ptr"].numel() - 1
        self.work = {k: torch.empty_like(inp[k]) for k in ("h", "g", "pos", "vel")}
        self.noise = torch.empty_like(inp["h"])
        self.ldj_mol = torch.empty(max(mols, 1), dtype=torch.float32, device=device)
        self.ldj = torch.empty(1, dtype=torch.float32, device=device)
        self.status = torch.zeros(2, dtype=torch.int32, device=device)   # error word, ldj ticket
        self.err = self.status[:1]
        self.calls = 0
        self.idx = torch.empty(max(n_atoms, 1), dtype=torch.int32, device=device)
        self.mx = torch.zeros(1, dtype=torch.int32, device=device)
        self.onehot = torch.empty((n_atoms, NF), dtype=torch.float32, device=device)
        model.packed_layers(device)
        model.dequantize.packed(device)
        self.src = inp
        if reverse:      # generate direction: invert a forward output (main.py:263-278)
            self.forward_once()
            torch.cuda.synchronize()
            self.src = {k: self.work[k].clone() for k in self.work}

    def forward_once(self, stats=None):
        # one launch: reads the input batch, writes the work buffers, draws the
        # ArgMax noise in the kernel (fresh Philox counters every call) and
        # reduces log|detJ| in the same launch (enflow_lf_forward_io_f32)
        i, w = self.inp, self.work
        self.calls += 1
        self.model.forward_buffers(w["h"], w["g"], w["pos"], w["vel"], i["box"], i["r_cut"], i["mol_ptr"],
                                   self.atoms, None, self.ldj_mol, self.ldj, self.err, stats,
                                   src=(i["h"], i["g"], i["pos"], i["vel"]),
                                   noise_key=(self.seed, self.calls * self.noise.numel()),
                                   ticket=self.status[1:])

    @property
    def seed(self):
        return 0x5eed0000 + int(self.gen.initial_seed())

    def step(self):
        if not self.reverse:
            return self.forward_once()
        from enflow_amd import _lib as L_
        i, w, s = self.inp, self.work, self.src
        self.model.reverse_buffers(w["h"], w["g"], w["pos"], w["vel"], i["box"], i["r_cut"], i["mol_ptr"],
                                   self.atoms, self.idx, self.mx, self.err,
                                   src=(s["h"], s["g"], s["pos"], s["vel"]))
        n = w["h"].shape[0]
        L_.check(L_.lib().enflow_one_hot_f32(L_.ptr(self.idx), n, NF, L_.ptr(self.onehot),
                                             L_.stream_ptr(self.dev)), "one_hot")

    def check(self):
        torch.cuda.synchronize()
        if int(self.err.item()) != 0:
            raise RuntimeError(f"flow kernel error flag {int(self.err.item())}")


PREWARM_S = 0.5   # untimed clock pre-warm (s) before the W warmup steps (--prewarm-s)


def set_prewarm(seconds):
    global PREWARM_S
    PREWARM_S = max(0.0, float(seconds))


def timed(step, steps, warmup, dist, device):
    """An untimed clock pre-warm (steps for PREWARM_S seconds: the MI355X
    ramps its shader clock over the first ~20 launches), W
    untimed steps, then K steps between barrier + synchronize on both sides;
    returns the MAX elapsed seconds over ranks."""
    from enflow_amd.distributed import max_over_ranks
    if PREWARM_S > 0:
        # the same number of steps on every rank (a training step holds a
        # collective): timed from 2 steps, max over ranks
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        n = min(4000, int(PREWARM_S / max((time.perf_counter() - t0) / 2, 1e-5)))
        n = int(max_over_ranks(float(n), device)) if dist else n
        for i in range(n):
            step()
            if i % 8 == 7:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, device)


def module_call_timing(model, b, device, steps, warmup, reverse=False):
    """The reference's own call surface, timed like timed(): ``model(data)``
    (``model.reverse(data)`` for the generate mode) on a Data with the
    reference's fields (enflow_amd.data.Data), under torch.no_grad(), per call:
    the host's input handling, output allocation, the launch, the error word's
    synchronous read (raised from the call, as the reference raises inside
    forward) and the output dtype -- for fp32 inputs and for the reference's
    own float64 (BaseFlow casts its model, enflow/flow/base.py:12).  Each call
    gets a shallow copy of the batch (the reference rebinds data's tensors to
    the outputs), so every call transforms the same inputs."""
    from enflow_amd.data import Data
    out = {}
    for name, dt in (("float32", torch.float32), ("float64", torch.float64)):
        d = Data.from_arrays(b, device=device, dtype=dt)
        if reverse:     # generate direction: invert one forward output (main.py:263-278)
            with torch.no_grad():
                d, _ = model(d._replace())
        call = (lambda: model.reverse(d._replace())) if reverse else (lambda: model(d._replace()))

        def step():
            with torch.no_grad():
                call()
        el = timed(step, steps, warmup, None, device)
        out[name] = {"ms_per_call": el / steps * 1e3, "calls": steps}
    out["note"] = ("model.reverse(data)" if reverse else "model(data)") + \
        " under torch.no_grad() on enflow_amd.data.Data, one synchronous error-word read per call"
    return out


def kernel_times(step, steps):
    """Per-kernel average launch duration (ms) over `steps` steps, from the
    library's HIP-event timer (events on each kernel's own launch stream)."""
    from enflow_amd import _lib as L_
    torch.cuda.synchronize()
    with L_.KernelTimer() as t:
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
    return {k: {"ms_per_launch": v[0] / v[1], "launches": v[1]} for k, v in t.stats.items()}


# ---------------------------------------------------------------------------
# CPU baseline (child process, no GPU)
# ---------------------------------------------------------------------------
_CPU = {}


def _cpu_chunk(bounds):
    from threadpoolctl import threadpool_limits
    from oracle import enflow_oracle as O
    from enflow_amd.data.synthetic import default_dt
    m0, m1 = bounds
    b = sub_batch(_CPU["b"], m0, m1)
    eps = _CPU["eps"][int(_CPU["b"]["mol_ptr"][m0]):int(_CPU["b"]["mol_ptr"][m1])]
    with threadpool_limits(1):
        t0 = time.perf_counter()
        O.lf_forward(_CPU["layers"], _CPU["dq"], b, eps, default_dt())
        return time.perf_counter() - t0


def cpu_baseline(per_core=192):
    """The CPU oracle (numpy float64 restatement of the reference path,
    oracle/enflow_oracle.py) on a bounded sample of the same workload:
    molecules are independent, so the sample is sharded over one single-thread
    worker process per host core (the box grants a one-GPU job 16)."""
    import multiprocessing as mp
    from enflow_amd.data.synthetic import make_molecules
    from enflow_amd.nn import EGCL, ArgMax
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    # the GPU box's affinity set shows the whole machine (shared with other jobs);
    # a one-GPU job is granted BOX_CPU_SHARE of them, exported as OMP_NUM_THREADS
    grant = int(os.environ.get("OMP_NUM_THREADS") or BOX_CPU_SHARE)
    cores = max(1, min(avail, grant))
    torch.manual_seed(0)
    nets = [EGCL(NF, NF, HID) for _ in range(LAYERS)]
    am = ArgMax(NF, HID)
    _CPU["layers"] = [{k: v.double().numpy() for k, v in n.state_dict().items()} for n in nets]
    _CPU["dq"] = {k: v.double().numpy() for k, v in am.state_dict().items()}
    total = cores * per_core
    _CPU["b"] = make_molecules(total, ATOMS, nf=NF, seed=4242)
    _CPU["eps"] = np.random.default_rng(0).normal(size=_CPU["b"]["h"].shape)
    chunks = [(c * per_core, (c + 1) * per_core) for c in range(cores)]
    ctx = mp.get_context("fork")          # this child never touches the GPU
    t0 = time.perf_counter()
    with ctx.Pool(cores) as pool:
        per = pool.map(_cpu_chunk, chunks)
    wall = time.perf_counter() - t0
    ref = None   # the reference itself (torch float64, build container; tools/ref_cpu_timing.py)
    try:
        with open(os.path.join(ROOT, "profiles", "r02", "r02_reference_cpu.json")) as f:
            r = json.load(f)
        ref = {"value": r["configs[1]_forward"]["value"], "unit": "molecule-transforms/s",
               "threads": r["host"]["torch_threads"], "cpu": r["host"]["cpu"],
               "sample": r["configs[1]_forward"]["sample"],
               "source": "profiles/r02/r02_reference_cpu.json (build container, not this host)"}
    except (OSError, KeyError, ValueError):
        pass
    return {"value": total / wall, "unit": "molecule-transforms/s", "cores": cores, "kind": "port",
            "cores_note": (f"{cores} single-thread worker processes = the host CPUs this job is granted "
                           f"(OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}); the affinity set "
                           f"lists {avail} logical CPUs of the whole machine, shared with other jobs"),
            "host_cpu": host_cpu_info(),
            "reference_torch": ref,
            "sample": f"{total} molecules x {ATOMS} atoms ({per_core} per core), {LAYERS} layers, hidden {HID}: "
                      f"numpy float64 oracle (oracle/enflow_oracle.py), one single-thread process per core, "
                      f"{wall:.1f} s wall (per-core {min(per):.1f}-{max(per):.1f} s); host CPUs visible "
                      f"{avail}, used {cores}"}


def host_cpu_info():
    """Model, logical CPUs and physical cores (distinct (package, core) pairs) of the host."""
    info = {"logical": os.cpu_count()}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
        cores = set()
        base = "/sys/devices/system/cpu"
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                t = os.path.join(base, d, "topology")
                with open(os.path.join(t, "physical_package_id")) as a, open(os.path.join(t, "core_id")) as b:
                    cores.add((a.read().strip(), b.read().strip()))
        info["physical_cores"] = len(cores)
    except OSError:
        pass
    return info


def run_cpu_baseline_child(per_core):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-only", "--cpu-per-core", str(per_core)]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    if r.returncode != 0:
        print(r.stderr[-2000:], file=sys.stderr)
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


# ---------------------------------------------------------------------------
# modes
# ---------------------------------------------------------------------------
def run_flow(args, world, rank, device, dist, cpu):
    c = MODES[args.mode]
    from enflow_amd.data.synthetic import make_molecules
    from enflow_amd.distributed import shard_range
    mols, atoms, layers = c["mols"], c["atoms"], c["layers"]
    model = build_model(device, layers)
    model.gemm_precision = c["prec"]
    gen = torch.Generator(device).manual_seed(rank)
    b = make_molecules(mols, atoms, nf=NF, seed=1000 + rank, chain=c["chain"])
    inp = batch_tensors(b, device)
    run = FlowRunner(model, inp, atoms, c["reverse"], device, gen)
    stats = torch.zeros(2, dtype=torch.int64, device=device)
    run.forward_once(stats)               # one counted forward: pair statistics for the FLOPs
    run.check()
    pairs, edges = (int(x) for x in stats.tolist())

    elapsed = timed(run.step, args.steps, args.warmup, dist, device)
    kt = kernel_times(run.step, max(args.steps, 5))
    kname = "lf_flow_kernel<rev>" if c["reverse"] else "lf_flow_kernel<fwd>"
    run.check()

    module_call = None
    if args.mode in ("forward", "generate") and world == 1:
        module_call = module_call_timing(model, b, device, args.steps, args.warmup, reverse=c["reverse"])
        module_call["bench_entry_ms_per_step"] = elapsed / args.steps * 1e3

    strong = None
    if args.mode == "forward":
        if world > 1:
            # strong scaling: the same global batch of 1024 molecules split over the ranks
            g = make_molecules(mols, atoms, nf=NF, seed=1000, chain=c["chain"])
            m0, m1 = shard_range(mols, rank, world)
            srun = FlowRunner(model, batch_tensors(sub_batch(g, m0, m1), device), atoms, False, device, gen)
            s_el = timed(srun.step, args.steps, args.warmup, dist, device)
            s_kt = kernel_times(srun.step, max(args.steps, 5))
            srun.check()
            # the instance the library picked for this shard (4-wave, 8-wave or split)
            sname = next((k for k in ("lf_fs_kernel<fwd>", "lf_flow_kernel<fwd,lat>", kname) if k in s_kt), None)
            strong = {"global_batch": mols, "molecules_per_gpu": m1 - m0, "value": mols * args.steps / s_el,
                      "ms_per_step": s_el / args.steps * 1e3, "flow_kernel": sname,
                      "flow_kernel_ms": s_kt[sname]["ms_per_launch"] if sname else None}
        else:
            strong = {"global_batch": mols, "molecules_per_gpu": mols, "value": mols * args.steps / elapsed,
                      "ms_per_step": elapsed / args.steps * 1e3, "note": "N=1: identical to the weak-scaling run"}

    if rank == 0:
        n_atoms = inp["h"].shape[0]
        alg, issued = flop_counts(pairs, n_atoms, layers, HID, NF, c["prec"], argmax=not c["reverse"])
        kern_ms = kt[kname]["ms_per_launch"]
        nmax = 32 if atoms <= 32 else (64 if atoms <= 64 else 256)
        sha, code = lib_sha(), code_sha()
        traffic, tsrc = load_traffic(workload_name(args.mode), sha, code)
        line = {
            "metric": c["metric"], "value": mols * world * args.steps / elapsed, "unit": c["unit"],
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if c["prec"] == "bf16" else "f32 (f16x3 GEMMs)",
            "data": f"synthetic (random-walk {atoms}-atom {'chains' if c['chain'] else 'molecules'}, "
                    f"random-init weights)",
            "config": {"workload": workload_name(args.mode), "molecules_per_gpu": mols,
                       "atoms_per_molecule": atoms, "coupling_layers": layers, "hidden_nf": HID,
                       "node_nf": NF, "global_batch": mols * world,
                       "parallelism": f"molecule-sharded x{world}" if world > 1 else "single GPU",
                       "unique_pairs_per_launch": pairs, "reference_edges_per_launch": edges},
            "roofline": roofline_mfma(alg, issued, kern_ms, c["prec"],
                                      f"lf_flow_kernel<{HID},{nmax},{str(c['reverse']).lower()},"
                                      f"{c['prec']}>", traffic,
                                      {"traffic_source": tsrc, "lib_sha": sha, "code_sha": code}),
            "kernels": kt,
            "cpu_baseline": cpu,
        }
        if strong is not None:
            line["strong_scaling"] = strong
        if module_call is not None:
            line["module_call"] = module_call
        print(json.dumps(line), flush=True)


TRAIN_METRIC = "molecule-train-steps/sec (fwd+NLL+bwd+Adam, RCCL grad all-reduce), batch 1024×64 atoms per GPU"
TRAIN_ATOMS = 64


def train_flops(pairs, atoms, layers, hid, nf):
    """Algorithmic FLOPs of one training step's flow part: the forward plus,
    per unique pair, the recomputed edge chain, its adjoint GEMMs
    (coord_nn.0^T, edge_nn.2^T, edge_nn.0^T) and the three weight-gradient
    outer products; per atom-layer the node MLP recompute, adjoint and weight
    gradients."""
    fwd_pair = 2 * hid * (2 * nf + 1) + 4 * hid * hid + 2 * hid
    bwd_pair = fwd_pair + (4 * hid * hid + 2 * hid * (2 * nf + 1)) + (4 * hid * hid + 2 * hid * (2 * nf + 2) + 2 * hid)
    node = (2 * hid * nf + 2 * hid) + (2 * hid * (hid + nf) + 2 * hid * nf)
    return (flops_per_launch(pairs, atoms, layers, hid, nf) + pairs * bwd_pair +
            atoms * layers * 3 * node)


def layer_bwd_flops(pairs, atoms, hid, nf):
    """lf_layer_bwd_kernel, summed over layers: per pair the recomputed edge
    chain (edge_nn.0, edge_nn.2, coord_nn.0) and the adjoint GEMMs
    coord_nn.0^T, edge_nn.2^T, edge_nn.0^T; per atom-layer the node MLP
    recompute + adjoint (node weight gradients run in outer_acc_kernel)."""
    rec = 2 * hid * (2 * nf + 1) + 4 * hid * hid
    adj = 4 * hid * hid + 2 * hid * (2 * nf + 1)
    node = 2 * (2 * hid * nf + 2 * hid * (hid + nf) + 2 * hid * nf)
    return pairs * (rec + adj) + atoms * node


def outer_x3_flops(pairs, hid, nf):
    """outer_x3_kernel, summed over layers: the pair-row weight gradients
    dW = sum_rows DY^T X of edge_nn.0, edge_nn.2, coord_nn.0 (+ coord_nn.2)."""
    return pairs * (2 * hid * (2 * nf + 1) + 4 * hid * hid + 2 * hid)


def run_train(args, world, rank, local, device, dist):
    """Config 3: a full training step (the reference's loop body,
    enflow/main.py:217-223) per GPU on 1024 synthetic 64-atom molecules,
    DDP (RCCL all-reduce of the gradients, main.py:159) across ranks."""
    from enflow_amd.data.synthetic import make_molecules, default_kBT
    from enflow_amd.flow import Alchemical_NLL
    from enflow_amd.data import Data
    from enflow_amd import _lib as L_
    atoms = args.atoms or TRAIN_ATOMS
    radius = 4.0 * (atoms / 22.0) ** (1.0 / 3.0)
    b = make_molecules(MOLS_PER_GPU, atoms, nf=NF, seed=2000 + rank, radius=radius)
    model = build_model(device, LAYERS)
    net = model
    if dist:
        from torch.nn.parallel import DistributedDataParallel as DDP
        net = DDP(model, device_ids=[local])      # main.py:159; backend nccl = RCCL
    model.defer_error_check = not args.sync_errors
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
        loss.backward()                     # a backward error NaN-poisons the grads; raised at the next check
        opt.step()
        return loss

    # pair statistics for the algorithmic FLOPs (one counted inference forward)
    stats = torch.zeros(2, dtype=torch.int64, device=device)
    with torch.no_grad():
        w = {k: getattr(base, k).clone() for k in ("h", "g", "pos", "vel")}
        ldj_mol = torch.empty(MOLS_PER_GPU, dtype=torch.float32, device=device)
        ldj = torch.empty(1, dtype=torch.float32, device=device)
        err = torch.zeros(1, dtype=torch.int32, device=device)
        model.forward_buffers(w["h"], w["g"], w["pos"], w["vel"], base.box, base.r_cut, base.mol_ptr, atoms,
                              torch.randn_like(w["h"]), ldj_mol, ldj, err, stats)
    torch.cuda.synchronize()
    if int(err.item()) != 0:
        raise RuntimeError(f"flow kernel error flag {int(err.item())}")
    pairs = int(stats[0].item())

    losses = []
    elapsed = timed(lambda: losses.append(step()), args.steps, args.warmup, dist, device)
    kt = kernel_times(step, max(args.steps, 3))
    if rank == 0:
        n_atoms = MOLS_PER_GPU * atoms
        flops = train_flops(pairs, n_atoms, LAYERS, HID, NF)
        ms = elapsed / args.steps * 1e3
        # dominant kernels priced against the F16 pipe they issue on (F16X3: 3 products per FLOP)
        roof = {}
        lb = kt.get("lf_layer_bwd_kernel")
        if lb:       # one launch per layer
            per = layer_bwd_flops(pairs, n_atoms, HID, NF) / LAYERS
            roof["lf_layer_bwd_kernel"] = roofline_mfma(per, 3 * per, lb["ms_per_launch"], "f16x3",
                                                        "lf_layer_bwd_kernel<128,64>")
        ox = kt.get("outer_x3_kernel")
        if ox:
            per = outer_x3_flops(pairs, HID, NF) / LAYERS
            roof["outer_x3_kernel"] = roofline_mfma(per, 3 * per, ox["ms_per_launch"], "f16x3", "outer_x3_kernel")
        fk = kt.get("lf_flow_kernel<fwd>")
        if fk:
            alg, issued = flop_counts(pairs, n_atoms, LAYERS, HID, NF, "f16x3")
            roof["lf_flow_kernel<fwd>"] = roofline_mfma(alg, issued, fk["ms_per_launch"], "f16x3",
                                                        "lf_flow_kernel<128,64,false,f16x3> (+tape)")
        dom = max(roof, key=lambda k: kt[k]["ms_per_launch"] * kt[k]["launches"]) if roof else None
        line = {
            "metric": TRAIN_METRIC, "value": MOLS_PER_GPU * world * args.steps / elapsed,
            "unit": "molecules/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32 (f16x3 GEMMs)",
            "data": f"synthetic (random-walk {atoms}-atom molecules, random-init weights)",
            "config": {"workload": f"lf_train_{MOLS_PER_GPU}x{atoms}_L{LAYERS}_H{HID}_nf{NF}_f32",
                       "molecules_per_gpu": MOLS_PER_GPU, "atoms_per_molecule": atoms,
                       "coupling_layers": LAYERS, "hidden_nf": HID, "node_nf": NF,
                       "global_batch": MOLS_PER_GPU * world,
                       "parallelism": f"molecule-sharded x{world}, DDP grad all-reduce" if world > 1
                       else "single GPU", "unique_pairs_per_layer_pass": pairs},
            "step_tflops": flops / (ms * 1e-3) / 1e12, "flops_per_step": flops,
            "roofline": roof.get(dom), "rooflines": roof, "kernels": kt,
            "final_loss": float(losses[-1]) if losses else None, "cpu_baseline": None,
        }
        print(json.dumps(line), flush=True)


LJ_METRIC = "LJ-box generations/sec (reverse/generate path, example/generate.yaml: 2944-atom periodic box)"


def run_lj(args, world, rank, device, dist):
    """The reference's example/generate.yaml system: one periodic 2944-atom
    Lennard-Jones box per GPU (batch 1), 8 coupling layers, hidden 128,
    generated by LFIntegrator.reverse (main.py:263-278) through the
    layer-by-layer large-system kernels (enflow_amd/csrc/enflow_large.hip).
    Not a BASELINE.json config: reported for the large-system path."""
    from enflow_amd.data.synthetic import make_lj_systems
    from enflow_amd.data import Data
    n = args.atoms or 2944
    b = make_lj_systems([n], seed=3000 + rank, nf=NF)
    b["pos"] = b["pos"] - np.round(b["pos"] / b["box"]) * b["box"]
    model = build_model(device, LAYERS)
    inp = batch_tensors(b, device)
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

    elapsed = timed(step, args.steps, args.warmup, dist, device)
    torch.cuda.synchronize()
    if int(err.item()) != 0:
        raise RuntimeError(f"flow kernel error flag {int(err.item())}")
    kt = kernel_times(step, max(args.steps, 5))
    if rank == 0:
        alg, issued = flop_counts(pairs, n, LAYERS, HID, NF, model.gemm_precision, argmax=False)
        lay = kt.get("lg_layer_kernel", {"ms_per_launch": float("nan"), "launches": 1})
        # the dominant kernel: the per-layer EGCL row-block kernel (one launch per layer)
        roof = roofline_mfma(alg / LAYERS, issued / LAYERS, lay["ms_per_launch"], model.gemm_precision,
                             "lg_layer_kernel<128,f16x3,false>")
        line = {
            "metric": LJ_METRIC, "value": world * args.steps / elapsed, "unit": "box-generations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 (f16x3 GEMMs)",
            "data": f"synthetic ({n}-atom LJ box, density 0.8, r_cut 2.5 sigma, random-init weights)",
            "config": {"workload": f"lf_reverse_1x{n}lj_L{LAYERS}_H{HID}_nf{NF}_f32", "atoms": n,
                       "coupling_layers": LAYERS, "hidden_nf": HID, "node_nf": NF,
                       "parallelism": f"independent boxes x{world}", "unique_pairs_per_launch": pairs},
            "roofline": roof, "kernels": kt, "cpu_baseline": None,
        }
        print(json.dumps(line), flush=True)


LJ_TRAIN_METRIC = "LJ-box training steps/sec (2944-atom periodic box, 8 layers, H=128: forward + NLL + backward + Adam)"


def run_lj_train(args, world, rank, local, device, dist):
    """Training on the reference's LJ system (enflow/data/lj.py:32-89 boxes
    through enflow/main.py:212-223): one 2944-atom periodic box per GPU, 8
    layers, hidden 128; the large-system tape and backward
    (enflow_lf_forward_large_f32 / enflow_lf_backward_large_f32).  Not a
    BASELINE.json config: reported for the large-system training path."""
    from enflow_amd.data.synthetic import make_lj_systems, default_kBT
    from enflow_amd.flow import Alchemical_NLL
    from enflow_amd.data import Data
    n = args.atoms or 2944
    b = make_lj_systems([n], seed=4000 + rank, nf=NF)
    b["pos"] = b["pos"] - np.round(b["pos"] / b["box"]) * b["box"]
    model = build_model(device, LAYERS)
    net = model
    if dist:
        from torch.nn.parallel import DistributedDataParallel as DDP
        net = DDP(model, device_ids=[local])
    model.defer_error_check = not args.sync_errors
    opt = torch.optim.Adam(model.parameters(), lr=1e-5)
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

    losses = []
    elapsed = timed(lambda: losses.append(step()), args.steps, args.warmup, dist, device)
    kt = kernel_times(step, max(args.steps, 3))
    from enflow_amd import _lib as L_
    L_.check_pending()
    if rank == 0:
        line = {
            "metric": LJ_TRAIN_METRIC, "value": world * args.steps / elapsed, "unit": "box-training-steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32 (f16x3 GEMMs)",
            "data": f"synthetic ({n}-atom LJ box, density 0.8, r_cut 2.5 sigma, random-init weights)",
            "config": {"workload": f"lf_train_1x{n}lj_L{LAYERS}_H{HID}_nf{NF}_f32", "atoms": n,
                       "coupling_layers": LAYERS, "hidden_nf": HID, "node_nf": NF,
                       "parallelism": f"independent boxes x{world}, DDP grad all-reduce" if world > 1
                       else "single GPU"},
            "kernels": kt, "final_loss": float(losses[-1]) if losses else None, "cpu_baseline": None,
        }
        print(json.dumps(line), flush=True)


def self_launch(n, argv):
    """Start N ranks under torch.distributed.run (a child process: this one has
    not touched the GPU) and return its exit code."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30,
                    help="untimed steps first: the first ~20 launches run while the clock ramps up")
    ap.add_argument("--prewarm-s", type=float, default=PREWARM_S,
                    help="untimed clock pre-warm (seconds of steps) before the warmup steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sync-errors", action="store_true",
                    help="train / lj_train: read the forward's error word before the forward returns (the module "
                         "default, LFIntegrator.defer_error_check = False) instead of at the start of "
                         "loss.backward(), which the reference's loop body calls right after (main.py:219-221)")
    ap.add_argument("--cpu-per-core", type=int, default=192,
                    help="cpu_baseline sample: molecules per host core (16 cores: ~15 s)")
    ap.add_argument("--cpu-baseline-only", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mode", choices=("forward", "generate", "chain", "train", "lj", "lj_train"), default="forward",
                    help="forward: the headline metric (configs[1]); generate: configs[2] (bf16 reverse); "
                         "chain: configs[4] (256-atom chains, 16 layers); train: configs[3] per GPU; "
                         "lj: example/generate.yaml's 2944-atom LJ box (large-system kernels); "
                         "lj_train: a training step on that box")
    ap.add_argument("--atoms", type=int, default=None,
                    help="train mode: atoms per molecule (default 64); lj mode: atoms per box (default 2944)")
    args = ap.parse_args()
    set_prewarm(args.prewarm_s)

    if args.cpu_baseline_only:
        print(json.dumps(cpu_baseline(args.cpu_per_core)), flush=True)
        return 0
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if torch.cuda.device_count() < args.gpus:      # device_count does not initialise HIP here
            print(f"bench.py: --gpus {args.gpus} but {torch.cuda.device_count()} GPUs visible", file=sys.stderr)
            return 2
        return self_launch(args.gpus, sys.argv[1:])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} differs from --gpus {args.gpus}; using {world}", file=sys.stderr)
    cpu = None
    if rank == 0 and world == 1 and args.mode == "forward" and not args.no_cpu_baseline:
        cpu = run_cpu_baseline_child(args.cpu_per_core)      # before this process initialises the GPU

    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=device)

    if args.mode == "train":
        run_train(args, world, rank, local, device, dist)
    elif args.mode == "lj":
        run_lj(args, world, rank, device, dist)
    elif args.mode == "lj_train":
        run_lj_train(args, world, rank, local, device, dist)
    else:
        run_flow(args, world, rank, device, dist, cpu)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
