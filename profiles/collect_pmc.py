"""Collect rocprofv3 PMC counters for the flow kernel, one counter group per
pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass;
never combined with any trace domain), and write

  gpurun_out/<tag>_pmc.json          every counter, averaged per flow-kernel dispatch
  gpurun_out/<tag>_pmc_traffic.json  HBM bytes per launch (bench.py reads the copy
                                     committed under profiles/)

This script never touches the GPU itself; it only launches rocprofv3
children (program after `--`, no exec hop).  Run on the GPU box:

    python profiles/collect_pmc.py r01
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PASSES = [
    ["FETCH_SIZE"],
    ["WRITE_SIZE"],
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
     "SQ_ACTIVE_INST_ANY", "GRBM_GUI_ACTIVE"],
    ["SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
     "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_VALU"],
    ["TCC_HIT_sum", "TCC_MISS_sum"],
    ["TCP_TCC_READ_REQ_sum", "TCP_TOTAL_CACHE_ACCESSES_sum", "TCC_REQ_sum"],
    ["SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_WAIT_INST_LDS", "SQ_INSTS_SMEM", "SQ_INST_CYCLES_VMEM_RD"],
]
# store-path diagnosis (collect_pmc.py TAG MODE KERNELS write)
PASSES_WRITE = [
    ["WRITE_SIZE"],
    ["TA_TA_BUSY_sum", "TA_BUFFER_WRITE_WAVEFRONTS_sum", "GRBM_GUI_ACTIVE"],
    ["TA_BUFFER_COALESCED_WRITE_CYCLES_sum", "TA_DATA_STALLED_BY_TC_CYCLES_sum"],
    ["TCP_TCC_WRITE_REQ_sum", "TCP_TCC_WRITE_REQ_LATENCY_sum", "TCP_PENDING_STALL_CYCLES_sum",
     "TCP_TCP_TA_DATA_STALL_CYCLES_sum"],
    ["TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_WRREQ_STALL_sum", "TCC_BUSY_sum"],
    ["TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "TCC_TOO_MANY_EA_WRREQS_STALL_sum"],
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_INSTS_VMEM_WR",
     "SQ_INSTS_VMEM_RD", "SQ_ACTIVE_INST_ANY"],
]
KERNEL = "lf_flow_kernel"


def run_pass(counters, outdir, mode="forward", kernels=(KERNEL,)):
    env = dict(os.environ, TMPDIR="/tmp")
    # an over-capacity counter request prints error 38 and then hangs: hard kill
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", outdir, "-o", "pmc", "--",
           sys.executable, os.path.join(ROOT, "bench.py"), "--mode", mode, "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=200)
    if r.returncode != 0:
        print(r.stderr[-3000:], file=sys.stderr)
        return {}
    vals = {}
    for path in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                kn = next((k for k in kernels if k in row.get("Kernel_Name", "")), None)
                if kn is None:
                    continue
                name = row.get("Counter_Name")
                v = float(row.get("Counter_Value", 0.0))
                key = (row.get("Dispatch_Id"), name if len(kernels) == 1 else f"{kn}:{name}")
                vals[key] = vals.get(key, 0.0) + v      # sum over dimensions of one dispatch
    per = {}
    for (disp, name), v in vals.items():
        per.setdefault(name, []).append(v)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    # usage: collect_pmc.py TAG [MODE [KERNEL,KERNEL,...]]   (traffic file: forward mode only)
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    mode = sys.argv[2] if len(sys.argv) > 2 else "forward"
    kernels = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else (KERNEL,)
    base = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    passes = PASSES_WRITE if len(sys.argv) > 4 and sys.argv[4] == "write" else PASSES
    allc = {}
    for i, counters in enumerate(passes):
        res = run_pass(counters, os.path.join(base, f"pass{i}"), mode, kernels)
        print(f"pass {i}: {res}", flush=True)
        allc.update(res)
    sys.path.insert(0, ROOT)
    import bench
    out = {"workload": bench.workload_name() if mode == "forward" else mode, "kernel": ",".join(kernels),
           "counters_per_dispatch": allc}
    dst = os.path.join(ROOT, "gpurun_out")      # merged back by gpurun; copied into profiles/
    with open(os.path.join(dst, f"{tag}_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    if mode == "forward" and "FETCH_SIZE" in allc and "WRITE_SIZE" in allc:
        # FETCH_SIZE / WRITE_SIZE are KiB.  gfx950 FETCH_SIZE under-reports wide
        # (16 B/lane) streaming reads by 2x (MI355X_MICROARCH.md, HBM); the
        # kernel's HBM reads are mostly narrow, so the raw value is reported and
        # the 2x-corrected one kept beside it as an upper bound.
        raw = (allc["FETCH_SIZE"] + allc["WRITE_SIZE"]) * 1024.0
        hi = (2 * allc["FETCH_SIZE"] + allc["WRITE_SIZE"]) * 1024.0
        tr = {"workload": bench.workload_name(), "kernel": KERNEL, "lib_sha": bench.lib_sha(), "code_sha": bench.code_sha(),
              "hbm_bytes_per_launch": raw,
              "hbm_bytes_per_launch_fetch_x2": hi, "fetch_kib": allc["FETCH_SIZE"],
              "write_kib": allc["WRITE_SIZE"]}
        with open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w") as fh:
            json.dump(tr, fh, indent=1)
        print(json.dumps(tr))


if __name__ == "__main__":
    main()
