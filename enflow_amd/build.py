"""Build libenflow_hip.so in-tree with hipcc for gfx950 (no JIT cache)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRCS = [os.path.join(CSRC, f) for f in ("enflow_flow.hip", "enflow_backward.hip", "enflow_large.hip", "enflow_timing.hip",
                                              "enflow_latency.hip")
        if os.path.exists(os.path.join(CSRC, f))]
HDRS = [os.path.join(CSRC, h) for h in ("flow_device.h", "flow_kernel.h", "enflow_timing.h", "enflow_large.h",
                                         "enflow_latency.h")] + [os.path.join(ROOT, "include", "enflow_hip.h")]
OUT = os.path.join(HERE, "libenflow_hip.so")
ARCH = os.environ.get("ENFLOW_OFFLOAD_ARCH", "gfx950")


OUT_NF16 = os.path.join(HERE, "libenflow_hip_nf16.so")
# the product libraries: (output, extra -D flags).  The 16-feature build is the
# same sources with ENFLOW_NFMAX=16 (node_nf 9..16); the 8-feature build keeps
# the smaller LDS images (two training workgroups per CU).
VARIANTS = [(OUT, ()), (OUT_NF16, ("ENFLOW_NFMAX=16",))]


def _start(force, verbose, out, defines):
    """Start the out-of-date compiles of one library; returns (procs, finish)."""
    deps = SRCS + HDRS
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return [], lambda: None
    # one hipcc per source, in parallel, then one link
    base = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-I", os.path.join(ROOT, "include"), *[f"-D{d}" for d in defines]]
    # objects are kept next to the library (git-ignored) and reused while they are
    # newer than their source, the shared headers and this build's flags
    objs = [out + "." + os.path.basename(src) + ".o" for src in SRCS]
    stamp = out + ".flags"
    flags = " ".join(base)
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags
    procs = []
    for src, obj in zip(SRCS, objs):
        if (not force and same_flags and os.path.exists(obj) and
                all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in [src] + HDRS)):
            continue
        cmd = base + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))

    def finish():
        with open(stamp, "w") as fh:
            fh.write(flags)
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return procs, finish


def build(force=False, verbose=False, out=OUT, defines=()):
    """One library (defines: extra -D flags; A/B and diagnostic variants are
    built to another `out`)."""
    procs, finish = _start(force, verbose, out, defines)
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    finish()
    return out


def build_all(force=False, verbose=False):
    """Every product library, all translation units compiled in parallel."""
    jobs = [_start(force, verbose, out, defs) for out, defs in VARIANTS]
    ok = all(p.wait() == 0 for procs, _ in jobs for p in procs)
    if not ok:
        raise subprocess.CalledProcessError(1, "hipcc")
    for _, finish in jobs:
        finish()
    return [out for out, _ in VARIANTS]


if __name__ == "__main__":
    import sys
    # python -m enflow_amd.build [OUT.so [DEFINE ...]]
    if len(sys.argv) > 1:
        print(build(force=True, verbose=True, out=os.path.abspath(sys.argv[1]), defines=sys.argv[2:]))
    else:
        print(build_all(force=True, verbose=True))
