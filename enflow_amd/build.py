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


def build(force=False, verbose=False, out=OUT, defines=()):
    """defines: extra -D flags (A/B and ablation variants built to another `out`)."""
    deps = SRCS + HDRS
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return out
    # one hipcc per source, in parallel, then one link
    base = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-I", os.path.join(ROOT, "include"), *[f"-D{d}" for d in defines]]
    # objects are kept next to the library (git-ignored) and reused while they are
    # newer than their source, the shared headers and this build's flags
    objs = [out + "." + os.path.basename(src) + ".o" for src in SRCS]
    stamp = out + ".flags"
    flags = " ".join(base)
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags
    hdrs = HDRS
    procs = []
    for src, obj in zip(SRCS, objs):
        if (not force and same_flags and os.path.exists(obj) and
                all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in [src] + hdrs)):
            continue
        cmd = base + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd))
    if any(p.wait() != 0 for p in procs):
        raise subprocess.CalledProcessError(1, "hipcc")
    with open(stamp, "w") as fh:
        fh.write(flags)
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import sys
    # python -m enflow_amd.build [OUT.so [DEFINE ...]]
    if len(sys.argv) > 1:
        print(build(force=True, verbose=True, out=os.path.abspath(sys.argv[1]), defines=sys.argv[2:]))
    else:
        print(build(force=True, verbose=True))
