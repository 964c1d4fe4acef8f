"""Build libenflow_hip.so in-tree with hipcc for gfx950 (no JIT cache).

Every translation unit is compiled with -save-temps=obj (the device assembly
of the same compilation; the code objects are identical to a plain compile)
and the device assembly goes through tools/asm_hazard_scan.py: an MFMA hazard
at an inline-asm boundary fails the build.  Objects and the scan reports live
in enflow_amd/build/<library>/ (git- and gpurun-ignored)."""
import glob
import importlib.util
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRCS = [os.path.join(CSRC, f) for f in ("enflow_flow.hip", "enflow_backward.hip", "enflow_large.hip", "enflow_timing.hip",
                                              "enflow_latency.hip", "enflow_split.hip")
        if os.path.exists(os.path.join(CSRC, f))]
HDRS = [os.path.join(CSRC, h) for h in ("flow_device.h", "flow_kernel.h", "enflow_timing.h", "enflow_large.h",
                                         "enflow_latency.h", "enflow_split.h")] + [os.path.join(ROOT, "include", "enflow_hip.h")]
OUT = os.path.join(HERE, "libenflow_hip.so")
ARCH = os.environ.get("ENFLOW_OFFLOAD_ARCH", "gfx950")
SCANNER = os.path.join(ROOT, "tools", "asm_hazard_scan.py")


OUT_NF16 = os.path.join(HERE, "libenflow_hip_nf16.so")
# the product libraries: (output, extra -D flags).  The 16-feature build is the
# same sources with ENFLOW_NFMAX=16 (node_nf 9..16); the 8-feature build keeps
# the smaller LDS images (two training workgroups per CU).
VARIANTS = [(OUT, ()), (OUT_NF16, ("ENFLOW_NFMAX=16",))]
# diagnostic / A-B switches that never go into a product library
DIAGNOSTIC = ("ENFLOW_STAMPS", "ENFLOW_DEV_ONLY", "ENFLOW_BWD_ABLATE", "ENFLOW_SKEW", "ENFLOW_PRIO",
              "ENFLOW_CHAIN_PRIO", "ENFLOW_AUX_PRIO", "ENFLOW_ABLATE_DEQUANT")


class HazardError(RuntimeError):
    pass


def _scanner():
    spec = importlib.util.spec_from_file_location("asm_hazard_scan", SCANNER)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def obj_dir(out):
    return os.path.join(HERE, "build", os.path.basename(out).replace(".", "_"))


def _start(force, verbose, out, defines):
    """Start the out-of-date compiles of one library; returns (procs, finish)."""
    if out in (OUT, OUT_NF16) and any(d.split("=")[0] in DIAGNOSTIC for d in defines):
        raise ValueError(f"diagnostic switches {defines} are not built into the product library {out}")
    deps = SRCS + HDRS
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps):
        return [], lambda: None
    odir = obj_dir(out)
    os.makedirs(odir, exist_ok=True)
    # one hipcc per source, in parallel, then one link
    base = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
            "-I", os.path.join(ROOT, "include"), *[f"-D{d}" for d in defines]]
    # objects are reused while they are newer than their source, the shared
    # headers and this build's flags
    objs = [os.path.join(odir, os.path.basename(src) + ".o") for src in SRCS]
    stamp = os.path.join(odir, "flags")
    flags = " ".join(base)
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags
    procs = []
    built = []
    for src, obj in zip(SRCS, objs):
        if (not force and same_flags and os.path.exists(obj) and
                all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in [src] + HDRS)):
            continue
        cmd = base + ["-save-temps=obj", "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd))
        procs.append(subprocess.Popen(cmd, cwd=odir))
        built.append(src)

    def finish():
        # the hazard gate over the device assembly of every TU compiled now
        scan = _scanner()
        hits = []
        for src in built:
            stem = os.path.splitext(os.path.basename(src))[0]
            s_files = glob.glob(os.path.join(odir, f"{stem}-hip-amdgcn-amd-amdhsa-*.s"))
            if not s_files:
                raise HazardError(f"no device assembly for {src} in {odir} (-save-temps=obj)")
            for sf in s_files:
                hits += [(sf, ln, kind, detail) for ln, kind, detail in scan.scan(sf)]
        report = os.path.join(odir, "hazard_scan.txt")
        with open(report, "a") as fh:
            for src in built:
                fh.write(f"scanned {os.path.basename(src)} ({' '.join(defines) or 'base'})\n")
            for h in hits:
                fh.write("%s:%d: %s: %s\n" % h)
        for pattern in ("*.hipi", "*.bc", "*.s", "*.out", "*.resolution.txt", "*.hipfb", "*-hip-amdgcn-*.o"):
            for f in glob.glob(os.path.join(odir, pattern)):
                os.remove(f)
        if hits:
            raise HazardError(f"{len(hits)} MFMA hazard(s) at inline-asm boundaries (see {report}):\n" +
                              "\n".join("%s:%d: %s: %s" % h for h in hits[:10]))
        if verbose:
            print(f"asm hazard scan: {len(built)} translation unit(s) of {os.path.basename(out)} clean")
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
