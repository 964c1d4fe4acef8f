"""Build libenflow_hip.so in-tree with hipcc for gfx950 (no JIT cache)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SRCS = [os.path.join(CSRC, f) for f in ("enflow_flow.hip", "enflow_backward.hip")
        if os.path.exists(os.path.join(CSRC, f))]
OUT = os.path.join(HERE, "libenflow_hip.so")
ARCH = os.environ.get("ENFLOW_OFFLOAD_ARCH", "gfx950")


def build(force=False, verbose=False):
    deps = SRCS + [os.path.join(CSRC, "flow_device.h"), os.path.join(ROOT, "include", "enflow_hip.h")]
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-o", OUT + ".tmp"] + SRCS
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
