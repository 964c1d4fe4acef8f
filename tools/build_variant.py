"""Build an A/B variant of libenflow_hip.so: enflow_flow.hip recompiled with
extra -D defines / hipcc flags, linked with the product build's other objects.

    python tools/build_variant.py NAME [--tu backward] [-DFOO=1 | -fflag ...]   ->  ab_libs/libenflow_NAME.so

--tu NAME recompiles enflow_NAME.hip instead (backward: the training kernels, latency: the
8-wave flow instances).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "enflow_amd", "libenflow_hip.so")


def main():
    name, flags = sys.argv[1], sys.argv[2:]
    tu = "enflow_flow.hip"
    if flags[:1] == ["--tu"]:
        tu, flags = f"enflow_{flags[1]}.hip", flags[2:]
    out_dir = os.path.join(ROOT, "ab_libs")   # shipped to the GPU box (enflow_amd/var is gpurun-ignored)
    os.makedirs(out_dir, exist_ok=True)
    obj = os.path.join(out_dir, f"{tu.split('.')[0]}_{name}.o")
    base = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I", os.path.join(ROOT, "include")]
    subprocess.run(base + flags + ["-c", os.path.join(ROOT, "enflow_amd", "csrc", tu), "-o", obj], check=True)
    sys.path.insert(0, ROOT)
    from enflow_amd.build import obj_dir
    odir = obj_dir(LIB)   # the product build's objects (enflow_amd/build/libenflow_hip_so)
    others = [os.path.join(odir, s + ".o") for s in ("enflow_flow.hip", "enflow_backward.hip", "enflow_large.hip",
                                                     "enflow_timing.hip", "enflow_latency.hip") if s != tu]
    so = os.path.join(out_dir, f"libenflow_{name}.so")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so, obj] + others, check=True)
    print(so)


if __name__ == "__main__":
    main()
