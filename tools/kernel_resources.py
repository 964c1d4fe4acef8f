"""Per-kernel register / scratch / LDS usage of a built library or object.

Extracts the gfx950 code object(s) from the clang offload bundle(s) inside the
file (the .hip_fatbin section), reads their AMDGPU metadata notes with
llvm-readelf and prints one line per kernel matching a name filter:

    python tools/kernel_resources.py enflow_amd/libenflow_hip.so lf_flow_kernel
"""
import os
import re
import subprocess
import sys
import tempfile

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def code_objects(path):
    data = open(path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        base = pos
        p = pos + len(MAGIC)
        n = int.from_bytes(data[p:p + 8], "little")
        p += 8
        for _ in range(n):
            off = int.from_bytes(data[p:p + 8], "little")
            size = int.from_bytes(data[p + 8:p + 16], "little")
            tl = int.from_bytes(data[p + 16:p + 24], "little")
            triple = data[p + 24:p + 24 + tl].decode(errors="replace")
            p += 24 + tl
            if "gfx" in triple and size:
                out.append((triple, data[base + off:base + off + size]))
        pos = data.find(MAGIC, p)
    return out


def kernels(path):
    res = []
    for triple, blob in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(blob)
            f.flush()
            txt = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
        cur = {}
        for line in txt.splitlines():
            m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if k == "agpr_count" and cur:
                pass
            cur[k] = v
            if k == "wavefront_size" and ".name" in line or k == "vgpr_spill_count":
                pass
            if k == "wavefront_size":
                res.append(dict(cur))
                cur = {}
    return res


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
    rows = []
    for k in kernels(path):
        name = k.get("name", "?")
        if not pat.search(name):
            continue
        rows.append((name, k.get("vgpr_count"), k.get("agpr_count"), k.get("sgpr_count"),
                     k.get("vgpr_spill_count"), k.get("sgpr_spill_count"), k.get("private_segment_fixed_size"),
                     k.get("group_segment_fixed_size")))
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'lds':>7}  kernel")
    for r in sorted(rows):
        print(f"{r[1]!s:>5} {r[2]!s:>5} {r[3]!s:>5} {r[4]!s:>6} {r[5]!s:>6} {r[6]!s:>7} {r[7]!s:>7}  {r[0]}")


if __name__ == "__main__":
    main()
