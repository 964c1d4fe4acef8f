"""Diagnostic: scan hipcc device assembly (.s) for inline-asm statements whose
first instructions read a VGPR an MFMA wrote within the last few instructions
with fewer than 12 s_nop wait states in between (hipcc pads no hazard into an
asm string: cdna_hip_programming.md 5.7 item 2).  Prints hits per kernel.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include --cuda-device-only -S \\
        -o /tmp/flow.s enflow_amd/csrc/enflow_flow.hip
    python tools/asm_hazard_scan.py /tmp/flow.s
"""
import re, sys
lines = open(sys.argv[1]).read().split("\n")
func = None
hits = {}
def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m: return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    if m: return {int(m.group(1))}
    return set()
recent = []   # (index, dest regs, is_mfma)
for i, l in enumerate(lines):
    s = l.strip()
    if re.match(r"^_Z\S+:", l):
        func = s[:-1]; recent = []
    if not s or s.startswith(";") or s.startswith("."):
        if s.startswith(";;#ASMSTART"):
            # look at the next asm instruction(s)
            j = i + 1; cnt = 0
            while j < len(lines) and not lines[j].strip().startswith(";;#ASMEND") and cnt < 4:
                ins = lines[j].strip()
                if ins and not ins.startswith(";"):
                    toks = [t.strip(",") for t in ins.split()]
                    srcs = set()
                    for t in toks[2:]:
                        srcs |= regs(t)
                    # distance in issued instructions since the producing MFMA
                    for k, (idx, dst, ismfma, dist_nops) in enumerate(reversed(recent)):
                        if ismfma and dst & srcs:
                            nops = sum(x[3] for x in recent[len(recent)-k:])
                            if k + cnt < 12 and nops < 12:
                                hits.setdefault(func, []).append((i, k + cnt, nops, ins))
                            break
                    cnt += 1
                j += 1
        continue
    toks = [t.strip(",") for t in s.split()]
    op = toks[0]
    nop = 0
    if op == "s_nop":
        nop = int(toks[1], 0) + 1
    dst = regs(toks[1]) if len(toks) > 1 else set()
    recent.append((i, dst, op.startswith("v_mfma"), nop))
    recent = recent[-40:]
for f, h in hits.items():
    print(len(h), str(f)[:120])
    for x in h[:3]:
        print("   line", x[0], "instr-dist", x[1], "nop-states", x[2], x[3])
