"""Build gate: MFMA hazards at inline-asm boundaries in hipcc device assembly.

hipcc pads the hazards of the instructions it generates, not those inside an
`asm` statement (cdna_hip_programming.md §5.7 item 2).  Two pairs cross that
boundary in this code base (the lock-step SiLU silu4 / silu4s, the operand
split split_lo8, the DPP segment scans, all in flow_device.h):

  (a) an MFMA's destination read by an instruction INSIDE an asm block before
      the MFMA has drained: 12 wait states for an 8-pass XDL op (32x32x16
      f16 / bf16; conservatively also for shorter shapes), 18 for a 16-pass
      one (32x32x2 f32);
  (b) a VGPR written inside an asm block and read as an MFMA A / B operand
      within 2 wait states after it (the block must end with `s_nop 1`).

Wait states between producer and consumer = instructions in between + the
extra states of every `s_nop N` (N + 1 each).  The scan is linear over the
.s text (straight-line code; every kernel resets the window) and flags, it
does not prove: a hit is a build failure to look at.

    python tools/asm_hazard_scan.py FILE.s [...]      (exit status 1 on a hit)

enflow_amd/build.py compiles with -save-temps=obj and runs scan() over the
device assembly of every translation unit of every library it builds
(identical code objects: the temporaries are the same compilation's).
"""
import re
import sys

_REG = re.compile(r"\b([va])\[(\d+):(\d+)\]|\b([va])(\d+)\b")


def _regs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(1):
            out |= {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
        else:
            out.add((m.group(4), int(m.group(5))))
    return out


def _mfma_states(op):
    """Wait states before a VALU may read an MFMA's destination: 18 for the
    16-pass fp32 32x32 shapes (32x32x1 / 32x32x2 f32), 12 otherwise (8-pass
    XDL ops such as 32x32x16 f16 / bf16, and conservatively the shorter ones)."""
    m = re.search(r"_(\d+)x(\d+)x(\d+)", op)
    if m and m.group(1) == "32" and int(m.group(3)) <= 2 and op.endswith("f32"):
        return 18
    return 12


def _split(line):
    s = line.split(";")[0].strip()
    if not s or s.endswith(":") or s.startswith("."):
        return None, None, None
    parts = s.split(None, 1)
    op = parts[0]
    args = parts[1] if len(parts) > 1 else ""
    toks = [t.strip() for t in args.split(",")]
    dst = _regs(toks[0]) if toks and toks[0] else set()
    src = set()
    for t in toks[1:]:
        src |= _regs(t)
    return op, dst, src


def scan(path):
    """[(line, kind, detail)] of every suspected hazard in one .s file."""
    hits = []
    lines = open(path, errors="replace").read().split("\n")
    recent = []          # (index in issue order, op, dst, states_needed) of the last MFMAs
    issue = 0            # wait-state clock: +1 per instruction, + N for s_nop N
    in_asm = False
    asm_writes = {}      # reg -> issue clock of the write (inside the current / last asm block)
    last_asm_end = None
    func = None
    for i, line in enumerate(lines):
        st = line.strip()
        if re.match(r"^[_A-Za-z][\w.$]*:\s*(;.*)?$", st) and not st.startswith(".") and "_Z" in st[:3]:
            func, recent, asm_writes, last_asm_end = st[:-1], [], {}, None
        if st.startswith(";;#ASMSTART"):
            in_asm, asm_writes = True, {}
            continue
        if st.startswith(";;#ASMEND"):
            in_asm, last_asm_end = False, issue
            continue
        op, dst, src = _split(line)
        if op is None:
            continue
        if op == "s_nop":
            issue += int(st.split()[1].rstrip(","), 0) + 1
            continue
        issue += 1
        if in_asm:
            for (k, o, d, need) in recent:
                reads = (src | (dst if op.startswith("v_fmac") or "_dpp" in op else set())) & d
                if reads and issue - k - 1 < need:
                    hits.append((i + 1, "mfma-result read in asm", f"{func}: {st} ({issue - k - 1} of {need} states "
                                 f"after {o})"))
            if op.startswith("v_"):
                for r in dst:
                    asm_writes[r] = issue
        elif op.startswith("v_mfma") and asm_writes:
            for r in src & set(asm_writes):
                if issue - asm_writes[r] - 1 < 2:
                    hits.append((i + 1, "asm write read by mfma", f"{func}: {st} ({issue - asm_writes[r] - 1} states "
                                 f"after the asm write of {r})"))
        if op.startswith("v_mfma"):
            recent.append((issue, op, dst, _mfma_states(op)))
            recent = [x for x in recent if issue - x[0] < 20]
        if not in_asm and last_asm_end is not None and issue - last_asm_end > 4:
            asm_writes = {}
    return hits


def main(paths):
    bad = 0
    for p in paths:
        for ln, kind, detail in scan(p):
            bad += 1
            print(f"{p}:{ln}: {kind}: {detail}")
    print(f"asm hazard scan: {len(paths)} file(s), {bad} hit(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
