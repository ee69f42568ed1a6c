#!/usr/bin/env python
"""Flag reads of AGPRs written by an (inline-asm) MFMA too soon after it, in a hipcc .s file.

hipcc does not model the latency of MFMAs issued from inline asm, so a compiler-placed
v_accvgpr_read / v_accvgpr_mov / scratch_store of the accumulator can read a stale value.
Counts wait states as issued instructions (s_nop N = N+1) between the MFMA and the reader along
the straight-line text (branches are ignored: conservative for fall-through code).

    python scripts/mfma_hazards.py file.s [kernel-filter] [--need 12]
"""
import re
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
need = 12
for a in sys.argv[1:]:
    if a.startswith("--need="):
        need = int(a.split("=")[1])
s = open(args[0]).read()
filt = args[1] if len(args) > 1 else ""


def regs(tok):
    m = re.match(r"a\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"a(\d+)$", tok)
    return {int(m.group(1))} if m else set()


for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
    name = m.group(1)
    if filt not in name:
        continue
    body = s[m.end():s.find(".Lfunc_end", m.end())].split("\n")
    last = {}  # agpr -> (line, ws counter at write)
    ws = 0
    bad = []
    for k, line in enumerate(body):
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.startswith("#"):
            continue
        op = t.split()[0]
        ops = [o.strip() for o in t[len(op):].split(",")]
        if op.startswith("s_nop"):
            ws += int(ops[0]) + 1
            continue
        if op.startswith("v_mfma"):
            for r in regs(ops[0]):
                last[r] = (k, ws + 1)
            ws += 4  # issue cycles of the MFMA itself (conservative low)
            continue
        reads = set()
        if op in ("v_accvgpr_read_b32", "v_accvgpr_mov_b32"):
            reads = regs(ops[1])
        elif op.startswith("scratch_store") or op.startswith("global_store") or op.startswith("buffer_store"):
            for o in ops[1:]:
                reads |= regs(o)
        for r in reads:
            if r in last and ws - last[r][1] < need:
                bad.append((k, r, ws - last[r][1], t))
        ws += 1
    print(f"{name[:80]}: {len(bad)} early AGPR reads")
    for b in bad[:6]:
        print("   line", b[0], "a%d" % b[1], "ws=%d" % b[2], b[3][:80])


# ---- --lds: registers written by inline-asm LDS reads (ds_read_b64_tr_b16, invisible to hipcc's
# wait-count pass) must not be read before an s_waitcnt lgkmcnt(0) retires them (gemm.hip lds_ready).
def vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


if "--lds" in sys.argv:
    for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
        name = m.group(1)
        if filt not in name:
            continue
        body = s[m.end():s.find(".Lfunc_end", m.end())].split("\n")
        pending = set()
        bad = []
        for k, line in enumerate(body):
            t = line.split(";")[0].strip()
            if not t or t.startswith(".") or t.startswith("#"):
                continue
            op = t.split()[0]
            ops = [o.strip() for o in t[len(op):].split(",")]
            if op == "s_waitcnt" and "lgkmcnt(0)" in t:
                pending.clear()
                continue
            if op == "ds_read_b64_tr_b16":
                srcs = vregs(ops[1].split()[0])
                if srcs & pending:
                    bad.append((k, t))
                pending |= vregs(ops[0])
                continue
            # every operand of any other instruction counts as a read (conservative; a plain
            # overwrite of a pending register is a WAW hazard too)
            used = set()
            for o in ops:
                used |= vregs(o.split()[0]) if o else set()
            if used & pending:
                bad.append((k, t))
        print(f"{name[:80]}: {len(bad)} early reads of asm LDS results")
        for b in bad[:6]:
            print("   line", b[0], b[1][:90])


# ---- --operands: VGPR / AGPR operands of inline-asm MFMAs (;;#ASMSTART blocks) written by a VALU
# instruction (v_mov, v_accvgpr_*, v_cndmask, ...) fewer than 2 wait states before the MFMA reads
# them, and their results read by a non-MFMA instruction fewer than 12 wait states after (hipcc
# pads only its own MFMAs; the asm statements open with s_nop where they expect it).
def anyregs(tok):
    m = re.match(r"([va])\[(\d+):(\d+)\]", tok)
    if m:
        return {(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    m = re.match(r"([va])(\d+)$", tok)
    return {(m.group(1), int(m.group(2)))} if m else set()


if "--operands" in sys.argv:
    for m in re.finditer(r"^(_Z\S+):\s*;", s, re.M):
        name = m.group(1)
        if filt not in name:
            continue
        body = s[m.end():s.find(".Lfunc_end", m.end())].split("\n")
        hist = []  # (wait-state counter, written registers) of recent VALU instructions
        dwrite = {}  # register -> (wait-state counter, text) of the asm MFMA that last wrote it
        ws, in_asm, bad = 0, False, []
        for k, line in enumerate(body):
            if ";;#ASMSTART" in line:
                in_asm = True
            if ";;#ASMEND" in line:
                in_asm = False
            t = line.split(";")[0].strip()
            if not t or t.startswith(".") or t.startswith("#"):
                continue
            op = t.split()[0]
            ops = [o.strip() for o in t[len(op):].split(",")]
            if op.startswith("s_nop"):
                ws += int(ops[0]) + 1
                continue
            if op.startswith("v_mfma") and in_asm:
                srcs = set()
                for o in ops[1:4]:
                    srcs |= anyregs(o.split()[0]) if o else set()
                for w_ws, regs_w, txt in hist:
                    if ws - w_ws < 2 and regs_w & srcs:
                        bad.append((k, ws - w_ws, txt, t))
                for r in anyregs(ops[0].split()[0]):
                    dwrite[r] = (ws, t)
            elif not op.startswith("v_mfma"):
                # a VGPR result of an asm MFMA read by anything but an MFMA within 12 wait states
                # (8-pass XDL write -> VALU / memory read; hipcc does not see the asm's latency)
                reads = set()
                for o in ops[1:]:
                    reads |= anyregs(o.split()[0]) if o else set()
                for r in reads & set(dwrite):
                    if ws - dwrite[r][0] < 12:
                        bad.append((k, ws - dwrite[r][0], dwrite[r][1], t))
                        break
            if op.startswith("v_") and not op.startswith("v_mfma"):
                hist.append((ws, anyregs(ops[0].split()[0]) if ops and ops[0] else set(), t))
                hist = hist[-8:]
            ws += 1
        print(f"{name[:80]}: {len(bad)} asm-MFMA operands written < 2 wait states before "
              "or results read < 12 after")
        for b in bad[:8]:
            print("   line", b[0], "ws=%d" % b[1], b[2][:60], "->", b[3][:70])
