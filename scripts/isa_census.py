#!/usr/bin/env python
"""Instruction census of a kernel's hottest loop, by purpose, from a hipcc --save-temps .s file.

    python scripts/isa_census.py attention_train-hip-amdgcn-amd-amdhsa-gfx950.s attn_bwd_kernelILi4ELi8ELb0E

The loop is the outermost one hipcc marks ``Loop Header: Depth=1`` (the body up to its back edge;
``--depth=2`` for loops nested once, ``--loop=N`` for the N-th of them);
within it, code behind the wave-uniform branches that only diagonal / tail tiles take is counted
separately: ``--cold=<regex>,...`` marks every block holding a matching instruction,
``--cold-blocks=<name>,...`` names blocks as ``--blocks`` lists them (label, ``#k`` = the k-th
fall-through after a branch).  Purposes
are by mnemonic (a census, not a dataflow analysis):

  mfma          v_mfma_*
  exp           v_exp_f32 (softmax recompute)
  softmax-math  float mul / fma / add / sub / max (max3), packed f32, v_bfe_i32 / v_and (dropout keep select)
  bf16-pack     v_cvt_pk_bf16_f32, v_perm_b32
  address       integer add / shift / xor / or / bitop3 / mad on addresses and indices
  compare-sel   v_cmp*, v_cndmask* (causal mask, bounds)
  move          v_mov*, v_readfirstlane, v_accvgpr*
  lds-read / lds-tr-read / lds-write, vmem-load / vmem-store, salu, s_nop, s_waitcnt, branch
"""
import collections
import re
import sys

CATS = [
    ("mfma", r"^v_mfma"),
    ("exp", r"^v_exp_f32"),
    ("bf16-pack", r"^v_cvt_pk_bf16|^v_perm_b32"),
    ("softmax-math", r"^v_(pk_)?(mul|fma|add|sub|max|min)_f32|^v_(max3|min3|med3)_f32|^v_bfe_i32|^v_and_b32"),
    ("compare-sel", r"^v_cmp|^v_cndmask"),
    ("move", r"^v_mov|^v_readfirstlane|^v_accvgpr|^v_readlane|^v_writelane"),
    ("address", r"^v_(add|sub|lshl|lshr|ashr|xor|or|and|bitop3|mad|mul_lo|mul_u32|bfe_u32|bfi|add3|lshl_add|lshl_or|add_lshl|and_or|or3|min|max)"),
    ("lds-tr-read", r"^ds_read_b64_tr"),
    ("lds-read", r"^ds_read"),
    ("lds-write", r"^ds_write"),
    ("vmem-load", r"^(buffer|global)_load|^scratch_load"),
    ("vmem-store", r"^(buffer|global)_store|^(buffer|global)_atomic|^scratch_store"),
    ("s_nop", r"^s_nop"),
    ("s_waitcnt", r"^s_waitcnt"),
    ("barrier", r"^s_barrier"),
    ("branch", r"^s_cbranch|^s_branch"),
    ("salu", r"^s_"),
    ("other-valu", r"^v_"),
]


def classify(m):
    for c, pat in CATS:
        if re.match(pat, m):
            return c
    return "other"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    opts = dict(a[2:].split("=", 1) for a in sys.argv[1:] if a.startswith("--") and "=" in a)
    src, name = args[0], args[1]
    s = open(src).read()
    m = re.search(r"^(_Z\S*" + re.escape(name) + r"\S*):", s, re.M)
    body = s[m.end():s.find(".Lfunc_end", m.end())].split("\n")
    # outermost loop: hipcc rotates it, so take the span from the earliest label any later branch
    # jumps back to (at or before the Depth=1 header) to the last such back edge
    depth = int(opts.get("depth", "1"))  # --depth=2: loops nested once (a persistent kernel's tile loops)
    hdrs = [i for i, l in enumerate(body) if re.search(r"Loop Header: Depth=%d\b" % depth, l)]
    hdr = hdrs[int(opts.get("loop", "0"))]  # --loop=N: the N-th loop of that depth
    lab = {l.split(":")[0].strip(): i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l.strip())}
    start, end = hdr, hdr
    nxt = min([h for h in hdrs if h > hdr] + [len(body)])
    # back edges of an enclosing (or earlier) loop jump to or before the nearest loop header ahead of it
    allh = [i for i, l in enumerate(body) if "Loop Header" in l]
    prev = max([h for h in allh if h < hdr] + [-1])
    for i, l in enumerate(body[:nxt]):
        mm = re.search(r"s_c?branch\w*\s+(\.LBB\w+)", l)
        if mm and i > hdr and prev < lab.get(mm.group(1), 1 << 30) <= hdr:
            start, end = min(start, lab[mm.group(1)]), max(end, i)
    label = body[hdr].split(":")[0].strip()
    # basic blocks: split at labels and after branches
    blocks, cur, k = {}, "entry", 0
    for l in body[start:end + 1]:
        t = l.strip()
        mm = re.match(r"^(\.LBB\w+):(.*)", t)
        if mm:
            cur = mm.group(1) + mm.group(2)
            continue
        if not t or t.startswith(";") or t.startswith("."):
            continue
        blocks.setdefault(cur, []).append(t.split(None, 1))
        if re.match(r"s_c?branch", t):
            k += 1
            cur = f"{cur.split()[0].split('#')[0]}#{k}"
    # cold: blocks holding an instruction that matches one of the --cold regexes (the causal-mask
    # compares of diagonal tiles, the zero stores of fully masked subtiles, ...)
    cold = [c for c in opts.get("cold", "").split(",") if c]
    cold_blocks = set(c for c in opts.get("cold-blocks", "").split(",") if c)
    tot, coldc = collections.Counter(), collections.Counter()
    for b, ins in blocks.items():
        text = [" ".join(x) for x in ins]
        is_cold = any(re.search(c, t) for c in cold for t in text) or b.split()[0] in cold_blocks
        tgt = coldc if is_cold else tot
        for x in ins:
            tgt[classify(x[0])] += 1
        if "--blocks" in sys.argv:
            c = collections.Counter(classify(x[0]) for x in ins)
            print(f"  {'cold' if is_cold else 'hot '} {b[:40]:40s} n={len(ins):4d} mfma={c['mfma']:3d} "
                  f"valu={sum(v for q, v in c.items() if q not in ('mfma', 'lds-read', 'lds-tr-read', 'lds-write', 'vmem-load', 'vmem-store', 's_nop', 's_waitcnt', 'barrier', 'branch', 'salu', 'other')):4d}")
    print(f"kernel {m.group(1)}\nloop {label}: lines {start}..{end}, {len(blocks)} basic blocks")
    for title, c in (("hot path", tot), ("cold blocks", coldc)):
        if not c:
            continue
        n_mfma = c["mfma"] or 1
        valu = sum(v for k, v in c.items() if k in ("exp", "bf16-pack", "softmax-math", "compare-sel", "move",
                                                     "address", "other-valu"))
        print(f"-- {title}: {sum(c.values())} instructions, {c['mfma']} MFMA, {valu} VALU "
              f"({valu / n_mfma:.2f} per MFMA)")
        for k, _ in CATS:
            if c[k]:
                print(f"   {k:14s} {c[k]:5d}" + (f"   {c[k] / n_mfma:5.2f}/MFMA" if k in (
                    "exp", "bf16-pack", "softmax-math", "compare-sel", "move", "address", "other-valu") else ""))


if __name__ == "__main__":
    main()
