#!/usr/bin/env python3
"""Per-loop instruction budget of one kernel in a gfx950 assembly listing
(hipcc --cuda-device-only -S): every backward branch's body (label ..
branch), its instructions counted by class -- VALU (with the half-rate
shifts / alignbit / add3 / perm, tools/valu_rate.hip), LDS reads by width,
VMEM loads / stores, SALU, waits.

  python3 tools/isa_loops.py <file.s> <kernel-symbol-substring>
"""
import collections
import re
import sys

HALF = ("v_alignbit", "v_lshlrev", "v_lshrrev", "v_add3", "v_perm",
        "v_lshl_or", "v_lshl_add", "v_bfe", "v_alignbyte")


def kernel_lines(path, sym):
    out, on = [], False
    for ln in open(path):
        if re.match(r"^_Z\S*:", ln):
            on = sym in ln.split(":")[0]
            continue
        if on and ln.startswith(".Lfunc_end"):
            break
        if on:
            out.append(ln.rstrip("\n"))
    return out


def classify(op):
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "lds_rd:" + op
    if op.startswith("ds_"):
        return "lds_other:" + op
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_ld:" + op
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_st:" + op
    if op.startswith("v_"):
        return "valu_half" if op.startswith(HALF) else "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other:" + op


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sym)
    labels = {}
    ins = []   # (index, label-or-None, opcode, text)
    for ln in lines:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if not s or s.startswith((";", ".")):
            continue
        ins.append(s.split()[0])
    # backward branches: a branch at k whose target label is at t <= k
    k = 0
    raw = [l.strip() for l in lines]
    pos = 0
    loops = []
    for ln in raw:
        if not ln or ln.startswith((";", ".")) or ln.endswith(":"):
            continue
        parts = ln.split()
        if parts[0].startswith("s_cbranch") or parts[0] == "s_branch":
            tgt = parts[1].rstrip(",") if len(parts) > 1 else ""
            if tgt in labels and labels[tgt] <= pos:
                loops.append((labels[tgt], pos, tgt))
        pos += 1
    print("kernel %s: %d instructions, %d loops" % (sym, len(ins), len(loops)))
    for a, b, tgt in loops:
        c = collections.Counter(classify(op) for op in ins[a:b + 1])
        tot = sum(c.values())
        valu = c["valu"] + c["valu_half"]
        lds = sum(v for k_, v in c.items() if k_.startswith("lds_rd"))
        print("\nloop %s: [%d, %d] %d instructions: VALU %d (half-rate %d), "
              "LDS reads %d, SALU %d, waits %d" %
              (tgt, a, b, tot, valu, c["valu_half"], lds, c["salu"], c["wait"]))
        for k_, v in sorted(c.items(), key=lambda kv: -kv[1]):
            if ":" in k_:
                print("   %-40s %d" % (k_, v))


if __name__ == "__main__":
    main()
