"""Instruction counts of a kernel's hot loop from hipcc assembly (-S).

    hipcc -O3 --offload-arch=gfx950 --offload-device-only -S -o k.s kernels_fx.hip
    python tools/isa_count.py k.s <symbol substring> [--block-exclude LABEL ...]

Finds the kernel, its basic blocks, and the outermost backward branch whose body
holds MFMAs (the tile loop); prints per-block and whole-loop counts by class
(VALU, MFMA, LDS read / write, LDS-DMA, VMEM, SALU, SMEM, waits, barriers) and
the kernel's register / LDS metadata.  Blocks passed with --block-exclude (rare
paths, e.g. a rescale branch) are listed but left out of the loop total.
"""
import argparse
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "MFMA"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "LDS_RD"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "LDS_WR"
    if op.startswith("ds_"):
        return "LDS_OTHER"
    if op.startswith(("global_load_lds", "buffer_load_lds")) or (op.startswith("buffer_load") and "lds" in op):
        return "LDS_DMA"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "VMEM_RD"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic", "buffer_atomic")):
        return "VMEM_WR"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "VALU_TRANS"
    if op.startswith(("v_permlane", "v_readlane", "v_readfirstlane", "v_writelane")):
        return "VALU_XLANE"
    if op.startswith("v_"):
        return "VALU"
    if op.startswith("s_waitcnt"):
        return "WAIT"
    if op.startswith("s_barrier"):
        return "BARRIER"
    if op.startswith(("s_load", "s_buffer_load")):
        return "SMEM"
    if op.startswith(("s_cbranch", "s_branch")):
        return "BRANCH"
    if op.startswith(("s_nop", "s_setprio", "s_sleep")):
        return "SCHED"
    if op.startswith("s_"):
        return "SALU"
    return "OTHER"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("symbol")
    ap.add_argument("--block-exclude", nargs="*", default=[])
    ap.add_argument("--loop", nargs=2, default=None, help="first and last block of the loop to count")
    a = ap.parse_args()
    lines = open(a.asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^\S*" + re.escape(a.symbol) + r"\S*:", l))
    sym = lines[start].split(":")[0]
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    order = [cur]
    for l in body[1:]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            order.append(cur)
            continue
        t = l.strip()
        if not t or t.startswith((";", ".", "//")):
            continue
        blocks[cur].append(t.split()[0])
    # backward branches: (span, target block index, source block index)
    back = []
    raw_targets = {}
    cur = "entry"
    for l in body[1:]:
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            cur = m.group(1)
            continue
        t = l.strip()
        mm = re.match(r"s_c?branch\S*\s+(\.LBB\d+_\d+)", t)
        if mm:
            raw_targets.setdefault(cur, []).append(mm.group(1))
    for src, tgts in raw_targets.items():
        for t in tgts:
            si, ti = order.index(src), order.index(t)
            if ti <= si:
                n_mfma = sum(1 for bb in order[ti:si + 1] for op in blocks[bb] if classify(op) == "MFMA")
                if n_mfma:
                    back.append((si - ti, ti, si))
    if not back:
        sys.exit("no loop with MFMAs found")
    for span, t, src in sorted(back):
        print(f"  backward edge {order[src]} -> {order[t]} ({span + 1} blocks)")
    if a.loop:
        ti, si = order.index(a.loop[0]), order.index(a.loop[1])
    else:
        _, ti, si = max(back)
    print(f"kernel {sym}")
    print(f"tile loop: blocks {order[ti]} .. {order[si]}")
    tot = Counter()
    for bb in order[ti:si + 1]:
        c = Counter(classify(op) for op in blocks[bb])
        ex = bb in a.block_exclude
        print(f"  {bb:14s} {'(excluded) ' if ex else ''}{len(blocks[bb]):5d} instr  " +
              " ".join(f"{k}={v}" for k, v in sorted(c.items())))
        if not ex:
            tot += c
    print("loop total (one pass of every non-excluded block): " + " ".join(f"{k}={v}" for k, v in sorted(tot.items())))
    print(f"  vector-issue class total: VALU+TRANS+XLANE={tot['VALU'] + tot['VALU_TRANS'] + tot['VALU_XLANE']}")
    text = "\n".join(lines)
    mi = text.find(".name:           " + sym)
    if mi >= 0:
        meta = text[max(0, mi - 1500): mi + 1500]
        for key in (".vgpr_count", ".agpr_count", ".sgpr_count", ".group_segment_fixed_size", ".vgpr_spill_count",
                    ".sgpr_spill_count", ".private_segment_fixed_size"):
            m = re.search(re.escape(key) + r":\s+(\d+)", text[mi:mi + 1500])
            if m:
                print(f"  {key[1:]} = {m.group(1)}")


if __name__ == "__main__":
    main()
