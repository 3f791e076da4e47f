"""Where a decode kernel's SGPR spill code sits: reads a device assembly file
(hipcc --cuda-device-only -S) and, for the named kernel, lists per loop depth
the spill stores / reloads (v_writelane / v_readlane with an immediate lane
into the spill VGPRs) and the inline-asm blocks, plus the code-object
metadata (vgpr_count, sgpr_spill_count).

usage: python tools/spill_map.py file.s [kernel-substring] [--blocks]
"""
import collections
import re
import sys


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "ctcx_beam_decode"
    show_blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    # the kernel body: from its label to the next top-level symbol
    start = end = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*%s\S*:" % re.escape(want), l):
            start = i
        elif start is not None and re.match(r"^(_Z|\.Lfunc_end)\S*", l):
            end = i
            break
    if start is None:
        sys.exit("kernel not found")
    spill = re.compile(r"^\s*v_(read|write)lane_b32\s+(\S+),\s*(\S+),\s*(\d+)\s*$")
    depth = 0
    header = None
    per_depth = collections.Counter()
    per_block = collections.Counter()
    asm_at = collections.Counter()
    block = None
    inasm = False
    spill_regs = collections.Counter()
    for l in lines[start:end]:
        m = re.match(r"^(\.LBB\S+):\s*(;.*)?$", l)
        if m:
            block = m.group(1)
            c = m.group(2) or ""
            d = re.search(r"Depth=(\d+)", c)
            depth = int(d.group(1)) if d else 0
            continue
        s = l.strip()
        if s.startswith(";;#ASMSTART"):
            inasm = True
            asm_at[depth] += 1
            continue
        if s.startswith(";;#ASMEND"):
            inasm = False
            continue
        if inasm:
            continue
        m = spill.match(l)
        if m:
            kind, a, b, lane = m.groups()
            reg = a if kind == "write" else b
            spill_regs[reg] += 1
            per_depth[(depth, kind)] += 1
            per_block[(block, depth)] += 1
    print("spill VGPRs:", dict(spill_regs))
    for d in sorted({k[0] for k in per_depth} | set(asm_at)):
        print("depth %d: writelane %4d readlane %4d   asm blocks %d" % (
            d, per_depth[(d, "write")], per_depth[(d, "read")], asm_at[d]))
    if show_blocks:
        for (b, d), n in sorted(per_block.items(), key=lambda kv: (-kv[0][1], -kv[1])):
            if d >= 2:
                print("  %-16s depth %d: %d" % (b, d, n))
    meta = "\n".join(lines[end:])
    for key in ("sgpr_spill_count", "vgpr_spill_count", "vgpr_count", "agpr_count", "sgpr_count",
                "private_segment_fixed_size"):
        m = re.search(r"\.%s:\s*(\d+)" % key, meta)
        if m:
            print("%s: %s" % (key, m.group(1)))


if __name__ == "__main__":
    main()
