"""Instruction mix per basic block of one kernel in a device assembly listing.

    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S quant_amd/csrc/k_mf32.hip -o /tmp/k_mf32.s
    python tools/isa_blocks.py /tmp/k_mf32.s assign_mf32_kernelILb1ELb1ELi4ELb1ELb0EE

prints each block's VALU / MFMA / LDS / VMEM counts and its five most frequent opcodes, so a
kernel's per-chunk VALU can be split into prologue, tile loop and epilogue parts.
"""
import collections
import re
import sys


def blocks(lines):
    name, ops = "entry", []
    for line in lines:
        m = re.match(r"^(\.LBB\d+_\d+):", line)
        if m:
            yield name, ops
            name, ops = m.group(1), []
            continue
        t = line.strip()
        if t and not t.startswith((";", ".")):
            ops.append(t.split()[0])
    yield name, ops


def kind(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_")):
        return "vmem"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    text = open(path).read().split("\n")
    start = next(i for i, l in enumerate(text) if l.startswith("_ZN") and sym in l.split(":")[0])
    end = next(i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end"))
    for name, ops in blocks(text[start + 1:end]):
        c = collections.Counter(kind(o) for o in ops)
        top = collections.Counter(ops).most_common(5)
        print("%-12s n=%4d valu=%4d mfma=%3d lds=%3d vmem=%3d  %s" %
              (name, len(ops), c["valu"], c["mfma"], c["lds"], c["vmem"], " ".join("%s:%d" % t for t in top)))


if __name__ == "__main__":
    main()
