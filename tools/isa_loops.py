"""Static instruction account of a kernel's loops in a gfx950 .s file
(hipcc --offload-device-only -S): per loop (the compiler's "Loop Header"
comments), its VALU / SALU / LDS / VMEM / SMEM instruction counts, the
v_readlane / v_writelane of spilled SGPRs, and the kernel's register and
spill metadata.

usage: python tools/isa_loops.py file.s KERNEL_SUBSTRING [--ops]
(--ops: the VALU opcode histogram of the largest loop)"""
import collections
import re
import sys


def kernel_text(lines, sub):
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sub in l)
    end = next(i for i in range(start, len(lines)) if ".amdhsa_kernel" in lines[i] or lines[i].startswith(".Lfunc_end"))
    return start, lines[start:end]


def meta(text_all, name):
    out = {}
    m = re.search(r"\.name:\s+" + re.escape(name) + r"\n(.*?)\.vgpr_spill_count:\s+(\d+)", text_all, re.S)
    block = text_all[text_all.find(".name:           " + name):]
    for key in ("sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count", "private_segment_fixed_size"):
        mm = re.search(r"\." + key + r":\s+(\d+)", block[:4000])
        if mm:
            out[key] = int(mm.group(1))
    return out


def classify(l):
    t = l.strip().split()
    if not t:
        return None
    op = t[0]
    if op.startswith("v_readlane") or op.startswith("v_writelane"):
        return "spill_lane"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return None


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start, body = kernel_text(lines, sub)
    name = body[0].rstrip(":").strip()
    heads = [i for i, l in enumerate(body) if "Loop Header" in l]
    print(name, meta("\n".join(lines), name))
    loops = []
    for j, h in enumerate(heads):
        e = heads[j + 1] if j + 1 < len(heads) else len(body)
        c = collections.Counter(classify(l) for l in body[h:e])
        depth = re.search(r"Depth=(\d+)", body[h])
        loops.append((h, e, c))
        print(f"  loop @{start + h:7d} len {e - h:5d} depth {depth.group(1) if depth else '?'}: "
              f"valu {c['valu']:4d} (+{c['spill_lane']} spill lanes) salu {c['salu']:4d} lds {c['lds']:3d} "
              f"vmem {c['vmem']:3d} smem {c['smem']:3d} scratch {c['scratch']}")
    if "--ops" in sys.argv and loops:
        h, e, _ = max(loops, key=lambda x: x[2]["valu"])
        ops = collections.Counter(l.strip().split()[0] for l in body[h:e] if l.strip().startswith("v_"))
        for op, k in ops.most_common(40):
            print(f"    {k:5d} {op}")


if __name__ == "__main__":
    main()
