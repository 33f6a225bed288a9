"""Where the fp32 argmax spills: compile cut_kernel.hip to gfx950 assembly with the given -D flags,
take cut_argmax3_kernel<KB> and count, per loop (a branch back to an earlier label), the MFMAs,
LDS reads, scratch loads / stores, VALU-ish and s_barrier instructions.  CPU only.
Usage: python tools/isa_cut.py [KB] [-DFLAG ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    KB = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else 30
    flags = [a for a in sys.argv[1:] if a.startswith("-")]
    src = os.path.join(ROOT, "sqlp_amd", "csrc", "cut_kernel.hip")
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "c.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                        "-I" + os.path.join(ROOT, "include")] + flags + [src, "-o", asm], check=True, capture_output=True)
        text = open(asm).read()
    sym = f"_ZN5twosd18cut_argmax3_kernelILi{KB}EEEvNS_9CutParamsE"
    body = text[text.index(sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    lines = [l.strip() for l in body.splitlines()]
    labels = {re.match(r"^(\.LBB[^:]+):", l).group(1): i for i, l in enumerate(lines) if re.match(r"^\.LBB[^:]+:", l)}
    loops = []
    for i, l in enumerate(lines):
        m = re.match(r"^s_cbranch_\w+\s+(\.LBB\S+)|^s_branch\s+(\.LBB\S+)", l)
        if m:
            t = m.group(1) or m.group(2)
            if t in labels and labels[t] < i:
                loops.append((labels[t], i))

    def count(a, b):
        seg = lines[a:b + 1]
        c = {"mfma": 0, "ds_read": 0, "scratch_ld": 0, "scratch_st": 0, "v_": 0, "s_": 0, "barrier": 0, "global": 0, "waitcnt": 0}
        for l in seg:
            if l.startswith("v_mfma"): c["mfma"] += 1
            elif l.startswith("ds_read"): c["ds_read"] += 1
            elif l.startswith("scratch_load") or (l.startswith("buffer_load") and "off, s[0:3]" in l): c["scratch_ld"] += 1
            elif l.startswith("scratch_store"): c["scratch_st"] += 1
            elif l.startswith("s_barrier"): c["barrier"] += 1
            elif l.startswith("s_waitcnt"): c["waitcnt"] += 1
            elif l.startswith("global_"): c["global"] += 1
            elif l.startswith("v_"): c["v_"] += 1
            elif l.startswith("s_"): c["s_"] += 1
        return c
    print("flags", flags, "whole kernel", count(0, len(lines) - 1))
    for a, b in [lp for lp in sorted(loops, key=lambda t: t[1] - t[0]) if count(*lp)['mfma'] > 0][:3]:
        print(f"loop lines {a}-{b} ({b - a}):", count(a, b))


if __name__ == "__main__":
    main()
