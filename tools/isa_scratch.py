"""Where the LP kernel spills: compile lp_hyper.hip to gfx950 assembly, take one instantiation
(default storm: R = 9 row slots, C = 28 column slots) and count the scratch loads / stores of
every loop (a back edge: a branch to an earlier label), plus the kernel's resource usage.
The pivot loop is the largest loop inside the per-scenario loop.
Usage: python tools/isa_scratch.py [R] [C] [full]   (CPU only: hipcc cross-compiles; full = 1: the
instantiation with the recovery / eta-file epilogue)"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 28
    FULL = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    src = os.path.join(ROOT, "sqlp_amd", "csrc", "lp_hyper.hip")
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "lp.s")
        r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                            "-I" + os.path.join(ROOT, "include"), "-Rpass-analysis=kernel-resource-usage", src, "-o", asm],
                           capture_output=True, text=True)
        text = open(asm).read()
    sym = f"_ZN5twosd15lp_hyper_kernelILi{R}ELi{C}ELb{FULL}EEEvNS_11HyperParamsE"
    usage = []
    lines_r = r.stderr.splitlines()
    for i, l in enumerate(lines_r):
        if sym in l:
            usage = [x.split("remark:")[1].split(" [-Rpass")[0].strip() for x in lines_r[i + 1:i + 10] if "remark:" in x and "Function Name" not in x]
            break
    body = text[text.index(sym + ":"):]
    body = body[:body.index(".Lfunc_end")]
    lines = body.splitlines()
    labels = {m.group(1): i for i, l in enumerate(lines) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
    loops = []
    for i, l in enumerate(lines):
        m = re.search(r"\bs_(?:c)?branch\w*\s+(\.LBB\d+_\d+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            loops.append((labels[m.group(1)], i))
    merged = {}
    for a, b in loops:                       # one entry per loop header: its farthest back edge
        merged[a] = max(merged.get(a, a), b)
    loops = sorted(merged.items(), key=lambda t: -(t[1] - t[0]))

    def cnt(a, b, pat):
        return sum(1 for l in lines[a:b + 1] if pat in l)

    def ninstr(a, b):
        return sum(1 for l in lines[a:b + 1] if l.startswith("\t") and not l.startswith(("\t.", "\t;")))

    print(f"lp_hyper_kernel<{R}, {C}, {'true' if FULL else 'false'}>: " + "; ".join(usage))
    print(f"whole kernel: {ninstr(0, len(lines))} instructions, scratch stores {cnt(0, len(lines), 'scratch_store')}, "
          f"loads {cnt(0, len(lines), 'scratch_load')}")
    scen = loops[0]
    piv = next(((a, b) for a, b in loops[1:] if scen[0] <= a and b <= scen[1]), None)
    print(f"scenario loop (lines {scen[0]}-{scen[1]}): {ninstr(*scen)} instructions, scratch stores {cnt(*scen, 'scratch_store')}, "
          f"loads {cnt(*scen, 'scratch_load')}")
    if piv:
        print(f"pivot loop    (lines {piv[0]}-{piv[1]}): {ninstr(*piv)} instructions, scratch stores {cnt(*piv, 'scratch_store')}, "
              f"loads {cnt(*piv, 'scratch_load')}")
        pre = (scen[0], piv[0] - 1)
        post = (piv[1] + 1, scen[1])
        print(f"  per scenario before the pivot loop: scratch stores {cnt(*pre, 'scratch_store')}, loads {cnt(*pre, 'scratch_load')}")
        print(f"  per scenario after the pivot loop:  scratch stores {cnt(*post, 'scratch_store')}, loads {cnt(*post, 'scratch_load')}")
    outside = (cnt(0, scen[0] - 1, "scratch_store"), cnt(0, scen[0] - 1, "scratch_load"))
    print(f"kernel prologue (once per wave): scratch stores {outside[0]}, loads {outside[1]}")


if __name__ == "__main__":
    main()
