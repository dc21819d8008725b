"""Per-kernel main-loop census of a hipcc -S listing: MFMA count, instruction count and
compiler-inserted s_waitcnt vmcnt(0) in every basic block with >= 32 MFMAs.
    python tools/asm_loops.py file.s [name-regex]"""
import re
import sys

L = open(sys.argv[1]).read().split("\n")
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else r"k_gemm[38]")
for i, l in enumerate(L):
    m = re.match(r"^(_Z\w+):", l)
    if not m or not pat.search(m.group(1)):
        continue
    end = i
    while not L[end].startswith(".Lfunc_end"):
        end += 1
    blocks, cur = [], ("entry", [])
    for x in L[i + 1:end]:
        mb = re.match(r"^(\.LBB\w+):", x)
        if mb:
            blocks.append(cur)
            cur = (mb.group(1), [])
            continue
        t = x.strip()
        if t and not t.startswith((";", ".")):
            cur[1].append(t)
    blocks.append(cur)
    for bn, ins in blocks:
        n = sum(1 for x in ins if x.startswith("v_mfma"))
        if n >= int(__import__("os").environ.get("MINMFMA", "32")):
            v0 = sum(1 for x in ins if x.startswith("s_waitcnt") and "vmcnt(0)" in x)
            print(f"{m.group(1)[14:80]:66s} {bn:10s} mfma {n:4d} ins {len(ins):5d} vmcnt0 {v0}")
