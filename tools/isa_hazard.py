"""ISA check of the asm-MFMA GEMM kernels: no read of an MFMA's accumulator registers within
the XDL result latency after it.

The GEMM main loops issue their MFMAs through inline asm with AGPR accumulators (gemm.hip
mfma_agpr / mfma_f8).  The compiler's hazard recognizer does not see inside asm, so it never
inserts the wait states a VALU / memory read of an MFMA result needs; a register-allocator
copy of an accumulator placed right after the last MFMA of a tile (at the k-loop exit) read
the pre-MFMA value once.  The kernels now put the wait states inside the same asm
statement as each tile's last MFMA (mfma_agpr_last / mfma_f8_last).  This tool scans the
disassembly of every k_gemm8 / k_gemm9 / k_gemm8f8 instantiation: for each v_mfma it walks
the following instructions in layout order, counting wait states (s_nop N = N + 1, anything
else = 1), and reports any non-MFMA instruction that reads an AGPR of the MFMA's destination
before REQ wait states have passed.  (MFMAs that chain on the same accumulator as srcC are
interlocked by the hardware and are not reported.)

    python tools/isa_hazard.py [libkdstep.so | object.o]        # exit 1 on a violation
"""
from __future__ import annotations

import re
import shutil
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = Path("/opt/rocm/lib/llvm/bin")
KERNELS = re.compile(r"k_gemm8f8|k_gemm8I|k_gemm8nI|k_gemm9I|k_gemm11I|k_gemm12I")
REQ = 19   # wait states before a non-XDL read of a 16-pass XDL result (the 8-pass ones need fewer)

_AREG = re.compile(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b")


def _aregs(text: str) -> set[int]:
    out = set()
    for m in _AREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(binary: Path) -> str:
    """Device disassembly of the gfx950 code objects bundled in a .so / .o."""
    with tempfile.TemporaryDirectory() as td:
        local = Path(td) / binary.name
        shutil.copy(binary, local)
        subprocess.run([str(LLVM / "llvm-objdump"), "--offloading", str(local)], cwd=td, check=True,
                       capture_output=True)
        out = []
        for co in sorted(Path(td).glob(f"{binary.name}.*gfx950*")):
            r = subprocess.run([str(LLVM / "llvm-objdump"), "-d", "--no-show-raw-insn", str(co)], check=True,
                               capture_output=True, text=True)
            out.append(r.stdout)
        return "\n".join(out)


def functions(dis: str):
    """(name, [(address, instruction text, branch target address or None)]) per function
    symbol of a disassembly (llvm-objdump prints each instruction's address and a branch's
    target as <symbol+offset> in the trailing comment)."""
    name, base, ins = None, 0, []
    for line in dis.split("\n"):
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
        if m:
            if name:
                yield name, ins
            name, base, ins = m.group(2), int(m.group(1), 16), []
            continue
        t = line.strip()
        if not name or not t or t.startswith(";"):
            continue
        text, _, comment = t.partition("//")
        ma = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        mt = re.search(r"<\S+\+0x([0-9a-f]+)>", comment)
        ins.append((int(ma.group(1), 16) if ma else -1, text.strip(), base + int(mt.group(1), 16) if mt else None))
    if name:
        yield name, ins


def check(dis: str, kernels=KERNELS):
    """[(kernel, mfma index, offending instruction, wait states seen)] and the count of
    kernels / MFMAs scanned."""
    bad, nk, nm = [], 0, 0
    for name, ins in functions(dis):
        if not kernels.search(name):
            continue
        nk += 1
        at = {a: k for k, (a, _, _) in enumerate(ins)}
        for i, (_, x, _) in enumerate(ins):
            if not x.startswith("v_mfma"):
                continue
            nm += 1
            ops = x.split(None, 1)[1] if " " in x else ""
            dst = _aregs(ops.split(",")[0])
            if not dst:
                continue
            # walk the fall-through path (and the target of an unconditional branch)
            ws, j, steps = 0, i + 1, 0
            while j < len(ins) and ws < REQ and dst and steps < 4096:
                steps += 1
                _, y, tgt = ins[j]
                op = y.split(None, 1)[0]
                if op == "s_endpgm":
                    break
                if op == "s_branch":
                    ws += 1
                    j = at.get(tgt, len(ins))
                    continue
                if op == "s_nop":
                    ws += int(y.split()[1], 0) + 1
                    j += 1
                    continue
                if op.startswith("v_mfma"):
                    ws += 1
                    j += 1
                    continue
                # a non-MFMA instruction: does it READ one of the accumulators? (the first
                # operand of a VALU / v_accvgpr_* / load is its destination)
                rest = y.split(None, 1)[1] if " " in y else ""
                dest = ""
                if op.startswith(("v_", "buffer_load", "global_load", "ds_read", "scratch_load")):
                    dest, _, rest = rest.partition(",")
                if _aregs(rest) & dst:
                    bad.append((name, i, y, ws))
                    break
                dst -= _aregs(dest)   # overwritten before being read: no longer a hazard
                ws += 1
                j += 1
    return bad, nk, nm


def main(argv):
    path = Path(argv[1]) if len(argv) > 1 else (Path(__file__).resolve().parent.parent /
                                                "knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd"
                                                / "libkdstep.so")
    bad, nk, nm = check(disassemble(path))
    for name, i, y, ws in bad[:50]:
        print(f"HAZARD {name[:90]} mfma #{i}: '{y}' after {ws} wait states (< {REQ})")
    print(f"{nk} kernels, {nm} MFMAs scanned, {len(bad)} hazards")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
