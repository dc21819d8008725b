"""The built library's asm-MFMA GEMM kernels (k_gemm8 / k_gemm9 / k_gemm8f8, every
instantiation) never read an MFMA accumulator within the XDL result latency after the MFMA
that writes it (tools/isa_hazard.py: disassembly of the gfx950 code object).
CPU only: reads the .so that build() produced."""
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "tools"))
LIB = REPO / "knowledge_distillation_for_sensory_substitution_in_multimodal_models_amd" / "libkdstep.so"


@pytest.mark.skipif(not LIB.exists() or not (Path("/opt/rocm/lib/llvm/bin/llvm-objdump")).exists(),
                    reason="needs the built library and llvm-objdump")
def test_no_accumulator_read_inside_mfma_latency():
    import isa_hazard as H
    bad, nk, nm = H.check(H.disassemble(LIB))
    assert nk >= 10 and nm > 1000, (nk, nm)   # every GEMM kernel build was scanned
    assert not bad, [f"{n[:60]} #{i}: {y} after {ws}" for n, i, y, ws in bad[:10]]


def test_checker_flags_a_read_inside_the_latency():
    import isa_hazard as H
    dis = "\n".join([
        "0000000000001000 <_ZN2kd12_GLOBAL__N_17k_gemm8ILb0ELb0ELi0EEEvNS0_5GemmPE>:",
        "\tv_mfma_f32_16x16x32_bf16 a[0:3], v[0:3], v[4:7], a[0:3]  // 000000001000: 00",
        "\ts_nop 3  // 000000001008: 00",
        "\tv_accvgpr_read_b32 v9, a2  // 00000000100C: 00",
        "\tv_mfma_f32_16x16x32_bf16 a[4:7], v[0:3], v[4:7], a[4:7]  // 000000001010: 00",
        "\ts_nop 15  // 000000001018: 00",
        "\ts_nop 15  // 00000000101C: 00",
        "\tv_accvgpr_read_b32 v9, a5  // 000000001020: 00",
    ])
    bad, nk, nm = H.check(dis)
    assert nk == 1 and nm == 2 and len(bad) == 1 and "a2" in bad[0][2]
