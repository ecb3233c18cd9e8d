"""CPU: the shipping library's gfx950 code pinned against the config-5 wrong scores of round 4.

The fused config-5 kernel (decoder_bf16_cs16_kernel<768, true>, dg_slot_score_hinge_bf16) once
returned wrong positive scores for a tile's first 16 pairs on ~1 % of half tiles, at random.
Round 5 traced them to one instruction form ("The config-5 miscompile"):
`v_pk_mul_f32 vD, vA, vB op_sel:[0,1]`, a packed multiply whose LOW result reads src1's HIGH
dword, intermittently returned 0 for lanes 48-63 of the wave in that kernel.  Every failing
score equals the reference minus exactly one such product of lane group 3; unpacking those
four instructions, or swapping their operands so the high dword is read through src0, removed
every failure (scripts/hazard_variants.py + scripts/hazard_harness).  These tests disassemble the
shipping library and assert that no kernel contains that form, and that config 5's epilogue is
the validated scalar form, so a compiler or source change that brings it back fails on the CPU,
before any GPU run.
"""
import re
import shutil
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scripts"))

import isa_scan  # noqa: E402

LIB = ROOT / "decagon_amd" / "lib" / "libdecagon_hip.so"
FUSED = "_ZN12_GLOBAL__N_124decoder_bf16_cs16_kernelILi768ELb1EEEvNS_11Bf16DecArgsE"


@pytest.fixture(scope="module")
def kernels():
    if not LIB.exists():
        pytest.skip("libdecagon_hip.so not built")
    if not (isa_scan.LLVM / "llvm-objdump").exists():
        pytest.skip("ROCm llvm-objdump not available")
    import tempfile

    out = {}
    with tempfile.TemporaryDirectory() as td:
        for co in isa_scan.extract_code_objects(LIB, Path(td)):
            for k in isa_scan.parse(isa_scan.disassemble(co)):
                out[k.name] = k
    return out


def _score_epilogue(k):
    """The instructions of the q loop after its last MFMA, up to the loop's back-edge."""
    ins = k.insns
    mf = [i for i, x in enumerate(ins) if x.op.startswith("v_mfma")]
    assert mf, "no MFMA in the kernel"
    back = next(i for i in range(mf[len(mf) // 2], len(ins)) if ins[i].op == "s_cbranch_scc0")
    last = max(i for i in mf if i < back)
    return ins[last + 1:back]


def test_library_has_the_fused_config5_kernel(kernels):
    assert FUSED in kernels


def test_config5_score_epilogue_is_not_packed(kernels):
    epi = _score_epilogue(kernels[FUSED])
    packed = [x.text for x in epi if re.match(r"v_pk_(fma|mul|add)_f32", x.op)]
    scalar = [x for x in epi if x.op in ("v_fma_f32", "v_fmac_f32", "v_fmac_f32_e32", "v_fma_f32_e64")]
    assert not packed, f"packed fp32 ops back in the config-5 score epilogue: {packed[:4]}"
    # the validated form: the 32 fmas of the four per-half sums (2 halves x {pos, neg} x 8 terms)
    assert len(scalar) >= 32, [x.text for x in epi][:10]


def _src1_high_low_result(k):
    """Packed fp32 instructions whose low result reads src1's high dword (op_sel bit 1 set)."""
    out = []
    for x in k.insns:
        if not (x.op.startswith("v_pk_") and x.op.endswith("_f32")):
            continue
        m = re.search(r"op_sel:\[([01,]+)\]", x.text)
        if m and m.group(1).split(",")[1] == "1":
            out.append(x.text)
    return out


def test_no_kernel_has_a_packed_fp32_op_reading_src1_high_for_its_low_result(kernels):
    bad = {name: _src1_high_low_result(k) for name, k in kernels.items()}
    bad = {n: v for n, v in bad.items() if v}
    assert not bad, bad


def test_scanner_finds_the_failing_form_in_failing_build():
    """The failing round-4 build (reassembled from commit 3b0d266's source without the opaque
    copy) has exactly the four op_sel:[0,1] multiplies per q loop that the GPU attribution named:
    the scan is not vacuous."""
    hz = ROOT / "scripts" / "hazard" / "failing.hsaco"
    if not hz.exists():
        pytest.skip("scripts/hazard_variants.py not run")
    ks = {k.name: k for k in isa_scan.parse(isa_scan.disassemble(hz))}
    found = _src1_high_low_result(ks[FUSED])
    assert len(found) == 4 and all(t.startswith("v_pk_mul_f32") for t in found), found


def test_scanner_finds_packed_epilogue_in_failing_build(tmp_path):
    """The check above recognises the failing round-4 build (reassembled from the source of
    commit 3b0d266 without the opaque copy): the scanner is not vacuous."""
    hz = ROOT / "scripts" / "hazard" / "failing.hsaco"
    if not hz.exists():
        pytest.skip("scripts/hazard_variants.py not run")
    ks = {k.name: k for k in isa_scan.parse(isa_scan.disassemble(hz))}
    epi = _score_epilogue(ks[FUSED])
    assert sum(bool(re.match(r"v_pk_(fma|mul)_f32", x.op)) for x in epi) >= 16
