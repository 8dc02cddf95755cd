"""Inline-asm hazard lint of the product code (VERDICT r5 item 3;
tools/isa_hazards.py).  hipcc pads the MFMA / VALU / memory hazards of the
instructions it generates, never those of an `asm volatile` string
(cdna_hip_programming.md 5.7): these tests check, on the device assembly of
every product source (build.py build_asm: hipcc -S with the product flags,
;;#ASMSTART / ;;#ASMEND markers kept), that no pair with an asm instruction
on either side is closer than the rule allows, and on the product library's
disassembly that no pair at all breaks R1-R3.  The rules are pinned on
synthetic sequences first, and on the one hazard the lint found in round 6:
the exact-fp32 mask head's asm leaky_relu (v_max_f32) fed an MFMA B operand
one wait state later (mask_head.hip epilogue, fixed: fmaxf in that form)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "segment-anything-nerf_amd"))

import isa_hazards as ih  # noqa: E402

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
LIB = os.path.join(REPO, "segment-anything-nerf_amd", "samnerf_amd", "libsamnerf_hip.so")


def lint_text(body, asm_only=True):
    found = []
    ih.lint(ih.parse(body.splitlines()), "synthetic", found, asm_only)
    return [(f[0], f[1], f[2]) for f in found]


def test_r1_valu_write_into_mfma_operand():
    bad = """
        ;;#ASMSTART
        v_max_f32 v18, v2, v3
        ;;#ASMEND
        v_mov_b32_e32 v40, 0
        v_mfma_f32_32x32x2_f32 a[80:95], v5, v18, a[80:95]
    """
    assert lint_text(bad) == [("R1", 2, 1)]
    good = bad.replace("v_mov_b32_e32 v40, 0", "s_nop 1")
    assert lint_text(good) == []
    # the same pair with no asm on either side is hipcc's to pad: not counted in .s mode
    assert lint_text(bad.replace(";;#ASMSTART", "").replace(";;#ASMEND", "")) == []
    assert lint_text(bad.replace(";;#ASMSTART", "").replace(";;#ASMEND", ""), asm_only=False) == [("R1", 2, 1)]


def test_r2_mfma_result_read_early_and_accumulation_chain_allowed():
    seq = """
        ;;#ASMSTART
        v_mfma_f32_32x32x16_f16 v[0:15], v[16:19], v[20:23], v[0:15]
        v_mfma_f32_32x32x16_f16 v[0:15], v[24:27], v[28:31], v[0:15]
        s_nop 7
        v_max_i32_e32 v1, 0, v1
        ;;#ASMEND
    """
    # 8-pass XDL: the back-to-back accumulation is legal, the VALU read after 8 states is not (needs 12)
    assert lint_text(seq) == [("R2", 12, 8)]
    assert lint_text(seq.replace("s_nop 7", "s_nop 11")) == []


def test_r2_asm_overwrites_an_mfma_result_in_flight():
    """The second hazard the lint found (round 6, k_sam_head_w8 once it became
    the product): hipcc scheduled the f16x3 split's asm right behind a 4-pass
    MFMA chain and gave its outputs the chain's result registers, so the
    split's first v_mul wrote v0 / v1 while the MFMA writing v[0:3] was in
    flight (the split now opens with s_nop 7 there: split8_f16<true>)."""
    seq = """
        v_mfma_f32_16x16x32_f16 v[0:3], v[8:11], v[58:61], v[0:3]
        v_mfma_f32_16x16x32_f16 v[78:81], v[8:11], v[62:65], v[0:3]
        ;;#ASMSTART
        v_mul_f32 v0, v82, v182
        v_mul_f32 v1, v57, v182
        ;;#ASMEND
    """
    found = lint_text(seq)
    assert found and all(f[0] in ("R2", "R3") for f in found), found
    fixed = seq.replace(";;#ASMSTART", ";;#ASMSTART\n        s_nop 7")
    assert lint_text(fixed) == []


def test_r3_write_after_mfma_srcc_read():
    seq = """
        ;;#ASMSTART
        v_mfma_f32_32x32x16_f16 v[32:47], v[16:19], v[20:23], v[0:15]
        v_mov_b32_e32 v3, 0
        ;;#ASMEND
    """
    assert ("R3", 7, 0) in lint_text(seq)
    assert lint_text(seq.replace("v_mov_b32_e32 v3, 0", "s_nop 6\n        v_mov_b32_e32 v3, 0")) == []


def test_mfma_passes_of_the_product_shapes():
    assert ih.mfma_passes("v_mfma_f32_32x32x16_f16") == 8
    assert ih.mfma_passes("v_mfma_f32_16x16x32_f16") == 4
    assert ih.mfma_passes("v_mfma_f32_32x32x2_f32") == 16
    assert ih.mfma_passes("v_mfma_f32_16x16x4_f32") == 8


@pytest.fixture(scope="module")
def product_asm():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    import build
    return build.build_asm()


def test_product_asm_statements_pad_their_hazards(product_asm):
    """Every inline-asm statement of the product sources (the f16x3 split,
    the LDS-DMA weight streams and their hand-counted waits, the leaky_relu
    max, the max3 / permlane helpers) keeps R1-R3 with the instructions
    around it."""
    bad = {}
    n_kernels = 0
    for path in product_asm:
        res = ih.run(path)
        n_kernels += len(res)
        for k, found in res.items():
            hard = [f for f in found if f[0] in ("R1", "R2", "R3")]
            if hard:
                bad[k] = hard[:4]
    assert n_kernels > 200
    assert not bad, bad


def test_product_library_has_no_mfma_hazard_pair(product_asm):
    """The disassembled product library, every pair (compiler and asm):
    no R1-R3 pair in any of its kernels."""
    if not os.path.exists(LIB):
        pytest.skip("product library not built")
    res = ih.run(LIB)
    assert len(res) > 200
    hard = {k: [f for f in v if f[0] in ("R1", "R2", "R3")][:3] for k, v in res.items()}
    hard = {k: v for k, v in hard.items() if v}
    assert not hard, hard
