"""ISA guard (CPU): the hot kernels of libvge.so carry no FLAT memory instructions and no scratch.

A FLAT instruction reaching an LDS operand through a generic pointer is the one instruction class in these kernels that
can raise a memory violation from an LDS-intended address (ds_read / ds_write past the allocation read zeros / drop;
the weight rings use buffer loads inside their images), and it is what the dropped 16x16x32 conv build used for its A
fragments (the build that faulted once).  Scratch in a streaming kernel means registers held
across its MFMA streams spilled.  tools/isa_guard.py extracts the gfx950 code objects from the library's offload
bundles and reads each kernel's disassembly and metadata; no GPU and no compiler run.
"""
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

LIB = os.path.join(REPO, "video-gen-evals_amd", "vge", "libvge.so")

# kernel name fragments: the config-2 headline kernels, the gate detector's own kernels, the generic-shape path, the
# extractor GEMM and grouped conv
HOT = [
    "conv_encoder_x3s_kernel",
    "transformer_x3_kernelILb1ELb1ELi1ELi1E",   # f32x3, one window per workgroup
    "transformer_x3_kernelILb1ELb0ELi1ELi1E",
    "transformer_x3_kernelILb0ELb0ELi1ELi1E",   # single fp16, one window per workgroup, one workgroup per CU
    "featurize_tiles_kernel",
    "fuse_kernel",
    "score_videos_kernel",
    "rpn_select_kernel",
    "rpn_nms_kernel",
    "roi_align_kernel",
    "det_post_kernel",
    "gen_conv_kernel",
    "gen_attn_kernel",
    "gemm_bf16_kernel",    # the extractors' GEMM (ViT-H, the detector's 1x1 convs): every epilogue / shape variant
    "gemm2_bf16_kernel",
    "gemmp_bf16_kernel",   # its persistent form (its hand-counted vmcnt waits assume no scratch traffic)
    "gconv3_kernel",       # the detector's grouped 3x3 convs
]

# Variants that spill by design, pinned to their current scratch (B/lane) so that growth fails here instead of going
# unnoticed (round 5: the config-5 variants grew from 172 / 216-320 to 252 / 276-372 with no test noticing).  They fit
# their per-wave state into what their occupancy leaves: the single-fp16 transformer at two
# workgroups per CU (config 5's 4,096-window chunks: 256 registers per wave for a state that needs 343 at one per CU;
# 1.5x faster than the spill-free one-per-CU kernel there) and the two-windows-per-workgroup variants (3xfp16 / split
# chunks of >= 2,048 windows).
SPILL_BUDGET = {
    "transformer_x3_kernelILb0ELb0ELi1ELi2E": 252,
    "transformer_x3_kernelILb1ELb1ELi2ELi1E": 372,
    "transformer_x3_kernelILb1ELb0ELi2ELi1E": 280,
    "transformer_x3_kernelILb0ELb0ELi2ELi1E": 276,
}


@pytest.fixture(scope="module")
def table():
    if not os.path.exists(LIB):
        pytest.skip("libvge.so not built")
    if not shutil.which("objcopy") or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump"):
        pytest.skip("objcopy / ROCm llvm-objdump not available")
    import isa_guard
    return isa_guard.kernels(LIB)


@pytest.mark.parametrize("frag", HOT)
def test_hot_kernel_isa(table, frag):
    hits = {k: v for k, v in table.items() if frag in k}
    assert hits, f"no kernel matching {frag} in libvge.so"
    for name, r in hits.items():
        assert r["flat"] == 0, f"{name}: {r['flat']} FLAT memory instructions"
        assert r["scratch"] == 0 and r["scratch_ops"] == 0, f"{name}: {r['scratch']} B/lane scratch"


def test_guard_sees_the_library(table):
    """The extraction finds the code objects (every HIP translation unit's kernels)."""
    assert len(table) > 60
    assert any("conv_bf16_kernel" in k for k in table) and any("gemm_bf16_kernel" in k for k in table)


@pytest.mark.parametrize("frag,budget", sorted(SPILL_BUDGET.items()))
def test_spilling_variants_stay_within_their_pinned_scratch(table, frag, budget):
    hits = {k: v for k, v in table.items() if frag in k}
    assert hits, f"no kernel matching {frag} in libvge.so"
    for name, r in hits.items():
        assert r["flat"] == 0, f"{name}: {r['flat']} FLAT memory instructions"
        assert r["scratch"] <= budget, f"{name}: {r['scratch']} B/lane scratch, pinned at {budget}"


def test_every_transformer_variant_is_guarded(table):
    """Each transformer_x3_kernel instantiation in the library is either scratch-free (HOT) or pinned (SPILL_BUDGET)."""
    names = [k for k in table if "transformer_x3_kernel" in k]
    assert len(names) >= 7
    for k in names:
        assert any(f in k for f in HOT) or any(f in k for f in SPILL_BUDGET), k
