"""Static resource guard for the hot MFMA kernels (a CPU test: hipcc cross-compiles gfx950).

A kernel that starts spilling to scratch, or outgrows its occupancy budget, is a silent
performance regression the numerics tests cannot see. The budgets are the ones the kernels are
designed for (docs/PERFORMANCE.md, MI355X_MICROARCH.md register table): two waves per SIMD
(<= 256 VGPRs incl. AGPRs) for the 32x32 gemm_softmax kernel; no scratch at all in the class-split
and wide (f64 MFMA) serving kernels; no scratch access inside the MFMA loop of the 32x32 kernel (its
KS = 8 OvR instantiations spill 28 bytes around the loop - stored before it, reloaded for the split
merge after it - not in it).
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

from mlapi_amd import _build

ROOT = Path(__file__).resolve().parent.parent
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
pytestmark = pytest.mark.skipif(not Path(HIPCC).exists(), reason="no hipcc")


def _compile(src: str, tmp_path) -> str:
    out = tmp_path / (Path(src).stem + ".s")
    cmd = [HIPCC, "-O3", "-std=c++17", f"--offload-arch={_build.ARCH}", "--cuda-device-only", "-S",
           f"-I{ROOT / 'csrc' / 'include'}", f"-I{ROOT / 'csrc'}", "-o", str(out)]
    cmd += _build.FILE_FLAGS.get(src, []) + [str(ROOT / "csrc" / src)]
    subprocess.run(cmd, check=True, capture_output=True)
    return out.read_text()


def _resources(text: str) -> dict:
    res = {}
    for key in ("num_vgpr", "num_agpr", "private_seg_size"):
        for name, v in re.findall(r"\.set (\w+)\." + key + r", (\d+)", text):
            res.setdefault(name, {})[key] = int(v)
    return res


def _pick(res: dict, pattern: str) -> dict:
    got = {k: v for k, v in res.items() if re.search(pattern, k)}
    assert got, f"no kernel matching {pattern}"
    return got


def _mfma_loop_blocks(text: str, kernel: str):
    """Basic blocks of `kernel` inside a loop (between a label and a later branch back to it) that
    issue >= 16 MFMAs: the pipelined class loop (2 x F/16 per chunk), not the prologue's first chunk."""
    start = text.index(kernel + ":")
    body = text[start:text.index(".Lfunc_end", start)]
    parts = re.split(r"\n(\.LBB\w+):", body)
    labels = [None] + parts[1::2]
    blocks = [parts[0]] + parts[2::2]
    pos = {lab: i for i, lab in enumerate(labels) if lab}
    in_loop = [False] * len(blocks)
    for j, blk in enumerate(blocks):
        for target in re.findall(r"s_c?branch\w*\s+(\.LBB\w+)", blk):
            i = pos.get(target)
            if i is not None and i <= j:
                for k in range(i, j + 1):
                    in_loop[k] = True
    for blk, loop in zip(blocks, in_loop):
        if loop and blk.count("v_mfma") >= 16:
            yield blk


def test_gemm_softmax_kernels_fit_two_waves_per_simd_without_spills(tmp_path):
    text = _compile("kernels/gemm_softmax.hip", tmp_path)
    res = _resources(text)
    assert "gemm_softmax_ws" not in text  # the measured-losing W-stationary kernel stays archived
    for name, r in _pick(res, r"gemm_softmax32_kernelILi[48]ELi4ELi1E").items():
        assert r.get("num_vgpr", 0) + r.get("num_agpr", 0) <= 256, (name, r)
        loops = list(_mfma_loop_blocks(text, name))
        assert loops, name
        assert not any("scratch_" in blk for blk in loops), name


def test_rows_g2_kernel_keeps_its_logits_without_spilling_in_the_loop(tmp_path):
    """The wide-F training G kernel that holds two class chunks of logits in registers (128 VGPRs of
    accumulators) fits 2 waves per SIMD; its few spilled registers live outside the MFMA loop."""
    text = _compile("kernels/gemm_softmax.hip", tmp_path)
    res = _resources(text)
    got = _pick(res, r"softmax_rows_g2_kernel")
    assert len(got) == 4, sorted(got)  # softmax / OvR x row-major / fragment-packed W
    for name, r in got.items():
        assert r.get("num_vgpr", 0) + r.get("num_agpr", 0) <= 256, (name, r)
        assert r.get("private_seg_size", 0) <= 16, (name, r)
        loops = list(_mfma_loop_blocks(text, name))
        assert loops, name
        assert not any("scratch_" in blk for blk in loops), name


def test_class_split_serving_kernel_has_no_scratch(tmp_path):
    res = _resources(_compile("kernels/linear_split.hip", tmp_path))
    for name, r in _pick(res, r"linear_split_kernel").items():
        assert r.get("private_seg_size", 0) == 0, (name, r)


def test_wide_serving_kernel_has_no_scratch(tmp_path):
    res = _resources(_compile("kernels/linear_wide.hip", tmp_path))
    got = _pick(res, r"linear_wide_kernel")
    assert len(got) == 4, sorted(got)  # f64 / f32 storage x one / two row tiles per wave
    for name, r in got.items():
        assert r.get("private_seg_size", 0) == 0, (name, r)
