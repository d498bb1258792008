"""tools/check_lds_waits.py: the static in-flight-LDS-register check, on synthetic ISA and on the
real fused-gradient kernels (whose LDS reads are inline asm with hand-counted lgkmcnt waits)."""
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import check_lds_waits as chk  # noqa: E402


def _run(asm: str):
    lines = list(enumerate(asm.strip().splitlines(), 1))
    return chk.check(lines, "k")


def test_copy_before_wait_is_flagged():
    bad = _run("""
        ds_read_b128 v[4:7], v1
        ds_read_b128 v[8:11], v1 offset:16
        s_waitcnt lgkmcnt(1)
        v_mov_b32_e32 v20, v4
        v_mov_b32_e32 v21, v8
        s_endpgm""")
    assert [b[0] for b in bad] == [5]  # v8 is still in flight, v4 retired by lgkmcnt(1)


def test_overwrite_of_pending_destination_is_flagged():
    assert len(_run("""
        ds_read_b64_tr_b16 v[2:3], v0
        v_add_u32_e32 v3, 1, v9
        s_endpgm""")) == 1


def test_pending_state_follows_branches():
    asm = """
        ds_read_b32 v5, v0
        s_cbranch_scc1 .LBB0_2
        s_waitcnt lgkmcnt(0)
    .LBB0_2:
        v_add_u32_e32 v6, v5, v5
        s_endpgm"""
    assert len(_run(asm)) == 1  # the taken branch skips the wait
    assert _run(asm.replace("s_cbranch_scc1 .LBB0_2\n", "")) == []


@pytest.mark.skipif(shutil.which("hipcc") is None and not Path("/opt/rocm/bin/hipcc").exists(), reason="no hipcc")
def test_fused_gradient_kernels_have_no_in_flight_reads(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "gdw.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    f"-I{ROOT / 'csrc' / 'include'}", f"-I{ROOT / 'csrc'}", "-o", str(out),
                    str(ROOT / "csrc" / "kernels" / "softmax_grad_dw.hip")], check=True, capture_output=True)
    names = []
    for name, body in chk.kernels(str(out), "softmax_grad_dw_kernel"):
        names.append(name)
        assert chk.check(body, name) == [], name
    # F 128/256 x multinomial/OvR x {16, 32} classes per wave + F 512 x 2 kinds x 16
    assert len(names) == 10


@pytest.mark.skipif(shutil.which("hipcc") is None and not Path("/opt/rocm/bin/hipcc").exists(), reason="no hipcc")
def test_wide_gradient_dma_kernel_has_no_in_flight_reads(tmp_path):
    """The wide-F G^T X kernel's transposed LDS reads are inline asm too (softmax_grad_wide.hip)."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    out = tmp_path / "gdw_wide.s"
    subprocess.run([hipcc, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    f"-I{ROOT / 'csrc' / 'include'}", f"-I{ROOT / 'csrc'}", "-o", str(out),
                    str(ROOT / "csrc" / "kernels" / "softmax_grad_wide.hip")], check=True, capture_output=True)
    names = []
    for name, body in chk.kernels(str(out), "gdw_gemm_dma_kernel"):
        names.append(name)
        assert chk.check(body, name) == [], name
    assert len(names) == 1
