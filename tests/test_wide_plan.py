"""Host plan of the f64-accumulating wide serving kernel (csrc/kernels/wide_plan.h, a CPU test):
class blocks of 16, feature splits only when one split would need more than 32 wave steps, rows
padded to a whole number of (4 waves x 16-byte loads x splits), 16-byte aligned, and one
workspace region per row group (16 rows while the grid fits one block per CU, else 32) whose
layout does not depend on B."""
import pytest

from mlapi_amd._native import C, available

pytestmark = pytest.mark.skipif(not available(), reason="native extension not built")

F64, F32 = 0, 1


@pytest.mark.parametrize("dt", [F64, F32])
@pytest.mark.parametrize("F", [1, 3, 40, 127, 256, 1000, 1024, 1025, 2048, 2049, 4096, 5000, 16384])
@pytest.mark.parametrize("K", [1, 2, 16, 17, 1000])
def test_wide_plan_invariants(dt, F, K):
    p = C().linear_wide_plan(dt, F, K)
    E = 2 if dt == F64 else 4  # elements per 16-byte load
    unit = 4 * 4 * E           # features one step of every wave covers
    assert p["ncb"] == (K + 15) // 16
    assert p["ldx"] >= F and p["ldx"] % (unit * p["nfs"]) == 0
    assert p["ldx"] * (8 if dt == F64 else 4) % 16 == 0
    assert 1 <= p["fsteps"] <= 32 and p["fsteps"] * unit * p["nfs"] == p["ldx"]
    # splits only when needed, and never more than needed
    assert p["nfs"] == max(1, -(-F // (unit * 32)))
    assert p["ldx"] - F < unit * p["nfs"]  # padding below one step of every split


@pytest.mark.parametrize("dt", [F64, F32])
def test_wide_workspace_is_per_row_group(dt):
    for F, K in ((256, 1000), (4096, 40), (300, 1)):
        one = C().linear_wide_workspace(1, dt, F, K)
        assert one % 256 == 0 and one >= (-(-K // 16)) * 32 * 32  # >= the row states of one group
        for B in (1, 15, 16, 17, 31, 32, 33, 100, 1000):  # sized for 16-row groups: the most a launch uses
            assert C().linear_wide_workspace(B, dt, F, K) == -(-B // 16) * one


def test_wide_plan_rejects_other_dtypes():
    with pytest.raises(Exception):
        C().linear_wide_plan(2, 256, 10)  # bf16 storage has its own kernels
    with pytest.raises(Exception):
        C().linear_wide_plan(F64, 0, 10)
