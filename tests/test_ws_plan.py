"""Host plan of the W-stationary gemm_softmax kernel (gemm_softmax.hip, `gemm_softmax_ws_plan`),
checked on CPU by replaying the kernel's block -> (XCD, slice, row group) and wave -> tile mapping:
every (tile, class slice) pair is computed exactly once, the NS slice blocks of a row group sit on
one XCD, the slices cover the classes, and the grid never exceeds the CUs."""
import pytest

from mlapi_amd._native import C

WS_WAVES = 8


def _replay(B, K, F, cus_per_xcd):
    plan = C().gemm_softmax_ws_plan(B, K, F, cus_per_xcd)
    assert plan is not None
    ns, gpx, tpg, grid = plan["slices"], plan["groups_per_xcd"], plan["tiles_per_group"], plan["grid"]
    T = (B + 31) // 32
    seen = {}
    xcd_of_group = {}
    for blk in range(grid):  # the kernel's prologue
        xcd, j = blk & 7, blk >> 3
        slc, gx = j % ns, j // ns
        if gx >= gpx:
            continue
        group = gx * 8 + xcd
        assert xcd_of_group.setdefault(group, xcd) == xcd  # a row group's slices share one XCD
        t_begin, t_end = group * tpg, min(T, (group + 1) * tpg)
        for wave in range(WS_WAVES):
            for tile in range(t_begin + wave, t_end, WS_WAVES):
                seen[(tile, slc)] = seen.get((tile, slc), 0) + 1
    assert set(seen) == {(t, s) for t in range(T) for s in range(ns)}
    assert all(v == 1 for v in seen.values())
    assert plan["slice_classes"] * ns >= K > plan["slice_classes"] * (ns - 1)
    assert grid <= 8 * cus_per_xcd
    return plan


@pytest.mark.parametrize("B,K,F", [(262144, 1000, 256), (65536, 1000, 256), (16384, 130, 256), (1, 1000, 256),
                                   (70000, 1100, 128), (5000, 600, 256), (33, 3000, 256)])
def test_every_tile_and_slice_once(B, K, F):
    plan = _replay(B, K, F, 32)
    if (B, K, F) == (262144, 1000, 256):  # BASELINE-scale: 4 slices of 256 classes, 64 row groups
        assert plan["slices"] == 4 and plan["slice_classes"] == 256 and plan["grid"] == 256


def test_partitioned_device_and_limits():
    _replay(100000, 1000, 256, 4)  # a CPX-style partition: 32 CUs -> 4 per "XCD"
    assert C().gemm_softmax_ws_plan(1000, 1000, 64, 32) is None    # F = 64: the 32x32 kernel
    assert C().gemm_softmax_ws_plan(1000, 40000, 256, 32) is None  # more slices than CUs per XCD
    assert C().gemm_softmax_ws_plan(600000, 1000, 256, 32) is None  # counters: B <= 524288
