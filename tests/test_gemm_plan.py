"""The automatic gemm_softmax plans (a CPU test: host code only), as tuned on an MI355X with the
tagged-granule split merge (profiles/r4_gemm_merge/: F = 256, K = 1000 sweeps): one block per CU
up to 64 row blocks of the 16x16 kernel (B = 1024 -> 16 splits of one 64-class chunk), two per CU
beyond; the 32x32 kernel from B = 8192 for wide K (B = 8192, K = 1000: 4 splits) and from 16384
otherwise, one block per CU up to 128 of its row blocks."""
import pytest

from mlapi_amd._native import C, available

pytestmark = pytest.mark.skipif(not available(), reason="native extension not built")


@pytest.mark.parametrize("B,K,kernel,splits", [
    (1, 1000, "tiles", 16), (100, 1000, "tiles", 16), (1024, 1000, "tiles", 16), (2048, 1000, "tiles", 8),
    (4096, 1000, "tiles", 4), (8192, 1000, "t32", 4), (16384, 1000, "t32", 2), (32768, 1000, "t32", 2),
    (65536, 1000, "t32", 1), (262144, 1000, "t32", 1), (8192, 100, "tiles", 2), (1024, 100, "tiles", 2),
    (1024, 10, "tiles", 1),
])
def test_gemm_softmax_plan(B, K, kernel, splits):
    p = C().gemm_softmax_plan(B, K, 256)
    assert (p["kernel"], p["splits"]) == (kernel, splits), p
    assert p["splits"] * p["classes_per_split"] >= K and p["classes_per_split"] % 64 == 0
    assert p["splits"] <= 16  # the merging block loads at most 16 granules per row in one pass


def test_gemm_softmax_plan_wide_features_use_the_row_group_kernel():
    assert C().gemm_softmax_plan(1024, 1000, 1024)["kernel"] == "rows"
