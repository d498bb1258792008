"""The completer's host merge of class-split row states (csrc/runtime/split_merge.h, used by
Engine::collect for serving batches of <= host_merge_rows rows) against the float64 oracle, on CPU.
The per-block states are built the way linear_split.hip builds them: per 64-class block the f32
max, its first index and the f32 sum of exp(z - max) (OvR: sum of sigmoids)."""
import numpy as np
import pytest

from mlapi_amd._native import C


def _block_states(z: np.ndarray, ovr: bool):
    bis, ms, ss = [], [], []
    for c0 in range(0, z.size, 64):
        blk = z[c0:c0 + 64].astype(np.float32)
        j = int(np.argmax(blk))
        m = np.float32(blk[j])
        if ovr:
            s = np.float32(np.sum(1.0 / (1.0 + np.exp(-blk.astype(np.float64)))))
        else:
            s = np.float32(np.sum(np.exp(blk.astype(np.float64) - np.float64(m))))
        bis.append(c0 + j)
        ms.append(float(m))
        ss.append(float(s))
    return bis, ms, ss


@pytest.mark.parametrize("K", [2, 3, 64, 65, 1000])
@pytest.mark.parametrize("ovr", [False, True])
def test_host_merge_matches_fp64_oracle(K, ovr):
    rng = np.random.default_rng(K + 7 * ovr)
    for _ in range(50):
        z = rng.standard_normal(K) * 3
        label, p = C().merge_split_records(*_block_states(z, ovr), ovr)
        zf = z.astype(np.float32).astype(np.float64)
        assert label == int(np.argmax(zf))
        if ovr:
            sig = 1.0 / (1.0 + np.exp(-zf))
            want = sig.max() / sig.sum()
        else:
            want = 1.0 / np.exp(zf - zf.max()).sum()
        assert p == pytest.approx(want, rel=1e-6)


def test_host_merge_ties_go_to_the_first_class():
    z = np.zeros(200)
    z[70] = z[150] = z[199] = 5.0  # equal maxima in blocks 1, 2 and 3: class 70 wins (numpy argmax)
    label, _ = C().merge_split_records(*_block_states(z, False), False)
    assert label == 70
    z[10] = 5.0  # an earlier block with the same max
    assert C().merge_split_records(*_block_states(z, False), False)[0] == 10


def test_host_merge_extreme_logits_stay_finite():
    z = np.array([-80.0] * 100 + [80.0] + [-80.0] * 99)
    label, p = C().merge_split_records(*_block_states(z, False), False)
    assert label == 100 and p == pytest.approx(1.0, rel=1e-12)
    label, p = C().merge_split_records(*_block_states(z, True), True)
    assert label == 100 and np.isfinite(p) and 0 < p <= 1


def test_host_merge_rejects_bad_shapes():
    with pytest.raises(ValueError):
        C().merge_split_records([], [], [], False)
    with pytest.raises(ValueError):
        C().merge_split_records([0] * 65, [0.0] * 65, [1.0] * 65, False)
