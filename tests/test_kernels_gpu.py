"""T3: every HIP kernel vs a plain PyTorch fp64/fp32 reference of the same op."""
import os

import numpy as np
import pytest
import torch

from mlapi_amd.models.linear import Kind
from mlapi_amd.ops import linear as ops
from mlapi_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _rand(shape, dtype, seed, scale=1.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(shape, generator=g, dtype=torch.float64) * scale).to(dtype).to(DEV)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("kind,K", [(Kind.BINARY, 1), (Kind.BINARY_SOFTMAX, 1), (Kind.MULTINOMIAL, 3),
                                    (Kind.OVR, 3), (Kind.MULTINOMIAL, 16), (Kind.OVR, 7)])
@pytest.mark.parametrize("B,F", [(1, 4), (64, 4), (1000, 4), (333, 31)])
def test_linear_small(dtype, kind, K, B, F):
    X, W, b = _rand((B, F), dtype, 1), _rand((K, F), dtype, 2), _rand((K,), dtype, 3)
    idx, p = ops.linear_small(X, W, b, kind)
    ridx, rp = ref.predict_ref(X, W, b, kind)
    torch.cuda.synchronize()
    tol = 1e-12 if dtype == torch.float64 else 2e-6
    assert torch.equal(idx.cpu(), ridx.cpu())
    torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=tol, atol=tol)


def test_linear_generic_wide():
    X, W, b = _rand((257, 100), torch.float64, 4), _rand((40, 100), torch.float64, 5), _rand((40,), torch.float64, 6)
    for kind in (Kind.MULTINOMIAL, Kind.OVR):
        idx, p = ops.linear_small(X, W, b, kind)
        ridx, rp = ref.predict_ref(X, W, b, kind)
        assert torch.equal(idx.cpu(), ridx.cpu())
        torch.testing.assert_close(p.cpu(), rp.cpu(), rtol=1e-12, atol=1e-12)


def test_linear_small_iris_parity(iris_sklearn_model, iris_data):
    """fp64 GPU path reproduces sklearn's predict / predict_proba().max() (main.py:21-22)."""
    m = iris_sklearn_model
    _, Xte, _, yte = iris_data
    X = torch.tensor(Xte, device=DEV)
    W = torch.tensor(m.coef_, device=DEV)
    b = torch.tensor(m.intercept_, device=DEV)
    idx, p = ops.linear_small(X, W, b, Kind.MULTINOMIAL)
    pred = m.classes_[idx.cpu().numpy()]
    np.testing.assert_array_equal(pred, m.predict(Xte))
    np.testing.assert_allclose(p.cpu().numpy(), m.predict_proba(Xte).max(1), rtol=1e-14, atol=0)
    assert np.mean(pred == yte) == pytest.approx(0.9666666666666667, abs=0)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,F", [(1, 256), (17, 256), (4099, 256), (1000, 64), (513, 128), (300, 1024), (77, 8)])
@pytest.mark.parametrize("kind", [Kind.BINARY, Kind.BINARY_SOFTMAX])
def test_gemv_binary(dtype, B, F, kind):
    if dtype == torch.float32 and F == 8:
        F = 8
    X, w = _rand((B, F), dtype, 7), _rand((F,), dtype, 8, scale=1 / np.sqrt(F))
    bias = 0.125
    idx, p = ops.gemv_binary(X, w, bias, kind)
    z = X.double() @ w.double() + bias
    ridx = (z > 0).to(torch.int32)
    rp = torch.sigmoid(z.abs() * (2 if kind == Kind.BINARY_SOFTMAX else 1))
    torch.cuda.synchronize()
    near = z.abs() < 1e-4  # sign of a near-zero logit may flip under f32 accumulation
    assert torch.equal(idx[~near].cpu(), ridx[~near].cpu())
    torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=1e-5, atol=1e-5)


def test_gemv_binary_large_stream():
    B, F = 1 << 20, 256
    X = torch.randn(B, F, device=DEV, dtype=torch.bfloat16)
    w = (torch.randn(F, device=DEV) / 16).to(torch.bfloat16)
    idx, p = ops.gemv_binary(X, w, -0.5)
    z = X.float() @ w.float() - 0.5
    near = z.abs() < 1e-3
    assert torch.equal(idx[~near], (z > 0).to(torch.int32)[~near])
    torch.testing.assert_close(p, torch.sigmoid(z.abs()), rtol=1e-4, atol=1e-4)


@pytest.fixture(params=[0, 1, 2, 3], ids=["auto", "tiles", "rows", "t32"])
def gemm_kernel(request):
    """Run a multiclass test under the automatic plan and with each kernel forced (tiles: the
    LDS-staged, chunk-pipelined 16x16x32 kernel; rows: the row-group kernel; t32: the 32x32x16
    large-batch kernel, F in {64, 128, 256}, else tiles)."""
    from mlapi_amd._native import C

    C().gemm_softmax_force_plan(0, 0, request.param)
    yield request.param
    C().gemm_softmax_force_plan(0, 0, 0)


@pytest.mark.parametrize("B,F,K", [(1024, 256, 1000), (1, 256, 1000), (130, 64, 10), (2048, 128, 37),
                                   (4096, 256, 3), (100, 512, 200), (37, 32, 65), (20000, 256, 130),
                                   (300, 1024, 100), (65, 4096, 1000), (5, 700, 12), (5000, 256, 600),
                                   (3000, 128, 1100)])
@pytest.mark.parametrize("kind", [Kind.MULTINOMIAL, Kind.OVR])
def test_gemm_softmax(B, F, K, kind, gemm_kernel):
    """Both multiclass kernels vs the fp64 oracle on bf16 operands; F > 512 (row-group kernel, F
    looped in 256-feature slices inside one launch) and F not a kernel width (zero-padded)."""
    X = _rand((B, F), torch.bfloat16, 9)
    W = _rand((K, F), torch.bfloat16, 10, scale=1 / np.sqrt(F))
    b = _rand((K,), torch.float32, 11, scale=0.1)
    idx, p = ops.gemm_softmax(X, W, b, kind)
    Z = ref.logits_ref(X, W, b, dtype=torch.float64)
    ridx, rp = ref.predict_ref(X, W, b, kind)
    top2 = torch.topk(Z, min(2, K), dim=1).values
    clear = (top2[:, 0] - top2[:, -1]) > 1e-3 if K > 1 else torch.ones(B, dtype=torch.bool, device=DEV)
    torch.cuda.synchronize()
    assert torch.equal(idx[clear].cpu(), ridx[clear].cpu())
    torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("F,B", [(1024, 777), (4096, 777), (1024, 20000), (768, 16384)])
def test_predict_wide_multiclass_matches_fp64_oracle(F, B):
    """ops.predict on F = 768 / 1024 / 4096 multiclass models against the float64
    oracle of the same bf16-rounded operands; B >= 16384 at F <= 1024 runs the row-group kernel
    with X staged in LDS."""
    from mlapi_amd.models.linear import LinearModel
    from mlapi_amd.serve.loadgen import bf16_oracle

    m = LinearModel.random(F, 300, seed=F, kind=Kind.MULTINOMIAL)
    Xn = np.random.default_rng(F).standard_normal((B, F))
    idx, p = ops.predict(torch.tensor(Xn, device=DEV, dtype=torch.bfloat16), torch.tensor(m.W, device=DEV),
                         torch.tensor(m.b, device=DEV), Kind.MULTINOMIAL)
    om, Xr = bf16_oracle(m, Xn)
    ridx, rp = om.predict_max(Xr)
    zs = np.sort(om.decision_function(Xr), axis=1)
    clear = zs[:, -1] - zs[:, -2] > 1e-3
    np.testing.assert_array_equal(idx.cpu().numpy()[clear], ridx[clear])
    np.testing.assert_allclose(p.cpu().numpy(), rp, rtol=2e-4, atol=2e-5)


def test_gemm_softmax_large_batch_and_rearm():
    """NT=2 multi-chunk path (double-buffered LDS) and the split path launched repeatedly on one
    workspace (the in-kernel merge counters must re-arm themselves)."""
    F, K = 256, 1000
    W = _rand((K, F), torch.bfloat16, 21, scale=1 / 16)
    b = _rand((K,), torch.float32, 22, scale=0.1)
    for B in (70000, 1024):
        X = _rand((B, F), torch.bfloat16, 20)
        op = ops.GemmSoftmax(B, K, F, DEV)
        Z = ref.logits_ref(X, W, b, dtype=torch.float32)
        top2 = torch.topk(Z, 2, dim=1).values
        clear = (top2[:, 0] - top2[:, 1]) > 1e-3
        rp = torch.softmax(Z.double(), dim=1).max(dim=1).values
        for _ in range(3):
            idx, p = op(X, W, b)
            assert torch.equal(idx[clear], torch.argmax(Z, dim=1).to(torch.int32)[clear])
            torch.testing.assert_close(p.double(), rp, rtol=2e-4, atol=2e-5)
        assert op.xcd_errors() == 0


@pytest.mark.parametrize("kind", [Kind.MULTINOMIAL, Kind.OVR])
@pytest.mark.parametrize("B", [1024, 8192])
def test_gemm_softmax_xcd_local_merge_repeated(B, kind):
    """BASELINE config 3 (B = 1024, K = 1000, F = 256) and a 4-split plan: the row blocks' splits meet
    in one XCD's L2 (gemm_softmax.hip, put_granule). Twenty back-to-back launches on fresh inputs all
    match the oracle, and every merged partial came from the merging block's XCD."""
    F, K = 256, 1000
    W = _rand((K, F), torch.bfloat16, 61, scale=1 / 16)
    b = _rand((K,), torch.float32, 62, scale=0.1)
    op = ops.GemmSoftmax(B, K, F, DEV)
    Xs = [_rand((B, F), torch.bfloat16, 200 + i) for i in range(20)]
    outs = [tuple(t.clone() for t in op(X, W, b, kind)) for X in Xs]
    torch.cuda.synchronize()
    from mlapi_amd._native import C

    # the placement probe ran before the first XCD-local launch and found the round-robin order
    assert C().xcd_placement_state(torch.cuda.current_device()) == 1
    assert C().xcd_placement_mismatches(torch.cuda.current_device()) == 0
    for X, (idx, p) in zip(Xs, outs):
        Z = ref.logits_ref(X, W, b, dtype=torch.float64)
        ridx, rp = ref.predict_ref(X, W, b, kind)
        top2 = torch.topk(Z, 2, dim=1).values
        clear = (top2[:, 0] - top2[:, 1]) > 1e-3
        assert torch.equal(idx[clear].cpu(), ridx[clear].cpu())
        torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=2e-4, atol=2e-5)
    assert op.xcd_errors() == 0


@pytest.mark.parametrize("B", [100, 1024, 8192])
def test_gemm_softmax_split_merge_graph_replay(B):
    """A HIP graph bakes the split merge's granule tag into its arguments: every replay runs with
    the same epoch, so the merging block must clear the tags it consumed or the next replay would
    merge the previous replay's partials. Five replays on new inputs copied into the captured
    tensor all match the oracle."""
    F, K = 256, 1000
    W = _rand((K, F), torch.bfloat16, 71, scale=1 / 16)
    b = _rand((K,), torch.float32, 72, scale=0.1)
    op = ops.GemmSoftmax(B, K, F, DEV)
    X = _rand((B, F), torch.bfloat16, 73)
    out = (torch.empty(B, dtype=torch.int32, device=DEV), torch.empty(B, dtype=torch.float32, device=DEV))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        op(X, W, b, Kind.MULTINOMIAL, out=out)  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        op(X, W, b, Kind.MULTINOMIAL, out=out)
    for i in range(5):
        Xi = _rand((B, F), torch.bfloat16, 300 + i)
        X.copy_(Xi)
        g.replay()
        torch.cuda.synchronize()
        Z = ref.logits_ref(Xi, W, b, dtype=torch.float64)
        ridx, rp = ref.predict_ref(Xi, W, b, Kind.MULTINOMIAL)
        top2 = torch.topk(Z, 2, dim=1).values
        clear = (top2[:, 0] - top2[:, 1]) > 1e-3
        assert torch.equal(out[0][clear].cpu(), ridx[clear].cpu()), i
        torch.testing.assert_close(out[1].double().cpu(), rp.cpu(), rtol=2e-4, atol=2e-5)


@pytest.mark.parametrize("kernel", [1, 2])
def test_gemm_logits_asymmetric(kernel):
    """A = I-style check with an asymmetric operand: catches a transposed C write (guide S3)."""
    B, F, K = 64, 64, 48
    X = torch.zeros(B, F, device=DEV, dtype=torch.bfloat16)
    X[torch.arange(B), torch.arange(B) % F] = 1
    W = (torch.arange(K * F, device=DEV, dtype=torch.float32).reshape(K, F) % 13 - 6).to(torch.bfloat16)
    b = torch.arange(K, device=DEV, dtype=torch.float32) * 0.5
    from mlapi_amd._native import C

    C().gemm_softmax_force_plan(0, 0, kernel)
    try:
        Z = ops.gemm_logits(X, W, b)
    finally:
        C().gemm_softmax_force_plan(0, 0, 0)
    torch.testing.assert_close(Z, ref.logits_ref(X, W, b), rtol=0, atol=0)


@pytest.mark.parametrize("F", [32, 64, 256])
def test_gemm_ties_first_max(gemm_kernel, F):
    B, K = 256, 130
    X = torch.ones(B, F, device=DEV, dtype=torch.bfloat16)
    W = torch.zeros(K, F, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(K, device=DEV)
    b[[5, 77, 129]] = 1.0  # three-way tie for the max
    idx, p = ops.gemm_softmax(X, W, b)
    assert (idx == 5).all()
    torch.testing.assert_close(p, torch.full_like(p, float(torch.softmax(b.double(), 0).max())), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,F", [(1, 256), (5000, 256), (1 << 16, 256), (999, 64), (333, 1024)])
def test_train_binary_grad(dtype, B, F):
    X = _rand((B, F), dtype, 12)
    y = (torch.rand(B, device=DEV) > 0.5).float()
    w = _rand((F,), torch.float32, 13, scale=0.05)
    b = torch.tensor([0.1], device=DEV)
    out = ops.train_binary_grad(X, y, w, b)
    r = ref.train_binary_ref(X, y, w, b)
    torch.testing.assert_close(out.double().cpu(), r.cpu(), rtol=2e-4, atol=2e-3 * max(1.0, np.sqrt(B) / 30))
    out2 = ops.train_binary_grad(X, y, w, b)
    assert torch.equal(out, out2), "gradient must be bitwise deterministic"


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
@pytest.mark.parametrize("kind,K", [(Kind.MULTINOMIAL, 3), (Kind.BINARY, 1), (Kind.BINARY_SOFTMAX, 1),
                                    (Kind.OVR, 3), (Kind.MULTINOMIAL, 16)])
@pytest.mark.parametrize("B,F", [(120, 4), (5000, 10), (64, 64)])
def test_train_small_grad(dtype, kind, K, B, F):
    if K * F > 1024:
        pytest.skip("outside train_small range")
    X = _rand((B, F), dtype, 14)
    W = _rand((K, F), dtype, 15, scale=0.3)
    b = _rand((K,), dtype, 16, scale=0.3)
    ncls = 2 if K == 1 else K
    y = torch.randint(0, ncls, (B,), device=DEV, dtype=torch.int32)
    out = ops.train_small_grad(X, y, W, b, kind)
    r = ref.train_small_ref(X, y, W, b, kind)
    tol = 1e-10 if dtype == torch.float64 else 3e-4
    torch.testing.assert_close(out.double().cpu(), r.cpu(), rtol=tol, atol=tol * max(1, B / 100))


def test_sgd_update():
    p = torch.randn(1001, device=DEV)
    g = torch.randn(1001, device=DEV)
    exp = p.clone()
    exp[:1000] -= 0.1 * (g[:1000] / 8 + 0.01 * exp[:1000])
    exp[1000:] -= 0.1 * g[1000:] / 8
    ops.sgd_update(p, g, 1000, 0.1, 1 / 8, 0.01)
    torch.testing.assert_close(p, exp)


@pytest.mark.parametrize("src,dst", [(torch.float64, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.float32), (torch.float64, torch.bfloat16)])
def test_cast(src, dst):
    x = _rand((4097,), src, 17, scale=100)
    torch.testing.assert_close(ops.cast(x, dst), x.to(dst), rtol=0, atol=0)


def test_ops_reject_cpu_tensors():
    with pytest.raises(ValueError):
        ops.linear_small(torch.zeros(2, 4, dtype=torch.float64), torch.zeros(3, 4, dtype=torch.float64),
                         torch.zeros(3, dtype=torch.float64), Kind.MULTINOMIAL)


def test_train_binary_step_fused_equals_unfused():
    from mlapi_amd._native import C

    B, F = 50000, 256
    X = _rand((B, F), torch.bfloat16, 30)
    y = (torch.rand(B, device=DEV) > 0.5).float()
    p1 = _rand((F + 1,), torch.float32, 31, scale=0.01)
    p2 = p1.clone()
    m1 = torch.zeros_like(p1)
    m2 = torch.zeros_like(p2)
    ws = torch.empty(C().train_binary_workspace(B, F), dtype=torch.uint8, device=DEV)
    g1 = torch.empty(F + 3, device=DEV)
    for _ in range(3):
        C().train_binary_step(2, X.data_ptr(), y.data_ptr(), p1.data_ptr(), m1.data_ptr(), B, F, g1.data_ptr(),
                              ws.data_ptr(), ws.numel(), 0.3, 1.0 / B, 1e-3, 0.9, torch.cuda.current_stream().cuda_stream)
        g2 = ops.train_binary_grad(X, y, p2[:F], p2[F:])
        ops.sgd_update(p2, g2, F, 0.3, 1.0 / B, 1e-3, 0.9, m2)
    torch.cuda.synchronize()
    assert torch.equal(p1, p2) and torch.equal(g1, g2)


@pytest.mark.parametrize("nc", [1, 2])
@pytest.mark.parametrize("B,F,K,kind,groups", [
    (1000, 256, 1000, Kind.MULTINOMIAL, 0), (8192, 256, 1000, Kind.MULTINOMIAL, 0),
    (4099, 128, 37, Kind.MULTINOMIAL, 0), (77, 128, 10, Kind.OVR, 0), (300, 256, 130, Kind.OVR, 0),
    (64, 256, 3, Kind.MULTINOMIAL, 0), (20000, 128, 200, Kind.OVR, 3), (65, 256, 64, Kind.MULTINOMIAL, 1),
    (9000, 256, 300, Kind.OVR, 0),
    # widths the kernel trains zero-padded (32, 64 -> 128) and F = 512 (16 classes per wave only)
    (77, 32, 10, Kind.OVR, 0), (64, 64, 3, Kind.MULTINOMIAL, 0), (5000, 64, 300, Kind.MULTINOMIAL, 0),
    (300, 512, 130, Kind.OVR, 0), (4099, 512, 1000, Kind.MULTINOMIAL, 0), (65, 512, 64, Kind.MULTINOMIAL, 1)])
def test_softmax_grad_dw_fused(B, F, K, kind, groups, nc):
    """Fused G + dW kernel (softmax_grad_dw.hip) vs the fp32 oracle at 16 and 32 classes per wave:
    all five served widths (32/64 run
    zero-padded at 128), ragged row tiles, partial class groups, both kinds, forced row-group
    counts; reruns are bitwise identical (slab sums, no atomics)."""
    from mlapi_amd._native import C

    if F == 512 and nc != 1:
        pytest.skip("F = 512 runs 16 classes per wave")
    Fa = ops.softmax_train_faug(F)
    Fk = Fa - 8
    X = _rand((B, F), torch.float32, 41)
    W, b = _rand((K, F), torch.float32, 42, scale=2 / np.sqrt(F)), _rand((K,), torch.float32, 43)
    y = torch.randint(0, K, (B,), generator=torch.Generator().manual_seed(44), dtype=torch.int32).to(DEV)
    Xa = ops.augment_features(X, Fa)
    Wb = torch.zeros(K, Fk, dtype=torch.bfloat16, device=DEV)
    Wb[:, :F] = W.to(torch.bfloat16)
    C().softmax_grad_dw_force_plan(groups, nc)
    try:
        bufs = ops.SoftmaxTrainBuffers(B, K, Fk, X.device)
        dW1, st1 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs)
        dW1, st1 = dW1.clone(), st1.clone()
        dW2, st2 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs)
        torch.cuda.synchronize()
    finally:
        C().softmax_grad_dw_force_plan(0, 0)
    assert torch.equal(dW1, dW2) and torch.equal(st1, st2)
    _, dW_ref, loss_ref, corr_ref = ref.softmax_train_ref(Xa, y, ops.augment_weights(Wb.float(), b, Fa), kind)
    scale = dW_ref.abs().max().item() + 1e-6
    err = (dW2 - dW_ref).abs().max().item()
    assert err < 1e-2 * scale + 1e-2 * np.sqrt(B / 1000), (err, scale)
    torch.testing.assert_close(dW2[:, Fk], dW_ref[:, Fk], atol=2e-2 * np.sqrt(B / 100), rtol=1e-2)  # intercept
    assert st2[0].item() == pytest.approx(loss_ref.item(), rel=1e-4)
    assert abs(st2[1].item() - corr_ref.item()) <= max(2, B // 2000)
    assert torch.all(dW2[:, F:Fk] == 0) and torch.all(dW2[:, Fk + 1:] == 0)  # padded features, pad columns


@pytest.mark.parametrize("B,F,K,kind", [(2048, 1024, 100, Kind.MULTINOMIAL), (777, 700, 37, Kind.OVR),
                                        (4099, 1024, 1000, Kind.MULTINOMIAL), (65, 2048, 3, Kind.MULTINOMIAL),
                                        (20000, 1024, 130, Kind.OVR),  # B >= 16384, F <= 1024: X staged in LDS
                                        (16384, 768, 1000, Kind.MULTINOMIAL),
                                        (16400, 1024, 1000, Kind.MULTINOMIAL)])
def test_softmax_grad_wide(B, F, K, kind):
    """Wide multiclass gradient (F > 512, softmax_grad_wide.hip: row stats + logits by the row-group
    kernel, G in bf16, G^T X_aug by the transposed-LDS MFMA kernel, slab sum) vs the fp32 oracle;
    reruns bitwise identical; padded feature columns get exactly zero gradient."""
    Fa = ops.softmax_train_faug(F)
    Fk = Fa - 8
    assert Fk % 256 == 0 and Fk > 512
    X = _rand((B, F), torch.float32, 51)
    W, b = _rand((K, F), torch.float32, 52, scale=2 / np.sqrt(F)), _rand((K,), torch.float32, 53)
    y = torch.randint(0, K, (B,), generator=torch.Generator().manual_seed(54), dtype=torch.int32).to(DEV)
    Xa = ops.augment_features(X, Fa)
    Wb = torch.zeros(K, Fk, dtype=torch.bfloat16, device=DEV)
    Wb[:, :F] = W.to(torch.bfloat16)
    bufs = ops.SoftmaxTrainBuffers(B, K, Fk, X.device)
    assert bufs.wide
    dW1, st1 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs)
    dW1, st1 = dW1.clone(), st1.clone()
    dW2, st2 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs)
    torch.cuda.synchronize()
    assert torch.equal(dW1, dW2) and torch.equal(st1, st2)
    _, dW_ref, loss_ref, corr_ref = ref.softmax_train_ref(Xa, y, ops.augment_weights(Wb.float(), b, Fa), kind)
    scale = dW_ref.abs().max().item() + 1e-6
    err = (dW2 - dW_ref).abs().max().item()
    assert err < 1e-2 * scale + 1e-2 * np.sqrt(B / 1000), (err, scale)
    torch.testing.assert_close(dW2[:, Fk], dW_ref[:, Fk], atol=2e-2 * np.sqrt(B / 100), rtol=1e-2)  # intercept
    assert st2[0].item() == pytest.approx(loss_ref.item(), rel=1e-4)
    assert abs(st2[1].item() - corr_ref.item()) <= max(2, B // 2000)
    assert torch.all(dW2[:, F:Fk] == 0) and torch.all(dW2[:, Fk + 1:] == 0)
    # the second pass reads the first pass's logits back (default) or recomputes them: same bits
    from mlapi_amd._native import C

    C().softmax_grad_wide_set_zbuf(0)
    try:
        dW3, st3 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs)
        torch.cuda.synchronize()
    finally:
        C().softmax_grad_wide_set_zbuf(-1)
    assert torch.equal(dW2, dW3) and torch.equal(st2, st3)
    # logits kept in registers (softmax_rows_g2_kernel, where it applies) vs the XLDS kernel with the
    # logits buffer: the same MFMA and merge order, so the same bits
    C().gemm_softmax_set_rows_g2(0)
    try:
        bufs0 = ops.SoftmaxTrainBuffers(B, K, Fk, X.device)
        dW4, st4 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs0)
        torch.cuda.synchronize()
    finally:
        C().gemm_softmax_set_rows_g2(-1)
    assert torch.equal(dW2, dW4) and torch.equal(st2, st4)
    # W read in MFMA-fragment order (the packed copy, default) vs row-major: the same fragments,
    # so the same bits
    C().gemm_softmax_set_w_packed(0)
    try:
        dW5, st5 = ops.softmax_train_grad(Xa, Wb, b, y, kind, bufs=bufs)
        torch.cuda.synchronize()
    finally:
        C().gemm_softmax_set_w_packed(-1)
    assert torch.equal(dW2, dW5) and torch.equal(st2, st5)


def test_sgd_wide_multiclass_estimator_one_gpu():
    """LogisticRegression(solver='sgd') on an F = 1024 multiclass problem trains on ONE GPU (no
    sharding, no vendor GEMM) and learns it."""
    from mlapi_amd.models.estimator import LogisticRegression
    from mlapi_amd.train.softmax_sgd import synthetic_multiclass

    X, y = synthetic_multiclass(6000, 1024, 5, seed=3, noise=0.1)
    est = LogisticRegression(solver="sgd", epochs=8, device="cuda:0").fit(X.numpy(), y.numpy())
    acc = (est.predict(X.numpy()) == y.numpy()).mean()
    assert acc > 0.9, acc


def test_sgd_update_2d():
    K, Fa, F = 9, 40, 32
    p = _rand((K, Fa), torch.float32, 20)
    g = _rand((K * Fa + 2,), torch.float32, 21)
    mom = torch.zeros(K, Fa, device=DEV)
    shadow_w = torch.empty(K, F, dtype=torch.bfloat16, device=DEV)
    shadow_b = torch.empty(K, dtype=torch.float32, device=DEV)
    p0 = p.clone()
    ops.sgd_update_2d(p, g, F, 0.1, 0.5, 0.01, 0.9, mom, shadow_w, shadow_b)
    d = g[: K * Fa].view(K, Fa) * 0.5
    d[:, :F] += 0.01 * p0[:, :F]
    torch.testing.assert_close(p, p0 - 0.1 * d)
    torch.testing.assert_close(mom, d)
    assert torch.equal(shadow_w, p[:, :F].to(torch.bfloat16))
    assert torch.equal(shadow_b, p[:, F])


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_softmax_fused_update_equals_separate_update(momentum):
    """The SGD update fused into the gradient's final slab sum (one replica) is bit-identical to
    softmax_train_grad followed by sgd_update_2d, including the bf16 / f32 shadow copies."""
    from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass

    X, y = synthetic_multiclass(4096, 256, 300, seed=4, noise=0.3, device=DEV)
    a = SoftmaxSGDTrainer(256, 300, lr=0.3, l2=1e-3, momentum=momentum, device=torch.device(DEV))
    b = SoftmaxSGDTrainer(256, 300, lr=0.3, l2=1e-3, momentum=momentum, device=torch.device(DEV))
    Xa = a.prepare(X)
    for _ in range(4):
        a.step(Xa, y)  # fused
        b._local_grad(Xa, y)
        b._update(Xa.shape[0])
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params) and torch.equal(a.shadow_w, b.shadow_w) and torch.equal(a.shadow_b, b.shadow_b)
    assert torch.equal(a.grad, b.grad)
    if momentum:
        assert torch.equal(a.mom, b.mom)


def test_binary_sgd_graph_replay_is_exact():
    """BinarySGDTrainer.capture: the replayed HIP graph runs the same two launches as eager steps."""
    from mlapi_amd.train.sgd import BinarySGDTrainer, synthetic_binary

    X, y = synthetic_binary(4096, 256, seed=3, dtype=torch.bfloat16, device=DEV)
    eager = BinarySGDTrainer(256, lr=0.5, l2=1e-3, momentum=0.9, device=torch.device(DEV))
    graphed = BinarySGDTrainer(256, lr=0.5, l2=1e-3, momentum=0.9, device=torch.device(DEV))
    graphed.capture(X, y)
    assert torch.equal(graphed.params, eager.params)  # capture leaves the parameters untouched
    for _ in range(25):
        eager.step(X, y)
        graphed.step(X, y)
    torch.cuda.synchronize()
    assert torch.equal(eager.params, graphed.params) and eager.last_accuracy() > 0.8


def test_softmax_sgd_gpu_trains_and_graph_replay_is_exact():
    from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass

    X, y = synthetic_multiclass(16384, 64, 20, seed=2, noise=0.3, device=DEV)
    eager = SoftmaxSGDTrainer(64, 20, lr=0.5, momentum=0.9, device=torch.device(DEV))
    graphed = SoftmaxSGDTrainer(64, 20, lr=0.5, momentum=0.9, device=torch.device(DEV))
    Xa = eager.prepare(X)
    xs, ys = Xa[:8192].contiguous(), y[:8192].contiguous()
    graphed.capture(xs, ys)
    for _ in range(30):
        eager.step(xs, ys)
        graphed.step(xs, ys)
    torch.cuda.synchronize()
    assert torch.equal(eager.params, graphed.params), "graph replay must run the same kernels"
    loss, acc = eager.evaluate(Xa[8192:].contiguous(), y[8192:].contiguous())
    assert acc > 0.7, (loss, acc)
    cpu = SoftmaxSGDTrainer(64, 20, lr=0.5, momentum=0.9, device=torch.device("cpu"))
    Xc = cpu.prepare(X.cpu())
    for _ in range(30):
        cpu.step(Xc[:8192], y[:8192].cpu())
    np.testing.assert_allclose(eager.params.cpu().numpy(), cpu.params.numpy(), atol=0.05, rtol=0.05)


# ---- class-split multiclass predict (linear_split.h): small serving batches, f32 MFMA path
@pytest.mark.parametrize("kind", [Kind.MULTINOMIAL, Kind.OVR])
@pytest.mark.parametrize("K", [3, 17, 64, 65, 1000, 4100])
@pytest.mark.parametrize("B", [1, 5, 8, 16, 17, 32, 33, 200])
def test_linear_split_bf16(B, K, kind):
    """bf16 operands vs the fp64 oracle of the same rounded values, B = 1..32 (one row group) and
    beyond (several row groups, one merge counter each); labels compared where the top-2 gap is clear."""
    F = 256
    X = _rand((B, F), torch.bfloat16, 31)
    W = _rand((K, F), torch.bfloat16, 32, scale=1 / np.sqrt(F))
    b = _rand((K,), torch.float32, 33, scale=0.1)
    op = ops.LinearSplit(B, K, DEV)
    for _ in range(2):  # the second launch checks the in-kernel counter re-arm
        idx, p = op(X, W, b, kind)
        Z = ref.logits_ref(X, W, b, dtype=torch.float64)
        ridx, rp = ref.predict_ref(X, W, b, kind)
        top2 = torch.topk(Z, min(2, K), dim=1).values
        clear = (top2[:, 0] - top2[:, -1]) > 1e-3
        torch.cuda.synchronize()
        assert torch.equal(idx[clear].cpu(), ridx[clear].cpu())
        torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=2e-5, atol=2e-6)
    assert op.xcd_errors() == 0


@pytest.mark.parametrize("kind", [Kind.MULTINOMIAL, Kind.OVR])
@pytest.mark.parametrize("B", [1024, 2048])
def test_linear_split_xcd_local_merge_repeated(B, kind):
    """BASELINE config 3 shape (K = 1000, F = 256): 32 / 64 row groups whose 16 splits meet in one
    XCD's L2 (linear_split.h, XCD-local merge). Twenty back-to-back launches on fresh inputs: every
    one matches the oracle (a counter not re-armed or a stale L2 read would show up as a wrong row),
    and every merged partial came from the merging block's XCD."""
    F, K = 256, 1000
    W = _rand((K, F), torch.bfloat16, 52, scale=1 / np.sqrt(F))
    b = _rand((K,), torch.float32, 53, scale=0.1)
    op = ops.LinearSplit(B, K, DEV)
    outs = []
    Xs = [_rand((B, F), torch.bfloat16, 100 + i) for i in range(20)]
    for X in Xs:
        idx, p = op(X, W, b, kind)
        outs.append((idx.clone(), p.clone()))
    torch.cuda.synchronize()
    for X, (idx, p) in zip(Xs, outs):
        Z = ref.logits_ref(X, W, b, dtype=torch.float64)
        ridx, rp = ref.predict_ref(X, W, b, kind)
        top2 = torch.topk(Z, 2, dim=1).values
        clear = (top2[:, 0] - top2[:, 1]) > 1e-3
        assert torch.equal(idx[clear].cpu(), ridx[clear].cpu())
        torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=2e-5, atol=2e-6)
    assert op.xcd_errors() == 0


@pytest.mark.parametrize("kind", [Kind.MULTINOMIAL, Kind.OVR])
@pytest.mark.parametrize("B,F,K", [(1, 256, 1000), (8, 256, 1000), (32, 256, 1000), (256, 256, 1000), (7, 16, 3),
                                   (64, 100, 40), (19, 512, 129)])
def test_linear_split_f32_matches_fp64(B, F, K, kind):
    """f32 MFMA path (v_mfma_f32_16x16x4_f32) within rel 1e-6 of the fp64 oracle on the same f32
    operands (F=256, K=1000 served in f32)."""
    X = _rand((B, F), torch.float32, 41)
    W = _rand((K, F), torch.float32, 42, scale=1 / np.sqrt(F))
    b = _rand((K,), torch.float32, 43, scale=0.1)
    idx, p = ops.linear_split(X, W, b, kind)
    Z = ref.logits_ref(X, W, b, dtype=torch.float64)
    ridx, rp = ref.predict_ref(X, W, b, kind)
    top2 = torch.topk(Z, min(2, K), dim=1).values
    clear = (top2[:, 0] - top2[:, -1]) > 1e-5
    torch.cuda.synchronize()
    assert torch.equal(idx[clear].cpu(), ridx[clear].cpu())
    torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_linear_split_ties_and_asymmetric(dtype):
    """Three-way tie -> the first max; an asymmetric operand catches a transposed C layout."""
    B, F, K = 12, 64, 130
    X = torch.ones(B, F, device=DEV, dtype=dtype)
    W = torch.zeros(K, F, device=DEV, dtype=dtype)
    b = torch.zeros(K, device=DEV)
    b[[5, 77, 129]] = 1.0
    idx, p = ops.linear_split(X, W, b)
    assert (idx == 5).all()
    torch.testing.assert_close(p, torch.full_like(p, float(torch.softmax(b.double(), 0).max())), rtol=1e-5, atol=1e-6)
    # row i selects feature i: logits z[i, k] = W[k, i] + b[k] with W[k, i] distinct per (k, i)
    X = torch.zeros(B, F, device=DEV, dtype=dtype)
    X[torch.arange(B), torch.arange(B)] = 1
    W = ((torch.arange(K * F, device=DEV, dtype=torch.float32).reshape(K, F) * 7) % 61 / 8.0).to(dtype)
    idx, p = ops.linear_split(X, W, b)
    ridx, rp = ref.predict_ref(X, W, b, Kind.MULTINOMIAL)
    assert torch.equal(idx.cpu(), ridx.cpu())
    torch.testing.assert_close(p.double().cpu(), rp.cpu(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("xcd", [1, 0], ids=["xcd_local", "agent_scope"])
@pytest.mark.parametrize("B", [40, 200])
def test_linear_split_graph_replay(B, xcd):
    """a captured class-split launch replays ONE granule epoch, so its merging blocks clear
    the tags they consumed (capture-only clears, linear_split.hip). B > 32 (the in-kernel merge,
    several row groups), K = 1000 (16 splits), under the XCD-local and the agent-scope protocol:
    five replays on new rows copied into the captured input all match the oracle."""
    from mlapi_amd._native import C

    F, K = 256, 1000
    W = _rand((K, F), torch.bfloat16, 81, scale=1 / np.sqrt(F))
    b = _rand((K,), torch.float32, 82, scale=0.1)
    C().linear_split_set_xcd(xcd)
    try:
        op = ops.LinearSplit(B, K, DEV)
        X = _rand((B, F), torch.bfloat16, 83)
        out = (torch.empty(B, dtype=torch.int32, device=DEV), torch.empty(B, dtype=torch.float32, device=DEV))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            op(X, W, b, Kind.MULTINOMIAL, out=out)  # warm-up outside the capture (placement probe)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            op(X, W, b, Kind.MULTINOMIAL, out=out)
        for i in range(5):
            Xi = _rand((B, F), torch.bfloat16, 400 + i)
            X.copy_(Xi)
            g.replay()
            torch.cuda.synchronize()
            Z = ref.logits_ref(Xi, W, b, dtype=torch.float64)
            ridx, rp = ref.predict_ref(Xi, W, b, Kind.MULTINOMIAL)
            top2 = torch.topk(Z, 2, dim=1).values
            clear = (top2[:, 0] - top2[:, 1]) > 1e-3
            assert torch.equal(out[0][clear].cpu(), ridx[clear].cpu()), i
            torch.testing.assert_close(out[1].double().cpu(), rp.cpu(), rtol=2e-5, atol=2e-6)
        assert op.xcd_errors() == 0
    finally:
        C().linear_split_set_xcd(-1)
