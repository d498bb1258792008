"""f64-accumulating wide predict (csrc/kernels/linear_wide.h, v_mfma_f64_16x16x4_f64) against the
float64 oracle: f64 storage must agree with sklearn's float64 math (reference main.py:21-22) to
rounding (rel 1e-12 on p_max, labels exact away from 1e-9 ties); f32 storage with the oracle of
the f32-rounded inputs to the same tolerance (the products are exact in f64, so f32 storage only
rounds the inputs). Shapes cover single / several class blocks, feature splits over blocks
(F > 1024 f64, > 2048 f32), unaligned F and K, 1..100 rows (one and several row groups, one and
two row tiles per wave) and every sklearn kind."""
import numpy as np
import pytest
import torch

from mlapi_amd.models.linear import Kind, LinearModel

pytestmark = pytest.mark.gpu


def _oracle_check(m: LinearModel, X, idx, p, rtol=1e-12, tie=1e-9):
    ridx, rp = m.predict_max(X)
    z = m.decision_function(X)
    margin = np.abs(z) if z.ndim == 1 else np.diff(np.sort(z, axis=1)[:, -2:], axis=1)[:, 0]
    bad = (idx != ridx) & (margin > tie)
    assert not bad.any(), f"{int(bad.sum())} labels differ away from ties"
    np.testing.assert_allclose(p, rp, rtol=rtol, atol=0)


SHAPES = [  # F, K, kind
    (40, 3, Kind.MULTINOMIAL),
    (256, 40, Kind.MULTINOMIAL),
    (256, 1000, Kind.MULTINOMIAL),
    (257, 17, Kind.OVR),
    (1024, 40, Kind.MULTINOMIAL),
    (1500, 33, Kind.OVR),
    (4096, 1000, Kind.MULTINOMIAL),
    (5000, 7, Kind.MULTINOMIAL),
    (128, 300, Kind.MULTINOMIAL),   # 19 class blocks: 32 lanes per row in the merge
    (512, 3000, Kind.MULTINOMIAL),  # 188 class blocks: 64 lanes per row, 3 blocks per lane
    (64, 4500, Kind.MULTINOMIAL),   # 282 class blocks: the merge's two-pass path (> 4 x 64 blocks)
    (300, 1100, Kind.OVR),
    (256, 1, Kind.BINARY),
    (4096, 1, Kind.BINARY),
    (300, 1, Kind.BINARY_SOFTMAX),
]


@pytest.mark.parametrize("dtype", ["f64", "f32"])
@pytest.mark.parametrize("F,K,kind", SHAPES)
def test_linear_wide_matches_fp64_oracle(dtype, F, K, kind):
    from mlapi_amd.ops.linear import LinearWide

    td = torch.float64 if dtype == "f64" else torch.float32
    m = LinearModel.random(F, 2 if K == 1 else K, seed=F * 7 + K, kind=kind)
    rng = np.random.default_rng(F + K)
    op = LinearWide(100, F, m.W.shape[0], td, "cuda")
    for B in (1, 7, 16, 17, 32, 100):
        X = rng.standard_normal((B, F))
        Xg = torch.tensor(X, device="cuda").to(td).contiguous()
        Wg = torch.tensor(m.W, device="cuda").to(td).contiguous()
        bg = torch.tensor(m.b, device="cuda", dtype=torch.float64)
        idx, p = op(Xg, Wg, bg, int(kind))
        torch.cuda.synchronize()
        if dtype == "f32":  # the oracle of the inputs the kernel reads
            om = LinearModel(m.W.astype(np.float32).astype(np.float64), m.b, m.classes, m.kind)
            Xo = X.astype(np.float32).astype(np.float64)
        else:
            om, Xo = m, X
        _oracle_check(om, Xo, idx.cpu().numpy(), p.cpu().numpy())


def test_linear_wide_grid_far_beyond_the_chip():
    """B = 6000 rows x K = 1000: 188 row groups x 63 class blocks = 11,844 blocks, ~6x what the chip
    holds at once - every row group's merging block still sees all its producers' granules (none
    times out), and the answers match the oracle."""
    from mlapi_amd.ops.linear import LinearWide

    F, K, B = 256, 1000, 6000
    m = LinearModel.random(F, K, seed=77)
    X = np.round(np.random.default_rng(8).standard_normal((B, F)), 3)
    op = LinearWide(B, F, K, torch.float64, "cuda")
    for _ in range(2):
        idx, p = op(torch.tensor(X, device="cuda"), torch.tensor(m.W, device="cuda"), torch.tensor(m.b, device="cuda"))
        torch.cuda.synchronize()
        assert op.failed(idx) == 0, "a class merge timed out"
        idx = idx.cpu().numpy()
        _oracle_check(m, X, idx, p.cpu().numpy())


def test_linear_wide_is_deterministic_and_tie_first():
    """Repeated launches are bitwise identical (fixed merge orders) and exact ties go to the lowest
    class index across class blocks (numpy argmax)."""
    from mlapi_amd.ops.linear import LinearWide

    F, K = 512, 100
    W = np.zeros((K, F))
    W[3, 0] = W[40, 0] = W[99, 0] = 1.0  # classes 3, 40, 99 tie for the max (three class blocks)
    b = np.zeros(K)
    X = np.zeros((20, F))
    X[:, 0] = np.linspace(0.5, 2, 20)
    op = LinearWide(20, F, K, torch.float64, "cuda")
    args = [torch.tensor(a, device="cuda") for a in (X, W)] + [torch.tensor(b, device="cuda")]
    outs = [op(*args, int(Kind.MULTINOMIAL)) for _ in range(3)]
    torch.cuda.synchronize()
    for idx, p in outs[1:]:
        assert torch.equal(idx, outs[0][0]) and torch.equal(p, outs[0][1])
    assert (outs[0][0].cpu().numpy() == 3).all()
    m = LinearModel(W, b, np.array([f"c{i}" for i in range(K)], dtype=object), Kind.MULTINOMIAL)
    _oracle_check(m, X, outs[0][0].cpu().numpy(), outs[0][1].cpu().numpy())


def test_linear_wide_nonfinite_rows():
    """+inf logits in two classes give a NaN probability (HTTP 500, reference A13); a finite row
    in the same batch is unaffected."""
    from mlapi_amd.ops.linear import LinearWide

    F, K = 64, 40
    m = LinearModel.random(F, K, seed=1)
    W = np.abs(m.W)
    X = np.stack([np.full(F, 1e308), np.ones(F)])
    op = LinearWide(2, F, K, torch.float64, "cuda")
    idx, p = op(torch.tensor(X, device="cuda"), torch.tensor(W, device="cuda"), torch.tensor(m.b, device="cuda"))
    p = p.cpu().numpy()
    assert not np.isfinite(p[0]) and np.isfinite(p[1])


# ---- served through the engine: wide_dtype f64 (the reference's precision) ------------------------
def _engine(native, **kw):
    cfg = native.EngineConfig()
    cfg.device = 0
    for k, v in kw.items():
        setattr(cfg, k, v)
    return native.Engine(cfg)


@pytest.mark.parametrize("merge", ["host", "kernel"])
@pytest.mark.parametrize("F", [256, 1024, 4096])
@pytest.mark.parametrize("K", [2, 40, 1000])
def test_engine_f64_wide_models_match_sklearn_math(native, F, K, merge):
    """wide_dtype = f64: every batch size class (host-merged records <= 16 rows or in-kernel class
    merge) agrees with the float64 oracle to rel 1e-12 and exact labels."""
    kind = Kind.BINARY if K == 2 else Kind.MULTINOMIAL
    m = LinearModel.random(F, K, seed=F + K, kind=kind)
    e = _engine(native, max_batch=64, max_features=F, wide_dtype=0, host_merge_rows=16 if merge == "host" else 0,
                wide_host_merge_blocks=64 if merge == "host" else 0)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        assert e.model_path() == "wide"
        rng = np.random.default_rng(K)
        for n in (1, 3, 16, 40):
            X = np.round(rng.standard_normal((n, F)), 3)
            idx, p, st = e.predict(X)
            assert (st == 0).all()
            _oracle_check(m, X, idx, p)
        s = e.stats()
        assert s["path_batches"]["wide"] == s["batches"] and s["generic_models"] == 0
    finally:
        e.stop()


@pytest.mark.parametrize("K", [40, 1000])
def test_engine_f64_host_merge_17_to_32_rows(native, K):
    """Host-merged WIDE batches of 17-32 rows (host_merge_rows = 32) run as ONE 32-row group even
    where the planner would pick 16-row groups for a batch that small; answers match the float64
    oracle (those batches used to throw in the launcher)."""
    F = 256
    m = LinearModel.random(F, K, seed=K + 5)
    e = _engine(native, max_batch=64, max_features=F, wide_dtype=0, host_merge_rows=32, wide_host_merge_blocks=64)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        assert e.model_path() == "wide"
        rng = np.random.default_rng(K)
        for n in (17, 24, 32):
            X = np.round(rng.standard_normal((n, F)), 3)
            idx, p, st = e.predict(X)
            assert (st == 0).all(), st
            _oracle_check(m, X, idx, p)
    finally:
        e.stop()


def test_engine_f32_k40_model_meets_1e6(native):
    """The K = 40 f32 model that missed rel 1e-6 on the f32-accumulating class-split kernel
    (profiles/r3_final4/prof_serve_wide_k40_f32_direct_failure.txt: 7 / 1024 rows, max 2.08e-6):
    bench.py serve_wide's exact model and rows. With f64 accumulation it meets 1e-11."""
    from mlapi_amd.serve.loadgen import make_workload

    F, K = 256, 40
    m = LinearModel.random(F, K, seed=0, labels=[f"class_{i}" for i in range(K)])
    rows = np.round(np.random.default_rng(7).standard_normal((1024, F)), 3)
    f32 = lambda a: np.asarray(a, dtype=np.float32).astype(np.float64)  # noqa: E731
    e = _engine(native, max_batch=256, max_features=F, wide_dtype=1)
    try:
        e.load_model(int(m.kind), m.W, m.b, m.label_json())
        assert e.model_path() == "wide"
        make_workload(e, m, [f"f{i}" for i in range(F)], rows, rtol_oracle=1e-11, label_margin=1e-9,
                      oracle=(LinearModel(f32(m.W), f32(m.b), m.classes, m.kind), f32(rows)))
    finally:
        e.stop()


def test_class_merge_timeout_fails_rows_not_answers(native):
    """Fault injection (linear_wide_set_probe(3)): the merging block never sees the other blocks'
    states. After its bounded 1 s poll every row comes back as WIDE_TIMEOUT_IDX / NaN from the op,
    and through the engine as a failed row (ST_DEVICE_ERROR -> HTTP 500), never as an answer; the
    next launch is normal again."""
    from mlapi_amd.ops.linear import LinearWide

    F, K = 64, 200
    m = LinearModel.random(F, K, seed=4)
    X = np.random.default_rng(1).standard_normal((5, F))
    op = LinearWide(5, F, K, torch.float64, "cuda")
    args = [torch.tensor(a, device="cuda") for a in (X, m.W, m.b)]
    native.linear_wide_set_probe(3)
    try:
        idx, p = op(*args)
        torch.cuda.synchronize()
        assert op.failed(idx) == 5 and (idx == LinearWide.WIDE_TIMEOUT_IDX).all() and torch.isnan(p).all()
        e = _engine(native, max_batch=16, max_features=F, wide_dtype=0)
        try:
            e.load_model(int(m.kind), m.W, m.b, m.label_json())
            _, _, st = e.predict(X)
            assert (st == 4).all(), st
        finally:
            e.stop()
    finally:
        native.linear_wide_set_probe(0)
    idx, p = op(*args)
    torch.cuda.synchronize()
    assert op.failed(idx) == 0
    _oracle_check(m, X, idx.cpu().numpy(), p.cpu().numpy())


@pytest.mark.parametrize("B", [8, 100])
def test_linear_wide_graph_replay(B):
    """A captured HIP graph replays the WIDE launch with ONE class-merge epoch baked in: the merging
    block clears the tags it consumed, so five replays on new rows copied into the captured input
    all match the oracle (without the clear, replay k would merge replay k - 1's states)."""
    from mlapi_amd.ops.linear import LinearWide

    F, K = 256, 1000
    m = LinearModel.random(F, K, seed=91, kind=Kind.MULTINOMIAL)
    op = LinearWide(B, F, K, torch.float64, "cuda")
    Wg = torch.tensor(m.W, device="cuda", dtype=torch.float64).contiguous()
    bg = torch.tensor(m.b, device="cuda", dtype=torch.float64)
    X = torch.zeros(B, F, device="cuda", dtype=torch.float64)
    out = (torch.empty(B, dtype=torch.int32, device="cuda"), torch.empty(B, dtype=torch.float64, device="cuda"))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        op(X, Wg, bg, int(Kind.MULTINOMIAL), out=out)  # warm-up outside the capture
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        op(X, Wg, bg, int(Kind.MULTINOMIAL), out=out)
    rng = np.random.default_rng(92)
    for i in range(5):
        Xn = rng.standard_normal((B, F))
        X.copy_(torch.tensor(Xn, device="cuda"))
        g.replay()
        torch.cuda.synchronize()
        _oracle_check(m, Xn, out[0].cpu().numpy(), out[1].cpu().numpy())


def test_wide_overlapping_launches_with_concurrent_training(native):
    """the WIDE class merge waits for its row group's class blocks, which the
    dispatcher placed before the merging block. Here several WIDE batches are in flight at once
    (slot-private workspaces: unordered packets that overlap on the GPU) while a 1000-class training
    step loop keeps the CUs busy from another thread - the case where block residency is not a
    given. Every one of the served bodies must still be the engine's own f64 answer (checked against
    the fp64 oracle first), with no merge timeout (500)."""
    import threading

    from mlapi_amd.serve.loadgen import make_workload
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass
    from mlapi_amd.utils.config import Config

    F, K = 256, 1000
    names = [f"f{i}" for i in range(F)]
    m = LinearModel.random(F, K, seed=77, kind=Kind.MULTINOMIAL, labels=[f"c{i}" for i in range(K)])
    X = np.round(np.random.default_rng(78).standard_normal((256, F)), 3)
    stop = threading.Event()
    steps = [0]
    errors = []

    def train():
        try:
            dev = torch.device("cuda:0")
            tr = SoftmaxSGDTrainer(256, 1000, lr=0.1, device=dev)
            Xt, yt = synthetic_multiclass(16384, 256, 1000, seed=5)
            Xa, yt = tr.prepare(Xt.to(dev)), yt.to(dev)
            s = torch.cuda.Stream(dev)
            with torch.cuda.stream(s):
                while not stop.is_set():
                    tr.step(Xa, yt)
                    steps[0] += 1
                    if steps[0] % 8 == 0:
                        s.synchronize()
            s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    cfg = Config.from_env(port=0, device="cuda:0", feature_names=names, reload="off", missing_model="keep",
                          model_path="/nonexistent/overlap.pkl", io_threads=4, wide_dtype="f64", slots=4)
    with NativeServer(cfg) as srv:
        srv.runtime.handle.load(m)
        reqs, exp = make_workload(srv.runtime.handle.engine, m, names, X, rtol_oracle=1e-12, label_margin=1e-9)
        th = threading.Thread(target=train)
        th.start()
        try:
            import time

            t_end = time.time() + 60
            while steps[0] < 2 and not errors and time.time() < t_end:  # training is under way
                time.sleep(0.01)
            lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), 48, 3)
            lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
            s0 = srv.runtime.handle.stats()
            st0 = steps[0]
            res = lg.run(400, True)
            st1 = steps[0]
            lg.close()
            s1 = srv.runtime.handle.stats()
        finally:
            stop.set()
            th.join()
    assert not errors, errors
    assert st1 > st0, "the training loop did not run alongside the serving batches"
    assert res["failed"] == 0 and res["body_mismatches"] == 0 and res["status_counts"] == {200: 48 * 400}, res
    nb = s1["batches"] - s0["batches"]
    assert s1["path_batches"]["wide"] - s0["path_batches"]["wide"] == nb and nb < 48 * 400  # coalesced, WIDE
    assert s1["errors"] == s0["errors"]
