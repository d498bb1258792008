"""Training: L-BFGS parity with sklearn, estimator API, notebook CLI, SGD checkpoint/resume."""
import json
import os
import pickle
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

ENV = {**os.environ, "PYTHONPATH": str(ROOT)}


def test_lbfgs_binary_matches_sklearn(iris_data):
    from sklearn.linear_model import LogisticRegression as SK

    from mlapi_amd.train.lbfgs import fit_logistic_lbfgs

    Xtr, _, ytr, _ = iris_data
    yb = (ytr == "Iris-versicolor")
    sk = SK().fit(Xtr, yb)
    m = fit_logistic_lbfgs(Xtr, yb)
    np.testing.assert_allclose(m.W, sk.coef_, atol=1e-6)
    np.testing.assert_allclose(m.b, sk.intercept_, atol=1e-6)


def test_lbfgs_multinomial_reproduces_notebook(iris_data):
    """`Logistic Regression.ipynb:13`: hold-out accuracy 0.9666666666666667."""
    from sklearn.linear_model import LogisticRegression as SK

    from mlapi_amd.models.estimator import LogisticRegression

    Xtr, Xte, ytr, yte = iris_data
    ours = LogisticRegression(device="cpu").fit(Xtr, ytr)
    sk = SK().fit(Xtr, ytr)
    assert ours.score(Xte, yte) == 0.9666666666666667
    np.testing.assert_array_equal(ours.predict(Xte), sk.predict(Xte))
    np.testing.assert_allclose(ours.predict_proba(Xte), sk.predict_proba(Xte), atol=2e-3)
    assert list(ours.classes_) == ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]


def test_lbfgs_ovr(iris_data):
    from sklearn.linear_model import LogisticRegression as SK
    from sklearn.multiclass import OneVsRestClassifier

    from mlapi_amd.train.lbfgs import fit_logistic_lbfgs

    Xtr, Xte, ytr, _ = iris_data
    m = fit_logistic_lbfgs(Xtr, ytr, multi_class="ovr")
    sk = OneVsRestClassifier(SK()).fit(Xtr, ytr)
    np.testing.assert_array_equal(m.predict(Xte), sk.predict(Xte))


def test_estimator_save_formats(tmp_path, iris_data):
    from mlapi_amd.models.estimator import LogisticRegression

    Xtr, Xte, ytr, yte = iris_data
    clf = LogisticRegression(device="cpu").fit(Xtr, ytr)
    clf.save(str(tmp_path / "a.pkl"))
    clf.save(str(tmp_path / "a.safetensors"), format="native")
    for p in ("a.pkl", "a.safetensors"):
        assert LogisticRegression.load(str(tmp_path / p), device="cpu").score(Xte, yte) == clf.score(Xte, yte)
    sk = pickle.loads((tmp_path / "a.pkl").read_bytes())  # our own file, readable by real sklearn
    np.testing.assert_array_equal(sk.predict(Xte), clf.predict(Xte))


def test_cli_iris_prints_reference_score(tmp_path):
    out = subprocess.run([sys.executable, "-m", "mlapi_amd.train", "iris", "--device", "cpu"], cwd=tmp_path, env=ENV,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == "0.9666666666666667"
    assert (tmp_path / "LRClassifier.pkl").exists()


def test_cli_sgd_checkpoint_resume(tmp_path):
    ck = str(tmp_path / "s.safetensors")
    base = [sys.executable, "-m", "mlapi_amd.train", "sgd", "--features", "16", "--rows-per-rank", "8000",
            "--batch", "1000", "--log-every", "1000", "--ckpt", ck, "--ckpt-every", "20"]
    env = {**ENV, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}
    full = subprocess.run(base + ["--steps", "40"], env=env, capture_output=True, text=True, timeout=300)
    assert full.returncode == 0, full.stderr
    final_full = json.loads(full.stdout.strip().splitlines()[-1])
    os.remove(ck)
    a = subprocess.run(base + ["--steps", "20"], env=env, capture_output=True, text=True, timeout=300)
    assert a.returncode == 0, a.stderr
    b = subprocess.run(base + ["--steps", "40", "--resume"], env=env, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0 and "resumed" in b.stdout, b.stdout + b.stderr
    final_resumed = json.loads(b.stdout.strip().splitlines()[-1])
    assert final_resumed["final_loss"] == pytest.approx(final_full["final_loss"], rel=1e-6)


@pytest.mark.gpu
def test_lbfgs_gpu_kernel_path_matches_cpu(iris_data):
    import torch

    from mlapi_amd.train.lbfgs import fit_logistic_lbfgs

    Xtr, Xte, ytr, yte = iris_data
    cpu = fit_logistic_lbfgs(Xtr, ytr)
    gpu = fit_logistic_lbfgs(Xtr, ytr, device=torch.device("cuda", 0))
    # same optimizer + objective; the ill-conditioned multinomial Iris problem amplifies last-bit
    # differences of the objective sums (GPU tree order vs numpy) like it does vs sklearn itself
    np.testing.assert_allclose(gpu.W, cpu.W, atol=1e-2)
    np.testing.assert_array_equal(gpu.predict(Xte), cpu.predict(Xte))
    assert gpu.score(Xte, yte) == 0.9666666666666667
    yb = ytr == "Iris-versicolor"  # well-conditioned binary problem: tight agreement
    np.testing.assert_allclose(fit_logistic_lbfgs(Xtr, yb, device=torch.device("cuda", 0)).W,
                               fit_logistic_lbfgs(Xtr, yb).W, atol=1e-6)


@pytest.mark.gpu
def test_estimator_gpu_predict_and_sgd(iris_data):
    from mlapi_amd.models.estimator import LogisticRegression

    Xtr, Xte, ytr, yte = iris_data
    clf = LogisticRegression(device="cuda").fit(Xtr, ytr)
    assert clf.score(Xte, yte) == 0.9666666666666667
    sgd = LogisticRegression(device="cuda", solver="sgd").fit(Xtr, ytr == "Iris-setosa")
    assert sgd.score(Xte, yte == "Iris-setosa") == 1.0
    mc = LogisticRegression(device="cuda", solver="sgd", lr=0.05, batch_size=20, epochs=200).fit(Xtr, ytr)
    assert mc.score(Xte, yte) >= 0.9


def test_softmax_ref_gradient_matches_autograd():
    """The multiclass oracle (also the trainer's CPU path) is the true gradient of the objective."""
    import torch

    from mlapi_amd.models.linear import Kind
    from mlapi_amd.ops.reference import softmax_train_ref

    torch.manual_seed(0)
    X, y = torch.randn(64, 10, dtype=torch.float64), torch.randint(0, 5, (64,), dtype=torch.int32)
    for kind in (Kind.MULTINOMIAL, Kind.OVR):
        W = torch.randn(5, 10, dtype=torch.float64, requires_grad=True)
        z = X @ W.T
        Y = torch.nn.functional.one_hot(y.long(), 5).double()
        if kind == Kind.MULTINOMIAL:
            loss = (torch.logsumexp(z, 1) - (z * Y).sum(1)).sum()
        else:
            loss = torch.nn.functional.binary_cross_entropy_with_logits(z, Y, reduction="sum")
        loss.backward()
        _, dW, lref, _ = softmax_train_ref(X, y, W.detach(), kind, dtype=torch.float64)
        torch.testing.assert_close(dW, W.grad)
        assert float(lref) == pytest.approx(float(loss.detach()), rel=1e-12)


@pytest.mark.parametrize("kind_name", ["MULTINOMIAL", "OVR"])
def test_softmax_sgd_cpu_learns(kind_name):
    import torch

    from mlapi_amd.models.linear import Kind
    from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass

    X, y = synthetic_multiclass(6000, 32, 7, seed=1, noise=0.3)
    tr = SoftmaxSGDTrainer(32, 7, kind=Kind[kind_name], lr=0.5, momentum=0.9, device=torch.device("cpu"))
    Xa = tr.prepare(X)
    assert Xa.shape == (6000, 136) and torch.all(Xa[:, 128] == 1)  # F=32 trains zero-padded to 128
    for s in range(60):
        lo = (s * 500) % 5000
        tr.step(Xa[lo:lo + 500], y[lo:lo + 500])
    loss, acc = tr.evaluate(Xa[5000:], y[5000:])
    assert acc > 0.8, (loss, acc)
    m = tr.to_model()
    pred = m.predict(X[5000:].double().numpy())
    assert np.mean(pred == y[5000:].numpy()) == pytest.approx(acc, abs=0.01)  # f64 model vs f32 training math


def test_estimator_sgd_multiclass_cpu(iris_data):
    from mlapi_amd.models.estimator import LogisticRegression

    Xtr, Xte, ytr, yte = iris_data
    clf = LogisticRegression(solver="sgd", device="cpu", lr=0.05, batch_size=20, epochs=200).fit(Xtr, ytr)
    assert list(clf.classes_) == ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]
    assert clf.coef_.shape == (3, 4)
    assert clf.score(Xte, yte) >= 0.9


def test_cli_sgd_multiclass_checkpoint_resume(tmp_path):
    ck = str(tmp_path / "m.safetensors")
    base = [sys.executable, "-m", "mlapi_amd.train", "sgd", "--features", "32", "--classes", "5",
            "--rows-per-rank", "4000", "--batch", "500", "--log-every", "1000", "--ckpt", ck, "--ckpt-every", "10",
            "--noise", "0.3"]
    env = {**ENV, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}
    full = subprocess.run(base + ["--steps", "20"], env=env, capture_output=True, text=True, timeout=300)
    assert full.returncode == 0, full.stderr
    final_full = json.loads(full.stdout.strip().splitlines()[-1])
    assert final_full["classes"] == 5 and final_full["final_acc"] > 0.5
    os.remove(ck)
    a = subprocess.run(base + ["--steps", "10"], env=env, capture_output=True, text=True, timeout=300)
    assert a.returncode == 0, a.stderr
    b = subprocess.run(base + ["--steps", "20", "--resume", "--out", str(tmp_path / "m.pkl")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0 and "resumed" in b.stdout, b.stdout + b.stderr
    final_resumed = json.loads(b.stdout.strip().splitlines()[-1])
    assert final_resumed["final_loss"] == pytest.approx(final_full["final_loss"], rel=1e-6)
    sk = pickle.loads((tmp_path / "m.pkl").read_bytes())  # our own export, readable by sklearn
    assert sk.coef_.shape == (5, 32)


def test_batch_schedule_resume_visits_the_same_batches():
    from mlapi_amd.train.schedule import BatchSchedule

    full = BatchSchedule(7, seed=3)
    seq = [full.next() for _ in range(30)]
    assert sorted(seq[:7]) == list(range(7)) and seq[:7] != list(range(7))  # a permutation per epoch
    a = BatchSchedule(7, seed=3)
    head = [a.next() for _ in range(17)]
    b = BatchSchedule(7, seed=99)  # a fresh process with the checkpointed state
    b.restore(a.epoch, a.cursor, a.rng_state())
    assert head + [b.next() for _ in range(13)] == seq


def test_cli_sgd_checkpoint_holds_rng_and_cursor(tmp_path):
    from mlapi_amd.ckpt.native import load_native

    ck = str(tmp_path / "s.safetensors")
    env = {**ENV, "CUDA_VISIBLE_DEVICES": "", "HIP_VISIBLE_DEVICES": ""}
    out = subprocess.run([sys.executable, "-m", "mlapi_amd.train", "sgd", "--features", "8", "--rows-per-rank", "3000",
                          "--batch", "1000", "--steps", "7", "--ckpt", ck, "--ckpt-every", "7", "--log-every", "100"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    _, st = load_native(ck)
    assert (st.step, st.epoch, st.data_cursor) == (7, 2, 1)  # 3 batches per epoch
    assert st.rng_state is not None and st.rng_state.dtype == np.uint8 and st.rng_state.size > 0
