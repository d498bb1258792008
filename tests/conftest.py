import os
import pickle
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
FIXTURES = ROOT / "tests" / "fixtures"
IRIS_LABELS = np.array(["Iris-setosa", "Iris-versicolor", "Iris-virginica"], dtype=object)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def iris_split():
    """The notebook's data recipe (`Logistic Regression.ipynb:24-31`) on sklearn's bundled Iris."""
    from sklearn.datasets import load_iris
    from sklearn.model_selection import train_test_split

    d = load_iris()
    X, y = d.data.astype(object), IRIS_LABELS[d.target]
    return train_test_split(X, y, test_size=0.20, random_state=1, shuffle=True)


@pytest.fixture(scope="session")
def iris_data():
    Xtr, Xte, ytr, yte = iris_split()
    return Xtr.astype(np.float64), Xte.astype(np.float64), ytr, yte


@pytest.fixture(scope="session")
def iris_sklearn_model():
    from sklearn.linear_model import LogisticRegression

    Xtr, _, ytr, _ = iris_split()
    return LogisticRegression().fit(Xtr, ytr)


@pytest.fixture(scope="session")
def iris_pickle_bytes(iris_sklearn_model):
    return pickle.dumps(iris_sklearn_model, protocol=4)


@pytest.fixture
def iris_cwd(tmp_path, iris_pickle_bytes, monkeypatch):
    """A CWD holding LRClassifier.pkl, as the reference expects (`main.py:19`)."""
    (tmp_path / "LRClassifier.pkl").write_bytes(iris_pickle_bytes)
    monkeypatch.chdir(tmp_path)
    return tmp_path


@pytest.fixture(scope="session")
def native():
    from mlapi_amd._native import C, available

    if not available():
        pytest.skip("native extension not built")
    return C()
