"""Capture the reference app's HTTP behaviour as a golden fixture (run once, offline).

Runs an unmodified copy of the reference `main.py` (path given on the command line; nothing from
it is imported into this repo) under FastAPI's TestClient inside a scratch directory that holds:
  * `LRClassifier.pkl` produced by the notebook recipe (`Logistic Regression.ipynb:24-37`) on
    sklearn's bundled Iris relabelled to the UCI strings (the UCI URL is unreachable offline);
  * an empty stub `python_multipart` package, only so FastAPI's import check for `/files/`
    passes (`/predict` never touches it; `/files/` cases are therefore not captured here).

Writes tests/fixtures/reference_contract.json: a list of {name, request, status, content_type,
body} for SURVEY Appendix A cases A1-A15 and A18 (openapi.json).

Usage: python tools/capture_reference_contract.py /root/reference/main.py
"""
from __future__ import annotations

import json
import os
import pickle
import shutil
import sys
import tempfile
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent

CASES = [
    ("A1", "POST", "/predict", {"json": {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": 0.2}}),
    ("A2", "POST", "/predict", {"json": {"sepal_length": 6.7, "sepal_width": 3.0, "petal_length": 5.2, "petal_width": 2.3}}),
    ("A3", "POST", "/predict", {"json": {"sepal_length": "5.1", "sepal_width": "3.5", "petal_length": "1.4", "petal_width": "0.2"}}),
    ("A4", "POST", "/predict", {"json": {"sepal_length": 5, "sepal_width": 3, "petal_length": 1, "petal_width": 0}}),
    ("A5", "POST", "/predict", {"json": {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": 0.2, "foo": 1}}),
    ("A6", "POST", "/predict", {"json": {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4}}),
    ("A7", "POST", "/predict", {"json": {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": "abc"}}),
    ("A8", "POST", "/predict", {"json": {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": None}}),
    ("A9", "POST", "/predict", {"content": b"hello", "headers": {"content-type": "application/json"}}),
    ("A10", "POST", "/predict", {"json": [1, 2, 3, 4]}),
    ("A11", "POST", "/predict", {"content": b'{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
                                 "headers": {"content-type": "text/plain"}}),
    ("A12", "POST", "/predict", {"content": b'{"sepal_length":NaN,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}',
                                 "headers": {"content-type": "application/json"}}),
    ("A13", "POST", "/predict", {"json": {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": 1e308}}),
    ("A14", "GET", "/predict", {}),
    ("A15", "GET", "/nope", {}),
    ("A18", "GET", "/openapi.json", {}),
    ("A1b", "POST", "/predict", {"content": b'{"petal_width": 0.2, "petal_length": 1.4, "sepal_width": 3.5, "sepal_length": 5.1}',
                                 "headers": {"content-type": "application/json; charset=utf-8"}}),
    ("A1c", "POST", "/predict", {"content": b'{"sepal_length":4.9,"sepal_width":3.0,"petal_length":1.4,"petal_width":0.2,"sepal_length":7.7}',
                                 "headers": {"content-type": "application/json"}}),
]


def make_iris_pickle(path: Path) -> None:
    import numpy as np
    from sklearn.datasets import load_iris
    from sklearn.linear_model import LogisticRegression
    from sklearn.model_selection import train_test_split

    d = load_iris()
    names = np.array(["Iris-setosa", "Iris-versicolor", "Iris-virginica"], dtype=object)
    X, y = d.data.astype(object), names[d.target]
    Xtr, _, ytr, _ = train_test_split(X, y, test_size=0.20, random_state=1, shuffle=True)
    with open(path, "wb") as f:
        pickle.dump(LogisticRegression().fit(Xtr, ytr), f)


def main(ref_main: str) -> None:
    scratch = Path(tempfile.mkdtemp(prefix="refcap_"))
    (scratch / "stub" / "python_multipart").mkdir(parents=True)
    (scratch / "stub" / "python_multipart" / "__init__.py").write_text('__version__ = "0.0.20"\n')
    shutil.copy(ref_main, scratch / "ref_main.py")
    make_iris_pickle(scratch / "LRClassifier.pkl")
    sys.path[:0] = [str(scratch / "stub"), str(scratch)]
    os.chdir(scratch)
    from fastapi.testclient import TestClient

    import ref_main  # noqa: E402

    client = TestClient(ref_main.app, raise_server_exceptions=False)
    out = []
    for name, method, path, kw in CASES:
        r = client.request(method, path, **kw)
        req = {"method": method, "path": path}
        if "json" in kw:
            req["json"] = kw["json"]
        if "content" in kw:
            req["content"] = kw["content"].decode()
        if "headers" in kw:
            req["headers"] = kw["headers"]
        out.append({"name": name, "request": req, "status": r.status_code,
                    "content_type": r.headers.get("content-type"), "body": r.content.decode()})
    dst = REPO / "tests" / "fixtures" / "reference_contract.json"
    dst.parent.mkdir(parents=True, exist_ok=True)
    dst.write_text(json.dumps(out, indent=1) + "\n")  # key order preserved: 422 bodies echo it
    print(f"wrote {len(out)} cases to {dst}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/main.py")
