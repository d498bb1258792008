"""R7 parity: notebooks/Logistic Regression.ipynb (the reference notebook's recipe on mlapi_amd) runs
and prints the reference's recorded score (`Logistic Regression.ipynb:13`: 0.9666666666666667).
Code cells are executed in order in one namespace (nbformat/jupyter are not installed)."""
import contextlib
import io
import json
import os

from conftest import ROOT


def test_notebook_reproduces_reference_score(tmp_path):
    nb = json.loads((ROOT / "notebooks" / "Logistic Regression.ipynb").read_text())
    assert nb["nbformat"] == 4
    code = ["".join(c["source"]) for c in nb["cells"] if c["cell_type"] == "code"]
    assert code, "notebook has no code cells"
    out = io.StringIO()
    cwd = os.getcwd()
    os.chdir(tmp_path)
    try:
        ns = {"__name__": "__main__"}
        with contextlib.redirect_stdout(out):
            for src in code:
                exec(compile(src, "Logistic Regression.ipynb", "exec"), ns)
    finally:
        os.chdir(cwd)
    assert out.getvalue().strip().splitlines()[-1] == "0.9666666666666667"
    assert (tmp_path / "LRClassifier.pkl").exists()
