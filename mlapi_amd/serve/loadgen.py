"""Benchmark client side: validated /predict workloads and the out-of-process load generator.

The reference ships no benchmark; BASELINE.md measured it with a single aiohttp client that
caps at ~7.4k req/s. The framework's load generator is native (csrc/http/loadgen.cpp) and runs
either in-process (``_C.Loadgen``) or as its own process (``mlapi_amd/bin/mlapi-loadgen``,
:class:`LoadgenProcess`) so a benchmark rank can pin it to CPUs apart from its server, and a
data-parallel run drives the shared SO_REUSEPORT port like external clients would.

Every response is checked: :func:`make_workload` renders N distinct request bodies together with
the exact response each must produce (computed by the serving engine itself and cross-checked
against the float64 oracle), and the load generator counts any other body as a failure.
"""
from __future__ import annotations

import json
import os
import subprocess
import tempfile
from typing import List, Optional, Sequence, Tuple

import numpy as np

from mlapi_amd.models.linear import LinearModel


def render_request(names: Sequence[str], row, path: str = "/predict") -> bytes:
    body = json.dumps({n: float(v) for n, v in zip(names, row)}, separators=(",", ":")).encode()
    return (b"POST %s HTTP/1.1\r\nHost: 127.0.0.1\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
            % (path.encode(), len(body), body))


def render_response(model: LinearModel, idx: int, p: float) -> bytes:
    from mlapi_amd._native import C

    return ('{"prediction":%s,"probability":%s}' % (model.label_json()[int(idx)], C().py_float_repr(float(p)))).encode()


def bf16_round(a) -> np.ndarray:
    """float64 values rounded to bfloat16 (nearest even), as the bf16 serving kernels see them."""
    u = np.ascontiguousarray(np.asarray(a, dtype=np.float32)).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def bf16_oracle(model: LinearModel, X) -> Tuple[LinearModel, np.ndarray]:
    """The model and rows exactly as the bf16 GEMV / GEMM paths read them (f32 intercept)."""
    om = LinearModel(bf16_round(model.W), model.b.astype(np.float32).astype(np.float64), model.classes, model.kind)
    return om, bf16_round(X)


def make_workload(engine, model: LinearModel, names: Sequence[str], X: np.ndarray, *,
                  rtol_oracle: float = 1e-12, label_margin: float = 0.0,
                  oracle: Optional[Tuple[LinearModel, np.ndarray]] = None) -> Tuple[List[bytes], List[bytes]]:
    """(requests, expected bodies) for the rows of X. Expected bodies come from ``engine.predict``
    (the serving kernel the server will run); they are first checked against the float64 oracle
    (``oracle`` = (model, rows) as the kernel reads them, default the exact ones; labels exact
    unless the top-2 logit margin is below ``label_margin``; p within rtol_oracle)."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    idx, p, st = engine.predict(X)
    if not (st == 0).all():
        raise RuntimeError(f"engine failed {int((st != 0).sum())} workload rows")
    om, Xo = oracle if oracle is not None else (model, X)
    ridx, rp = om.predict_max(Xo)
    z = om.decision_function(Xo)
    if z.ndim == 1:
        margin = np.abs(z)
    else:
        zs = np.sort(z, axis=1)
        margin = zs[:, -1] - zs[:, -2]
    bad = (idx != ridx) & (margin > label_margin)
    if bad.any():
        raise RuntimeError(f"engine labels differ from the oracle on {int(bad.sum())} rows")
    np.testing.assert_allclose(p, rp, rtol=rtol_oracle, atol=1e-7 if rtol_oracle > 1e-9 else 0)
    reqs = [render_request(names, row) for row in X]
    exp = [render_response(model, i, q) for i, q in zip(idx, p)]
    return reqs, exp


def write_workload(path: str, requests: Sequence[bytes], expected: Sequence[bytes]) -> None:
    with open(path, "wb") as f:
        f.write(b"MLW1\n")
        for r, e in zip(requests, expected):
            f.write(b"%d %d\n" % (len(r), len(e)))
            f.write(r)
            f.write(e)


def binary_path() -> str:
    from mlapi_amd._build import loadgen_path

    p = str(loadgen_path())
    if not os.path.exists(p):
        raise RuntimeError(f"{p} is missing: run python -m mlapi_amd._build")
    return p


class LoadgenProcess:
    """One ``mlapi-loadgen`` child process, driven over its stdin/stdout line protocol.

    Start it before the GPU is touched (it is a plain fork+exec child, it never uses the GPU)."""

    def __init__(self):
        self.proc = subprocess.Popen([binary_path()], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                     bufsize=1)
        self._tmp: Optional[str] = None

    @property
    def pid(self) -> int:
        return self.proc.pid

    def cmd(self, line: str) -> dict:
        assert self.proc.stdin is not None and self.proc.stdout is not None
        self.proc.stdin.write(line + "\n")
        self.proc.stdin.flush()
        out = self.proc.stdout.readline()
        if not out:
            raise RuntimeError(f"mlapi-loadgen exited (rc={self.proc.poll()}) on {line!r}")
        r = json.loads(out)
        if not r.get("ok"):
            raise RuntimeError(f"mlapi-loadgen: {r.get('error')} ({line!r})")
        return r

    def pin(self, cpus: Sequence[int]) -> dict:
        return self.cmd("pin " + ",".join(str(c) for c in cpus)) if cpus else {"ok": True, "cpus": 0}

    def workload(self, requests: Sequence[bytes], expected: Sequence[bytes], rel_tol: float = 0.0) -> dict:
        fd, path = tempfile.mkstemp(prefix="mlapi-workload-", suffix=".bin")
        os.close(fd)
        write_workload(path, requests, expected)
        try:
            return self.cmd(f"workload {path} {rel_tol!r}")
        finally:
            os.unlink(path)

    def connect(self, host: str, port: int, conns: int, threads: int, timeout_s: float = 60.0,
                source: str = "") -> dict:
        """source: local IPv4 address to connect from ("" = the kernel's choice)."""
        return self.cmd(f"connect {host} {int(port)} {int(conns)} {int(threads)} {timeout_s} {source or '-'}")

    def conn_map(self, mode: str, seed: int = 1) -> dict:
        """rr: connection c on load-generator thread c % threads (connect order); shuffle: a seeded
        permutation, so a thread's connections are not paired with the server's IO threads."""
        return self.cmd(f"connmap {mode} {int(seed)}")

    def thread_cpus(self, cpus: Sequence[int]) -> dict:
        """Pin client thread i to cpus[i] for the following runs ([] = keep the process mask)."""
        return self.cmd("threadcpus " + (",".join(str(c) for c in cpus) if cpus else "-"))

    def run(self, requests_per_conn: int, record: bool = True) -> dict:
        return self.cmd(f"run {int(requests_per_conn)} {1 if record else 0}")

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.cmd("quit")
            except Exception:
                pass
            try:
                self.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
