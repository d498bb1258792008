"""T5: multi-process semantics on CPU with gloo (world_size 2), via torchrun."""
import json
import signal
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import numpy as np
import pytest

from conftest import ROOT

ENV = {**os.environ, "PYTHONPATH": str(ROOT), "OMP_NUM_THREADS": "1", "CUDA_VISIBLE_DEVICES": "",
       "HIP_VISIBLE_DEVICES": ""}


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def torchrun(nproc: int, script: str, env: dict, cwd=None, timeout=240, args=()):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", script, *args]
    return subprocess.Popen(cmd, env={**ENV, **env}, cwd=cwd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                            text=True)


def run(nproc, script, env, timeout=240, args=(), cwd=None):
    # free_port() releases its port before torchrun binds it: another process's ephemeral socket
    # (gloo opens many) can take it in between. Only that rendezvous failure is retried, on a new port.
    for attempt in range(3):
        p = torchrun(nproc, script, env, args=args, cwd=cwd)
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
            raise AssertionError("torchrun timed out:\n" + out[-3000:])
        if p.returncode != 0 and "EADDRINUSE" in out and attempt < 2:
            continue
        assert p.returncode == 0, out[-3000:]
        return out


def test_broadcast_and_dp_sgd_determinism(tmp_path):
    script = str(ROOT / "tests" / "dist" / "bcast_train.py")
    run(1, script, {"OUT": str(tmp_path)})
    run(2, script, {"OUT": str(tmp_path)})
    b0 = json.loads((tmp_path / "bcast_2_0.json").read_text())
    b1 = json.loads((tmp_path / "bcast_2_1.json").read_text())
    assert b0["W"] == b1["W"] and b0["b"] == b1["b"] and b0["classes"] == b1["classes"] == list("abcde")
    p0, p1 = np.load(tmp_path / "params_2_0.npy"), np.load(tmp_path / "params_2_1.npy")
    assert np.array_equal(p0, p1), "DP replicas must stay bitwise identical"
    single = np.load(tmp_path / "params_1_0.npy")
    np.testing.assert_allclose(p0, single, rtol=1e-4, atol=1e-5)  # DP == single-process on the global batch
    assert b0["acc"] > 0.8
    m0, m1 = np.load(tmp_path / "mc_params_2_0.npy"), np.load(tmp_path / "mc_params_2_1.npy")
    assert np.array_equal(m0, m1), "multiclass DP replicas must stay bitwise identical"
    np.testing.assert_allclose(m0, np.load(tmp_path / "mc_params_1_0.npy"), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world", [4, 8])
def test_dp_sgd_determinism_more_ranks(tmp_path, world):
    """N ranks == 1 rank on the same global batch (binary and multiclass), N = 4, 8."""
    script = str(ROOT / "tests" / "dist" / "bcast_train.py")
    run(1, script, {"OUT": str(tmp_path)})
    run(world, script, {"OUT": str(tmp_path)}, timeout=300)
    for name in ("params", "mc_params"):
        ranks = [np.load(tmp_path / f"{name}_{world}_{r}.npy") for r in range(world)]
        assert all(np.array_equal(ranks[0], x) for x in ranks[1:]), "replicas must stay bitwise identical"
        np.testing.assert_allclose(ranks[0], np.load(tmp_path / f"{name}_1_0.npy"), rtol=1e-4, atol=1e-5)


def test_fake_comm_collectives(tmp_path):
    """The framework communicator API (NativeComm's twin) over gloo, world_size 2 and 1."""
    script = str(ROOT / "tests" / "dist" / "comm_semantics.py")
    for n in (2, 1):
        run(n, script, {"OUT": str(tmp_path), "MLAPI_COMM": "fake"})
        for r in range(n):
            assert (tmp_path / f"OK_{r}").read_text() == "fake-gloo"
            (tmp_path / f"OK_{r}").unlink()


@pytest.mark.parametrize("world,comm", [(1, "torch"), (2, "torch"), (3, "fake")])
def test_tensor_parallel_matches_oracle(tmp_path, world, comm):
    """Class-sharded (TP over K) and feature-sharded (split-F) predict == the unsharded oracle."""
    run(world, str(ROOT / "tests" / "dist" / "tensor_parallel.py"), {"OUT": str(tmp_path), "MLAPI_COMM": comm})
    for r in range(world):
        assert (tmp_path / f"TP_OK_{r}").read_text() == str(world)


def test_shard_bounds():
    from mlapi_amd.parallel.tensor_parallel import shard_bounds

    assert shard_bounds(10, 3) == [(0, 4), (4, 7), (7, 10)]
    assert shard_bounds(4, 4) == [(0, 1), (1, 2), (2, 3), (3, 4)]
    assert shard_bounds(2, 3)[-1] == (2, 2)


def test_dp_sgd_through_fake_comm(tmp_path):
    script = str(ROOT / "tests" / "dist" / "bcast_train.py")
    run(2, script, {"OUT": str(tmp_path), "MLAPI_COMM": "fake"})
    p0, p1 = np.load(tmp_path / "mc_params_2_0.npy"), np.load(tmp_path / "mc_params_2_1.npy")
    assert np.array_equal(p0, p1)


def test_launcher_pins_and_runs_collectives(tmp_path):
    """python -m mlapi_amd.launch: rank env, disjoint CPU slices, store bootstrap, collectives."""
    from mlapi_amd.launch import cpu_slices

    assert cpu_slices(3, list(range(8))) == [[0, 1, 2], [3, 4, 5], [6, 7]]
    launch = [sys.executable, "-m", "mlapi_amd.launch", "--nproc", "2"]
    out = subprocess.run(launch[:-2] + ["--nproc", "2", "--pin", "cores", str(ROOT / "tests" / "dist" / "affinity.py")],
                         env={**ENV, "OUT": str(tmp_path)}, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    a = [json.loads((tmp_path / f"aff_{r}.json").read_text()) for r in range(2)]
    assert [x["rank"] for x in a] == [0, 1] and all(x["world"] == 2 for x in a)
    assert not set(a[0]["cpus"]) & set(a[1]["cpus"])
    assert a[0]["omp"] == str(len(a[0]["cpus"]))
    # default at N > 1: each rank on its GPU's NUMA node (tests/test_affinity.py); without the KFD
    # topology in sysfs (this container) the ranks are left unpinned rather than guessed
    import os

    if not os.path.isdir("/sys/class/kfd/kfd/topology/nodes"):
        out = subprocess.run(launch + [str(ROOT / "tests" / "dist" / "affinity.py")], env={**ENV, "OUT": str(tmp_path)},
                             capture_output=True, text=True, timeout=120)
        assert out.returncode == 0, out.stderr
        a = [json.loads((tmp_path / f"aff_{r}.json").read_text()) for r in range(2)]
        assert sorted(a[0]["cpus"]) == sorted(os.sched_getaffinity(0)) == sorted(a[1]["cpus"])
    out = subprocess.run(launch + [str(ROOT / "tests" / "dist" / "comm_semantics.py")],
                         env={**ENV, "OUT": str(tmp_path), "MLAPI_COMM": "fake"}, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr[-3000:]
    assert (tmp_path / "OK_1").read_text() == "fake-gloo"


def test_launcher_propagates_failure(tmp_path):
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, "-m", "mlapi_amd.launch", "--nproc", "2", "--grace", "2",
                          str(ROOT / "tests" / "dist" / "affinity.py")],
                         env={**ENV, "OUT": str(tmp_path), "FAIL_RANK": "1"}, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 7, out.stderr
    assert time.monotonic() - t0 < 30  # the sleeping rank was stopped, not waited for
    assert "rank 1 exited with 7" in out.stderr


def test_dp_serving_reload(tmp_path, iris_pickle_bytes):
    import httpx

    from mlapi_amd.ckpt import export_sklearn_pickle, load_sklearn_pickle

    (tmp_path / "LRClassifier.pkl").write_bytes(iris_pickle_bytes)
    base = free_port()
    while base + 1 == 0:
        base = free_port()
    p = torchrun(2, str(ROOT / "tests" / "dist" / "dp_serve.py"), {"OUT": str(tmp_path), "BASE_PORT": str(base)},
                 cwd=str(tmp_path))
    try:
        t0 = time.time()
        while not all((tmp_path / f"ready_{r}").exists() for r in (0, 1)):
            assert p.poll() is None, p.stdout.read()
            assert time.time() - t0 < 90
            time.sleep(0.1)
        a1 = {"sepal_length": 5.1, "sepal_width": 3.5, "petal_length": 1.4, "petal_width": 0.2}
        for r in (0, 1):
            res = httpx.post(f"http://127.0.0.1:{base + r}/predict", json=a1)
            assert res.json()["prediction"] == "Iris-setosa"
        m = load_sklearn_pickle(iris_pickle_bytes)
        m.b = m.b + np.array([-100.0, 0.0, 100.0])
        export_sklearn_pickle(m, tmp_path / "LRClassifier.pkl")
        deadline = time.time() + 20
        seen = set()
        while time.time() < deadline and len(seen) < 2:
            for r in (0, 1):
                if httpx.post(f"http://127.0.0.1:{base + r}/predict", json=a1).json()["prediction"] == "Iris-virginica":
                    seen.add(r)
            time.sleep(0.05)
        assert seen == {0, 1}, "both replicas must switch to the new weights (broadcast from rank 0)"
        os.remove(tmp_path / "LRClassifier.pkl")
        deadline = time.time() + 20
        codes = set()
        while time.time() < deadline and codes != {500}:
            codes = {httpx.post(f"http://127.0.0.1:{base + r}/predict", json=a1).status_code for r in (0, 1)}
            time.sleep(0.05)
        assert codes == {500}
    finally:
        (tmp_path / "stop").touch()
        try:
            out, _ = p.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
    assert p.returncode == 0, out[-3000:]


def test_bench_contract_two_ranks():
    out = run(2, str(ROOT / "bench.py"), {}, args=["--cpu", "--gpus", "2", "--steps", "10", "--warmup", "2",
                                                   "--c1-requests", "200", "--reqs-per-conn", "512"])
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["value"] > 0


def _post_new_conn(port, body):
    """One request on a NEW connection (SO_REUSEPORT balances connections, not requests)."""
    s = socket.create_connection(("127.0.0.1", port), timeout=10)
    try:
        s.sendall(b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\nConnection: close\r\n"
                  b"Content-Length: %d\r\n\r\n%s" % (len(body), body))
        data = b""
        while True:
            c = s.recv(65536)
            if not c:
                break
            data += c
        return int(data.split()[1])
    except (ConnectionError, IndexError):
        return 0
    finally:
        s.close()


def test_dp_health_dispatch_drops_and_readmits_rank(tmp_path, iris_pickle_bytes):
    """3 CPU ranks share one port; rank 1 is fault-injected ("drop a rank"). Once it has left the
    SO_REUSEPORT group, clients see 100% 200s; after recovery the probe re-admits it."""
    (tmp_path / "LRClassifier.pkl").write_bytes(iris_pickle_bytes)
    port = free_port()
    p = torchrun(3, str(ROOT / "tests" / "dist" / "dp_health.py"),
                 {"OUT": str(tmp_path), "PORT": str(port), "MLAPI_FAULT_DROP_RANK": "1"}, cwd=str(tmp_path))
    body = b'{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}'

    def state(r):
        try:
            return json.loads((tmp_path / f"state_{r}").read_text())
        except (OSError, ValueError):
            return None

    try:
        t0 = time.time()
        while not (all(state(r) for r in range(3)) and state(1)["listen_closes"] >= 1):
            assert p.poll() is None, p.stdout.read()
            assert time.time() - t0 < 90, [state(r) for r in range(3)]
            time.sleep(0.1)
        time.sleep(0.25)  # the group's acceptor learns of it over the member channel (<= one poll period)
        s1 = state(1)
        assert not s1["accepting"] and s1["listeners"] == 0 and not s1["healthy"]
        assert 'mlapi_engine_healthy{rank="1",backend="cpu"} 0' in s1["metrics"]
        assert 'mlapi_rank_accepting{rank="1",backend="cpu"} 0' in s1["metrics"]
        codes = [_post_new_conn(port, body) for _ in range(300)]
        assert codes == [200] * 300, {c: codes.count(c) for c in set(codes)}
        (tmp_path / "recover").touch()
        t0 = time.time()
        while not (state(1)["accepting"] and state(1)["listeners"] == 2):
            assert time.time() - t0 < 30, state(1)
            time.sleep(0.05)
        time.sleep(0.2)
        served = [state(r)["requests"] for r in range(3)]
        codes = [_post_new_conn(port, body) for _ in range(300)]
        assert codes == [200] * 300, {c: codes.count(c) for c in set(codes)}
        time.sleep(0.2)
        assert state(1)["requests"] > served[1], "re-admitted rank must receive connections again"
        assert state(0)["requests"] > served[0] and state(2)["requests"] > served[2]
    finally:
        (tmp_path / "stop").touch()
        try:
            out, _ = p.communicate(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
    assert p.returncode == 0, out[-3000:]


def test_launcher_restarts_a_crashed_replica(tmp_path, iris_pickle_bytes):
    """`mlapi_amd.launch --restart 1`, 3 CPU serving ranks on one port: rank 1 dies while serving
    (fault injection). Clients keep getting 200s from the survivors, the launcher brings rank 1 back
    as a standalone replica, and a replaced checkpoint is then picked up by every replica (the
    survivors' broken reload group falls back to per-rank file watching)."""
    from mlapi_amd.models.linear import LinearModel

    (tmp_path / "LRClassifier.pkl").write_bytes(iris_pickle_bytes)
    port = free_port()
    cmd = [sys.executable, "-m", "mlapi_amd.launch", "--nproc", "3", "--no-pin", "--restart", "1", "-m",
           "mlapi_amd.serve", "--device", "cpu", "--port", str(port), "--io-threads", "1",
           "--reload-interval-ms", "50"]
    env = {**ENV, "MLAPI_FAULT_EXIT_RANK": "1", "MLAPI_FAULT_EXIT_AFTER_MS": "1500",
           "PYTHONPATH": str(ROOT)}
    p = subprocess.Popen(cmd, env=env, cwd=str(tmp_path), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    body = b'{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}'
    try:
        t0 = time.time()
        while True:  # up
            assert p.poll() is None, p.stdout.read()
            assert time.time() - t0 < 90
            try:
                if _post_new_conn(port, body) == 200:
                    break
            except OSError:
                time.sleep(0.2)
        codes = []
        t0 = time.time()
        while time.time() - t0 < 8:  # across the crash and the restart
            try:
                codes.append(_post_new_conn(port, body))
            except OSError:
                codes.append(-1)  # a connection the dying rank had accepted
            time.sleep(0.01)
        assert p.poll() is None, "the launcher must keep the job alive"
        ok = codes.count(200)
        assert ok >= 0.97 * len(codes), {c: codes.count(c) for c in set(codes)}
        # hot reload after the restart: a model that always answers class 2 ("Iris-virginica")
        W = np.zeros((3, 4))
        b = np.array([0.0, 0.0, 5.0])
        m = LinearModel(W=W, b=b, classes=np.array(["Iris-setosa", "Iris-versicolor", "Iris-virginica"]),
                        kind=2)
        from mlapi_amd.ckpt.sklearn_pickle import export_sklearn_pickle

        export_sklearn_pickle(m, str(tmp_path / "new.pkl"))
        os.replace(tmp_path / "new.pkl", tmp_path / "LRClassifier.pkl")
        t0 = time.time()
        while True:
            labels = []
            for _ in range(60):
                s = socket.create_connection(("127.0.0.1", port), timeout=10)
                s.sendall(b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\n"
                          b"Connection: close\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body))
                data = b""
                while True:
                    c = s.recv(65536)
                    if not c:
                        break
                    data += c
                s.close()
                labels.append(json.loads(data.split(b"\r\n\r\n", 1)[1])["prediction"])
            if labels == ["Iris-virginica"] * 60:
                break
            assert time.time() - t0 < 20, labels
            time.sleep(0.2)
    finally:
        p.send_signal(signal.SIGTERM)
        try:
            out, _ = p.communicate(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
    assert "restart 1/1" in out, out[-3000:]


def test_p2p_verify_cpu_twin(tmp_path):
    """the CPU FakeComm twin of the fused-exchange verification (exact-sum check
    of a rank-tagged synthetic gradient, corruption caught, replica hash + rank-0 re-sync)."""
    run(2, str(ROOT / "tests" / "dist" / "p2p_verify_cpu.py"), {"OUT": str(tmp_path), "MLAPI_COMM": "fake"})
    assert (tmp_path / "OK_0").exists() and (tmp_path / "OK_1").exists()
