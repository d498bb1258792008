"""Round-robin connection dispatch (csrc/http/dispatch.h) and the self-launching multi-rank bench.

BASELINE config 4 asks for "round-robin dispatch" across the DP replicas; SO_REUSEPORT's 4-tuple
hash left ranks +-5-17% apart. These tests pin the acceptor protocol on CPU:
exact round-robin over replicas and IO threads, health-aware skipping, leader failover, and the
`bench.py --gpus N` self-launch contract.
"""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

from conftest import ROOT

A1 = b'{"sepal_length":5.1,"sepal_width":3.5,"petal_length":1.4,"petal_width":0.2}'
ENV = {**os.environ, "PYTHONPATH": str(ROOT), "OMP_NUM_THREADS": "1", "CUDA_VISIBLE_DEVICES": "",
       "HIP_VISIBLE_DEVICES": ""}
for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
    ENV.pop(k, None)


def _post(port, body=A1, keep=None):
    s = keep or socket.create_connection(("127.0.0.1", port), timeout=10)
    s.sendall(b"POST /predict HTTP/1.1\r\nHost: t\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
              % (len(body), body))
    buf = b""
    while b"\r\n\r\n" not in buf:
        c = s.recv(65536)
        if not c:
            raise ConnectionError("closed")
        buf += c
    head, rest = buf.split(b"\r\n\r\n", 1)
    n = int([l for l in head.split(b"\r\n") if l.lower().startswith(b"content-length")][0].split(b":")[1])
    while len(rest) < n:
        rest += s.recv(65536)
    return int(head.split()[1]), s


def _server(port, rank, io_threads=2, group="", dispatch="acceptor", claim=""):
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    os.environ["RANK"] = str(rank)  # the replica's rank, reported to the group's leader
    try:
        srv = NativeServer(Config.from_env(port=port, device="cpu", io_threads=io_threads, dispatch=dispatch,
                                           dispatch_group=group, dispatch_claim=claim)).start()
    finally:
        os.environ.pop("RANK", None)
    return srv


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_acceptor_round_robin_over_replicas_and_threads(iris_cwd):
    """Three replicas (in one process: the protocol is the same across processes) on one port:
    30 new connections -> exactly 10 per replica, and 5 per IO thread inside each."""
    port = _free_port()
    srvs = [_server(port, r) for r in range(3)]
    try:
        d0 = srvs[0].http.stats()["dispatch"]
        assert d0["leader"] and not srvs[1].http.stats()["dispatch"]["leader"]
        assert all(s.port == port for s in srvs)
        t0 = time.time()
        while len(srvs[0].http.stats()["dispatch"]["targets"]) < 3:  # members' hellos processed
            assert time.time() - t0 < 10
            time.sleep(0.01)
        socks = []
        for _ in range(30):
            st, s = _post(port)
            assert st == 200
            socks.append(s)
        tg = {r: n for r, n, _ in srvs[0].http.stats()["dispatch"]["targets"]}
        assert tg == {0: 10, 1: 10, 2: 10}, tg
        assert [s.http.stats()["dispatch"]["received"] for s in srvs] == [10, 10, 10]
        assert [s.http.stats()["connections"] for s in srvs] == [10, 10, 10]
        for s in socks:
            s.close()
    finally:
        for s in srvs:
            s.stop()


def _post_from(port, source):
    s = socket.socket()
    s.bind((source, 0))
    s.settimeout(10)
    s.connect(("127.0.0.1", port))
    return _post(port, keep=s)


def test_claimed_client_address_goes_to_its_replica(iris_cwd):
    """dispatch=source with claims: replica r claims 127.1.0.(r+1); the addresses then reach their own
    replicas whatever order they first connect in (without claims the first-seen address takes the
    leader) - the bench's rank-local load generators stay on their own rank's replica."""
    port = _free_port()
    srvs = [_server(port, r, io_threads=2, dispatch="source", claim=f"127.1.0.{r + 1}") for r in range(3)]
    try:
        t0 = time.time()
        while len(srvs[0].http.stats()["dispatch"]["targets"]) < 3:
            assert time.time() - t0 < 10
            time.sleep(0.01)
        socks = []
        for k in range(4):
            for a in ("127.1.0.3", "127.1.0.2", "127.1.0.1"):  # reverse of the claims' order
                st, s = _post_from(port, a)
                assert st == 200
                socks.append(s)
        assert [s.http.stats()["connections"] for s in srvs] == [4, 4, 4]
        assert [s.http.stats()["dispatch"]["received"] for s in srvs] == [4, 4, 4]
        # an unclaimed address still goes round robin
        st, s = _post_from(port, "127.1.0.9")
        assert st == 200
        socks.append(s)
        assert sum(x.http.stats()["connections"] for x in srvs) == 13
        for s in socks:
            s.close()
    finally:
        for s in srvs:
            s.stop()


def test_source_affinity_keeps_a_client_address_on_one_replica(iris_cwd):
    """dispatch=source: three client addresses x 8 connections, interleaved, over three replicas of
    4 IO threads -> each address's 8 connections on ONE replica (a different one per address, in
    first-seen round-robin order), and inside it on the IO threads in connect order (2 per thread:
    a load generator with 4 threads keeps each thread's connections on one IO thread)."""
    port = _free_port()
    srvs = [_server(port, r, io_threads=4, dispatch="source") for r in range(3)]
    try:
        t0 = time.time()
        while len(srvs[0].http.stats()["dispatch"]["targets"]) < 3:
            assert time.time() - t0 < 10
            time.sleep(0.01)
        socks = []
        for k in range(8):
            for a in ("127.1.0.1", "127.1.0.2", "127.1.0.3"):
                st, s = _post_from(port, a)
                assert st == 200
                socks.append(s)
        tg = {r: n for r, n, _ in srvs[0].http.stats()["dispatch"]["targets"]}
        assert tg == {0: 8, 1: 8, 2: 8}, tg
        assert [s.http.stats()["connections"] for s in srvs] == [8, 8, 8]
        for s in socks:
            s.close()
        # a new address takes the next replica in round-robin order (the fourth: replica 0 again);
        # a known one stays on its replica (127.1.0.2, seen second: replica 1)
        st, s = _post_from(port, "127.1.0.4")
        s.close()
        st, s2 = _post_from(port, "127.1.0.2")
        s2.close()
        tg = {r: n for r, n, _ in srvs[0].http.stats()["dispatch"]["targets"]}
        assert tg == {0: 9, 1: 9, 2: 8}, tg
    finally:
        for s in srvs:
            s.stop()


def test_acceptor_skips_unhealthy_replica_and_readmits(iris_cwd):
    port = _free_port()
    srvs = [_server(port, r) for r in range(2)]
    from mlapi_amd.serve.server import NativeServer  # noqa: F401

    try:
        t0 = time.time()
        while len(srvs[0].http.stats()["dispatch"]["targets"]) < 2:
            assert time.time() - t0 < 10
            time.sleep(0.01)
        # member 1 reports unhealthy: the health hook reads HttpServer.accepting(), driven by the
        # health thread from the engine; fault-inject the engine and enable health dispatch
        srvs[1].stop()
        srvs[1] = _server_health(port, 1)
        srvs[1].runtime.handle.engine.inject_drop(True)
        t0 = time.time()
        while True:
            tg = srvs[0].http.stats()["dispatch"]["targets"]
            if len(tg) == 2 and not tg[1][2]:
                break
            assert time.time() - t0 < 10, tg
            time.sleep(0.02)
        for _ in range(10):
            st, s = _post(port)
            assert st == 200
            s.close()
        tg = srvs[0].http.stats()["dispatch"]["targets"]
        assert tg[1][1] == 0, tg  # nothing went to the unhealthy replica
        srvs[1].runtime.handle.engine.inject_drop(False)
        t0 = time.time()
        while not srvs[0].http.stats()["dispatch"]["targets"][1][2]:
            assert time.time() - t0 < 10
            time.sleep(0.02)
        for _ in range(10):
            st, s = _post(port)
            assert st == 200
            s.close()
        assert srvs[0].http.stats()["dispatch"]["targets"][1][1] == 5
    finally:
        for s in srvs:
            s.stop()


def _server_health(port, rank):
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    os.environ["RANK"] = str(rank)
    try:
        srv = NativeServer(Config.from_env(port=port, device="cpu", io_threads=1, health_dispatch="on",
                                           dispatch="acceptor")).start()
    finally:
        os.environ.pop("RANK", None)
    return srv


def test_acceptor_leader_failover(iris_cwd):
    """The leader stops: the member wins the election, re-binds the port and keeps serving."""
    port = _free_port()
    a, b = _server(port, 0), _server(port, 1)
    try:
        assert a.http.stats()["dispatch"]["leader"]
        a.stop()
        t0 = time.time()
        while not b.http.stats()["dispatch"]["leader"]:
            assert time.time() - t0 < 10
            time.sleep(0.01)
        for _ in range(5):
            st, s = _post(port)
            assert st == 200
            s.close()
        assert b.http.stats()["dispatch"]["elections"] == 1
        c = _server(port, 2)  # a restarted replica joins the new leader
        assert not c.http.stats()["dispatch"]["leader"]
        c.stop()
    finally:
        a.stop()
        b.stop()


def test_reuseport_mode_still_available(iris_cwd):
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    srv = NativeServer(Config.from_env(port=0, device="cpu", io_threads=2, dispatch="reuseport")).start()
    try:
        st, s = _post(srv.port)
        assert st == 200 and "dispatch" not in srv.http.stats()
        s.close()
    finally:
        srv.stop()


def _bench(args, env=None, timeout=300):
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env={**ENV, **(env or {})},
                          capture_output=True, text=True, timeout=timeout, cwd=str(ROOT))


def test_bench_self_launches_n_ranks():
    """`python bench.py --cpu --gpus 4` (no torchrun): the bench starts 4 ranks itself; the line says
    n_gpus 4 / dp4, every rank served an equal share (source-affinity dispatch: one load generator per
    replica), and the communicator
    evidence fields are present."""
    r = _bench(["--cpu", "--gpus", "4", "--steps", "3", "--warmup", "1", "--reqs-per-conn", "64",
                "--c1-requests", "100"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp4"
    assert len(d["served_per_rank"]) == 4
    mean = sum(d["served_per_rank"]) / 4
    assert all(abs(v - mean) <= 0.02 * mean for v in d["served_per_rank"]), d["served_per_rank"]
    assert d["comm_nranks"] == 4 and d["rccl_nranks"] is None  # gloo on CPU: no RCCL claimed
    assert set(d["allreduce_us"]) == {"1KiB", "1MiB"} and d["c1_bcast_us"] > 0
    # the driver's line contract (task spec) and the round-3 host-CPU evidence
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    cb = d["cpu_breakdown_rank0"]
    assert cb["server_cpu_us_per_req"] > 0
    assert set(cb["io_stage_us_per_req"]) == {"poll", "recv", "parse", "submit", "idle_gpu", "render", "send",
                                              "handoff"}
    # engine-thread stage clocks per GPU batch (zero on the CPU backend, which has no GPU batches)
    assert set(cb["batcher_us_per_batch"]) == {"take", "slot", "launch", "book"}
    assert set(cb["completer_us_per_batch"]) == {"wait_gpu", "deliver"}
    assert d["dispatch"] == "source"  # each rank's load generator from an address of its own


def test_bench_self_launches_eight_ranks():
    """The driver's whole-node shape, rehearsed on the CPU: `bench.py --cpu --gpus 8` starts 8
    ranks (gloo), the acceptor deals the load generators' client addresses round robin to all of them, and the line reports
    dp8 with 8 balanced per-rank counts."""
    r = _bench(["--cpu", "--gpus", "8", "--steps", "2", "--warmup", "1", "--reqs-per-conn", "16",
                "--c1-requests", "50"], timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 8 and d["config"]["parallelism"] == "dp8" and d["comm_nranks"] == 8
    assert len(d["served_per_rank"]) == 8
    mean = sum(d["served_per_rank"]) / 8
    assert all(abs(v - mean) <= 0.02 * mean for v in d["served_per_rank"]), d["served_per_rank"]
    assert d["body_mismatches"] == 0


def test_bench_refuses_world_size_mismatch():
    r = _bench(["--cpu", "--gpus", "2", "--steps", "1", "--warmup", "0"], env={"WORLD_SIZE": "1"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_bench_refuses_more_ranks_than_gpus_without_p2p():
    """No GPU visible here: asking for 2 GPU ranks must fail loudly, not fall back to 1."""
    r = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2 and "GPU" in r.stderr
