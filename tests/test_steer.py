"""Connection steering by SO_INCOMING_CPU (csrc/http/server.h io_steer) and the load generator's
shuffled connection map / pinned client threads (csrc/http/loadgen.h), on the CPU backend.

VERDICT r5 next 1: the headline must hold when the load generator's threads are not paired with the
server's IO threads by connect order. The load generator deals its connections to its threads by a
seeded permutation (``shuffle``), each client thread pinned to a CPU of its own; the server learns
every connection's client CPU from SO_INCOMING_CPU and regroups connections so the ones driven from
one CPU share one IO thread (a CPU with more than a thread's share is split over two or three)."""
import os
import time

import numpy as np
import pytest

from mlapi_amd.models.linear import LinearModel

IRIS = ["sepal_length", "sepal_width", "petal_length", "petal_width"]
LABELS = ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]


def test_client_thread_cpus_disjoint_per_rank():
    from mlapi_amd.utils.affinity import client_thread_cpus

    mask = list(range(64))
    sysfs = "/nonexistent"  # no topology: core order = the mask's order
    a = client_thread_cpus(0, 4, 8, mask, [0, 0, 0, 0], sysfs=sysfs)
    b = client_thread_cpus(1, 4, 8, mask, [0, 0, 0, 0], sysfs=sysfs)
    c = client_thread_cpus(3, 4, 8, mask, [0, 0, 0, 0], sysfs=sysfs)
    assert len(a) == len(set(a)) == 8
    assert not set(a) & set(b) and not set(b) & set(c) and not set(a) & set(c)
    # ranks on another NUMA node restart at the beginning of their own mask
    assert client_thread_cpus(4, 8, 8, mask, [0, 0, 0, 0, 1, 1, 1, 1], sysfs=sysfs) == a
    assert client_thread_cpus(0, 1, 0, mask) == [] and client_thread_cpus(0, 1, 4, []) == []


def test_serve_thread_cpus_give_io_threads_cores_of_their_own():
    from mlapi_amd.utils.affinity import client_thread_cpus, serve_thread_cpus

    mask = list(range(64))
    sysfs = "/nonexistent"
    cl, io = serve_thread_cpus(0, 2, 8, 8, mask, [0, 0], sysfs=sysfs)
    assert cl == client_thread_cpus(0, 2, 8, mask, [0, 0], sysfs=sysfs)[:8] and len(io) == 8
    assert not set(cl) & set(io) and len(set(io)) == 8
    cl1, io1 = serve_thread_cpus(1, 2, 8, 8, mask, [0, 0], sysfs=sysfs)  # the other rank's stretch
    assert not (set(cl) | set(io)) & (set(cl1) | set(io1))
    assert serve_thread_cpus(0, 1, 4, 0, mask, sysfs=sysfs) == (client_thread_cpus(0, 1, 4, mask, sysfs=sysfs), [])
    assert serve_thread_cpus(0, 1, 4, 4, []) == ([], [])


def test_serve_thread_cpus_llc_and_sibling_modes(tmp_path):
    """A fake topology: 8 cores x 2 threads (CPU c and c + 8 siblings), two 4-core LLCs."""
    from mlapi_amd.utils.affinity import serve_thread_cpus

    for c in range(16):
        core = c % 8
        d = tmp_path / f"cpu{c}"
        (d / "topology").mkdir(parents=True)
        (d / "cache" / "index3").mkdir(parents=True)
        (d / "topology" / "core_id").write_text(str(core))
        (d / "topology" / "physical_package_id").write_text("0")
        (d / "topology" / "thread_siblings_list").write_text(f"{core},{core + 8}")
        lo = 0 if core < 4 else 4
        (d / "cache" / "index3" / "shared_cpu_list").write_text(f"{lo}-{lo + 3},{lo + 8}-{lo + 11}")
    mask = list(range(16))
    # four ranks on the node: each a stretch of 2 physical cores, client + IO on the same core,
    # no core shared between ranks (a stretch of LOGICAL CPUs would hand ranks 2-3 the siblings of
    # ranks 0-1's cores, i.e. their IO threads' CPUs)
    seen = set()
    for r in range(4):
        cl, io = serve_thread_cpus(r, 4, 2, 2, mask, [0, 0, 0, 0], sysfs=str(tmp_path), mode="sibling")
        assert io == [c + 8 for c in cl] and len(cl) == 2
        cores = {c % 8 for c in cl}
        assert not cores & seen
        seen |= cores
    cl, io = serve_thread_cpus(0, 1, 2, 2, mask, sysfs=str(tmp_path), mode="sibling")
    assert io == [c + 8 for c in cl]
    assert serve_thread_cpus(0, 1, 2, 5, mask, sysfs=str(tmp_path), mode="sibling")[1] == io  # no pair: unpinned
    cl, io = serve_thread_cpus(0, 1, 2, 2, mask, sysfs=str(tmp_path), mode="llc")
    assert len(set(io)) == 2 and not set(io) & set(cl)
    for c, i in zip(cl, io):
        assert (c % 8 < 4) == (i % 8 < 4) and i % 8 != c % 8  # same LLC, another core


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 2, reason="needs 2 CPUs")
def test_io_cpus_pin_the_io_threads(native):
    """Config.io_cpus: IO thread i runs on the i-th CPU of the list (bench.py --io-pin)."""
    cpus = sorted(os.sched_getaffinity(0))[:2]
    with _server(4, io_cpus=",".join(str(c) for c in cpus)):
        seen = {}
        deadline = time.time() + 10
        while len(seen) < 4 and time.time() < deadline:
            for tid in os.listdir("/proc/self/task"):
                try:
                    name = open(f"/proc/self/task/{tid}/comm").read().strip()
                except OSError:
                    continue
                if name.startswith("mlapi-io-"):
                    seen[int(name.rsplit("-", 1)[1])] = sorted(os.sched_getaffinity(int(tid)))
            time.sleep(0.05)
        assert sorted(seen) == [0, 1, 2, 3], seen
        for i, aff in seen.items():  # threads past the list keep the process mask
            assert aff == ([cpus[i]] if i < 2 else sorted(os.sched_getaffinity(0))), (i, aff)


def _server(io_threads, **kw):
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config

    return NativeServer(Config.from_env(port=0, device="cpu", reload="off", missing_model="keep", resident="off",
                                        model_path="/nonexistent/steer.pkl", feature_names=list(IRIS),
                                        io_threads=io_threads, **kw))


def _workload(srv):
    from mlapi_amd.serve.loadgen import make_workload

    m = LinearModel.random(4, 3, seed=21, labels=LABELS)
    srv.runtime.handle.load(m)
    X = np.round(np.random.default_rng(2).standard_normal((128, 4)) * 2 + 4, 1)
    return make_workload(srv.runtime.handle.engine, m, IRIS, X, rtol_oracle=1e-12, label_margin=1e-5)


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 4, reason="needs 4 CPUs")
def test_shuffled_pinned_clients_are_regrouped_by_cpu(native):
    """2 pinned client threads x 8 connections, dealt by a seeded permutation over 4 IO threads:
    the plan splits each client CPU's 8 connections over 2 IO threads (a thread's share is 4), the
    connections move there, and every body stays exact."""
    cpus = sorted(os.sched_getaffinity(0))[:2]
    with _server(4, steer_every=8, steer_stable=2) as srv:
        reqs, exp = _workload(srv)
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), 16, 2)
        lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
        lg.set_conn_map("shuffle", 7)
        lg.set_thread_cpus(cpus)
        t_end = time.time() + 20
        st = srv.http.stats()
        while time.time() < t_end:
            res = lg.run(100, False)
            assert res["failed"] == 0 and res["body_mismatches"] == 0 and res["status_counts"] == {200: 1600}, res
            st = srv.http.stats()
            plan = {p[0]: p for p in st["steer_plan"] if p[1] > 0}
            if st["steered"] > 0 and set(plan) == set(cpus) and sorted(st["conns_per_thread"]) == [4, 4, 4, 4]:
                break
        lg.close()
    plan = {p[0]: p for p in st["steer_plan"] if p[1] > 0}
    assert st["steered"] > 0, st
    assert set(plan) == set(cpus) and all(p[1] == 8 for p in plan.values()), st["steer_plan"]
    threads = [set(t for t in p[2:] if t >= 0) for p in plan.values()]
    assert all(len(t) == 2 for t in threads) and not threads[0] & threads[1], st["steer_plan"]
    assert sorted(st["conns_per_thread"]) == [4, 4, 4, 4], st


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 2, reason="needs 2 CPUs")
def test_steering_prefers_the_io_thread_pinned_on_the_clients_core(native):
    """io_cpus gives every CPU a home IO thread (the one pinned on its physical core): the plan sends
    a client CPU's connections there, even when connect order dealt them elsewhere."""
    cpus = sorted(os.sched_getaffinity(0))[:2]
    # IO thread 0 on the second client CPU, thread 1 on the first: the reverse of connect order
    with _server(2, steer_every=8, steer_stable=2, io_cpus=f"{cpus[1]},{cpus[0]}") as srv:
        reqs, exp = _workload(srv)
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), 8, 2)
        lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
        lg.set_thread_cpus(cpus)
        t_end = time.time() + 20
        st = srv.http.stats()
        while time.time() < t_end:
            res = lg.run(100, False)
            assert res["failed"] == 0 and res["body_mismatches"] == 0, res
            st = srv.http.stats()
            plan = {p[0]: p for p in st["steer_plan"] if p[1] > 0}
            if set(plan) == set(cpus) and st["conns_per_thread"] == [4, 4] and st["steered"] >= 8:
                break
        lg.close()
    plan = {p[0]: p for p in st["steer_plan"] if p[1] > 0}
    assert plan[cpus[0]][2] == 1 and plan[cpus[1]][2] == 0, st["steer_plan"]
    assert st["steered"] >= 8 and st["conns_per_thread"] == [4, 4], st


def test_steering_off_keeps_the_acceptor_deal(native):
    with _server(4, io_steer=0) as srv:
        reqs, exp = _workload(srv)
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), 16, 2)
        lg.set_workload([r.decode() for r in reqs], [e.decode() for e in exp], 0.0)
        lg.set_conn_map("shuffle", 3)
        res = lg.run(300, False)
        st = srv.http.stats()
        lg.close()
    assert res["status_counts"] == {200: 4800} and res["body_mismatches"] == 0, res
    assert st["steered"] == 0 and st["conns_per_thread"] == [4, 4, 4, 4], st


def test_conn_map_rejects_unknown_mode(native):
    with _server(1) as srv:
        reqs, exp = _workload(srv)
        lg = native.Loadgen("127.0.0.1", srv.port, reqs[0].decode(), 2, 1)
        with pytest.raises(Exception):
            lg.set_conn_map("sideways", 1)
        with pytest.raises(Exception):
            lg.set_thread_cpus([-1])
        lg.close()
