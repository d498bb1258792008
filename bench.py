"""Benchmark driver (BASELINE.json metric: "requests/sec (whole node) + p50 latency, logistic
/predict at batch=1/64").

    python bench.py --gpus N --steps K --warmup W            # default: --mode serve
    torchrun --nproc-per-node N bench.py --gpus N ...        # one rank per GPU (RCCL)

serve (flagship, BASELINE config 1/4): every rank runs the full production stack on its GPU -
native HTTP server -> batching engine -> fused fp64 HIP kernel -> JSON response - with the Iris
LogisticRegression architecture (F=4 features, K=3 classes; random-init weights, seeded,
broadcast from rank 0 over RCCL = collective C1). All ranks' servers share ONE SO_REUSEPORT port
(the dp_serve topology, health-aware dispatch at N > 1); each rank drives it with its own
out-of-process native load generator (mlapi-loadgen, pinned apart from the server threads when
the rank is pinned): 64 keep-alive connections ("batch=64": 64 concurrent single-row POST
/predict requests) cycling through 1024 distinct Iris-like requests, every response body checked
byte for byte against the engine's answer (itself checked against the fp64 oracle).
  step  = each of the 64 connections completes --reqs-per-conn (2048) requests = 131,072 requests
          per rank (~0.1-0.2 s, so the driver's --steps 20 times >= 2 s)
  value = whole-node requests/s = requests completed by all ranks / max-over-ranks elapsed
  p50/p99 at concurrency 64 come from the timed run; batch=1 latency (concurrency 1) is measured
  afterwards by rank 0 alone and reported as extra fields.
serve_wide: the same with an F=256 model (--wide-classes 1000: MFMA gemm_softmax; 2: bf16 GEMV).
Other modes (extra evidence, not the headline): gemv (config 2: 1M x 256 bf16 binary predict),
gemm (config 3: B=1024, F=256, K=1000 bf16 multiclass predict), train (config 5: binary LR
mini-batch SGD, F=256 bf16, DP gradient all-reduce).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

# Reference numbers (measured on the reference itself, CPU, no published numbers):
BASELINES = {
    "serve": 1494.0,       # req/s, 1 uvicorn worker, concurrency 64
    "serve_wide": None,    # the reference serves Iris only
    "gemv": 1.00e6,        # rows/s, sklearn binary 1M x 256 predict+proba
    "gemm": 87075.0,       # rows/s, sklearn 1000-class B=1024 F=256
    "train": 3.73e6,       # sample-gradients/s, sklearn lbfgs binary 100k x 256
    "train_softmax": None,  # no reference number for 1000-class training
}
IRIS_LABELS = ["Iris-setosa", "Iris-versicolor", "Iris-virginica"]


def _sync(info):
    import torch

    if info.device is not None:
        torch.cuda.synchronize(info.device)


def _timed(info, fn):
    """barrier + sync on both sides of fn(); returns max-over-ranks seconds."""
    from mlapi_amd.parallel.comm import all_reduce_max, barrier

    barrier(info)
    _sync(info)
    t0 = time.perf_counter()
    out = fn()
    _sync(info)
    t1 = time.perf_counter()
    barrier(info)
    return all_reduce_max(t1 - t0, info), out


def _comm_probe(info, model=None) -> dict:
    """Evidence of the job's communicator, measured before the timed region and reported in every
    bench line: how many ranks RCCL itself counts (ncclCommCount), the C1 model broadcast latency,
    and the C2 all-reduce latency at the two gradient sizes of SURVEY 2.4 (1 KiB binary, 1 MiB
    1000-class). All max over ranks."""
    import torch

    from mlapi_amd.models.linear import LinearModel
    from mlapi_amd.parallel.comm import _coll_device, all_reduce_max, all_reduce_sum_, barrier, broadcast_model

    out = {"comm_nranks": info.comm_nranks()}
    kind = getattr(info.comm, "kind", info.backend)
    out["rccl_nranks"] = (info.comm_nranks() if kind in ("native-rccl", "torch-rccl") or info.backend == "nccl"
                          else None)
    if info.world == 1:
        # one rank: a broadcast / all-reduce moves nothing over xGMI - no latency worth reporting
        out["collectives"] = "noop_world1"
        return out
    if model is None:
        model = LinearModel.random(256, 1000, seed=3) if info.is_main else None
    barrier(info)
    t0 = time.perf_counter()
    broadcast_model(model if info.is_main else None, info)
    out["c1_bcast_us"] = all_reduce_max(time.perf_counter() - t0, info) * 1e6
    out["c1_payload"] = "K=1000 x F=256 f64 W|b (2 MB) + label header"
    dev = _coll_device(info)
    ar = {}
    for name, nbytes in (("1KiB", 1 << 10), ("1MiB", 1 << 20)):
        t = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
        for _ in range(3):
            all_reduce_sum_(t, info)
        _sync(info)
        barrier(info)
        iters = 20
        t0 = time.perf_counter()
        for _ in range(iters):
            all_reduce_sum_(t, info)
        _sync(info)
        dt = (time.perf_counter() - t0) / iters
        if info.comm is not None and hasattr(info.comm, "wait"):
            info.comm.wait()
        ar[name] = all_reduce_max(dt, info) * 1e6
        want = float(info.world) ** (3 + iters)
        if info.world > 1 and abs(float(t[0].item()) - want) > 1e-4 * want:
            raise RuntimeError(f"all-reduce probe ({name}) returned {float(t[0].item())}")
    out["allreduce_us"] = ar
    return out


def _thread_cpus(args, info) -> tuple:
    """(load-generator thread CPUs, server IO-thread CPUs). --client-pin: one CPU per load-generator
    thread, from this rank's mask (disjoint stretches for ranks that share a NUMA-node mask);
    --io-pin (with --client-pin): the IO threads on the next physical cores of the same stretch.
    [] = those threads keep the process mask."""
    if args.client_pin == "off":
        return [], []
    from mlapi_amd.utils.affinity import client_thread_cpus, gpu_numa_nodes, serve_thread_cpus

    if getattr(args, "lg_mask", None):  # --pin on: the load generator has a core slice of its own
        return client_thread_cpus(0, 1, args.client_threads, args.lg_mask), []
    mask = sorted(os.sched_getaffinity(0))
    nodes = gpu_numa_nodes() if os.environ.get("MLAPI_PLACEMENT") == "numa" else None
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", info.world))
    n_io = args.io_threads if args.io_pin != "off" else 0
    return serve_thread_cpus(info.local_rank, local_world, args.client_threads, n_io, mask, nodes,
                             mode=args.io_pin if args.io_pin != "off" else "cores")


def _share_port(port: int, info) -> int:
    """Rank 0's bound port, known to every rank (the shared SO_REUSEPORT port of the DP group)."""
    from mlapi_amd.parallel.comm import all_gather_floats

    return int(all_gather_floats([float(port)], info)[0, 0])


def _serve_bench(args, info, model, names, rows, *, dtype_cfg, rel_tol, oracle_kw, model_desc, features):
    """Production topology on every rank: native HTTP server + batching engine + HIP kernel, all
    ranks in ONE SO_REUSEPORT group on a shared port (health-aware dispatch on at N > 1), driven by
    an out-of-process native load generator per rank (pinned apart from the server when the rank
    is pinned) whose every response body is validated."""
    from mlapi_amd.parallel.comm import all_gather_floats, barrier
    from mlapi_amd.serve.loadgen import make_workload
    from mlapi_amd.serve.server import NativeServer
    from mlapi_amd.utils.config import Config
    from mlapi_amd.utils.threads import cpu_by_group, utilization

    lg = args.lg_proc
    device = "cpu" if info.device is None else f"cuda:{info.device.index}"
    client_cpus, io_cpus = _thread_cpus(args, info)
    args.io_cpus = io_cpus
    # dispatch "source": this rank's load generator connects from an address of its own, and this
    # rank's replica claims it - its clients (pinned next to this replica's IO threads) are served
    # here from the first connection on, not by whichever replica the round robin reached first
    src = f"127.1.{info.rank // 250}.{info.rank % 250 + 1}" if args.dispatch == "source" else ""
    mk = lambda port: Config.from_env(port=port, device=device, reload="off", missing_model="keep",  # noqa: E731
                                      io_threads=args.io_threads, max_batch=args.max_batch, reuseport=True,
                                      dispatch=args.dispatch, io_cpus=",".join(str(c) for c in io_cpus),
                                      dispatch_claim=src,
                                      model_path="/nonexistent/bench.pkl", feature_names=list(names), **dtype_cfg)
    srv = None
    # everything from the server start on is inside the try: a failed workload pre-check (or any
    # error) stops the server and its threads before the exception leaves, so the process exits
    # non-zero through the normal path (tests/test_bench_cli.py)
    try:
        if info.is_main:  # rank 0 binds an ephemeral port, the other ranks join its SO_REUSEPORT group
            srv = NativeServer(mk(0))
            srv.runtime.handle.load(model)
            srv.start()
        port = _share_port(srv.port if srv is not None else 0, info)
        if srv is None:
            srv = NativeServer(mk(port))
            srv.runtime.handle.load(model)
            srv.start()
        reqs, exp = make_workload(srv.runtime.handle.engine, model, names, rows, **oracle_kw)
        lg.workload(reqs, exp, rel_tol)
        barrier(info)  # every rank's listeners are in the group before any client connects
        # "acceptor" deals every connection round robin over ranks; "source" keeps this rank's
        # connections together on the replica that claimed their address (see src above)
        lg.connect("127.0.0.1", port, args.conns, args.client_threads, source=src)
        lg.thread_cpus(client_cpus)
        if args.warmup:
            w = lg.run(args.warmup * args.reqs_per_conn, False)
            if w["failed"] or w["errors"]:
                raise RuntimeError(f"warmup failed: {w}")
        barrier(info)  # every rank's warmup traffic has drained before the counters are read

        def phase(steps):
            """One timed closed-loop phase: (elapsed, loadgen result, server CPU breakdown)."""
            s0, h0 = srv.runtime.handle.stats(), srv.http.stats()
            c0, l0 = cpu_by_group(), cpu_by_group(lg.pid)
            elapsed, res = _timed(info, lambda: lg.run(steps * args.reqs_per_conn, True))
            cpu_util = utilization(c0, cpu_by_group(), elapsed)
            cpu_util["loadgen_process"] = utilization(l0, cpu_by_group(lg.pid), elapsed).get("process_total", 0.0)
            s1, h1 = srv.runtime.handle.stats(), srv.http.stats()
            nreq = max(1, s1["requests"] - s0["requests"])
            nbat = max(1, (s1["batches"] - s0["batches"]) - (s1["idle_batches"] - s0["idle_batches"]))  # batcher launches
            # where this rank's server CPU goes, per request (IO-thread stage clock, exclusive; "poll"
            # is epoll_wait + loop overhead, mostly idle blocking) and the server-side HTTP latency
            cpu_breakdown = {
                "server_cpu_us_per_req": cpu_util.get("process_total", 0.0) * elapsed / nreq * 1e6,
                # requests this rank served per second of server CPU (all its threads): what decides the
                # whole-node number when the ranks share the node's CPUs
                "req_per_s_per_server_core": nreq / max(1e-9, cpu_util.get("process_total", 0.0) * elapsed),
                "io_stage_us_per_req": {k: (h1["stage_ns"][k] - h0["stage_ns"][k]) / nreq / 1e3 for k in h1["stage_ns"]},
                "engine_queue_wait_us_per_req": (s1["queue_wait_us_sum"] - s0["queue_wait_us_sum"]) / nreq,
                # engine threads, per GPU batch (launched by the batcher): where a batch's time goes
                "batcher_us_per_batch": {k: (s1["batcher_ns"][k] - s0["batcher_ns"][k]) / nbat / 1e3
                                         for k in s1["batcher_ns"]},
                "completer_us_per_batch": {k: (s1["completer_ns"][k] - s0["completer_ns"][k]) / nbat / 1e3
                                           for k in s1["completer_ns"]},
                # inside `launch`, zero-copy / BAR batches only (the wide models' paths), per such batch
                "wide_launch_us_per_batch": {k: (s1["launch_ns"][k] - s0["launch_ns"][k]) / nbat / 1e3
                                             for k in s1["launch_ns"]},
                "server_http_latency_us_mean": (h1["http_latency_sum_ns"] - h0["http_latency_sum_ns"]) / 1e3
                / max(1, h1["http_latency_count"] - h0["http_latency_count"]),
                "steered_conns": h1.get("steered", 0) - h0.get("steered", 0),
                "steer_pauses": h1.get("steer_pauses", 0) - h0.get("steer_pauses", 0),
                "io_conns_per_thread": h1.get("conns_per_thread"),
                "steer_plan": h1.get("steer_plan") or None,
            }
            want = steps * args.reqs_per_conn * args.conns
            if res["failed"] or res["errors"] or res["body_mismatches"] or res["ok200"] != want:
                raise RuntimeError(f"load generator saw errors: {res}")
            return elapsed, res, cpu_util, cpu_breakdown, s0, s1

        elapsed, res, cpu_util, cpu_breakdown, s0, s1 = phase(args.steps)
        shuffled = None
        if args.shuffle_steps > 0:
            # the same connections, dealt to the load generator's threads by a seeded permutation: a
            # client thread's connections then sit on several IO threads (not paired by connect
            # order), as independent clients' would. Measured after the headline phase, same run.
            lg.conn_map("shuffle", 1000 + info.rank)
            el2, res2, cu2, cb2, _, _ = phase(args.shuffle_steps)
            lg.conn_map("rr")
            tot2 = float(all_gather_floats([res2["completed"]], info)[:, 0].sum())
            shuffled = {"req_per_s": tot2 / el2, "p50_latency_ms_c64": res2["p50_ns"] / 1e6,
                        "p99_latency_ms_c64": res2["p99_ns"] / 1e6,
                        "server_cpu_us_per_req": cb2["server_cpu_us_per_req"],
                        "steered_conns": cb2["steered_conns"], "steer_pauses": cb2["steer_pauses"],
                        "io_conns_per_thread": cb2["io_conns_per_thread"], "steer_plan": cb2["steer_plan"],
                        "cpu_cores_busy_rank0": cu2,
                        "io_stage_us_per_req": cb2["io_stage_us_per_req"]}
        lg.cmd("close")
        # batch = 1: one client, closed loop, measured by rank 0 alone (the other ranks idle)
        r1 = {"p50_ns": 0, "p99_ns": 0, "completed": 0, "elapsed_s": 1.0}
        barrier(info)
        s2 = srv.runtime.handle.stats()
        if info.is_main:
            lg.connect("127.0.0.1", port, 1, 1, source=src)
            lg.run(200, False)
            s2 = srv.runtime.handle.stats()
            r1 = lg.run(args.c1_requests, True)
            lg.cmd("close")
            if r1["errors"] or r1["body_mismatches"]:
                raise RuntimeError(f"batch=1 run saw errors: {r1}")
        s3 = srv.runtime.handle.stats()
        barrier(info)
        nb = max(1, s1["batches"] - s0["batches"])
        # the batch=1 connection lands on whichever replica the dispatcher picks: sum its deltas over ranks
        per_rank = all_gather_floats([res["p50_ns"] / 1e6, res["p99_ns"] / 1e6, res["completed"],
                                      (s1["requests"] - s0["requests"]) / nb,
                                      (s1["device_us_sum"] - s0["device_us_sum"]) / nb,
                                      s3["device_us_sum"] - s2["device_us_sum"], s3["batches"] - s2["batches"],
                                      s1["requests"] - s0["requests"], s1["idle_batches"] - s0["idle_batches"],
                                      s3["idle_batches"] - s2["idle_batches"]], info)
        barrier(info)
        paths = {k: s1["path_batches"][k] - s0["path_batches"][k] for k in s1["path_batches"]}
        resident = {"rows": s1["resident_rows"] - s0["resident_rows"],
                    "stale": s1["resident_stale"] - s0["resident_stale"],
                    "launches": s1["resident_launches"], "rings": s1["resident_rings"],
                    "live": bool(s1["resident_live"])}
        idle = {"c64": int(per_rank[:, 8].sum()), "batch1": int(per_rank[:, 9].sum())}
    finally:
        if srv is not None:
            srv.stop()
    total = float(np.sum(per_rank[:, 2]))
    value = total / elapsed
    extra = {
        "p50_latency_ms_c64": float(np.max(per_rank[:, 0])),
        "p99_latency_ms_c64": float(np.max(per_rank[:, 1])),
        "p50_latency_ms_batch1": r1["p50_ns"] / 1e6,
        "p99_latency_ms_batch1": r1["p99_ns"] / 1e6,
        "req_per_s_batch1": r1["completed"] / r1["elapsed_s"],
        "timed_region_s": elapsed,
        "body_mismatches": 0,
        "validated_responses": int(total),
        "served_per_rank": [int(v) for v in per_rank[:, 7]],
        "mean_gpu_batch_rows": float(np.mean(per_rank[:, 3])),
        # launch -> completion seen by the completer thread, per batch (the GPU leg of a request)
        "gpu_leg_us_c64": float(np.mean(per_rank[:, 4])),
        "gpu_leg_us_batch1": float(per_rank[:, 5].sum() / max(1.0, per_rank[:, 6].sum())),
        "kernel_batches": paths,
        # batches the IO thread launched itself on an idle engine (Engine::run_idle)
        "idle_path_batches": idle,
        # rows answered by the resident kernel through the IO threads' rings (rank 0; no packet,
        # batcher or completer per request), bounced stale by a reload, instances launched, rings
        "resident_rank0": resident,
        "backend": srv.runtime.handle.backend,
        "cpu_cores_busy_rank0": cpu_util,
        "cpu_breakdown_rank0": cpu_breakdown,
        # the shuffled-connection phase (see phase() above): whole-node req/s and rank 0's server CPU
        "req_per_s_shuffled": None if shuffled is None else shuffled["req_per_s"],
        "shuffled_rank0": shuffled,
        "threads": {"io": args.io_threads, "loadgen": args.client_threads, "pinned_cpus": args.pinned_cpus,
                    # one CPU per load-generator thread (--client-pin): the loopback stand-in for NIC
                    # RX queues with pinned interrupts, so each connection arrives from a stable CPU
                    "client_cpus": client_cpus,
                    # --io-pin: the server's IO threads on physical cores of their own beside them
                    "io_cpus": io_cpus,
                    # launcher placement of this rank (numa: its GPU's NUMA-node mask) and its mask size
                    "placement": os.environ.get("MLAPI_PLACEMENT", "cores" if args.pinned_cpus else "none"),
                    "affinity_cpus": len(os.sched_getaffinity(0))},
        "requests_per_step": args.reqs_per_conn * args.conns * info.world,
        "topology": ("one port for all ranks, connections dealt by the group's acceptor "
                     "(csrc/http/dispatch.h; dispatch=source: round robin over client addresses, a "
                     "client address keeping its replica); one out-of-process load generator per "
                     "rank, connecting from an address of its own"),
        "dispatch": srv.config.dispatch,
    }
    return ("requests_per_sec_whole_node", value, "req/s", elapsed, extra,
            {"model": model_desc, "global_batch": args.conns * info.world, "seq_len": 1, "features": features,
             "parallelism": f"dp{info.world}", "concurrency_per_gpu": args.conns})


def bench_serve(args, info):
    """Headline: the reference's Iris /predict (F=4, K=3, fp64 = sklearn parity)."""
    from mlapi_amd.models.linear import LinearModel
    from mlapi_amd.parallel.comm import broadcast_model
    from mlapi_amd.utils.config import IRIS_FEATURES

    model = LinearModel.random(4, 3, seed=0, labels=IRIS_LABELS) if info.is_main else None
    model = broadcast_model(model, info)  # C1 over RCCL
    rng = np.random.default_rng(7)
    rows = np.round(np.array([5.84, 3.05, 3.76, 1.2]) + rng.standard_normal((args.workload_rows, 4))
                    * np.array([0.83, 0.43, 1.76, 0.76]), 1)  # Iris-like requests, 1 decimal like the dataset
    extra_note = {"baseline_note": "reference uvicorn+sklearn, 1 worker, c=64: 1494 req/s, p50 41.8 ms; "
                                   "c=1 p50 0.881 ms"}
    out = _serve_bench(args, info, model, IRIS_FEATURES, rows, dtype_cfg={"dtype": "f64"}, rel_tol=0.0,
                       oracle_kw={"rtol_oracle": 1e-12}, features=4,
                       model_desc="sklearn LogisticRegression (Iris: F=4, K=3) via POST /predict")
    out[4].update(extra_note)
    return out


def bench_serve_wide(args, info):
    """Wide model on the /predict hot path: F=--wide-features (256), K classes (2 -> binary).
    --wide-dtype f64 (default, the engine default): the reference's precision (f64 storage, f64 MFMA
    accumulation), every body within rel 1e-12 of sklearn's float64 math and byte-compared (rel 0)
    against the engine's own answers; f32: f32 storage on the same f64-accumulating kernel, within
    rel 1e-11 of the fp64 oracle of the f32-rounded model; bf16: the bf16 GEMV / MFMA GEMM kernels,
    within rel 1e-4 of the bf16-rounded oracle."""
    from mlapi_amd.models.linear import LinearModel
    from mlapi_amd.parallel.comm import broadcast_model
    from mlapi_amd.serve.loadgen import bf16_oracle

    F, K = args.wide_features, args.wide_classes
    names = [f"f{i}" for i in range(F)]
    model = LinearModel.random(F, K, seed=0, labels=[f"class_{i}" for i in range(K)]) if info.is_main else None
    model = broadcast_model(model, info)
    rows = np.round(np.random.default_rng(7).standard_normal((args.workload_rows, F)), 3)
    if args.wide_dtype == "bf16":
        okw = {"rtol_oracle": 1e-4, "label_margin": 1e-3, "oracle": bf16_oracle(model, rows)}
        rel = 1e-5
    elif args.wide_dtype == "f64":
        okw = {"rtol_oracle": 1e-12, "label_margin": 1e-9}
        rel = 0.0
    else:
        f32 = lambda a: np.asarray(a, dtype=np.float32).astype(np.float64)  # noqa: E731
        on = lambda v: os.environ.get(v, "0") not in ("0", "", "false")  # noqa: E731
        f32acc = K == 2 and on("MLAPI_F32_GEMV")  # the f32-accumulating GEMV (A/B)
        okw = {"rtol_oracle": 1e-6 if f32acc else 1e-11, "label_margin": 1e-5 if f32acc else 1e-9,
               "oracle": (LinearModel(f32(model.W), f32(model.b), model.classes, model.kind), f32(rows))}
        rel = 1e-6
    return _serve_bench(args, info, model, names, rows, dtype_cfg={"wide_dtype": args.wide_dtype}, rel_tol=rel,
                        oracle_kw=okw, features=F,
                        model_desc=f"LogisticRegression F={F} K={K} ({'binary' if K == 2 else 'softmax'}) "
                                   f"via POST /predict, {args.wide_dtype} kernels")


def _launcher(args, call):
    """The timed region of the kernel benches: args.steps calls of ``call``, either eager or
    captured once into a HIP graph (outside the timed region) and replayed in it."""
    import torch

    if args.launch == "eager" or not torch.cuda.is_available():
        return lambda: [call() for _ in range(args.steps)]
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        call()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(args.steps):
            call()
    g.replay()  # first replay uploads the graph: untimed
    torch.cuda.synchronize()
    return g.replay


def bench_gemv(args, info):
    import torch

    from mlapi_amd.ops import linear as ops

    B, F = args.rows, 256
    g = torch.Generator(device=info.device).manual_seed(info.rank)
    X = torch.randn(B, F, device=info.device, generator=g).to(torch.bfloat16)
    w = (torch.randn(F, device=info.device, generator=g) / 16).to(torch.bfloat16)
    idx = torch.empty(B, dtype=torch.int32, device=info.device)
    p = torch.empty(B, dtype=torch.float32, device=info.device)
    for _ in range(args.warmup):
        ops.gemv_binary(X, w, 0.1, out=(idx, p))
    elapsed, _ = _timed(info, _launcher(args, lambda: ops.gemv_binary(X, w, 0.1, out=(idx, p))))
    value = info.world * B * args.steps / elapsed
    gbps = B * F * 2 * args.steps / (elapsed) / 1e9
    return ("rows_per_sec_binary_predict", value, "rows/s", elapsed, {"hbm_GBps_per_gpu": gbps},
            {"model": "binary LogisticRegression F=256", "global_batch": B * info.world, "seq_len": 1,
             "features": F, "parallelism": f"dp{info.world}"})


def _xcd_placement(info):
    """Block -> XCD placement probe result of this device (csrc/kernels/xcd.hip): 'round-robin'
    when the XCD-local split merges are on, 'off' when the probe found another order."""
    from mlapi_amd._native import C

    st = C().xcd_placement_state(info.device.index if info.device is not None else 0)
    return {0: "not probed", 1: "round-robin", 2: "off"}.get(st, str(st))


def bench_gemm(args, info):
    import torch

    from mlapi_amd.ops import linear as ops

    B, F, K = args.batch, 256, 1000
    g = torch.Generator(device=info.device).manual_seed(info.rank)
    X = torch.randn(B, F, device=info.device, generator=g).to(torch.bfloat16)
    W = (torch.randn(K, F, device=info.device, generator=g) / 16).to(torch.bfloat16)
    b = torch.randn(K, device=info.device, generator=g) * 0.1
    if args.gemm_kernel == "split" or args.gemm_dtype == "f32":
        # class-split kernel (small serving batches; the f32 MFMA path)
        if args.gemm_dtype == "f32":
            X, W = X.float(), W.float()
        op = ops.LinearSplit(B, K, info.device)
    else:
        forced = {"tiles": 1, "rows": 2, "t32": 3}.get(args.gemm_kernel, 0)
        if forced:
            from mlapi_amd._native import C

            C().gemm_softmax_force_plan(0, 0, forced)
        op = ops.GemmSoftmax(B, K, F, info.device)
    out = (torch.empty(B, dtype=torch.int32, device=info.device), torch.empty(B, device=info.device))
    for _ in range(args.warmup):
        op(X, W, b, out=out)
    run = _launcher(args, lambda: op(X, W, b, out=out))
    elapsed, _ = _timed(info, run)
    value = info.world * B * args.steps / elapsed
    tflops = 2 * B * F * K * args.steps / elapsed / 1e12
    return ("rows_per_sec_softmax_predict", value, "rows/s", elapsed,
            {"tflops_per_gpu": tflops, "us_per_call": elapsed / args.steps * 1e6, "launch": args.launch,
             "kernel": "linear_split" if isinstance(op, ops.LinearSplit) else "gemm_softmax",
             "gemm_kernel": args.gemm_kernel, "dtype": args.gemm_dtype,
             "xcd_placement": _xcd_placement(info)},
            {"model": "softmax regression F=256 K=1000", "global_batch": B * info.world, "seq_len": 1,
             "features": F, "parallelism": f"dp{info.world}"})


def _replica_evidence(tr, info) -> dict:
    """DP replicas after the timed steps: a 48-bit hash of every rank's parameters, all-gathered
    (equal on every rank = bitwise-identical replicas), and the P2P exchange's start-up self-test."""
    import hashlib

    from mlapi_amd.parallel.comm import all_gather_floats

    tr.check()
    raw = tr.params.detach().cpu().numpy().tobytes()
    h = float(int.from_bytes(hashlib.sha256(raw).digest()[:6], "little"))
    hs = all_gather_floats([h], info)[:, 0]
    return {"replicas_bitwise_equal": bool((hs == hs[0]).all()),
            "p2p_selftest": info.__dict__.get("p2p_selftest", "n/a"),
            # the fused exchange checked against the exact sum / ncclAllReduce at start-up and by
            # the replica hash every MLAPI_DP_VERIFY_EVERY steps (mlapi_amd/parallel/p2p.py)
            "p2p_verify": info.__dict__.get("p2p_verify", "n/a")}


def bench_train(args, info):
    from mlapi_amd.train.sgd import BinarySGDTrainer, synthetic_binary

    F = 256
    X, y = synthetic_binary(args.train_batch * args.shards, F, seed=1234 + info.rank, device=info.device)
    tr = BinarySGDTrainer(F, info=info, lr=0.5, l2=1e-4, device=info.device)
    nb = args.shards

    def run(n):
        for s in range(n):
            j = s % nb
            tr.step(X[j * args.train_batch:(j + 1) * args.train_batch], y[j * args.train_batch:(j + 1) * args.train_batch])

    run(args.warmup)
    elapsed, _ = _timed(info, lambda: run(args.steps))
    value = info.world * args.train_batch * args.steps / elapsed
    extra = {"final_loss": tr.last_loss(), "dp_exchange": tr.dp_exchange,
             "launches_per_step": 2 if tr.dp_exchange in ("fused-p2p", "local") else 3}
    extra.update(_replica_evidence(tr, info))
    return ("train_samples_per_sec", value, "samples/s", elapsed, extra,
            {"model": "binary LogisticRegression F=256 (mini-batch SGD)", "global_batch": args.train_batch * info.world,
             "seq_len": 1, "features": F, "parallelism": f"dp{info.world}"})


def bench_train_softmax(args, info):
    """Multiclass (1000-class, F=256) DP SGD: MFMA row stats + fused G/dW kernel + RCCL all-reduce."""
    from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass

    F, K, B = args.softmax_features, 1000, args.softmax_batch
    nb = max(1, args.shards // 2)
    X, y = synthetic_multiclass(B * nb, F, K, seed=99 + info.rank, device=info.device)
    tr = SoftmaxSGDTrainer(F, K, info=info, lr=0.5, l2=1e-5, device=info.device)
    Xa = tr.prepare(X)
    del X
    shards = [(Xa[j * B:(j + 1) * B], y[j * B:(j + 1) * B]) for j in range(nb)]

    def run(n):
        for s in range(n):
            tr.step(*shards[s % nb])

    run(args.warmup)
    elapsed, _ = _timed(info, lambda: run(args.steps))
    value = info.world * B * args.steps / elapsed
    flops = 3 * 2 * B * K * tr.F_aug * info.world * args.steps / elapsed  # 2 logits passes + dW
    # F <= 512: row stats + fused G/dW + slab sum/update; wider: row stats with G (softmax_rows_kernel
    # MODE 5) + G^T X_aug + slab sum/update
    launches = 3
    extra = {"final_loss": tr.last_loss(), "tflops_incl_recompute": flops / 1e12, "dp_exchange": tr.dp_exchange,
             "launches_per_step": launches + (0 if tr.dp_exchange in ("fused-p2p", "local") else 1),
             "kernel_width": tr.Fk,
             "two_shot": os.environ.get("MLAPI_DP_TWO_SHOT", "auto")}
    extra.update(_replica_evidence(tr, info))
    return ("train_softmax_samples_per_sec", value, "samples/s", elapsed, extra,
            {"model": f"{K}-class softmax LogisticRegression F={F} (mini-batch SGD)", "global_batch": B * info.world,
             "seq_len": 1, "features": F, "classes": K, "parallelism": f"dp{info.world}"})


def _self_launch(args, argv) -> int:
    """Parent of a self-launched N-rank run. Refuses more ranks than GPUs unless the data plane is
    the P2P kernel (``MLAPI_COMM=p2p``, several ranks per device) or the run is on CPUs."""
    comm = os.environ.get("MLAPI_COMM", "auto").lower()
    if not args.cpu:
        import torch  # device_count() does not initialise the GPU on this image

        ndev = torch.cuda.device_count()
        if ndev == 0:
            print("bench.py: --gpus > 1 but no GPU is visible (use --cpu for a CPU rehearsal)", file=sys.stderr)
            return 2
        if args.gpus > ndev and comm != "p2p":
            print(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) visible; RCCL needs one GPU per rank "
                  "(MLAPI_COMM=p2p shares a device between ranks)", file=sys.stderr)
            return 2
    from mlapi_amd import launch

    # ranks on their GPU's NUMA node by default (a node mask, no core slices: core pinning lost at
    # N = 1, profiles/r2_pin/); --pin on = disjoint core slices, off = unpinned
    largv = ["--nproc", str(args.gpus), "--pin", {"auto": "numa", "numa": "numa", "on": "cores", "off": "off"}[args.pin]]
    return launch.main(largv + [os.path.abspath(__file__)] + list(argv))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--mode", default="serve",
                    choices=["serve", "serve_wide", "gemv", "gemm", "train", "train_softmax"])
    ap.add_argument("--conns", type=int, default=64)
    ap.add_argument("--reqs-per-conn", type=int, default=3072,
                    help="serve: one step = conns x this many requests per rank (~0.15-0.25 s, so the "
                         "driver's 20 steps time >= 2 s even at 1.3 M req/s)")
    ap.add_argument("--workload-rows", type=int, default=1024, help="serve: distinct validated requests")
    ap.add_argument("--io-pin", default="sibling", choices=["off", "cores", "llc", "sibling"],
                    help="serve (with --client-pin on): pin server IO thread i - sibling (default): on the SMT "
                         "sibling of load-generator thread i's CPU, the loopback stand-in for an IO thread beside "
                         "its NIC RX queue's CPU (2.44 M req/s median, p99 0.029 ms vs 1.62 M / 0.061 unpinned, "
                         "profiles/r6_iopin/); llc: another CPU of that CPU's last-level cache; cores: physical "
                         "cores of their own (1.27 M: every wake-up crosses cores); off: the scheduler places them")
    ap.add_argument("--client-pin", default="on", choices=["on", "off"],
                    help="serve: pin each load-generator thread to its own CPU of the rank's mask (on: like "
                         "NIC RX queues with pinned interrupts, a connection's segments arrive from one CPU, "
                         "which the server's SO_INCOMING_CPU steering groups by) or leave them floating")
    ap.add_argument("--shuffle-steps", type=int, default=-1,
                    help="serve: steps of the extra phase with the load generator's connections dealt to its "
                         "threads by a seeded permutation (req_per_s_shuffled); -1 = --steps, 0 = skip")
    ap.add_argument("--wide-classes", type=int, default=1000, help="serve_wide: 2 = binary GEMV, else softmax GEMM")
    ap.add_argument("--wide-dtype", default="f64", choices=["f64", "f32", "bf16"],
                    help="serve_wide: kernel operand dtype (f64 = the engine default, sklearn's precision)")
    ap.add_argument("--wide-features", type=int, default=256, help="serve_wide: F")
    ap.add_argument("--client-threads", type=int, default=0, help="0 = auto from the CPUs per rank")
    ap.add_argument("--io-threads", type=int, default=0, help="0 = auto from the CPUs per rank")
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--dispatch", default="source", choices=["source", "acceptor", "reuseport"],
                    help="serve: one acceptor deals connections round robin over client addresses, each "
                         "rank's load generator connecting from its own (default: a client host keeps its "
                         "replica), round robin per connection (acceptor), or hashed by SO_REUSEPORT")
    ap.add_argument("--c1-requests", type=int, default=3000)
    ap.add_argument("--rows", type=int, default=1 << 20)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--gemm-kernel", default="auto", choices=["auto", "split", "tiles", "rows", "t32"],
                    help="gemm: auto = the planner's choice; split = the class-split small-batch kernel; "
                         "tiles / rows / t32 = that gemm_softmax kernel forced (measurement)")
    ap.add_argument("--gemm-dtype", default="bf16", choices=["bf16", "f32"], help="gemm: f32 runs the split kernel")
    ap.add_argument("--launch", default="graph", choices=["graph", "eager"],
                    help="gemv/gemm: the timed K calls replayed from one captured HIP graph (GPU time) or "
                         "dispatched one by one from Python (adds host overhead per call)")
    ap.add_argument("--train-batch", type=int, default=1 << 18)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--softmax-batch", type=int, default=1 << 16)
    ap.add_argument("--softmax-features", type=int, default=256, help="train_softmax: F (any: <= 512 the fused G/dW kernel, wider the 3-launch wide path)")
    ap.add_argument("--cpu", action="store_true", help="force the CPU backend (testing without a GPU)")
    ap.add_argument("--pin", default="auto", choices=["auto", "on", "off", "numa"],
                    help="on: pin this rank to its share of physical cores on its GPU's NUMA node, server "
                         "and load generator on disjoint cores (measured interleaved on one box, core "
                         "pinning cost c=64 throughput at N=1 (0.65-0.80 M vs 0.98-1.06 M req/s) and N=2 "
                         "(0.83-0.85 M vs 0.92-1.02 M), profiles/r2_pin/); numa: this rank and its load "
                         "generator on the GPU's NUMA node (a node mask); auto: numa (N = 1 here, N > 1 "
                         "through mlapi_amd.launch); off: unpinned")
    args = ap.parse_args(argv)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.shuffle_steps < 0:
        args.shuffle_steps = args.steps
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # `python bench.py --gpus N`: start the N rank processes ourselves (one per GPU) through the
        # framework's launcher - fresh child processes, nothing re-exec'd, this parent never touches
        # the GPU. Rank 0's JSON line reaches stdout through the inherited descriptor.
        return _self_launch(args, sys.argv[1:] if argv is None else list(argv))
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks",
              file=sys.stderr)
        return 2
    if args.mode in ("serve", "serve_wide"):
        # the load generator is its own process, started before anything touches the GPU
        from mlapi_amd.serve.loadgen import LoadgenProcess

        args.lg_proc = LoadgenProcess()

    from mlapi_amd.parallel.comm import init_distributed, shutdown

    info = init_distributed(use_gpu=False if args.cpu else None)
    if info.backend == "gloo-fallback":
        # the RCCL communicator failed to initialise: a number measured over the host gloo group
        # would be mislabelled as a GPU-collective run
        print(f"bench.py: rank {info.rank}: RCCL unavailable (gloo fallback); refusing to benchmark", file=sys.stderr)
        return 3
    if info.world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {info.world} rank(s) initialised", file=sys.stderr)
        return 2
    local = int(os.environ.get("LOCAL_WORLD_SIZE", info.world))
    pinned = []
    if args.pin == "auto" and info.device is not None:
        # measured: numa 1.51-1.54 M vs unpinned 1.35-1.53 M req/s (profiles/r5_serve/); at N > 1
        # under torchrun too (bench's own launcher already placed the rank: MLAPI_PLACEMENT set)
        args.pin = "numa"
    if args.pin == "numa" and os.environ.get("MLAPI_PLACEMENT") != "numa":
        # this rank and its load generator on the GPU's NUMA node (a node mask, not core slices):
        # loopback TCP, the pinned request rings and the GPU's host link stay on one socket
        from mlapi_amd.utils.affinity import gpu_numa_nodes, numa_rank_cpus

        dev_index = info.local_rank if info.device is None else info.device.index
        mask = numa_rank_cpus(dev_index, gpu_numa_nodes())
        if mask:
            os.sched_setaffinity(0, mask)
            if getattr(args, "lg_proc", None) is not None:
                args.lg_proc.pin(mask)
            os.environ["MLAPI_PLACEMENT"] = "numa"
    if args.pin == "on":
        # before any native thread starts: the server / batcher / load-generator threads inherit it
        from mlapi_amd.utils.affinity import pin_this_rank

        pinned = pin_this_rank(info.local_rank, local, None if info.device is None else info.device.index)
    args.pinned_cpus = len(pinned)
    if args.io_threads <= 0 or args.client_threads <= 0:
        # Server IO threads and load-generator threads share this rank's CPUs (sweep on a 16-CPU
        # MI355X box share: 6 + 6 threads -> 519k req/s vs 3 + 3 -> 270k; tools/gpu_session.sh threads).
        # The CPU budget is the cgroup quota, not the affinity mask (a 1-GPU box: 256 CPUs in the
        # mask, cpu.max = 16 cores), shared by the ranks of this node.
        from mlapi_amd.parallel.comm import per_rank_cpus

        # core slice: the rank's own; NUMA-node mask: shared by the ranks on that node; both capped
        # by the rank's share of the cgroup quota
        per_rank = max(4, len(pinned) if pinned else per_rank_cpus())
        # measured on a 16-CPU share with the out-of-process load generator. Resident SMALL path
        # (round 5, profiles/r5_serve/ s22-s26, interleaved): equal IO and load-generator thread
        # counts win - the acceptor deals connection k to IO thread k % io and the load generator
        # gives it to its thread k % client, so with io == client each load-generator thread's
        # connections sit on one IO thread (3.7-3.9 us of server CPU per request instead of 4.8-5.1):
        # 8/8 -> 1.94 M req/s median of 9 (1.32-1.97), 10/5 1.76 M median of 11, 7/7 1.64, 6/6
        # 1.67, 8/4 1.52; ratios that are not whole (8/5, 7/5, 9/3, 8/6) 0.95-1.23 M. The batcher
        # path (resident off) had io=10/4 best (profiles/r2_serve_threads/: 0.99-1.11 M; 9/5
        # 0.89-0.93 M; 8/6 0.75-0.94 M)
        cl = max(2, min(6, per_rank // 4))
        # the resident kernel serves the headline's SMALL (Iris) model; serve_wide's F = 256 models
        # take the batcher path
        from mlapi_amd.parallel.comm import resident_auto_ok

        res_env = os.environ.get("MLAPI_RESIDENT", "auto").lower()
        resident = (args.mode == "serve" and info.device is not None
                    and (res_env == "on" or (res_env == "auto" and resident_auto_ok())))
        io = max(2, min(12, per_rank // 2 if resident else per_rank - cl - 2))
        if resident:
            cl = io
        elif args.mode == "serve_wide" and args.client_pin == "on" and args.io_pin != "off":
            # the batcher path with paired placement: half the CPUs to IO threads, two to the batcher
            # and completer, the rest to client threads (each paired with an IO thread on its core):
            # 8 : 6 0.90-0.95 M req/s at 9.7-10.1 us of server CPU per request vs 10 : 4 0.85-0.90 M
            # at 11.2-11.7 (profiles/r6_iopin/r6s18)
            io = max(2, min(12, per_rank // 2))
            cl = max(2, per_rank - io - 2)
        args.io_threads = args.io_threads if args.io_threads > 0 else io
        args.client_threads = args.client_threads if args.client_threads > 0 else cl
    if pinned and getattr(args, "lg_proc", None) is not None and len(pinned) > args.io_threads + 3:
        # server threads (IO + batcher + completer) and the load generator on disjoint CPUs
        import os as _os

        n_srv = args.io_threads + 2
        _os.sched_setaffinity(0, pinned[:n_srv])
        args.lg_proc.pin(pinned[n_srv:])
        args.lg_mask = list(pinned[n_srv:])
    if args.mode != "serve" and info.device is None:
        print(f"mode {args.mode} needs a GPU", file=sys.stderr)
        return 2
    probe = _comm_probe(info)
    if info.world > 1 and probe["comm_nranks"] != info.world:
        print(f"bench.py: communicator reports {probe['comm_nranks']} ranks, expected {info.world}", file=sys.stderr)
        return 2
    fn = {"serve": bench_serve, "serve_wide": bench_serve_wide, "gemv": bench_gemv, "gemm": bench_gemm,
          "train": bench_train, "train_softmax": bench_train_softmax}[args.mode]
    try:
        metric, value, unit, elapsed, extra, config = fn(args, info)
    finally:
        if getattr(args, "lg_proc", None) is not None:
            args.lg_proc.close()
    if info.is_main:
        line = {
            "metric": metric, "value": value, "unit": unit, "n_gpus": info.world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None if BASELINES[args.mode] is None else value / BASELINES[args.mode],
            "dtype": "fp64" if args.mode == "serve" else (args.wide_dtype if args.mode == "serve_wide" else "bf16"),
            "data": "synthetic (random-init weights, fixed synthetic inputs)", "config": config,
            "comm_backend": info.backend,
        }
        line.update(probe)
        line.update(extra)
        print(json.dumps(line), flush=True)
    shutdown(info)
    return 0


if __name__ == "__main__":
    sys.exit(main())
