"""Native RCCL communicator (csrc/dist/comm.cpp) on the GPU box (one GPU: world_size 1).

Multi-rank RCCL runs need one GPU per rank (RCCL rejects two ranks on one device); the same
collective code paths are covered at world_size 2 on CPU through FakeComm
(tests/test_distributed.py::test_fake_comm_collectives). The one-shot P2P all-reduce runs with
2 and 4 processes sharing the GPU."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
ENV = {**os.environ, "PYTHONPATH": str(ROOT)}


def _launch(nproc, script_args, env, cwd=None):
    """torchrun on a free 127.0.0.1 port. The port is released before torchrun binds it, so another
    process's ephemeral socket can take it in between: only that rendezvous failure (EADDRINUSE)
    is retried, on a new port."""
    import socket

    for attempt in range(3):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr=127.0.0.1", f"--master-port={port}", *script_args]
        out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=cwd)
        if out.returncode != 0 and "EADDRINUSE" in out.stdout + out.stderr and attempt < 2:
            continue
        return out


def test_native_comm_semantics_world1(tmp_path):
    out = _launch(1, [str(ROOT / "tests" / "dist" / "comm_semantics.py")],
                  {**ENV, "OUT": str(tmp_path), "MLAPI_COMM": "native"})
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    assert (tmp_path / "OK_0").read_text() == "native-rccl"


def test_native_comm_uses_torch_rccl_and_aborts():
    from mlapi_amd._native import C
    from mlapi_amd.parallel.rccl import NativeComm, measure_all_reduce

    c = NativeComm(0, 1, torch.device("cuda", 0))
    assert C().RcclComm.version() > 20000
    assert "rccl" in C().RcclComm.library_path()
    t = torch.arange(1 << 20, dtype=torch.float32, device="cuda:0")
    c.all_reduce_(t)
    c.wait(10_000)
    assert torch.equal(t, torch.arange(1 << 20, dtype=torch.float32, device="cuda:0"))
    assert measure_all_reduce(c, 1 << 20, iters=5) < 0.05
    c.abort()
    assert c.aborted
    with pytest.raises(RuntimeError, match="aborted"):
        c.all_reduce_(t)


@pytest.mark.parametrize("mode", ["train", "serve"])
def test_bench_defaults_to_native_comm(mode):
    """MLAPI_COMM unset on a GPU rank -> the framework's C++ RCCL communicator is the data plane."""
    env = {k: v for k, v in ENV.items() if k != "MLAPI_COMM"}
    args = ["--steps", "5", "--warmup", "1"] + (["--reqs-per-conn", "64"] if mode == "serve" else [])
    out = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--mode", mode, *args], env=env,
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["comm_backend"] == "native-rccl"


@pytest.mark.parametrize("world", [2, 4])
def test_p2p_allreduce_multiprocess(tmp_path, world):
    """One-shot P2P all-reduce (csrc/dist/p2p_allreduce.hip) across `world` processes: IPC handles
    exchanged over the TCP store, peers' buffers mapped, bitwise rank-order sums, double-buffered
    epochs, and a bounded wait (status 1, no hang) when a peer never arrives. On the 1-GPU box all
    ranks share the GPU (RCCL itself refuses that), which exercises the same code path."""
    out = _launch(world, [str(ROOT / "tests" / "dist" / "p2p_allreduce.py")],
                  {**ENV, "OUT": str(tmp_path), "OMP_NUM_THREADS": "1"}, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    res = [json.loads((tmp_path / f"P2P_{r}.json").read_text()) for r in range(world)]
    assert all(x["checks"] == 7 for x in res)
    assert res[0]["timed_out"] == 1
    print({"world": world, "us_per_call_256k": [round(x["us_per_call_256k"], 1) for x in res]})


def _torchrun(world, script, out_dir, args=(), env=None):
    path = script if script.endswith("bench.py") else str(ROOT / "tests" / "dist" / script)
    out = _launch(world, [path, *args], {**ENV, "OUT": str(out_dir), "OMP_NUM_THREADS": "1", **(env or {})}, cwd=ROOT)
    assert out.returncode == 0, (out.stdout + out.stderr)[-3000:]
    return out.stdout


def test_dp_sgd_on_gpu_with_p2p_allreduce(tmp_path):
    """Two GPU ranks (sharing the box's GPU) train with HIP gradient kernels and the P2P all-reduce
    as the data plane: replicas stay bitwise identical, match one rank on the global batch, and the
    model broadcast (C1) arrives intact."""
    import numpy as np

    _torchrun(1, "dp_train_gpu.py", tmp_path)
    _torchrun(2, "dp_train_gpu.py", tmp_path)
    _torchrun(2, "dp_train_gpu.py", tmp_path, env={"MLAPI_DP_FUSED": "0"})
    # two-shot exchange (the multiclass gradient: owner ranks reduce + update, the others copy)
    _torchrun(2, "dp_train_gpu.py", tmp_path, env={"MLAPI_DP_TWO_SHOT": "1"})
    for r in range(2):
        assert np.array_equal(np.load(tmp_path / f"mc_params_2_{r}_two.npy"), np.load(tmp_path / f"mc_params_2_{r}.npy")), \
            "two-shot exchange must give the one-shot replicas bitwise"
    for name in ("params", "mc_params"):
        a, b = np.load(tmp_path / f"{name}_2_0.npy"), np.load(tmp_path / f"{name}_2_1.npy")
        assert np.array_equal(a, b), f"{name}: DP replicas must stay bitwise identical"
        # the in-kernel exchange sums ranks in the same order as the all-reduce kernel: bitwise equal
        u = np.load(tmp_path / f"{name}_2_0_unfused.npy")
        assert np.array_equal(a, u), f"{name}: fused DP step must equal gradient + all-reduce + update bitwise"
        assert np.array_equal(u, np.load(tmp_path / f"{name}_2_1_unfused.npy"))
        np.testing.assert_allclose(a, np.load(tmp_path / f"{name}_1_0.npy"), rtol=2e-3, atol=2e-4)
    j0, j1 = (json.loads((tmp_path / f"bcast_2_{r}.json").read_text()) for r in range(2))
    assert j0["W"] == j1["W"] and j0["classes"] == list("abcde")
    assert j0["p2p_calls"] >= 35 and j0["acc"] > 0.8


def test_dp_fused_exchange_times_out_without_a_peer(tmp_path):
    """Rank 1 never joins a fused DP step: rank 0's in-kernel wait gives up (status 1, no hang),
    its update is skipped, and check() raises."""
    _torchrun(2, "dp_fused_timeout.py", tmp_path)
    res = json.loads((tmp_path / "timeout_0.json").read_text())
    assert res["raised"] and res["params_unchanged"] and res["elapsed_s"] < 30
    assert res["next_step_raised"], "the step after a missed exchange must stop the loop"


def test_p2p_selftest_failure_falls_back(tmp_path):
    """A rank whose IPC self-test pattern arrives wrong (MLAPI_P2P_SELFTEST_CORRUPT) makes every
    rank drop the fused in-kernel exchange for the unfused all-reduce path; training still runs and
    the replicas stay bitwise identical."""
    import numpy as np

    _torchrun(2, "p2p_selftest.py", tmp_path, env={"MLAPI_P2P_SELFTEST_CORRUPT": "1"})
    for r in range(2):
        res = json.loads((tmp_path / f"selftest_{r}.json").read_text())
        assert res["p2p_selftest"] == "failed" and res["dp_exchange"] == "rccl", res
        assert res["p2p_verify"] == "failed:ipc-pattern", res
    assert np.array_equal(np.load(tmp_path / "st_params_0.npy"), np.load(tmp_path / "st_params_1.npy"))


def test_p2p_verify_passes_on_a_healthy_exchange(tmp_path):
    """the fused exchange kernel itself, on a rank-tagged synthetic gradient, is
    bitwise equal to the exact sum before the first step; the job keeps the fused exchange."""
    import numpy as np

    _torchrun(2, "p2p_selftest.py", tmp_path, env={"MLAPI_DP_VERIFY_EVERY": "2"})
    for r in range(2):
        res = json.loads((tmp_path / f"selftest_{r}.json").read_text())
        assert res["p2p_verify"] == "ok" and res["dp_exchange"] == "fused-p2p", res
    assert np.array_equal(np.load(tmp_path / "st_params_0.npy"), np.load(tmp_path / "st_params_1.npy"))


def test_p2p_verify_stale_flag_falls_back(tmp_path):
    """A rank that skips one block's flag publish in the verification launch (a stale flag for its
    peer, MLAPI_P2P_VERIFY_FAULT): the peer's bounded wait times out, the verdict (max over ranks)
    is 'failed:fused-timeout' on every rank and the job trains on the unfused all-reduce path,
    replicas bitwise identical."""
    import numpy as np

    _torchrun(2, "p2p_selftest.py", tmp_path, env={"MLAPI_P2P_VERIFY_FAULT": "1", "MLAPI_P2P_VERIFY_TIMEOUT_MS": "500"})
    for r in range(2):
        res = json.loads((tmp_path / f"selftest_{r}.json").read_text())
        assert res["p2p_verify"] == "failed:fused-timeout" and res["dp_exchange"] == "rccl", res
    assert np.array_equal(np.load(tmp_path / "st_params_0.npy"), np.load(tmp_path / "st_params_1.npy"))


def test_p2p_periodic_replica_check_resyncs(tmp_path):
    """A replica that diverges mid-run (rank 1's parameters nudged after step 3) is caught by the
    replica-hash check at step 4 (MLAPI_DP_VERIFY_EVERY=2): fused exchange off, every replica re-synced
    to rank 0's parameters, training continues bitwise identical."""
    import numpy as np

    _torchrun(2, "p2p_selftest.py", tmp_path, env={"MLAPI_DP_VERIFY_EVERY": "2", "CORRUPT_AT_STEP": "3"})
    for r in range(2):
        res = json.loads((tmp_path / f"selftest_{r}.json").read_text())
        assert res["dp_exchange_first"] == "fused-p2p", res
        assert res["p2p_verify"] == "failed:param-hash" and res["dp_exchange"] == "rccl", res
    assert np.array_equal(np.load(tmp_path / "st_params_0.npy"), np.load(tmp_path / "st_params_1.npy"))


@pytest.mark.parametrize("mode", ["serve", "serve_wide"])
def test_dp_serving_bench_two_gpu_ranks(tmp_path, mode):
    """The driver's multi-GPU launch shape (torchrun, one rank per device) on the 1-GPU box: two
    ranks share the GPU (MLAPI_COMM=p2p: RCCL refuses two ranks on one device), each with its own
    engine and out-of-process load generator behind ONE SO_REUSEPORT port; every response body
    is validated and both ranks serve."""
    out = _torchrun(2, str(ROOT / "bench.py"), tmp_path,
                    args=["--gpus", "2", "--mode", mode, "--steps", "3", "--warmup", "1", "--reqs-per-conn", "64",
                          "--c1-requests", "200"], env={"MLAPI_COMM": "p2p"})
    line = json.loads(out.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["comm_backend"] == "p2p+gloo" and line["body_mismatches"] == 0
    assert line["config"]["parallelism"] == "dp2" and line["value"] > 0
    assert len(line["served_per_rank"]) == 2 and min(line["served_per_rank"]) > 0, line["served_per_rank"]
