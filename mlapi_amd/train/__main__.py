"""Training CLI.

``python -m mlapi_amd.train iris [--out LRClassifier.pkl]`` reproduces the reference notebook
(`Logistic Regression.ipynb:18-43`): load Iris (sklearn's bundled copy relabelled to the UCI class
names — the UCI URL is not reachable offline), 80/20 split with random_state=1, fit
LogisticRegression() (L-BFGS, C=1), pickle it to LRClassifier.pkl, reload it, print the test score
(0.9666666666666667).

``python -m mlapi_amd.train csv data.csv --target class [--out ...]`` does the same for any CSV.

``torchrun --nproc-per-node N -m mlapi_amd.train sgd --features 256 --rows-per-rank 1048576 ...``
runs data-parallel mini-batch SGD on synthetic data (BASELINE config 5) with checkpoint/resume
in the native format (``--ckpt``; ``--resume``). ``--classes K`` (K > 2) trains a softmax
(``--kind multinomial``) or one-vs-rest model with the MFMA gradient kernels; ``--graph``
captures a single-GPU step in a HIP graph.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

UCI_IRIS_LABELS = np.array(["Iris-setosa", "Iris-versicolor", "Iris-virginica"], dtype=object)


def iris_dataset():
    from sklearn.datasets import load_iris

    d = load_iris()
    return d.data.astype(np.float64), UCI_IRIS_LABELS[d.target]


def split(X, y, test_size=0.2, random_state=1):
    from sklearn.model_selection import train_test_split

    return train_test_split(X, y, test_size=test_size, random_state=random_state, shuffle=True)


def cmd_fit(X, y, args) -> int:
    from mlapi_amd.models.estimator import LogisticRegression

    Xtr, Xte, ytr, yte = split(X, y)
    clf = LogisticRegression(C=args.C, max_iter=args.max_iter, device=args.device).fit(Xtr, ytr)
    clf.save(args.out, format=args.format)
    loaded = LogisticRegression.load(args.out, device=args.device)
    print(loaded.score(Xte, yte))
    return 0


def cmd_sgd(args) -> int:
    import torch

    if args.classes > 2:
        return cmd_sgd_multiclass(args)

    from mlapi_amd.ckpt.native import TrainState, load_native, save_native
    from mlapi_amd.parallel.comm import barrier, init_distributed, shutdown
    from mlapi_amd.train.schedule import BatchSchedule
    from mlapi_amd.train.sgd import BinarySGDTrainer, synthetic_binary

    info = init_distributed()
    dev = info.device
    X, y = synthetic_binary(args.rows_per_rank, args.features, seed=1000 + info.rank, device=dev,
                            dtype=torch.bfloat16 if dev is not None else torch.float32)
    tr = BinarySGDTrainer(args.features, info=info, lr=args.lr, l2=args.l2, momentum=args.momentum, device=dev)
    nb = max(1, args.rows_per_rank // args.batch)
    sched = BatchSchedule(nb, seed=args.seed, shuffle=not args.no_shuffle)
    start = 0
    if args.resume and os.path.exists(args.ckpt):
        model, st = load_native(args.ckpt)
        tr.params.copy_(torch.as_tensor(np.concatenate([model.W[0], model.b]), dtype=torch.float32))
        if tr.mom is not None and "mom" in st.opt:
            tr.mom.copy_(torch.as_tensor(st.opt["mom"], dtype=torch.float32))
        start = st.step
        tr.steps = start
        sched.restore(st.epoch, st.data_cursor, st.rng_state)
        if info.is_main:
            print(f"resumed from {args.ckpt} at step {start} (epoch {st.epoch}, batch {st.data_cursor})", flush=True)
    t0 = time.perf_counter()
    for step in range(start, args.steps):
        j = sched.next()
        tr.step(X[j * args.batch:(j + 1) * args.batch], y[j * args.batch:(j + 1) * args.batch])
        if info.is_main and (step + 1) % args.log_every == 0:
            print(json.dumps({"step": step + 1, "loss": tr.last_loss(), "acc": tr.last_accuracy()}), flush=True)
        if args.ckpt and (step + 1) % args.ckpt_every == 0:
            barrier(info)
            if info.is_main:
                st = TrainState(step=step + 1, epoch=sched.epoch, data_cursor=sched.cursor,
                                rng_state=sched.rng_state(),
                                opt={} if tr.mom is None else {"mom": tr.mom.cpu().numpy()}, config=vars(args))
                save_native(args.ckpt, tr.to_model(), st)
    if dev is not None:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if info.is_main:
        n = (args.steps - start) * args.batch * info.world
        print(json.dumps({"samples_per_s": n / max(dt, 1e-9), "final_loss": tr.last_loss(),
                          "final_acc": tr.last_accuracy(), "world": info.world}), flush=True)
        if args.out:
            from mlapi_amd.ckpt.sklearn_pickle import export_sklearn_pickle

            export_sklearn_pickle(tr.to_model(), args.out)
    shutdown(info)
    return 0


def cmd_sgd_multiclass(args) -> int:
    import torch

    from mlapi_amd.ckpt.native import TrainState, load_native, save_native
    from mlapi_amd.models.linear import Kind
    from mlapi_amd.parallel.comm import barrier, init_distributed, shutdown
    from mlapi_amd.train.schedule import BatchSchedule
    from mlapi_amd.train.softmax_sgd import SoftmaxSGDTrainer, synthetic_multiclass

    info = init_distributed()
    dev = info.device
    kind = Kind.OVR if args.kind == "ovr" else Kind.MULTINOMIAL
    X, y = synthetic_multiclass(args.rows_per_rank, args.features, args.classes, seed=1000 + info.rank,
                                device=dev, noise=args.noise)
    tr = SoftmaxSGDTrainer(args.features, args.classes, kind=kind, info=info, lr=args.lr, l2=args.l2,
                           momentum=args.momentum, device=dev)
    Xa = tr.prepare(X)
    del X
    nb = max(1, args.rows_per_rank // args.batch)
    sched = BatchSchedule(nb, seed=args.seed, shuffle=not args.no_shuffle)
    start = 0
    if args.resume and os.path.exists(args.ckpt):
        model, st = load_native(args.ckpt)
        tr.set_params(torch.as_tensor(model.W, dtype=torch.float32), torch.as_tensor(model.b, dtype=torch.float32))
        if tr.mom is not None and "mom" in st.opt:
            tr.mom.copy_(torch.as_tensor(st.opt["mom"], dtype=torch.float32))
        start = tr.steps = st.step
        sched.restore(st.epoch, st.data_cursor, st.rng_state)
        if info.is_main:
            print(f"resumed from {args.ckpt} at step {start} (epoch {st.epoch}, batch {st.data_cursor})", flush=True)
    shards = [(Xa[j * args.batch:(j + 1) * args.batch], y[j * args.batch:(j + 1) * args.batch]) for j in range(nb)]
    if args.graph and dev is not None and info.world == 1 and nb == 1:  # one batch: order is moot
        tr.capture(*shards[0])  # one HIP graph launch per step
    t0 = time.perf_counter()
    for step in range(start, args.steps):
        tr.step(*shards[sched.next()])
        if info.is_main and (step + 1) % args.log_every == 0:
            print(json.dumps({"step": step + 1, "loss": tr.last_loss(), "acc": tr.last_accuracy()}), flush=True)
        if args.ckpt and (step + 1) % args.ckpt_every == 0:
            barrier(info)
            if info.is_main:
                st = TrainState(step=step + 1, epoch=sched.epoch, data_cursor=sched.cursor,
                                rng_state=sched.rng_state(),
                                opt={} if tr.mom is None else {"mom": tr.mom.cpu().numpy()}, config=vars(args))
                save_native(args.ckpt, tr.to_model(), st)
    if dev is not None:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if info.is_main:
        n = (args.steps - start) * args.batch * info.world
        print(json.dumps({"samples_per_s": n / max(dt, 1e-9), "final_loss": tr.last_loss(),
                          "final_acc": tr.last_accuracy(), "world": info.world, "classes": args.classes}),
              flush=True)
        if args.out:
            from mlapi_amd.ckpt.sklearn_pickle import export_sklearn_pickle

            export_sklearn_pickle(tr.to_model(), args.out)
    shutdown(info)
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m mlapi_amd.train")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("iris", "csv"):
        p = sub.add_parser(name)
        p.add_argument("--out", default="LRClassifier.pkl")
        p.add_argument("--format", default="sklearn", choices=["sklearn", "native"])
        p.add_argument("--C", type=float, default=1.0)
        p.add_argument("--max-iter", type=int, default=100)
        p.add_argument("--device", default="auto")
        if name == "csv":
            p.add_argument("path")
            p.add_argument("--target", required=True)
    p = sub.add_parser("sgd")
    p.add_argument("--features", type=int, default=256)
    p.add_argument("--rows-per-rank", type=int, default=1 << 20)
    p.add_argument("--batch", type=int, default=1 << 16)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--lr", type=float, default=0.5)
    p.add_argument("--l2", type=float, default=1e-6)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--log-every", type=int, default=50)
    p.add_argument("--ckpt", default="")
    p.add_argument("--ckpt-every", type=int, default=100)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--out", default="")
    p.add_argument("--classes", type=int, default=2, help="> 2: multiclass (softmax / one-vs-rest) SGD")
    p.add_argument("--kind", default="multinomial", choices=["multinomial", "ovr"])
    p.add_argument("--noise", type=float, default=1.0, help="multiclass synthetic label noise")
    p.add_argument("--graph", action="store_true", help="capture the single-GPU step in a HIP graph")
    p.add_argument("--seed", type=int, default=0, help="mini-batch order (epoch shuffles; same on every rank)")
    p.add_argument("--no-shuffle", action="store_true", help="visit the batches in order every epoch")
    args = ap.parse_args(argv)
    if args.cmd == "iris":
        X, y = iris_dataset()
        return cmd_fit(X, y, args)
    if args.cmd == "csv":
        import pandas as pd

        df = pd.read_csv(args.path)
        y = df.pop(args.target).to_numpy()
        return cmd_fit(df.to_numpy(dtype=np.float64), y, args)
    return cmd_sgd(args)


if __name__ == "__main__":
    sys.exit(main())
