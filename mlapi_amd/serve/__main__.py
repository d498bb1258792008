"""CLI: `python -m mlapi_amd.serve [--port 8000] [--device auto] [--uvicorn] ...`.

Under torchrun (WORLD_SIZE > 1) every rank serves one GPU; rank 0 loads the checkpoint and the
weights are broadcast over RCCL (see mlapi_amd.parallel.dp_serve).
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

from mlapi_amd.utils.config import Config


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m mlapi_amd.serve")
    Config.add_arguments(ap)
    ap.add_argument("--uvicorn", action="store_true", help="serve with uvicorn instead of the native front end")
    a = ap.parse_args(argv)
    cfg = Config.from_args(a)
    logging.basicConfig(level=getattr(logging, cfg.log_level.upper(), logging.WARNING),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from mlapi_amd.parallel.dp_serve import serve_dp, serve_replica

        if os.environ.get("MLAPI_REPLICA_RESTART"):  # relaunched by `mlapi_amd.launch --restart`
            return serve_replica(cfg)
        return serve_dp(cfg)
    if a.uvicorn:
        import uvicorn

        from mlapi_amd.api.app import create_app

        uvicorn.run(create_app(cfg), host=cfg.host, port=cfg.port, log_level=cfg.log_level)
        return 0
    from mlapi_amd.serve.server import NativeServer

    NativeServer(cfg).serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
