"""Build the native extension ``mlapi_amd._C`` in-tree with hipcc for gfx950.

Every source (HIP kernels, C++ runtime, HTTP server, bindings) is compiled by ``hipcc
--offload-arch=gfx950`` in parallel and linked into ``mlapi_amd/_C<ext-suffix>.so``. No hipify,
no torch cpp_extension: the extension links only libamdhip64 (resolved at import time to the
HIP runtime torch already loaded, see :mod:`mlapi_amd._native`).

Rebuilds are decided by content, not mtimes: every object, the extension, the load generator and
the serving code object carry a ``<file>.sha256`` stamp of the exact source bytes, headers, flags
and compiler they were built from (:func:`stamp_matches` lets callers check an in-tree binary).

Usage: ``python -m mlapi_amd._build [--force] [--jobs N]``.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("MLAPI_OFFLOAD_ARCH", "gfx950")
ROCM_LIB = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib"

SOURCES = [
    "kernels/linear_small.hip",
    "kernels/gemv_binary.hip",
    "kernels/gemm_softmax.hip",
    "kernels/linear_split.hip",
    "kernels/linear_wide.hip",
    "kernels/train.hip",
    "kernels/pack.hip",
    "kernels/shard.hip",
    "kernels/softmax_grad_dw.hip",
    "kernels/softmax_grad_wide.hip",
    "kernels/xcd.hip",
    "runtime/engine.cpp",
    "runtime/direct_dispatch.cpp",
    "http/server.cpp",
    "http/json_body.cpp",
    "http/dispatch.cpp",
    "http/loadgen.cpp",
    "dist/comm.cpp",
    "dist/p2p_allreduce.hip",
    "bindings.cpp",
]


# Per-source extra flags. gemm_softmax.hip: MFMA results in VGPRs (on gfx950 the register file is
# unified; hipcc's default put the accumulators in AGPRs and paid a v_accvgpr_read per element in
# the softmax epilogue - 96 extra moves per class chunk).
FILE_FLAGS = {
    "kernels/gemm_softmax.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build mlapi_amd._C)")


def ext_path() -> Path:
    return ROOT / "mlapi_amd" / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _includes() -> list:
    import pybind11

    return [f"-I{CSRC}", f"-I{CSRC / 'include'}", f"-I{pybind11.get_include()}",
            f"-I{sysconfig.get_paths()['include']}"]


def _flags() -> list:
    return ["-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"--offload-arch={ARCH}",
            "-Wno-unused-result", "-Wno-unused-command-line-argument"]


def _headers_digest() -> str:
    """Content hash of every header under csrc/ (any source may include any of them)."""
    h = hashlib.sha256()
    for p in sorted(CSRC.rglob("*.h")):
        h.update(str(p.relative_to(CSRC)).encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _digest(*parts) -> str:
    h = hashlib.sha256()
    for x in parts:
        h.update(x if isinstance(x, bytes) else str(x).encode())
        h.update(b"\0")
    return h.hexdigest()


def _stamp_ok(out: Path, digest: str) -> bool:
    st = Path(str(out) + ".sha256")
    return out.exists() and st.exists() and st.read_text().strip() == digest


def _write_stamp(out: Path, digest: str) -> None:
    Path(str(out) + ".sha256").write_text(digest + "\n")


def _compile(src: str, force: bool, hdig: str) -> Path:
    """Compile one source unless its object was built from exactly these bytes: the stamp is a
    content hash of the source, every header and the compiler flags (not mtimes: a tree copied
    with fresh timestamps - or an old object with a new mtime - is judged by what it contains)."""
    s = CSRC / src
    obj = BUILD / (src.replace("/", "__") + ".o")
    dig = _digest(s.read_bytes(), hdig, hipcc(), _flags(), FILE_FLAGS.get(src, []), _includes())
    if not force and _stamp_ok(obj, dig):
        return obj
    cmd = [hipcc()] + _flags() + FILE_FLAGS.get(src, []) + _includes()
    if s.suffix == ".cpp":
        cmd += ["-x", "hip"] if src == "bindings.cpp" else []
    cmd += ["-c", str(s), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    _write_stamp(obj, dig)
    return obj


def loadgen_path() -> Path:
    return ROOT / "mlapi_amd" / "bin" / "mlapi-loadgen"


def _build_loadgen(force: bool, verbose: bool) -> Path:
    """The standalone load-generator process (csrc/http/loadgen_main.cpp + loadgen.cpp): host-only
    C++, no HIP, so benchmarks can run it on CPUs apart from the server."""
    out = loadgen_path()
    srcs = [CSRC / "http" / "loadgen_main.cpp", CSRC / "http" / "loadgen.cpp"]
    cxx = shutil.which("g++") or shutil.which("c++") or hipcc()
    dig = _digest(*[p.read_bytes() for p in srcs], _headers_digest(), cxx)
    if not force and _stamp_ok(out, dig):
        return out
    out.parent.mkdir(parents=True, exist_ok=True)
    cmd = [cxx, "-O2", "-std=c++17", f"-I{CSRC}", "-o", str(out) + ".tmp"] + [str(p) for p in srcs] + ["-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"loadgen build failed:\n{r.stderr[-4000:]}")
    os.replace(str(out) + ".tmp", out)
    _write_stamp(out, dig)
    if verbose:
        print(f"[mlapi_amd] built {out.relative_to(ROOT)}", file=sys.stderr)
    return out


def hsaco_path() -> Path:
    return ROOT / "mlapi_amd" / "serve_kernels.hsaco"


def _build_hsaco(force: bool, verbose: bool) -> Path:
    """The engine's directly dispatched serving kernels (csrc/kernels/serve_direct.hip) as a plain
    gfx950 code object the HSA loader reads (csrc/runtime/direct_dispatch.cpp); not part of _C."""
    out = hsaco_path()
    src = CSRC / "kernels" / "serve_direct.hip"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "--cuda-device-only", "--no-gpu-bundle-output", "-O3", "-std=c++17"] + \
        _includes() + [str(src), "-o", str(out) + ".tmp"]
    dig = _digest(src.read_bytes(), _headers_digest(), cmd[:-3])
    if not force and _stamp_ok(out, dig):
        return out
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for serve_direct.hip:\n{r.stderr[-4000:]}")
    os.replace(str(out) + ".tmp", out)
    _write_stamp(out, dig)
    if verbose:
        print(f"[mlapi_amd] built {out.relative_to(ROOT)}", file=sys.stderr)
    return out


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    BUILD.mkdir(parents=True, exist_ok=True)
    hdig = _headers_digest()
    jobs = jobs or min(len(SOURCES), max(1, min(8, os.cpu_count() or 1)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, hdig), SOURCES))
    out = ext_path()
    link = [f"-L{ROCM_LIB}", "-lhsa-runtime64", "-lpthread", "-ldl"]
    dig = _digest(*[Path(str(o) + ".sha256").read_text() for o in objs], link)
    if force or not _stamp_ok(out, dig):
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(out) + ".tmp"] + \
              [str(o) for o in objs] + link
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        os.replace(str(out) + ".tmp", out)
        _write_stamp(out, dig)
        if verbose:
            print(f"[mlapi_amd] built {out.relative_to(ROOT)}", file=sys.stderr)
    _build_loadgen(force, verbose)
    _build_hsaco(force, verbose)
    return out


def stamp_matches() -> bool:
    """True when the in-tree extension was built from the current sources (by content)."""
    hdig = _headers_digest()
    digs = []
    for src in SOURCES:
        s = CSRC / src
        obj = BUILD / (src.replace("/", "__") + ".o")
        d = _digest(s.read_bytes(), hdig, hipcc(), _flags(), FILE_FLAGS.get(src, []), _includes())
        if not _stamp_ok(obj, d):
            return False
        digs.append(d)
    link = [f"-L{ROCM_LIB}", "-lhsa-runtime64", "-lpthread", "-ldl"]
    return _stamp_ok(ext_path(), _digest(*[d + "\n" for d in digs], link))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build(force=a.force, jobs=a.jobs)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
