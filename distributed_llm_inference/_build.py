"""In-tree build of the native extensions (no JIT cache, no hipify, no setuptools magic).

* ``_C``        — CDNA4 kernels (``csrc/kernels/*.hip``, compiled by hipcc for gfx950 only),
                  their torch bindings and the RCCL communicator (``csrc/bindings.hip``,
                  ``csrc/comm/rccl_p2p.hip``).
* ``_runtime``  — torch-free C++ host runtime (block manager, shared-memory channels), built with
                  g++ so CPU-only tests can use it.

Both land next to this file so the built ``.so`` travels with the repository snapshot to the GPU
box.  Rebuilds are incremental (object files are cached under ``build/``).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List, Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
BUILD_DIR = os.path.join(REPO_DIR, "build", "native")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("DLI_OFFLOAD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

KERNEL_SOURCES = ["kernels/norm.hip", "kernels/activation.hip", "kernels/rope_cache.hip",
                  "kernels/attention.hip", "kernels/attn_prefill32.hip", "kernels/sampling.hip", "kernels/quant.hip",
                  "kernels/gemv.hip", "kernels/gemm_tile.hip", "kernels/gemm4.hip",
                  "kernels/int8_outlier.hip", "kernels/digest.hip"]
TORCH_SOURCES = ["bindings.hip", "comm/rccl_p2p.hip", "comm/streams.hip"]
RUNTIME_SOURCES = ["runtime/block_manager.cpp", "runtime/shm_channel.cpp"]


def kernels_so_path() -> str:
    return os.path.join(PKG_DIR, "_C" + EXT_SUFFIX)


def runtime_so_path() -> str:
    return os.path.join(PKG_DIR, "_runtime" + EXT_SUFFIX)


def _headers() -> List[str]:
    out = []
    for root, _, files in os.walk(CSRC):
        out += [os.path.join(root, f) for f in files if f.endswith((".h", ".hpp", ".cuh"))]
    return out


def _mtime(paths) -> float:
    return max((os.path.getmtime(p) for p in paths if os.path.exists(p)), default=0.0)


def _content_hash(paths: List[str], extra: str = "") -> str:
    h = hashlib.sha1(extra.encode())
    for p in sorted(paths):
        if os.path.exists(p):
            h.update(os.path.relpath(p, PKG_DIR).encode())
            with open(p, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def _up_to_date(out: str, deps: List[str], extra: str) -> bool:
    """The built ``out`` matches the sources: by the content hash recorded next to it at build
    time (robust to a copy that does not preserve mtimes, e.g. a repository snapshot shipped to
    another machine), else — no record yet — by modification times."""
    if not os.path.exists(out):
        return False
    rec = out + ".srchash"
    if os.path.exists(rec):
        with open(rec) as f:
            return f.read().strip() == _content_hash(deps, extra)
    return os.path.getmtime(out) >= _mtime(deps)


def _record(out: str, deps: List[str], extra: str) -> None:
    with open(out + ".srchash", "w") as f:
        f.write(_content_hash(deps, extra) + "\n")


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    if verbose and r.stdout.strip():
        print(r.stdout)


def _py_includes() -> List[str]:
    import pybind11
    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = [f"-I{p}" for p in inc + _py_includes()] + [
        "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-DHIPBLAS_V2",
        "-D__HIP_PLATFORM_AMD__=1",
    ]
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-ltorch", "-ltorch_cpu",
               "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64", "-lrccl"]
    return cflags, ldflags


def _compile_many(jobs, verbose: bool, workers: int) -> None:
    if not jobs:
        return
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        futs = [ex.submit(_run, cmd, verbose) for cmd in jobs]
        for f in futs:
            f.result()


def _check_own_symbols(so: str) -> None:
    """A shared object may link with undefined symbols; one of our own (namespace ``dli``) left
    undefined means a launcher was declared but not compiled in, and would only fail at import on
    the GPU box -- fail the build here instead."""
    nm = shutil.which("nm") or os.path.join(ROCM, "lib", "llvm", "bin", "llvm-nm")
    if not os.path.exists(nm):
        return
    r = subprocess.run([nm, "-D", "--undefined-only", "-C", so], capture_output=True, text=True)
    missing = [l.split(None, 1)[-1] for l in r.stdout.splitlines() if " dli::" in f" {l.split(None, 1)[-1]}"]
    if missing:
        os.remove(so)
        raise RuntimeError("native kernels: undefined dli symbols (declared, never defined): "
                           + "; ".join(missing[:8]))


def build_kernels(force: bool = False, verbose: bool = False, workers: Optional[int] = None) -> str:
    """Compile the gfx950 kernels + torch bindings into ``_C``; returns the .so path."""
    hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    out = kernels_so_path()
    srcs = [os.path.join(CSRC, s) for s in KERNEL_SOURCES + TORCH_SOURCES]
    srcs = [s for s in srcs if os.path.exists(s)]
    deps = srcs + _headers() + [__file__]
    if not force and _up_to_date(out, deps, ARCH):
        return out
    os.makedirs(BUILD_DIR, exist_ok=True)
    tcflags, ldflags = _torch_flags()
    base = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast",
            f"-I{CSRC}", "-Wno-unused-result", "-Wno-deprecated-declarations"]
    hdr_m = _mtime(_headers() + [__file__])
    jobs, objs = [], []
    for s in srcs:
        rel = os.path.relpath(s, CSRC)
        is_torch = rel in TORCH_SOURCES
        flags = base + (tcflags if is_torch else [])
        key = hashlib.sha1(" ".join(flags).encode()).hexdigest()[:8]
        obj = os.path.join(BUILD_DIR, rel.replace("/", "_") + f".{key}.o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(s), hdr_m):
            jobs.append(flags + ["-c", s, "-o", obj])
    _compile_many(jobs, verbose, workers or min(8, os.cpu_count() or 4))
    tmp = out + ".tmp"
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ldflags, verbose)
    _check_own_symbols(tmp)
    os.replace(tmp, out)
    _record(out, deps, ARCH)
    return out


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    """Compile the torch-free host runtime into ``_runtime`` with the system C++ compiler."""
    out = runtime_so_path()
    srcs = [os.path.join(CSRC, s) for s in RUNTIME_SOURCES]
    deps = srcs + _headers() + [__file__]
    if not force and _up_to_date(out, deps, "runtime"):
        return out
    cxx = os.environ.get("CXX") or shutil.which("g++") or "c++"
    tmp = out + ".tmp"
    cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden"] + \
          [f"-I{p}" for p in _py_includes()] + srcs + ["-o", tmp, "-lrt", "-pthread"]
    _run(cmd, verbose)
    os.replace(tmp, out)
    _record(out, deps, "runtime")
    return out


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_runtime(force=force, verbose=verbose)
    build_kernels(force=force, verbose=verbose)


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--runtime-only", action="store_true")
    a = ap.parse_args()
    build_runtime(a.force, a.verbose)
    if not a.runtime_only:
        build_kernels(a.force, a.verbose)
    print("built:", runtime_so_path(), "" if a.runtime_only else kernels_so_path())
    sys.exit(0)
