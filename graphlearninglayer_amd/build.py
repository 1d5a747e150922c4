"""Build libgll.so (HIP kernels + C ABI) for gfx950 with hipcc, in-tree.

    python graphlearninglayer_amd/build.py [--force] [--verbose] [--trace] [--digest]
    (or python -m graphlearninglayer_amd.build once the package imports, i.e. after a build:
    the package refuses to import without its .so files -- there is no CPU fallback)

The shared library lands next to this file so it travels to the GPU box with the repo
snapshot (it is git-ignored).  Each translation unit is compiled separately (in parallel)
and then linked; a unit is rebuilt only when it or a header is newer than its object.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OBJ = os.path.join(HERE, "_obj")
LIB = os.path.join(HERE, "libgll.so")
ARCH = os.environ.get("GLL_OFFLOAD_ARCH", "gfx950")
UNITS = ["knn.hip", "rows.hip", "solve.hip", "gridcg.hip", "grad.hip", "api.hip"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
         "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm >= 7 required)")


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(INCLUDE, "gll.h"))
    return max(os.path.getmtime(h) for h in hs)


def _compile(unit, force, verbose, extra, objdir=OBJ):
    src = os.path.join(CSRC, unit)
    obj = os.path.join(objdir, unit.replace(".hip", ".o"))
    stamp = obj + ".id"
    if unit == "api.hip":
        # api.hip carries the build identity (gll_build_id): rebuilt whenever any input changed
        bid = source_digest()
        extra = [*extra, f'-DGLL_BUILD_ID="{bid}"']
        fresh_id = os.path.exists(stamp) and open(stamp).read() == bid
    else:
        fresh_id = True
    if (not force and fresh_id and os.path.exists(obj)
            and os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime())):
        return obj
    cmd = [hipcc(), *FLAGS, *extra, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    for _ in range(3):
        # hipcc reads the source once per pass (host, device): a file edited mid-compile gives an
        # object whose host stubs and device code disagree, and a newer mtime than the edit.
        # Compare the inputs before and after; on a change, compile again.
        before = _inputs_digest(src)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed on {unit}:\n{r.stdout}\n{r.stderr}")
        if _inputs_digest(src) == before:
            break
    else:
        os.remove(obj)
        raise RuntimeError(f"{unit} kept changing while it compiled")
    if verbose and r.stderr.strip():
        print(r.stderr, file=sys.stderr)
    if unit == "api.hip":
        with open(stamp, "w") as fh:
            fh.write(bid)
    return obj


def source_digest() -> str:
    """Build identity of libgll.so: sha256 (16 hex) over every source and header it is built
    from and the compile flags.  Profile sessions record it (profiles/<tag>_build.json) and
    bench.py cites only the summaries whose identity equals the library it measures."""
    import hashlib
    h = hashlib.sha256(" ".join(FLAGS).encode())
    hs = sorted(f for f in os.listdir(CSRC) if f.endswith(".h"))
    for f in [*UNITS, *hs]:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(INCLUDE, "gll.h"), "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def _inputs_digest(src):
    import hashlib
    h = hashlib.sha256()
    hs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h"))
    for f in [src, *hs, os.path.join(INCLUDE, "gll.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


TRACE_OBJ = os.path.join(OBJ, "trace")
TRACE_LIB = os.path.join(OBJ, "libgll_trace.so")


def build_trace(force=False, verbose=False):
    """Diagnostic variant with in-kernel timestamps (-DGLL_TRACE): _obj/libgll_trace.so,
    loaded only by tools/trace_probe.py -- never by the package."""
    os.makedirs(TRACE_OBJ, exist_ok=True)
    with cf.ThreadPoolExecutor(len(UNITS)) as ex:
        objs = list(ex.map(lambda u: _compile(u, force, verbose, ["-DGLL_TRACE"], TRACE_OBJ),
                           UNITS))
    cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", TRACE_LIB]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return TRACE_LIB


def build(force=False, verbose=False, extra=()):
    os.makedirs(OBJ, exist_ok=True)
    jobs = min(len(UNITS), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda u: _compile(u, force, verbose, list(extra)), UNITS))
    if (force or not os.path.exists(LIB)
            or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs)):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", LIB]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    build_torch_ext(force=force, verbose=verbose)
    return LIB


TORCH_EXT_SRC = os.path.join(CSRC, "torch_ext.cpp")
TORCH_EXT = os.path.join(HERE, "_gll_torch.so")


def build_torch_ext(force=False, verbose=False):
    """The C++ autograd node (csrc/torch_ext.cpp) as a Python extension module linked
    against libgll.so and libtorch; built in-tree so it travels with the repo."""
    if (not force and os.path.exists(TORCH_EXT)
            and os.path.getmtime(TORCH_EXT) >= max(os.path.getmtime(TORCH_EXT_SRC),
                                                   os.path.getmtime(LIB), _headers_mtime())):
        return TORCH_EXT
    import sysconfig

    import torch
    from torch.utils import cpp_extension

    tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared",
           "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_API_INCLUDE_EXTENSION_H",
           "-DTORCH_EXTENSION_NAME=_gll_torch", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           *[f"-I{p}" for p in cpp_extension.include_paths()],
           f"-I{sysconfig.get_paths()['include']}", f"-I{rocm}/include", f"-I{INCLUDE}",
           TORCH_EXT_SRC, "-o", TORCH_EXT,
           f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           "-ltorch_python", f"-L{HERE}", "-lgll", f"-L{rocm}/lib", "-lamdhip64",
           f"-Wl,-rpath,{tlib}", "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"torch extension build failed:\n{r.stdout}\n{r.stderr[-4000:]}")
    return TORCH_EXT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--resource-usage", action="store_true",
                    help="print per-kernel VGPR/SGPR/LDS/occupancy (-Rpass-analysis)")
    ap.add_argument("--trace", action="store_true",
                    help="also build the in-kernel timestamp variant _obj/libgll_trace.so")
    ap.add_argument("--digest", action="store_true", help="print the build identity and exit")
    a = ap.parse_args()
    if a.digest:
        print(source_digest())
        return
    if a.trace:
        print(build_trace(force=a.force, verbose=a.verbose))
    extra = ["-Rpass-analysis=kernel-resource-usage"] if a.resource_usage else []
    print(build(force=a.force or a.resource_usage, verbose=a.verbose or a.resource_usage,
                extra=extra))


if __name__ == "__main__":
    main()
