"""In-tree native build: HIP kernels (hipcc, gfx950) + C++ host runtime (g++).

Outputs go to ``dnn_page_vectors_amd/lib/`` so they travel with the repo
snapshot to the GPU box (``*.so`` is git-ignored, not gpurun-ignored).
Rebuilds are incremental: each object is keyed by a hash of its source, the
shared headers and the compile flags.

    python -m dnn_page_vectors_amd._build          # build everything
    python -m dnn_page_vectors_amd._build --hip    # kernels only
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List, Sequence

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib")
OBJ = os.path.join(PKG, "lib", "obj")

HIP_LIB = os.path.join(LIB, "libpagevec_hip.so")
HIP_DEBUG_LIB = os.path.join(LIB, "libpagevec_hip_debug.so")  # PV_CHECK preconditions compiled in
RT_LIB = os.path.join(LIB, "libpagevec_rt.so")

ARCH = os.environ.get("PAGEVEC_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")

HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-ffp-contract=fast"]
RT_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-sign-compare"]


def _digest(paths: Sequence[str], flags: Sequence[str]) -> str:
    h = hashlib.sha1()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _headers(d: str) -> List[str]:
    out = []
    for root, _, files in os.walk(d):
        for fn in sorted(files):
            if fn.endswith((".h", ".hpp", ".cuh", ".inc")):
                out.append(os.path.join(root, fn))
    return sorted(out)


def _sources(d: str, ext: str) -> List[str]:
    if not os.path.isdir(d):
        return []
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(ext))


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build command failed ({r.returncode}):\n{' '.join(cmd)}\n{r.stdout}")
    if verbose and r.stdout.strip():
        print(r.stdout)


def _objects(srcs: List[str], compiler: str, flags: List[str], incdir: str, tag: str) -> List[str]:
    """Object paths of the sources: each keyed by a digest of its source, the shared headers and
    the flags, so the list (and the link stamp over it) changes with any input."""
    hdrs = _headers(incdir)
    return [os.path.join(OBJ, f"{tag}_{os.path.splitext(os.path.basename(s))[0]}_{_digest([s] + hdrs, flags + [compiler])}.o")
            for s in srcs]


def _stamp_of(objs: List[str]) -> str:
    # object BASENAMES (each carries its source digest): the stamp is the same wherever the tree
    # lives (the GPU box unpacks the snapshot under another absolute path)
    return hashlib.sha1("\n".join(os.path.basename(o) for o in objs).encode()).hexdigest()


def _hip_inputs(debug: bool):
    srcs = _sources(os.path.join(CSRC, "kernels"), ".hip")
    flags = list(HIP_FLAGS) + (["-DPAGEVEC_DEBUG=1"] if debug else [])
    return srcs, flags, os.path.join(CSRC, "kernels"), "hipdbg" if debug else "hip"


def hip_stale(debug: bool = False) -> bool:
    """True when the kernel library is missing or was linked from other sources than the ones in
    the tree (its link stamp differs from the stamp the current sources / headers / flags give)."""
    out = HIP_DEBUG_LIB if debug else HIP_LIB
    stamp = out + ".stamp"
    if not (os.path.exists(out) and os.path.exists(stamp)):
        return True
    srcs, flags, incdir, tag = _hip_inputs(debug)
    with open(stamp) as f:
        return f.read().strip() != _stamp_of(_objects(srcs, HIPCC, flags, incdir, tag))


def hip_stamp(debug: bool = False) -> str:
    """The link stamp of the built kernel library ('' if none)."""
    stamp = (HIP_DEBUG_LIB if debug else HIP_LIB) + ".stamp"
    return open(stamp).read().strip() if os.path.exists(stamp) else ""


def _compile_all(srcs: List[str], compiler: str, flags: List[str], incdir: str, tag: str,
                 jobs: int, verbose: bool) -> List[str]:
    os.makedirs(OBJ, exist_ok=True)
    objs = _objects(srcs, compiler, flags, incdir, tag)
    todo = [(s, o) for s, o in zip(srcs, objs) if not os.path.exists(o)]
    def one(so):
        s, o = so
        tmp = o + ".tmp.o"
        _run([compiler] + flags + ["-I", incdir, "-c", s, "-o", tmp], verbose)
        os.replace(tmp, o)
    if todo:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(one, todo))
    keep = set(objs)
    for f in os.listdir(OBJ):  # drop objects of older source versions
        p = os.path.join(OBJ, f)
        if f.startswith(tag + "_") and f.endswith(".o") and p not in keep:
            os.remove(p)
    return objs


def _link(objs: List[str], out: str, linker: List[str], verbose: bool) -> bool:
    stamp = out + ".stamp"
    key = _stamp_of(objs)
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return False
    tmp = out + ".tmp"
    _run(linker + ["-shared", "-o", tmp] + objs, verbose)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return True


def build_runtime(verbose: bool = False, jobs: int = 4) -> str:
    srcs = _sources(os.path.join(CSRC, "runtime"), ".cpp")
    objs = _compile_all(srcs, CXX, RT_FLAGS, os.path.join(CSRC, "runtime"), "rt", jobs, verbose)
    _link(objs, RT_LIB, [CXX, "-pthread"], verbose)
    return RT_LIB


class _BuildLock:
    """Inter-process lock around a build (ranks of one job may find the library stale together)."""

    def __enter__(self):
        import fcntl

        os.makedirs(LIB, exist_ok=True)
        self.f = open(os.path.join(LIB, ".build.lock"), "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl

        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def build_hip(verbose: bool = False, jobs: int = 4, debug: bool = False) -> str:
    with _BuildLock():
        return _build_hip(verbose, jobs, debug)


def _build_hip(verbose: bool = False, jobs: int = 4, debug: bool = False) -> str:
    """Release kernels -> libpagevec_hip.so; debug=True -> libpagevec_hip_debug.so with the
    PV_CHECK precondition flags (out-of-range ids / keys, LDS indices) compiled in."""
    if not os.path.exists(HIPCC):
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    srcs, flags, incdir, tag = _hip_inputs(debug)
    out = HIP_DEBUG_LIB if debug else HIP_LIB
    objs = _compile_all(srcs, HIPCC, flags, incdir, tag, jobs, verbose)
    _link(objs, out, [HIPCC, f"--offload-arch={ARCH}", "-fPIC"], verbose)
    return out


def build_all(verbose: bool = False, jobs: int = 0) -> None:
    jobs = jobs or min(8, os.cpu_count() or 4)
    build_runtime(verbose, jobs)
    build_hip(verbose, jobs)


def clean() -> None:
    shutil.rmtree(LIB, ignore_errors=True)


def main(argv: Sequence[str] = ()) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hip", action="store_true")
    ap.add_argument("--rt", action="store_true")
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--debug", action="store_true", help="also build libpagevec_hip_debug.so")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(list(argv) or sys.argv[1:])
    if a.clean:
        clean()
    jobs = a.jobs or min(8, os.cpu_count() or 4)
    if a.hip or not a.rt:
        if not a.hip:
            build_runtime(a.verbose, jobs)
        build_hip(a.verbose, jobs)
    elif a.rt:
        build_runtime(a.verbose, jobs)
    if a.debug:
        build_hip(a.verbose, jobs, debug=True)


if __name__ == "__main__":
    main()
