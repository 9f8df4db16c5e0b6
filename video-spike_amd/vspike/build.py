"""Build libvspike.so (hipcc, gfx950 only) in-tree: video-spike_amd/vspike/_build/libvspike.so.

No torch extension machinery: the library is a plain C-ABI shared object (include/vspike.h)
loaded with ctypes, so it builds in seconds and travels with the repo snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.join(os.path.dirname(PKG_DIR), "csrc")
ROOT = os.path.dirname(os.path.dirname(PKG_DIR))
INCLUDE = os.path.join(ROOT, "include")
BUILD_DIR = os.path.join(PKG_DIR, "_build")
LIB_PATH = os.path.join(BUILD_DIR, "libvspike.so")
ARCH = "gfx950"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libvspike)")


def _flags():
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", SRC_DIR,
            "-Wno-unused-result", "-munsafe-fp-atomics"]


def _sources():
    srcs = sorted(glob.glob(os.path.join(SRC_DIR, "*.hip"))) + sorted(glob.glob(os.path.join(SRC_DIR, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(SRC_DIR, "*.h"))) + [os.path.join(INCLUDE, "vspike.h")]
    return srcs, headers


def source_hash(defines=()) -> str:
    """sha256 prefix over every source and header the library is compiled from (by file name and
    content, in name order) plus the target, any extra -D defines and the compile flags: the id
    `vs_build_id()` of a library built from exactly these sources with these flags returns."""
    h = hashlib.sha256()
    srcs, headers = _sources()
    for f in sorted(srcs + headers, key=os.path.basename):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    h.update(("|".join([ARCH] + sorted(defines))).encode())
    # the compile flags too (a flags-only change must change the id); the include directories by
    # their repo-relative names, so the id is the same in every checkout of the tree
    rel = {INCLUDE: "include", SRC_DIR: "csrc"}
    h.update(("|".join(rel.get(f, f) for f in _flags())).encode())
    return h.hexdigest()[:16]


def _needs(obj: str, deps) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = True, jobs: int = 8, variant: str = "", defines=()) -> str:
    """Compile + link.  `variant` builds a diagnostic copy (objects under _build/<variant>/, library
    _build/libvspike_<variant>.so) with extra `-D` defines, e.g. ("wt", ["VS_WT_STORES"])."""
    obj_dir = os.path.join(BUILD_DIR, variant) if variant else BUILD_DIR
    lib_path = os.path.join(BUILD_DIR, f"libvspike_{variant}.so") if variant else LIB_PATH
    os.makedirs(obj_dir, exist_ok=True)
    hipcc = _hipcc()
    dflags = [f"-D{d}" for d in defines]
    srcs, headers = _sources()
    bid = source_hash(defines)
    stamp = os.path.join(obj_dir, "build_id")
    old_bid = open(stamp).read().strip() if os.path.exists(stamp) else ""
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(obj_dir, os.path.splitext(os.path.basename(s))[0] + ".o")
        objs.append(o)
        # runtime.hip carries the build id: recompiled whenever any source changed
        if force or _needs(o, [s] + headers) or (os.path.basename(s) == "runtime.hip" and old_bid != bid):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        if s.endswith(".cpp"):     # host-only code (shard reader): plain C++
            cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-I", INCLUDE, "-c", s, "-o", o]
        else:
            cmd = [hipcc, *_flags(), *dflags, "-c", s, "-o", o]
            if os.path.basename(s) == "runtime.hip":
                cmd.insert(-4, f'-DVS_BUILD_ID="{bid}"')
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed for {os.path.basename(s)}:\n{r.stderr[-6000:]}")
        return s

    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            for s in ex.map(compile_one, todo):
                if verbose:
                    print(f"[vspike.build] compiled {os.path.basename(s)}", file=sys.stderr)
    if force or todo or _needs(lib_path, objs):
        rocm_lib = os.path.join(os.path.dirname(os.path.dirname(hipcc)), "lib")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib_path, *objs, "-lpthread",
               f"-L{rocm_lib}", "-lrccl", f"-Wl,-rpath,{rocm_lib}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        if verbose:
            print(f"[vspike.build] linked {lib_path} (build id {bid})", file=sys.stderr)
    with open(stamp, "w") as fh:
        fh.write(bid + "\n")
    return lib_path


if __name__ == "__main__":
    build(force="--force" in sys.argv)
