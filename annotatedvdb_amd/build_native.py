"""Compile ``libavdb_hip.so`` for gfx950 in-tree (``annotatedvdb_amd/_lib``).

``hipcc`` cross-compiles without a GPU, so this runs in the build container;
the resulting ``.so`` travels to the GPU box with the repository snapshot.
"""

from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(OUT_DIR, "libavdb_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
ARCH = os.environ.get("AVDB_OFFLOAD_ARCH", "gfx950")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


PERCALL_SRC = os.path.join(CSRC, "avdb_percall.c")


def percall_path() -> str:
    import sysconfig
    return os.path.join(HERE, "avdb_percall" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_percall(force: bool = False, verbose: bool = True) -> str:
    """The CPython binding of the per-call host entries (``avdb_percall``,
    plain C against Python.h: it calls into libavdb_hip.so through the function
    pointers ``_native`` hands it, so it links against nothing else)."""
    import sysconfig
    out = percall_path()
    deps = [PERCALL_SRC, os.path.join(INCLUDE, "avdb.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    cc = os.environ.get("CC") or shutil.which("gcc") or "cc"
    cmd = [cc, "-O2", "-shared", "-fPIC", "-Wall", "-I", sysconfig.get_paths()["include"], "-I", INCLUDE,
           PERCALL_SRC, "-o", out + ".tmp"]
    if verbose:
        print("[avdb] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libavdb_hip.so)")


def _obj(src: str, flags, objdir: str = "obj") -> str:
    tag = "".join(f for f in flags if f.startswith("-D")).replace("-D", "_").replace("=", "")
    return os.path.join(OUT_DIR, objdir, os.path.basename(src)[:-4] + tag + ".o")


def _obj_stale(src: str, obj: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    deps = [src] + glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def _reap(job) -> None:
    pr, obj = job
    if pr.wait() != 0:
        raise subprocess.CalledProcessError(pr.returncode, "hipcc -c -> " + obj)
    os.replace(obj + ".tmp", obj)


def build(force: bool = False, verbose: bool = True, out: str = None, flags=(), objdir: str = "obj",
          link_flags=()) -> str:
    """One object per source, compiled concurrently (each .hip is its own
    translation unit: no device code crosses files), then one link."""
    out = out or LIB
    if not force and out == LIB and not flags and not _stale():
        return LIB
    os.makedirs(os.path.join(OUT_DIR, objdir), exist_ok=True)
    base = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I", INCLUDE] + list(flags)
    procs = []
    objs = []
    jobs = max(1, min(len(sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    for src in sources():
        obj = _obj(src, flags, objdir)
        objs.append(obj)
        if force or _obj_stale(src, obj):
            cmd = base + ["-c", src, "-o", obj + ".tmp"]
            if verbose:
                print("[avdb] " + " ".join(cmd), file=sys.stderr)
            if len(procs) >= jobs:
                _reap(procs.pop(0))
            procs.append((subprocess.Popen(cmd), obj))
    for job in procs:
        _reap(job)
    tmp = out + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + list(link_flags) + objs
    if verbose:
        print("[avdb] " + " ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    build_percall(force="--force" in sys.argv)
    print(LIB)
