"""Build recipe for the in-tree native libraries (hipcc for gfx950; no JIT cache).

  burn_raymarching_amd/lib/libraymarch_hip.so  <- csrc/rm_kernels.hip   (the product: C ABI of include/raymarch.h)
  burn_raymarching_amd/lib/librm_host.so        <- csrc/host/{io,data,driver,comm}.cpp (C ABI of include/rm_host.h; RCCL)
  burn_raymarching_amd/lib/rm_train             <- csrc/host/main.cpp    (CLI: train / generate / preview)

Run ``python -m burn_raymarching_amd._build`` or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import hashlib
import os
import re
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
ARCH = os.environ.get("RM_OFFLOAD_ARCH", "gfx950")
LIB = os.path.join(LIBDIR, "libraymarch_hip.so")
HOST_LIB = os.path.join(LIBDIR, "librm_host.so")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP toolchain is required to build libraymarch_hip.so")


def _stale(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


# The kernel library's sources; their hash is compiled into rm_version() ("src <hash>"), so that a
# shipped .so names the source it came from (tests/test_abi.py compares it with the tree).
KERNEL_SOURCES = [os.path.join(CSRC, "rm_kernels.hip"), os.path.join(CSRC, "rm_device.h"),
                  os.path.join(CSRC, "rm_small.h"), os.path.join(ROOT, "include", "raymarch.h")]


def source_hash(paths=None) -> str:
    """sha256 (first 16 hex digits) over the kernel sources' names and bytes, in order."""
    h = hashlib.sha256()
    for p in paths or KERNEL_SOURCES:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def lib_source_hash(path: str = LIB, tag: bytes = rb"\(gfx950\) src "):
    """The source hash compiled into a built artefact (read from the file, not loaded): the kernel
    library's rm_version() string by default; HOST_TAG / EXE_TAG for librm_host.so / rm_train."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = re.search(tag + rb"([0-9a-f]{16})", f.read())
    return m.group(1).decode() if m else None


HOST_DIR = os.path.join(CSRC, "host")
EXE = os.path.join(LIBDIR, "rm_train")
# librm_host.so's sources (rmh_version(): "host 0.1.0 src <hash>") and rm_train's ("rm_train src
# <hash>"): each artefact carries the hash of what it was built from, as the kernel library does
HOST_SOURCES = [os.path.join(HOST_DIR, f) for f in ("io.cpp", "data.cpp", "driver.cpp", "comm.cpp", "rmh_common.hpp")] + \
    [os.path.join(ROOT, "include", "rm_host.h"), os.path.join(ROOT, "include", "raymarch.h")]
EXE_SOURCES = [os.path.join(HOST_DIR, "main.cpp"), os.path.join(ROOT, "include", "rm_host.h")]
HOST_TAG = rb"host 0\.1\.0 src "
EXE_TAG = rb"rm_train src "


def build_lib(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIBDIR, exist_ok=True)
    srcs = KERNEL_SOURCES
    sha = source_hash(srcs)
    # rebuilt when the embedded hash differs from the tree's (mtimes alone miss a checkout of
    # older sources), or when a source is newer than the library
    if force or _stale(LIB, srcs) or lib_source_hash(LIB) != sha:
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-result", f'-DRM_SOURCE_SHA="{sha}"', "-o", LIB, srcs[0]]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return LIB


def build_host(force: bool = False, verbose: bool = False) -> str:
    """librm_host.so (include/rm_host.h: files, dataset, prune_and_split, train driver) and the
    rm_train CLI, both C++ host code linked against libraymarch_hip.so."""
    host_dir = HOST_DIR
    if not os.path.isdir(host_dir):
        return ""
    lib = build_lib(force=force, verbose=verbose)
    inc = os.path.join(ROOT, "include")
    lib_srcs = [p for p in HOST_SOURCES if p.endswith(".cpp")]
    # -ffp-contract=off: the host f32 arithmetic (camera rays, prune_and_split) keeps the
    # reference's rounding, no fused multiply-adds
    common = [_hipcc(), "-O2", "-std=c++17", "-Wall", "-fPIC", "-ffp-contract=off", "-I", inc]
    rpath = ["-Wl,-rpath,$ORIGIN"]
    # rebuilt when the embedded hash differs from the tree's (not on mtimes alone), or when a
    # source or the library it links is newer
    hsha = source_hash(HOST_SOURCES)
    if force or _stale(HOST_LIB, HOST_SOURCES + [lib]) or lib_source_hash(HOST_LIB, HOST_TAG) != hsha:
        cmd = common + [f'-DRMH_SOURCE_SHA="{hsha}"', "-shared", "-o", HOST_LIB] + lib_srcs + \
            ["-L", LIBDIR, "-lraymarch_hip", "-lz", "-lrccl"] + rpath
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    esha = source_hash(EXE_SOURCES)
    if force or _stale(EXE, EXE_SOURCES + [HOST_LIB]) or lib_source_hash(EXE, EXE_TAG) != esha:
        cmd = common + [f'-DRMT_SOURCE_SHA="{esha}"', "-o", EXE, EXE_SOURCES[0], "-L", LIBDIR, "-lrm_host",
                        "-lraymarch_hip"] + rpath
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
    return EXE


def build_all(force: bool = False, verbose: bool = False) -> None:
    build_lib(force=force, verbose=verbose)
    build_host(force=force, verbose=verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv, verbose=True)
