"""In-tree build of the native pieces of lazzaro_amd.

Two shared objects are produced next to the package sources (never in
site-packages, so the GPU box loads exactly what this tree built):

* ``lazzaro_amd/_lib/liblzk.so`` -- every HIP kernel under ``csrc/kernels`` for
  gfx950 (CDNA4), one translation unit per file, C ABI (``extern "C" lzk_*``),
  loaded with ctypes after ``import torch`` so it binds to the same HIP runtime
  (``libamdhip64.so.7``) torch already mapped.
* ``lazzaro_amd/_lib/_lzrt*.so`` -- the host runtime (columnar versioned store,
  WordPiece/hash tokenizer, CSR/graph utilities, tenant placement), C++20 +
  pybind11, built with g++ and linked against the Arrow C++ library inside
  pyarrow (the store's fragments are Arrow IPC files).

* ``lazzaro_amd/_lib/liblzk_debug.so`` -- the same kernels with
  ``-DLZK_DEBUG=1`` device bounds asserts. ``build_all`` always produces it
  (in a second, parallel compile) because the GPU tier's debug-build test loads
  it on a box that never builds; the release ``liblzk.so`` is what every other
  process loads.

Usage: ``python -m lazzaro_amd._build`` (or ``__graft_entry__.build()``).
Incremental: a target is rebuilt only when a source or header is newer.
"""
from __future__ import annotations

import glob
import os
import re
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
LIBDIR = os.path.join(ROOT, "lazzaro_amd", "_lib")
BUILDDIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("LZK_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_kernels(verbose: bool = False, jobs: int = 8, debug: bool = False, sanitize: str = "") -> str:
    """Compile every csrc/kernels/*.hip for gfx950 into one C-ABI library.

    debug=True   -> ``liblzk_debug.so`` with ``-DLZK_DEBUG=1``: device-side
                    bounds asserts (``LZK_DASSERT``) in the index-driven kernels
                    (graph ops, gathers); loaded instead of liblzk.so when
                    ``LZK_DEBUG=1``.
    sanitize="address" (or "undefined") -> host-side sanitizer on the launcher
                    code only (``-Xarch_host -fsanitize=...``); GPU sanitizers are
                    not available on this pool. Implies the debug library.
    """
    os.makedirs(LIBDIR, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "include", "*.h"))
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    flags = [
        f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
        "-fvisibility=hidden", "-mcode-object-version=5",
        "-I" + os.path.join(CSRC, "include"),
    ]
    tag = ""
    if debug or sanitize:
        flags.append("-DLZK_DEBUG=1")
        tag = "_debug"
    for san in filter(None, sanitize.split(",")):
        flags += ["-Xarch_host", f"-fsanitize={san}"]
        tag += "_" + san
    if sanitize:
        flags += ["-Xarch_host", "-fno-omit-frame-pointer", "-g"]
    bdir = BUILDDIR + tag
    os.makedirs(bdir, exist_ok=True)
    objs = []
    todo = []
    for s in srcs:
        o = os.path.join(bdir, os.path.basename(s) + ".o")
        objs.append(o)
        if _newer(o, [s] + headers):
            todo.append((s, o))

    def comp(so):
        s, o = so
        if verbose:
            print("[hipcc]", os.path.relpath(s, ROOT), flush=True)
        _run([HIPCC] + flags + ["-c", s, "-o", o])

    if todo:
        with ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            list(ex.map(comp, todo))
    out = os.path.join(LIBDIR, f"liblzk{tag}.so")
    if _newer(out, objs) or not objs:
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs
        for san in filter(None, sanitize.split(",")):
            link += ["-Xarch_host", f"-fsanitize={san}"]
        _run(link)
    return out


def build_runtime(verbose: bool = False, sanitize: str = "", outdir: str = "") -> str:
    """Build the pybind11 host runtime. ``sanitize`` ("address", "undefined"
    or both, comma separated) builds an instrumented copy into ``outdir``
    (default ``_lib/san``) -- load it with the sanitizer runtime preloaded
    (see tests/unit/test_sanitizers.py)."""
    import pybind11

    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    headers = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    odir = outdir or (os.path.join(LIBDIR, "san") if sanitize else LIBDIR)
    os.makedirs(odir, exist_ok=True)
    out = os.path.join(odir, "_lzrt" + suffix)
    if not srcs:
        return ""
    if _newer(out, srcs + headers):
        if verbose:
            print("[g++] runtime" + (f" (sanitize={sanitize})" if sanitize else ""), flush=True)
        cxx = shutil.which("g++") or "c++"
        opt = ["-O3"]
        if sanitize:
            opt = ["-O1", "-g", "-fno-omit-frame-pointer"] + [f"-fsanitize={x}" for x in sanitize.split(",") if x]
        # the columnar store writes / memory-maps Arrow IPC fragments with the
        # Arrow C++ library that ships inside pyarrow (linked by soname + rpath)
        import pyarrow as pa

        pa_dir = pa.get_library_dirs()[0]
        arrow_so = sorted(f for f in os.listdir(pa_dir) if re.fullmatch(r"libarrow\.so\.\d+", f))
        if not arrow_so:
            raise RuntimeError(f"no libarrow.so.<N> in {pa_dir} (pyarrow wheel)")
        # -ffp-contract=off: the batch planner replays the device kernels'
        # fp32 / fp64 rounding operation by operation (no fma contraction)
        cmd = [cxx] + opt + ["-std=c++20", "-ffp-contract=off", "-shared", "-fPIC", "-fvisibility=hidden",
                             "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
                             "-I" + pa.get_include(), "-I" + os.path.join(CSRC, "runtime")] + srcs + [
            "-o", out, "-L" + pa_dir, "-l:" + arrow_so[0], "-Wl,-rpath," + pa_dir, "-lpthread"]
        _run(cmd)
    return out


def build_all(verbose: bool = True) -> None:
    """Release kernels, host runtime and the device-bounds-checked debug twin
    (loaded only by the LZK_DEBUG tests), the three built concurrently."""
    with ThreadPoolExecutor(max_workers=3) as ex:
        fk = ex.submit(build_kernels, verbose, 4)
        fr = ex.submit(build_runtime, verbose)
        fd = ex.submit(build_kernels, verbose, 4, True)
        k, r, d = fk.result(), fr.result(), fd.result()
    if verbose:
        print("built:", k, r, d)


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser(description="build the lazzaro_amd native libraries in-tree")
    ap.add_argument("--debug", action="store_true", help="(build_all already builds liblzk_debug.so; kept for compatibility)")
    ap.add_argument("--sanitize", default="", help="host sanitizer(s) for debug builds, e.g. address,undefined")
    a = ap.parse_args()
    build_all(verbose=True)
    if a.debug or a.sanitize:
        print("built:", build_kernels(verbose=True, debug=True, sanitize=a.sanitize))
    if a.sanitize:
        print("built:", build_runtime(verbose=True, sanitize=a.sanitize))
    sys.exit(0)
