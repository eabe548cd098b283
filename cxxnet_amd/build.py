"""In-tree native build for cxxnet_amd.

Produces, under ``cxxnet_amd/_native/``:
  * ``_cxxnet_rt<EXT_SUFFIX>``  -- pybind11 module: config parser, NetConfig,
    checkpoint PODs, data IO, metrics (g++, no GPU dependency).
  * ``libcxxnet_kernels.so``     -- every hand-written HIP kernel for gfx950,
    exported through a flat C ABI (hipcc --offload-arch=gfx950).
  * ``libcxxnetwrapper.so``      -- the CXN* C ABI (embeds CPython).

Run ``python -m cxxnet_amd.build`` (or ``__graft_entry__.build()``).  Builds are
incremental: a target is rebuilt when any of its sources/headers is newer.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
# CXXNET_NATIVE_DIR selects another output / load directory (the --asan build goes to
# cxxnet_amd/_native_asan so the production libraries are never replaced by it)
OUT = os.environ.get("CXXNET_NATIVE_DIR") or os.path.join(PKG, "_native")
ASAN_DIR = os.path.join(PKG, "_native_asan")
# host sanitizer flags (--asan): AddressSanitizer + UBSan on the host C++ (runtime, C ABI)
SAN_FLAGS = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-g"]
_san = {"on": False}
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("CXXNET_OFFLOAD_ARCH", "gfx950")

RT_NAME = "_cxxnet_rt" + sysconfig.get_config_var("EXT_SUFFIX")
KERNEL_LIB = "libcxxnet_kernels.so"
WRAPPER_LIB = "libcxxnetwrapper.so"


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def build_runtime(verbose=False, force=False) -> str:
    import pybind11

    src = os.path.join(CSRC, "runtime", "bindings.cpp")
    deps = [src] + glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    target = os.path.join(OUT, RT_NAME)
    if force or _newer(target, deps):
        os.makedirs(OUT, exist_ok=True)
        cmd = ["g++", "-O1" if _san["on"] else "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall",
               "-Wno-unused-result", "-fvisibility=hidden"] + (SAN_FLAGS if _san["on"] else []) + [
               "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
               src, "-o", target + ".tmp", "-lz", "-lpthread", "-ldl"]
        _run(cmd, verbose)
        os.replace(target + ".tmp", target)
    return target


def build_kernels(verbose=False, force=False, jobs=8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    target = os.path.join(OUT, KERNEL_LIB)
    objdir = os.path.join(OUT, "obj")
    os.makedirs(objdir, exist_ok=True)
    common = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
              "-munsafe-fp-atomics", "-Wno-unused-result",
              "-I" + os.path.join(CSRC, "kernels")]
    objs = []
    jobs_list = []
    for s in srcs:
        o = os.path.join(objdir, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            jobs_list.append(common + ["-c", s, "-o", o])
    if jobs_list:
        with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            list(ex.map(lambda c: _run(c, verbose), jobs_list))
    if force or _newer(target, objs) or jobs_list:
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", target + ".tmp"], verbose)
        _check_stubs(target + ".tmp")
        os.replace(target + ".tmp", target)
    return target


def _check_stubs(lib):
    """Fail the build when a kernel's host launch stub is undefined: hipcc's host pass can drop
    one silently (gemm_4w.hip lds_dma16), and the library would then fail only at dlopen on a
    GPU box."""
    nm = os.path.join(ROCM, "lib", "llvm", "bin", "llvm-nm")
    if not os.path.exists(nm):
        return
    out = subprocess.run([nm, "-D", "--undefined-only", lib], stdout=subprocess.PIPE, text=True).stdout
    bad = [l.split()[-1] for l in out.splitlines() if "__device_stub__" in l]
    if bad:
        raise RuntimeError(f"build failed: {len(bad)} undefined kernel launch stub(s) in {lib}, e.g. {bad[0]}")


def build_wrapper(verbose=False, force=False) -> str:
    src = os.path.join(CSRC, "capi", "cxxnet_wrapper.cpp")
    if not os.path.exists(src):
        return ""
    deps = [src] + glob.glob(os.path.join(CSRC, "capi", "*.h"))
    target = os.path.join(OUT, WRAPPER_LIB)
    if force or _newer(target, deps):
        libdir = sysconfig.get_config_var("LIBDIR")
        ver = sysconfig.get_config_var("LDVERSION")
        cmd = ["g++", "-O1" if _san["on"] else "-O2", "-std=c++17", "-shared", "-fPIC", "-Wall"] + \
              (SAN_FLAGS if _san["on"] else []) + [
               "-I" + sysconfig.get_paths()["include"], "-I" + os.path.join(CSRC, "capi"),
               src, "-o", target + ".tmp", "-L" + libdir, "-lpython" + ver,
               "-Wl,-rpath," + libdir]
        _run(cmd, verbose)
        os.replace(target + ".tmp", target)
    return target


def build_im2bin(verbose=False, force=False) -> str:
    """The native im2bin executable (csrc/tools/im2bin.cpp)."""
    src = os.path.join(CSRC, "tools", "im2bin.cpp")
    deps = [src] + glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    target = os.path.join(OUT, "im2bin")
    if force or _newer(target, deps):
        os.makedirs(OUT, exist_ok=True)
        _run(["g++", "-O2", "-std=c++17", "-Wall", "-Wno-unused-result"] + (SAN_FLAGS if _san["on"] else []) +
             [src, "-o", target + ".tmp", "-lz", "-lpthread", "-ldl"], verbose)
        os.replace(target + ".tmp", target)
    return target


def build_all(verbose=False, force=False):
    rt = build_runtime(verbose, force)
    k = build_kernels(verbose, force)
    w = build_wrapper(verbose, force)
    build_im2bin(verbose, force)
    return rt, k, w


def build_asan(verbose=False, force=False):
    """Host-sanitizer build (AddressSanitizer + UBSan) of the C++ runtime and the CXN* C ABI into
    cxxnet_amd/_native_asan; the HIP kernel library is linked in unchanged (device code is not
    sanitized: GPU ASan is not available on this pool).  Use it with
        CXXNET_NATIVE_DIR=cxxnet_amd/_native_asan LD_PRELOAD="$(g++ -print-file-name=libasan.so)
        $(g++ -print-file-name=libubsan.so)" ASAN_OPTIONS=detect_leaks=0 python -m pytest -m "not gpu"
    (tools/asan_cpu_tests.sh)."""
    global OUT
    saved = OUT
    OUT = ASAN_DIR
    _san["on"] = True
    try:
        os.makedirs(OUT, exist_ok=True)
        rt = build_runtime(verbose, force)
        w = build_wrapper(verbose, force)
        k = os.path.join(OUT, KERNEL_LIB)
        src = os.path.join(saved, KERNEL_LIB)
        if not os.path.exists(src):
            OUT = saved
            build_kernels(verbose)
            OUT = ASAN_DIR
        if not os.path.exists(k) or os.path.getmtime(k) < os.path.getmtime(src):
            import shutil
            shutil.copy2(src, k)
        return rt, k, w
    finally:
        OUT = saved
        _san["on"] = False


if __name__ == "__main__":
    force = "--force" in sys.argv
    built = build_asan(verbose=True, force=force) if "--asan" in sys.argv else build_all(verbose=True, force=force)
    for p in built:
        if p:
            print("built", p)
