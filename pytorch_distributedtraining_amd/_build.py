"""Ahead-of-time build of the native parts of pytorch_distributedtraining_amd.

Two artefacts, both built IN-TREE so they travel with the repository snapshot to the GPU box:

* ``lib/libpdt_kernels.so`` -- every HIP kernel under ``csrc/kernels/*.hip``, compiled by ``hipcc``
  for gfx950 (MI355X / CDNA4) only.  Plain C ABI (``pdt_*``), loaded with ctypes after ``import torch``
  so it binds to the same HIP runtime (soname ``libamdhip64.so.7``) torch already mapped.
* ``_pdt_runtime*.so`` -- the host-side C++ runtime (bucket planner, ZeRO/FSDP shard planners,
  collective sequence tracer, pinned prefetch ring), a pybind11 module compiled by g++.

No hipify, no torch cpp_extension, no CUDA: the sources are written for CDNA4 directly.
Incremental: an artefact is rebuilt only when a source or header is newer than it.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pytorch_distributedtraining_amd")
KERNEL_DIR = os.path.join(ROOT, "csrc", "kernels")
RUNTIME_DIR = os.path.join(ROOT, "csrc", "runtime")
BUILD_DIR = os.path.join(ROOT, "build", "native")
KERNEL_LIB = os.path.join(PKG, "lib", "libpdt_kernels.so")
ARCH = os.environ.get("PDT_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}",
    "-munsafe-fp-atomics", "-ffp-contract=fast", "-Wno-unused-result",
]
# MFMA kernels whose accumulators are post-processed by VALU (softmax / gradient tiles): keep the MFMA
# results in arch VGPRs (no v_accvgpr_read/write shuttling through AGPRs).
PER_FILE_FLAGS = {
    # no-NaN float mode: fmaxf on MFMA outputs compiles to bare v_max3 (no canonicalising v_max x,x first)
    "flash_attn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-honor-nans", "-mno-amdgpu-ieee"],
}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the gfx950 kernels)")


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
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_kernels(verbose: bool = False, jobs: int | None = None) -> str:
    # generated sources (hand-scheduled asm main loops): regenerate when the generator changed
    for gen in sorted(glob.glob(os.path.join(KERNEL_DIR, "gen_*.py"))):
        inc = os.path.join(KERNEL_DIR, os.path.basename(gen)[4:-3] + ".inc")
        if _newer(inc, [gen]):
            _run([sys.executable, gen], verbose)
    srcs = sorted(glob.glob(os.path.join(KERNEL_DIR, "*.hip")))
    headers = sorted(glob.glob(os.path.join(KERNEL_DIR, "*.h")))
    incs = sorted(glob.glob(os.path.join(KERNEL_DIR, "*.inc")))
    os.makedirs(BUILD_DIR, exist_ok=True)
    os.makedirs(os.path.dirname(KERNEL_LIB), exist_ok=True)
    hipcc = _hipcc()
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(BUILD_DIR, os.path.basename(s)[:-4] + f".{ARCH}.o")
        objs.append(o)
        with open(s) as f:
            text = f.read()
        deps = [s] + headers + [i for i in incs if os.path.basename(i) in text] + [__file__]
        if _newer(o, deps):
            todo.append((s, o))
    jobs = jobs or min(8, os.cpu_count() or 4, max(1, len(todo)))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_run, [hipcc, *HIPCC_FLAGS, *PER_FILE_FLAGS.get(os.path.basename(s), []),
                                        "-I", KERNEL_DIR, "-c", s, "-o", o], verbose)
                    for s, o in todo]
            for f in futs:
                f.result()
    if _newer(KERNEL_LIB, objs):
        # hipBLASLt (epilogue GEMMs, blaslt.hip): resolves at run time to the copy torch already mapped
        # (same soname libhipblaslt.so.1), like libamdhip64
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", KERNEL_LIB,
              "-L/opt/rocm/lib", "-lhipblaslt"], verbose)
        _check_no_missing_stubs(KERNEL_LIB)
    return KERNEL_LIB


def _check_no_missing_stubs(lib: str) -> None:
    """A kernel whose host-side stub was not emitted links fine and only fails at dlopen on the GPU box
    ("undefined symbol: ...__device_stub__..."): catch it at build time."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-D", "--undefined-only", lib], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    missing = [ln.split()[-1] for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if missing:
        os.remove(lib)
        raise RuntimeError("kernel library has unresolved host stubs (device-only code leaked into the host "
                           "pass?):\n  " + "\n  ".join(missing[:10]))


def runtime_ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_pdt_runtime" + suffix)


def build_runtime(verbose: bool = False, out_dir: str | None = None, sanitize: bool | None = None) -> str:
    """``out_dir``: build the module there instead of in-tree (the sanitizer test's private copy, loaded
    through ``PDT_RUNTIME_DIR``); ``sanitize``: ASan + UBSan instrumented host code (default: env
    ``PDT_SANITIZE``)."""
    import pybind11

    srcs = sorted(glob.glob(os.path.join(RUNTIME_DIR, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(RUNTIME_DIR, "*.h")))
    out = runtime_ext_path() if out_dir is None else os.path.join(out_dir, os.path.basename(runtime_ext_path()))
    if sanitize is None:
        sanitize = bool(os.environ.get("PDT_SANITIZE"))
    if not srcs:
        return out
    if _newer(out, srcs + headers + [__file__]):
        cxx = os.environ.get("CXX", "g++")
        inc = [pybind11.get_include(), sysconfig.get_paths()["include"]]
        cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-Wall",
               "-Wno-unused-function", "-pthread"]
        for i in inc:
            cmd += ["-I", i]
        cmd += ["-I", RUNTIME_DIR, *srcs, "-o", out]
        if sanitize:
            cmd[1:1] = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
                        "-fno-omit-frame-pointer", "-g"]
        _run(cmd, verbose)
    return out


HOOKS_DIR = os.path.join(ROOT, "csrc", "hooks")


def hooks_ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_pdt_hooks" + suffix)


def build_hooks(verbose: bool = False) -> str:
    """``_pdt_hooks``: C++ AccumulateGrad post hooks for the reducers, compiled by g++ against the installed
    torch's headers and libraries (host code only; no HIP)."""
    import torch

    srcs = sorted(glob.glob(os.path.join(HOOKS_DIR, "*.cpp")))
    out = hooks_ext_path()
    if not srcs or not _newer(out, srcs + [__file__]):
        return out
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           sysconfig.get_paths()["include"]]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", "-w",
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_EXTENSION_NAME=_pdt_hooks", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    for i in inc:
        cmd += ["-isystem", i]
    cmd += [*srcs, "-o", out, "-L", os.path.join(tdir, "lib"), "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python",
            f"-Wl,-rpath,{os.path.join(tdir, 'lib')}"]
    _run(cmd, verbose)
    return out


def build_all(verbose: bool = False) -> None:
    with cf.ThreadPoolExecutor(max_workers=3) as ex:
        a = ex.submit(build_runtime, verbose)
        b = ex.submit(build_kernels, verbose)
        c = ex.submit(build_hooks, verbose)
        a.result()
        b.result()
        c.result()


if __name__ == "__main__":
    build_all(verbose="-v" in sys.argv)
    print("built:", KERNEL_LIB, runtime_ext_path())
