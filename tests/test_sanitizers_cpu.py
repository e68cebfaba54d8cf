"""SURVEY.md §5.2 race / memory-safety checks of the native host runtime (csrc/runtime/runtime.cpp: the
BucketPlanner, ReadyTracker, ZeroLayout, FlatLayout and CollectiveTracer every engine drives).

The runtime is rebuilt with ``-fsanitize=address,undefined`` into a private directory and loaded through
``PDT_RUNTIME_DIR``; the runtime unit tests and a world-2 gloo pass over the DDP / OSS+ShardedDDP / FSDP
engines then run under it (ASan first in the preload list, UBSan errors fatal).  Any report makes the
child exit non-zero.  The reference has no native code and no such checks ("Reference:
none"); this covers the C++ this framework adds."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gcc_lib(name):
    r = subprocess.run(["g++", f"-print-file-name={name}"], capture_output=True, text=True)
    path = os.path.realpath(r.stdout.strip())
    return path if r.returncode == 0 and os.path.isabs(path) and os.path.exists(path) else None


def _asan_runtime():
    return _gcc_lib("libasan.so")


def _preload(env):
    """ASan first (the interpreter is not instrumented), then libstdc++ so ASan's __cxa_throw interceptor can
    resolve the real one at start-up (python itself does not link libstdc++); anything already preloaded
    stays, after them."""
    libs = [_asan_runtime(), _gcc_lib("libstdc++.so")]
    return ":".join([x for x in libs if x] + ([env["LD_PRELOAD"]] if env.get("LD_PRELOAD") else []))


@pytest.fixture(scope="module")
def sanitized_runtime(tmp_path_factory):
    if _asan_runtime() is None:
        pytest.skip("libasan not available to g++")
    sys.path.insert(0, ROOT)
    from pytorch_distributedtraining_amd import _build
    d = str(tmp_path_factory.mktemp("asan_rt"))
    out = _build.build_runtime(out_dir=d, sanitize=True)
    assert os.path.exists(out)
    nm = subprocess.run(["nm", "-D", out], capture_output=True, text=True).stdout
    assert "__asan_" in nm and "__ubsan_" in nm, "runtime was not built with the sanitizers"
    return d


def _run_sanitized(rt_dir, args, timeout=600):
    env = dict(os.environ)
    env["LD_PRELOAD"] = _preload(env)
    env.update(PDT_RUNTIME_DIR=rt_dir, OMP_NUM_THREADS="2",
               # CPython and torch keep allocations alive at exit by design: leak checking is off, everything
               # else (heap/stack overflow, use-after-free, UB) aborts the process
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:exitcode=86:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=87")
    return subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", *args], cwd=ROOT,
                          env=env, capture_output=True, text=True, timeout=timeout)


def test_runtime_unit_tests_clean_under_asan_ubsan(sanitized_runtime):
    r = _run_sanitized(sanitized_runtime, ["tests/test_runtime.py"])
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]


def test_engines_world2_clean_under_asan_ubsan(sanitized_runtime):
    """The engines' hot host paths (bucket plan + rebuild, readiness per gradient hook, owner layouts,
    flat-parameter pieces, tracer) at world 2 over gloo, every rank on the instrumented runtime."""
    r = _run_sanitized(sanitized_runtime, [
        "tests/test_engines_dist_cpu.py", "-k",
        "(test_ddp_matches_single_process and 2-2) or (test_zero_oss_sddp_match_single_process and 2-True) or "
        "(test_fsdp_matches_single_process and 2-full_shard) or (test_zero2_reduce_to_owner and 2-reduce-2)"])
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "4 passed" in out, out[-2000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]


def test_sanitized_runtime_rejects_bad_index(sanitized_runtime):
    """Bounds checks hold in the instrumented build too: an out-of-range ReadyTracker index raises."""
    code = ("from pytorch_distributedtraining_amd.utils.native import require_runtime\n"
            "t = require_runtime().ReadyTracker([[0, 1]], 2)\n"
            "try:\n    t.mark_ready(5)\nexcept (RuntimeError, IndexError, ValueError):\n    print('rejected')\n")
    env = dict(os.environ)
    env["LD_PRELOAD"] = _preload(env)
    env.update(PDT_RUNTIME_DIR=sanitized_runtime, ASAN_OPTIONS="detect_leaks=0:exitcode=86:verify_asan_link_order=0")
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "rejected" in r.stdout, (r.stdout + r.stderr)[-3000:]


def test_harness_reports_a_planted_heap_overflow(tmp_path):
    """The harness itself is live: a one-past-the-end write in a library built with the same flags and loaded
    the same way (preload + options, into an uninstrumented python) must end the process with ASan's report."""
    if _asan_runtime() is None:
        pytest.skip("libasan not available to g++")
    src = tmp_path / "bad.cpp"
    src.write_text('#include <cstdlib>\nextern "C" int pdt_planted(int n) {\n'
                   '  int* a = (int*)std::malloc(n * sizeof(int));\n  a[n] = 1;\n  int v = a[0];\n'
                   '  std::free(a);\n  return v;\n}\n')
    lib = tmp_path / "libbad.so"
    subprocess.run(["g++", "-shared", "-fPIC", "-O0", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    str(src), "-o", str(lib)], check=True)
    env = dict(os.environ)
    env["LD_PRELOAD"] = _preload(env)
    env["ASAN_OPTIONS"] = "detect_leaks=0:exitcode=86:verify_asan_link_order=0"
    r = subprocess.run([sys.executable, "-c", f"import ctypes; ctypes.CDLL({str(lib)!r}).pdt_planted(4)"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 86 and "heap-buffer-overflow" in r.stderr, (r.returncode, r.stderr[-2000:])
