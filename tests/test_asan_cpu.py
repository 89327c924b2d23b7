"""the extension's host code under AddressSanitizer + UndefinedBehaviorSanitizer, on CPU.

`make -C freeze-omni_amd/csrc asan` builds libfo_hip_asan.so: the same sources with every host function instrumented
(`-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined`, recovery off; device code unchanged -- GPU
sanitizers are not used on this pool).  This test runs the C-ABI's CPU tests -- the argument checks and pack-extent
refusals of test_pack_abi_cpu.py, the symbol table and host policy functions of test_capi_symbols.py -- in a child
Python that has the ASan runtime preloaded and loads the instrumented library (FO_LIB_PATH): any heap / stack /
global overflow, use-after-free or undefined behaviour on those paths aborts the child."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_LIB = os.path.join(ROOT, "freeze-omni_amd", "fo", "libfo_hip_asan.so")
RT = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))


@pytest.mark.skipif(not os.path.exists(ASAN_LIB) or not RT,
                    reason="libfo_hip_asan.so not built (make -C freeze-omni_amd/csrc asan) or no ASan runtime")
def test_c_abi_host_paths_clean_under_asan_and_ubsan():
    nm = subprocess.run(["nm", "-D", "--undefined-only", ASAN_LIB], capture_output=True, text=True, check=True).stdout
    assert "__asan_report" in nm and "__ubsan_handle" in nm, "the library is not instrumented"
    env = dict(os.environ, LD_PRELOAD=RT[-1], FO_LIB_PATH=ASAN_LIB,
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_pack_abi_cpu.py"),
                        os.path.join(ROOT, "tests", "test_capi_symbols.py")],
                       env=env, capture_output=True, text=True, cwd=ROOT, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert " passed" in out and "skipped" not in out, out[-2000:]
