"""Race / memory-error detection for the host native runtime: the runtime's
self-test (tests/native/rt_selftest.cpp) under AddressSanitizer + UndefinedBehaviorSanitizer,
and a deterministic-replay check that the OpenMP build returns bitwise the same results as
the serial one.  (GPU sanitizers are not available on this pool; device kernels are checked
against fp64 oracles in the -m gpu suite, and reruns of the grid search are compared
bitwise there.)"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "rt_selftest.cpp")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")


def _build(tmp_path, name, flags):
    exe = str(tmp_path / name)
    subprocess.run(["g++", "-std=c++17", *flags, SRC, "-o", exe], check=True,
                   capture_output=True, text=True, timeout=300)
    return exe


def test_runtime_asan_ubsan(tmp_path):
    exe = _build(tmp_path, "rt_asan", ["-O1", "-g", "-fno-omit-frame-pointer",
                                       "-fsanitize=address,undefined",
                                       "-fno-sanitize-recover=all"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe, "12"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "failures 0" in r.stdout


def test_runtime_openmp_matches_serial(tmp_path):
    ser = _build(tmp_path, "rt_serial", ["-O3"])
    omp = _build(tmp_path, "rt_omp", ["-O3", "-fopenmp"])
    outs = []
    for exe, threads in ((ser, "1"), (omp, "4"), (omp, "3")):
        r = subprocess.run([exe, "4"], capture_output=True, text=True, timeout=300,
                           env=dict(os.environ, OMP_NUM_THREADS=threads))
        assert r.returncode == 0, r.stdout + r.stderr[-2000:]
        outs.append(r.stdout.split()[1])
    assert outs[0] == outs[1] == outs[2], outs
