"""Host sanitizers over the C++ IO runtime: csrc/tests/sanitize_io.cpp drives the
TFRecord framing/CRC walk, the Example decoder, the threaded batch loader and the libsvm converter
on valid data (checked value by value) and on corrupted data (truncations, bit flips, forged
lengths), built with -fsanitize=address,undefined and with -fsanitize=thread.  Any out-of-bounds
access, undefined behaviour or data race fails the test.  (GPU sanitizers are not available on
this pool; the device-side id guard is ROCFM_CHECK_IDS, tests/test_fused_kernels_gpu.py.)"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
SRCS = [os.path.join(CSRC, "tests", "sanitize_io.cpp"), os.path.join(CSRC, "io", "tfrecord.cpp"),
        os.path.join(CSRC, "io", "loader.cpp"), os.path.join(CSRC, "io", "record_index.cpp")]


def _build_and_run(tmp_path, flags, iters):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "harness")
    r = subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-msse4.2", "-pthread", "-fno-omit-frame-pointer", *flags,
                        "-I", CSRC, *SRCS, "-o", exe], capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "sanitize" in r.stderr and "cannot find" in r.stderr:
        pytest.skip("sanitizer runtime not installed")
    assert r.returncode == 0, r.stderr[-3000:]
    d = tmp_path / "data"
    d.mkdir()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(d), str(iters)], capture_output=True, text=True, timeout=900, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "sanitize harness ok" in r.stdout, out[-4000:]
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "LeakSanitizer"):
        assert bad not in out, out[-4000:]


def test_io_runtime_asan_ubsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], 300)


def test_io_runtime_tsan(tmp_path):
    _build_and_run(tmp_path, ["-fsanitize=thread"], 40)
