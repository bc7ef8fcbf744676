"""Sanitizer runs of the native host runtime (SURVEY.md §5 "race detection / sanitizers").

GPU sanitizers (xnack / GPU ASan) are unavailable on this hardware pool, so the host half of the
runtime -- TCP store (csrc/runtime/store.cpp) and host collectives (hostcomm.cpp), i.e. everything a
CPU/"gloo" job and the rendezvous of every GPU job runs -- is compiled into a standalone stress
driver (tests/native/runtime_stress.cpp, W ranks as threads over real sockets) with
ASan + UBSan and, separately, TSan, and must finish clean.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "runtime", f) for f in ("store.cpp", "hostcomm.cpp")]
DRIVER = os.path.join(ROOT, "tests", "native", "runtime_stress.cpp")


def _build(tmp_path, flags, name):
    exe = str(tmp_path / name)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-pthread",
           "-I" + os.path.join(ROOT, "csrc", "runtime"), *flags, DRIVER, *SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    return exe


def _run(exe, env_extra, world=4, iters=2):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([exe, str(world), str(iters)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-6000:])
    assert "runtime stress ok" in r.stdout
    return r


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_runtime_asan_ubsan(tmp_path):
    exe = _build(tmp_path, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"], "stress_asan")
    _run(exe, {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0:verify_asan_link_order=0", "UBSAN_OPTIONS": "print_stacktrace=1"})


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_runtime_tsan(tmp_path):
    exe = _build(tmp_path, ["-fsanitize=thread"], "stress_tsan")
    _run(exe, {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}, world=3, iters=1)
