"""ASan + UBSan over the host code that parses untrusted files and prepares scenes:
tests/native/sanitize_driver.cpp linked with dae_loader.cpp, exr_loader.cpp, bdpt_scene.cpp and the
device core's CPU build (core_cpu.cpp), compiled with g++ -fsanitize=address,undefined, run on the
real scenes / environment maps / camera files and on truncated and byte-flipped copies of them.
CPU only (no device code is involved)."""
import glob
import os
import shutil
import subprocess

import pytest

from _util import REPO

CSRC = os.path.join(REPO, "bidirectional-pathtracing_amd", "csrc")
NATIVE = os.path.join(REPO, "tests", "native")
OUT = os.path.join(REPO, "build", "sanitize", "sanitize_driver")
SRCS = [os.path.join(NATIVE, "sanitize_driver.cpp"), os.path.join(NATIVE, "core_cpu.cpp")] + [
    os.path.join(CSRC, f) for f in ("dae_loader.cpp", "exr_loader.cpp", "bdpt_scene.cpp")]


def _build():
    deps = SRCS + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "bdpt", "*.h"))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(p) for p in deps):
        return
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-ffp-contract=off", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-static-libasan",
           "-I" + os.path.join(REPO, "include"), "-I" + CSRC, "-o", OUT] + SRCS + ["-lz"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=600)


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_parsers_under_asan_ubsan(tmp_path):
    _build()
    files = sorted(glob.glob(os.path.join(REPO, "scenes", "CB*.dae")))
    files = [f for f in files if "standin" not in f and "bunny" not in f.lower()]   # the large meshes: slow under ASan
    files += [os.path.join(REPO, "scenes", "teapot.dae"), os.path.join(REPO, "scenes", "banana.dae")]
    files += sorted(glob.glob(os.path.join(REPO, "tests", "golden", "env", "*.exr")))
    files += [os.path.join(REPO, "tests", "golden", "cam", "CBspheres_orbit.txt")]
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([OUT, str(tmp_path)] + files, capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "no sanitizer report" in r.stdout
