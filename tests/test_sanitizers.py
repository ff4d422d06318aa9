"""Host-code sanitizers: the garbler + host evaluator built with
ASan+UBSan and with TSan, driven multi-threaded by tests/native/sanitize_main.cpp.
GPU sanitizers are not available on the target pool; GPU/CPU bit-exact parity
tests are the device-side race detector."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "dash_amd" / "csrc"
CXX = "/opt/rocm/llvm/bin/clang++" if os.path.exists("/opt/rocm/llvm/bin/clang++") else shutil.which("clang++")
SOURCES = [str(CSRC / f) for f in ("core.cpp", "gadgets.cpp", "garbler.cpp", "evaluator.cpp", "serialize.cpp")]


@pytest.mark.skipif(CXX is None, reason="clang++ not available")
def test_host_sanitizers(tmp_path):
    common = ["-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-maes", "-msse4.2", "-mavx2", "-mpclmul",
              f"-I{CSRC}", str(ROOT / "tests" / "native" / "sanitize_main.cpp"),
              str(ROOT / "tests" / "native" / "gpu_garbler_stub.cpp"), *SOURCES, "-lpthread"]
    builds = {"asan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"],
              "tsan": ["-fsanitize=thread"]}
    procs = {k: subprocess.Popen([CXX, *flags, *common, "-o", str(tmp_path / k)], stdout=subprocess.PIPE,
                                 stderr=subprocess.STDOUT, text=True) for k, flags in builds.items()}
    for k, p in procs.items():
        out, _ = p.communicate(timeout=600)
        assert p.returncode == 0, f"{k} build failed:\n{out[-3000:]}"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1",
               DASH_NUM_THREADS="8")
    for k in builds:
        r = subprocess.run([str(tmp_path / k)], capture_output=True, text=True, timeout=600, env=env)
        log = r.stdout + r.stderr
        assert r.returncode == 0, f"{k} run failed:\n{log[-4000:]}"
        assert "runtime error" not in log and "ThreadSanitizer" not in log and "AddressSanitizer" not in log, log
        assert log.count(" ok") == 3
