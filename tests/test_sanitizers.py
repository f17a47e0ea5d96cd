"""the C++ runtime under AddressSanitizer + UBSan (host code only).

tests/native/featurize_fuzz.cpp is linked straight against csrc/runtime/featurize.cpp
with -fsanitize=address,undefined (ASan runtime linked statically into the executable)
and run as a subprocess; any heap overflow, use after free, leak or undefined behaviour
aborts it with a non-zero status.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ missing")
def test_featurizer_asan_ubsan(tmp_path):
    exe = tmp_path / "fuzz"
    src = [os.path.join(REPO, "tests", "native", "featurize_fuzz.cpp"),
           os.path.join(REPO, "dnn_page_vectors_amd", "csrc", "runtime", "featurize.cpp")]
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-static-libasan", "-pthread", "-o", str(exe)] + src
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(tmp_path / "f.jsonl"), "200"], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-6000:])
    assert r.stdout.startswith("ok")
