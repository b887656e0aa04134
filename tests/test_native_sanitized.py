"""Host code under AddressSanitizer + UBSan.  tests/native/bits_fuzz.cpp
round-trips random field sequences through the bit cursors (fse_bits.cpp):
BitStackWriter, BitStackReader and BitStreamReader, from exact-size buffers
at every alignment, plus short and corrupt inputs.  tests/native/oracle_fuzz.c
runs the oracle's codecs on random, truncated and corrupted blocks."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_bit_cursors_sanitized(tmp_path):
    exe = tmp_path / "bits_fuzz"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "bits_fuzz.cpp"),
                    os.path.join(ROOT, "entropy_coders_amd", "csrc", "fse_bits.cpp")],
                   check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0")
    r = subprocess.run([str(exe), "1500"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("ok"), r.stdout


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_sanitized(tmp_path):
    exe = tmp_path / "oracle_fuzz"
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "oracle_fuzz.c"),
                    os.path.join(ROOT, "oracle", "fse_oracle.c"), "-lm"],
                   check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0")
    r = subprocess.run([str(exe), "600"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.startswith("ok"), r.stdout
