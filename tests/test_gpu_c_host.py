"""The drop-in boundary from plain C (tests/native/c_abi_host.c): a host
program with no Python and no PyTorch in the process calls the C ABI the way
the crate's Rust FFI would -- host buffers, the crate's
append-to-dst convention -- and checks every result against the C oracle
linked in as the checker: fse_compress2 / fse_compress bytes and payload
bits, their statuses, fse_decompress2 / fse_decompress round trips and
statuses, fse_decompress2_many over 40 streams, and zero rank-check
fallbacks."""
import os
import shutil
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_plain_c_host_program(tmp_path):
    lib_dir = os.path.join(ROOT, "entropy_coders_amd")
    if not os.path.exists(os.path.join(lib_dir, "libfsehip.so")):
        pytest.skip("libfsehip.so not built")
    exe = tmp_path / "c_abi_host"
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Werror", "-o", str(exe),
                    os.path.join(ROOT, "tests", "native", "c_abi_host.c"), os.path.join(ROOT, "oracle", "fse_oracle.c"),
                    f"-L{lib_dir}", "-lfsehip", f"-Wl,-rpath,{lib_dir}", "-lm"],
                   check=True, capture_output=True, timeout=120)
    env = {k: v for k, v in os.environ.items() if not k.startswith("FSEHIP_")}
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=240, env=env)
    print(r.stdout)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    assert r.stdout.startswith("ok 54 cases")
