"""The C ABI from a C++ caller (tests/c_abi/c_abi_demo.cpp): compiles against include/ and the
built library on CPU; on the GPU it runs and checks bit-identity with the plain-C oracle."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "c_abi", "c_abi_demo.cpp")
LIB_DIR = os.path.join(ROOT, "quantizers_amd")
ORACLE_DIR = os.path.join(ROOT, "oracle", "build")


def _build(out_dir):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    if not os.path.exists(os.path.join(LIB_DIR, "libquantizers_amd.so")):
        pytest.skip("library not built (run __graft_entry__.build())")
    if not os.path.exists(os.path.join(ORACLE_DIR, "libquant_ref.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    exe = os.path.join(out_dir, "c_abi_demo")
    cmd = [hipcc, "--offload-arch=gfx950", "-O2", "-std=c++17", SRC, "-I", os.path.join(ROOT, "include"),
           "-L", LIB_DIR, "-lquantizers_amd", "-L", ORACLE_DIR, "-lquant_ref", "-o", exe]
    subprocess.run(cmd, check=True, timeout=300, capture_output=True)
    return exe


def test_c_abi_demo_compiles(tmp_path):
    assert os.path.exists(_build(str(tmp_path)))


@pytest.mark.gpu
def test_c_abi_demo_runs(cuda, tmp_path):
    exe = _build(str(tmp_path))
    env = dict(os.environ, LD_LIBRARY_PATH=f"{LIB_DIR}:{ORACLE_DIR}:" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([exe, "1024", "4096"], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert "bit-identical" in r.stdout
