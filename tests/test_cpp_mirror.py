"""The C++ host-side mirror of the reference surface (zig-tfhe_amd/cpp/tfhe.hpp):
it compiles against the C ABI header on CPU, and its gate tests — written as
src/gates.zig's own tests — pass on the GPU (zig-tfhe_amd/cpp/test_gates.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zig-tfhe_amd")


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_cpp_mirror_header_compiles():
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror", f"-I{ROOT}/include",
                        f"-I{PKG}/cpp", os.path.join(PKG, "cpp", "test_gates.cpp")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_cpp_gate_tests_pass_on_gpu():
    exe = os.path.join(PKG, "lib", "test_gates")
    assert os.path.exists(exe), "build first: make -C zig-tfhe_amd"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "PASSED" in r.stdout, r.stdout + r.stderr
