"""The C++ host API (include/mav_tube_trajectory_generation_amd/) built and
run as a program, mirroring the reference's gtest suite
(test/test_polynomial_optimization.cpp).  tests/cpp/test_polynomial_optimization.cpp
holds the cases; the "host" group needs no GPU, the "gpu" group is the
parity run through the C ABI on the device."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mav_tube_trajectory_generation_amd")
ORACLE = os.path.join(REPO, "oracle")
SRC = os.path.join(REPO, "tests", "cpp", "test_polynomial_optimization.cpp")


@pytest.fixture(scope="module")
def cpp_test_binary(tmp_path_factory):
    subprocess.run(["make", "-s", "-C", ORACLE], check=True)
    if not os.path.exists(os.path.join(PKG, "libmtg_hip.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    out = str(tmp_path_factory.mktemp("cpp") / "test_polynomial_optimization")
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-Werror",
           "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(REPO, "include"), "-I" + ORACLE,
           "-I/opt/rocm/include", SRC, "-o", out, "-L" + PKG, "-lmtg_hip", "-L" + ORACLE,
           "-loracle", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{PKG}:{ORACLE}:/opt/rocm/lib"]
    subprocess.run(cmd, check=True)
    return out


def _run(binary, group, timeout):
    p = subprocess.run([binary, group], capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-4000:]
    return p.stdout


def test_cpp_api_host(cpp_test_binary):
    out = _run(cpp_test_binary, "host", 120)
    assert "0 failed tests" in out


@pytest.mark.gpu
def test_cpp_api_gpu(cpp_test_binary):
    out = _run(cpp_test_binary, "gpu", 600)
    assert "0 failed tests" in out
