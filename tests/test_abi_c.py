"""The C ABI from plain C99 (tests/native/abi_c.c), CPU tier.

abi_c.c includes include/vclassify.h and links libvclassify.so with
gcc -std=c99 -Wall -Wextra -Werror -pedantic: the header must compile as
strict C and every function the shim sequence calls must link.  Without a
GPU, vc_create must fail with VC_EDEVICE (no CPU path) and the program
exits 3 before classifying anything.  tests/test_gpu_abi_c.py runs the same
binary on the MI355X box.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BIN = os.path.join(NATIVE, "build", "abi_c")


def build_abi_c():
    subprocess.check_call(["make", "-s", "-C", NATIVE, "build/abi_c"])
    return BIN


def test_abi_c_builds_strict_c99():
    assert os.access(build_abi_c(), os.X_OK)


def test_abi_c_without_gpu_fails_loudly(tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: tests/test_gpu_abi_c.py covers this box")
    r = subprocess.run([build_abi_c(), str(tmp_path / "out.bin")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 3, r.stdout + r.stderr
    assert "VC_EDEVICE" in r.stdout
    assert not (tmp_path / "out.bin").exists()
