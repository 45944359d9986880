"""The C-ABI library loads (no GPU needed) and exports every symbol that
include/vclassify.h declares."""
import ctypes
import subprocess

from vproxy_amd import _lib


def test_header_symbols_exported():
    syms = _lib.header_symbols()
    assert len(syms) >= 40
    L = _lib.lib()
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_exports_are_c_abi():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in _lib.header_symbols():
        assert s in exported, s          # unmangled extern "C" names


def test_version():
    assert b"gfx950" in _lib.lib().vc_version()


def test_product_does_not_link_oracle():
    out = subprocess.check_output(["ldd", _lib.LIB_PATH]).decode()
    assert "oracle" not in out and "imgcheck" not in out
    strings = open(_lib.LIB_PATH, "rb").read()
    assert b"vo_sg_allow" not in strings and b"ic_acl" not in strings
