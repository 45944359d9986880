"""The JNI shim (jni/) against the C ABI and its Java class, CPU tier.

No JDK is in this image, so the shim is not compiled here (jni/Makefile
builds it where JAVA_HOME is set; tests/native/abi_c.c runs the same C call
sequence).  These checks keep the three files consistent: every native
method GpuClassifier.java declares has its Java_..._<name> export in the C
file and vice versa, and every vc_* function the shim calls is declared in
include/vclassify.h (and exported by libvclassify.so, test_capi_symbols.py).
"""
import os
import re

from vproxy_amd._lib import header_symbols

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JNI = os.path.join(ROOT, "jni")


def _read(name):
    with open(os.path.join(JNI, name)) as f:
        return f.read()


def test_java_natives_match_c_exports():
    java = _read("GpuClassifier.java")
    c = _read("vproxy_component_secure_GpuClassifier.c")
    natives = set(re.findall(r"public static native [\w\[\]]+ (\w+)\(", java))
    exports = set(re.findall(r"Java_vproxy_component_secure_GpuClassifier_(\w+)", c))
    assert natives and natives == exports


def test_shim_calls_only_header_functions():
    c = _read("vproxy_component_secure_GpuClassifier.c")
    called = set(re.findall(r"\b(vc_[a-z0-9_]+)\s*\(", c))
    assert called <= set(header_symbols()), called - set(header_symbols())
    # the shim's sequence for the drain-loop batch and the metrics endpoint
    assert {"vc_create", "vc_pipeline", "vc_counters_prometheus", "vc_host_register"} <= called
