"""The JNI shim (jni/) against the C ABI and its Java class, CPU tier.

No JDK is in this image: jni/Makefile builds the shim where JAVA_HOME is
set.  Here the C file is compiled (gcc -Wall -Wextra -Werror) against
tests/native/jni_spec/jni.h, the subset of the JNI specification's types
and function table it uses, and run under a fake JNIEnv
(tests/native/jni_harness.c): without a GPU, create throws IOException,
buffers shorter than their batch throw IllegalArgumentException before the
library is called, and compileUpstream leaves the caller's buffer as it was
(the GPU tier runs the same harness against the C ABI,
tests/test_gpu_abi_c.py).  These checks also keep the three files
consistent: every native method GpuClassifier.java declares has its
Java_..._<name> export in the C file and vice versa, and every vc_* function
the shim calls is declared in include/vclassify.h (and exported by
libvclassify.so, test_capi_symbols.py).
"""
import os
import re
import subprocess

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


def test_shim_compiles_and_runs_under_fake_jnienv():
    native = os.path.join(ROOT, "tests", "native")
    subprocess.check_call(["make", "-s", "-C", native, "build/jni_harness"])
    r = subprocess.run([os.path.join(native, "build", "jni_harness"), "cpu"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "JNI OK" in r.stdout, r.stdout + r.stderr
