"""The JNI shim without a JDK (the image has no javac and no
jni.h): integration/jni/lda_jni.c compiles, warning-free, against the JNI
types and function signatures restated from the JNI specification
(tests/jni/stub/jni.h, declarations only), and its exported function matches
the Java class's native declaration -- the JNI-mangled name of
cmu_gpu.GpuParallelTopicModel.nativeEstimate and one parameter of the
corresponding JNI type per Java parameter, in order.  The native logic under
it (lda_jni_core.c) is compiled and GPU-tested by test_jni_harness_gpu.py."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "integration", "jni", "lda_jni.c")
JAVA = os.path.join(ROOT, "integration", "java", "src", "main", "java", "cmu_gpu",
                    "GpuParallelTopicModel.java")
JNI_TYPE = {"int": "jint", "long": "jlong", "double": "jdouble", "int[]": "jintArray",
            "long[]": "jlongArray", "double[]": "jdoubleArray"}


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_shim_compiles_against_the_jni_declarations():
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(ROOT, "tests", "jni", "stub"),
                        "-I", os.path.join(ROOT, "include"),
                        "-I", os.path.join(ROOT, "integration", "jni"), SHIM],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def _java_native(name):
    src = open(JAVA).read()
    m = re.search(r"static\s+native\s+(\w+)\s+" + name + r"\s*\(([^)]*)\)", src, re.S)
    assert m, "native declaration not found"
    params = [p.strip().rsplit(None, 1) for p in m.group(2).split(",")]
    return m.group(1), [t.replace(" ", "") for t, _ in params]


def test_shim_matches_the_java_native_declaration():
    ret, jtypes = _java_native("nativeEstimate")
    src = open(SHIM).read()
    m = re.search(r"JNIEXPORT\s+(\w+)\s+JNICALL\s+(Java_\w+)\s*\(([^)]*)\)", src, re.S)
    assert m
    assert m.group(2) == "Java_cmu_1gpu_GpuParallelTopicModel_nativeEstimate"   # cmu_gpu -> cmu_1gpu
    assert m.group(1) == JNI_TYPE[ret]
    cparams = [p.strip().rsplit(None, 1)[0].replace(" ", "") for p in m.group(3).split(",")]
    # JNIEnv* and the jclass of a static method, then one per Java parameter
    assert cparams[:2] == ["JNIEnv*", "jclass"]
    assert cparams[2:] == [JNI_TYPE[t] for t in jtypes]
