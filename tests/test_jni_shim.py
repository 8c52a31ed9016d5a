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


# ---------------------------------------------------------------- fake JNIEnv
# integration/jni/lda_jni.c itself, run through the fake JNIEnv of
# tests/jni/fake_env.c (HotSpot-like copying arrays, failure injection; the
# program checks that every pinned array is released exactly once and that
# outputs are copied back only on success).  The failure paths never reach the
# GPU, so they run here; the success path is test_jni_harness_gpu.py's.
FAKE = os.path.join(ROOT, "tests", "jni", "bin", "fake_env")


def _write_input(path, K=8, V=30, D=12, seed=3):
    import numpy as np
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 15, size=D)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    N = int(off[-1])
    with open(path, "wb") as f:
        f.write(np.array([K, V, D], np.int32).tobytes())
        f.write(off.tobytes())
        f.write(rng.integers(0, V, size=N).astype(np.int32).tobytes())
        f.write(rng.integers(0, K, size=N).astype(np.int32).tobytes())
        f.write(np.full(K, 0.1).tobytes())
        f.write(np.array([0.1 * K, 0.01, 0.01 * V]).tobytes())
        f.write(np.array([0], np.int64).tobytes())
        f.write(np.array([20, 200, 0, 10, 0, 1, 0], np.int32).tobytes())
        f.write(np.array([seed], np.int64).tobytes())


def _fake(*args):
    if not os.path.exists(FAKE):
        # built by build() / `make -C integration/jni harness`, which links the
        # HIP libraries: a checkout without the HIP build skips, as the gcc
        # check above does without gcc
        pytest.skip("tests/jni/bin/fake_env not built (build() / make -C integration/jni harness)")
    return subprocess.run([FAKE, *args], capture_output=True, text=True, timeout=60)


@pytest.mark.parametrize("n", list(range(1, 13)))
def test_failed_pin_releases_everything_and_leaves_the_oom_pending(tmp_path, n):
    """The n-th of the 12 Get<Type>ArrayElements calls (options, then the
    eleven arrays) returns NULL: the glue returns 0, throws nothing of its own,
    and releases every array it had pinned (JNI_ABORT: z unchanged)."""
    fin = str(tmp_path / "in.bin")
    _write_input(fin)
    r = _fake("--fail-pin", str(n), fin)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pending=java/lang/OutOfMemoryError" in r.stdout and "throws=0" in r.stdout
    assert f"pins={n - 1} releases={n - 1}" in r.stdout and "copies=0" in r.stdout


def test_estimate_error_throws_runtime_exception(tmp_path):
    """ldaj_estimate fails (K = 0): every array released with JNI_ABORT, one
    RuntimeException carrying ldaj_last_error()."""
    fin = str(tmp_path / "in.bin")
    _write_input(fin)
    r = _fake("--bad-k", fin)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pins=12 releases=12 aborts=12 copies=0 throws=1" in r.stdout
    assert "pending=java/lang/RuntimeException" in r.stdout and "bad argument" in r.stdout


def test_java_loads_the_library_lazily():
    """Loading a serialized model (src/cmu_ron/TrainAndPredict.java:191-196,
    :246: predict() on a host without the GPU library) must not need the
    .so: no static initializer of the class itself loads it."""
    src = open(JAVA).read()
    head = src[:src.index("private static final class NativeLibrary")]
    assert "System.loadLibrary" not in head
    assert "NativeLibrary.load()" in src[src.index("public void estimate()"):]
