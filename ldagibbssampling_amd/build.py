"""Build the in-tree HIP library (hipcc, gfx950) and the CPU oracle (gcc)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def build_library(jobs: int = 2) -> str:
    subprocess.run(["make", "-s", f"-j{jobs}", "-C", os.path.join(HERE, "csrc")], check=True)
    return os.path.join(HERE, "lib", "liblda_mi355x.so")


def build_jni_harness() -> str:
    """The Java drop-in's native half (integration/jni/lda_jni_core.c) linked
    into the C harness that tests it (tests/jni/estimate_harness.c)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "integration", "jni"), "harness"],
                   check=True)
    return os.path.join(ROOT, "tests", "jni", "bin", "estimate_harness")


def build_native_tests() -> str:
    """GPU test programs over the sampler ABI (tests/native/: the device RNG
    against rocRAND's philox4x32_10)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "native")], check=True)
    return os.path.join(ROOT, "tests", "native", "bin", "philox_vs_rocrand")


def build_oracle() -> str:
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return os.path.join(ROOT, "oracle", "lib", "liblda_oracle.so")


if __name__ == "__main__":
    print(build_library())
    print(build_jni_harness())
    print(build_oracle())
