"""CPU-side checks of the C ABI library (no compute without a GPU): it
loads, exports exactly what include/lda_mi355x.h declares, and fails loudly
(status + message) when no device is present."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from ldagibbssampling_amd import capi

HEADER = capi.HEADER_PATH


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(lda_[a-z_0-9]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(capi.LIB_PATH):
        from ldagibbssampling_amd.build import build_library
        build_library()
    return capi.load()


def test_header_and_binding_agree():
    assert declared_functions() == sorted(capi.SIGNATURES)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", capi.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (lda_\w+)", out))
    missing = set(declared_functions()) - exported
    assert not missing, missing
    for name in declared_functions():
        assert getattr(lib, name) is not None


def test_library_is_gfx950_code():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", capi.LIB_PATH],
                         capture_output=True, text=True)
    blob = open(capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"k_sample" in blob


def test_host_only_entry_points(lib):
    assert lib.lda_version().decode().startswith("lda_mi355x")
    assert capi.padded_topics(1) == 64
    assert capi.padded_topics(64) == 64
    assert capi.padded_topics(65) == 128
    assert capi.padded_topics(1024) == 1024
    assert capi.padded_topics(300) == 512          # Kp = 64 x power of two
    assert capi.padded_topics(1025) == 2048
    assert capi.padded_topics(4096) == 4096


def test_config_struct_layout():
    # lda_config is shared with C: field offsets must match the header's order
    assert C.sizeof(capi.lda_config) == 4 + 4 + 8 + 8 + 8 + 8 + 4 + 4 + 8 + 8
    assert capi.lda_config.token_base.offset == 48


def test_invalid_arguments_fail_loudly(lib):
    h = C.c_void_p()
    cfg = capi.lda_config()
    cfg.num_topics = 0                       # invalid before any device call
    off = np.array([0, 1], dtype=np.int64)
    w = np.array([0], dtype=np.int32)
    st = lib.lda_create(C.byref(h), C.byref(cfg), off, w.ctypes.data, None)
    assert st == -1
    assert b"num_topics" in lib.lda_last_error()
    with pytest.raises(capi.LdaError, match="LDA_ERR_INVALID_ARG"):
        capi.check(st, "lda_create")
    assert lib.lda_sweep(None, 1) == -1
    assert lib.lda_sample(None) == -1
    # the dense sampler indexes nw cells with 32 bits: V * Kp >= 2^32 is refused
    alpha = np.full(1024, 0.1)
    cfg.num_topics = 1024
    cfg.num_types = 1 << 22
    cfg.alpha = alpha.ctypes.data_as(C.POINTER(C.c_double))
    cfg.beta = 0.01
    cfg.sampler = capi.SAMPLERS["dense"]
    st = lib.lda_create(C.byref(h), C.byref(cfg), off, w.ctypes.data, None)
    assert st == -5 and b"2^32" in lib.lda_last_error()


def test_no_cpu_fallback_without_library(tmp_path):
    import importlib
    saved = capi._lib
    try:
        capi._lib = None
        with pytest.raises(ImportError):
            capi.load(str(tmp_path / "missing.so"))
    finally:
        capi._lib = saved


def test_bench_traffic_record_matches_its_sweep_window():
    """bench.py prices a line's PMC traffic only with a profile of the same
    window: the committed C5 profile of the bench command near init is found
    for burn-in 0 on the kernel sources in the tree, the after-30-sweeps one
    (shorter rows) for burn-in 30, and none for a window nobody profiled."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rec, src = bench.pmc_record(250_000_000, "k_sample_sparse_big<", 4096, 0)
    if rec is None:
        pytest.skip("no C5 profile of the kernel sources in the tree")
    assert src.endswith("traffic_c5.json")
    assert rec.get("burnin", 0) == 0
    rec30, src30 = bench.pmc_record(250_000_000, "k_sample_sparse_big<", 4096, 30)
    if rec30 is not None:
        assert src30.endswith("traffic_c5_b30.json") and rec30["burnin"] == 30
        assert rec30["bytes_per_token"] < rec["bytes_per_token"]
    assert bench.pmc_record(250_000_000, "k_sample_sparse_big<", 4096, 7) == (None, None)
