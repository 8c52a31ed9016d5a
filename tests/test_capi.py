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
    rec, src = bench.pmc_record(250_000_000, "k_sample_big<", 4096, 0, C=64)
    if rec is None:
        pytest.skip("no C5 profile of the kernel sources in the tree")
    assert "traffic_c5" in src and "_b30" not in src
    assert rec.get("burnin", 0) == 0
    rec30, src30 = bench.pmc_record(250_000_000, "k_sample_big<", 4096, 30, C=64)
    if rec30 is not None:
        assert "traffic_c5" in src30 and src30.endswith("_b30.json") and rec30["burnin"] == 30
        assert rec30["bytes_per_token"] < rec["bytes_per_token"]
    assert bench.pmc_record(250_000_000, "k_sample_big<", 4096, 7, C=64) == (None, None)


def test_version_string_carries_the_abi_number(lib):
    """lda_version() had said "ABI 3" while the header said 4."""
    v = lib.lda_version().decode()
    assert v.endswith(f"; ABI {lib.lda_abi_version()})"), v


def _warm_tokens(lib, doc_off, parts, token_base, g0, gn):
    import numpy as np
    off = np.ascontiguousarray(doc_off, dtype=np.int64)
    out = np.zeros(parts, dtype=np.int64)
    capi.check(lib.lda_warm_part_tokens(off.ctypes.data, len(off) - 1, parts, int(token_base),
                                        int(g0), int(gn), out.ctypes.data), "lda_warm_part_tokens")
    return out


def test_warm_start_parts_keep_every_shard_busy(lib):
    """the warm start's parts are interleaved segments of
    the corpus, so at G = 8 shards and P = 4 parts every shard samples in
    every step (round 3's contiguous parts left 6 of 8 GPUs idle per step),
    and the product's cuts equal the oracle's (cpu_exact _warm_runs)."""
    import numpy as np
    from ldagibbssampling_amd.distributed import shard_corpus
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    lens = rng.integers(20, 400, size=40_000)
    doc_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    words = np.zeros(int(doc_off[-1]), dtype=np.int32)
    N = int(doc_off[-1])
    for G, P in [(8, 4), (8, 2), (3, 4), (1, 3)]:
        tot = np.zeros(P, dtype=np.int64)
        for r in range(G):
            sh = shard_corpus(doc_off, words, G, r)
            t = _warm_tokens(lib, sh.doc_off, P, sh.token_base, 0, N)
            assert t.sum() == len(sh.words)
            # every shard has ~1/P of its tokens in each part
            assert (t > 0).all() and t.min() >= 0.15 * len(sh.words), (G, P, r, t)
            o = O.ExactSampler(4, 1, sh.doc_off, sh.words, 0.1, 0.01, 1, token_base=sh.token_base)
            o.set_warm_start(P, 1, 0, N)
            off = sh.doc_off - sh.doc_off[0]
            ot = [sum(int(off[b] - off[a]) for a, b in runs) for runs in o._warm_runs()]
            assert list(t) == ot
            tot += t
        # the global parts do not depend on the sharding
        one = _warm_tokens(lib, doc_off, P, 0, 0, N)
        np.testing.assert_array_equal(tot, one)
        assert (abs(one - N / P) < 0.02 * N).all()


def test_staleness_schedule_matches_mallet_threads(lib):
    """lda_staleness_schedule (host-only): the sequential-sweep schedule whose
    mean live fraction is that of Mallet's T worker threads, 1/(2T) -- two
    parts, the first f of every block with f (1 - f) = 1/(2T) -- and the
    oracle's restatement of it, fraction for fraction."""
    import ctypes as C
    import numpy as np
    from oracle import oracle as O
    for T in (1, 2, 3, 4, 8, 64):
        n = C.c_int32()
        fr = np.zeros(capi.MAX_EXCHANGE_PARTS, dtype=np.float64)
        capi.check(lib.lda_staleness_schedule(T, C.byref(n), fr.ctypes.data), "lda_staleness_schedule")
        parts, ofr = O.staleness_schedule(T)
        assert n.value == parts and list(fr[:parts]) == ofr
        live = sum(ofr[i] * sum(ofr[:i]) for i in range(parts))
        if T > 1:
            assert abs(live - 1 / (2 * T)) < 1e-12 and parts == 2
        else:
            assert parts == capi.MAX_EXCHANGE_PARTS and abs(live - 3 / 8) < 1e-12
    # the quantised cuts are exact for equal parts
    assert O.quantise_fractions([1 / 3] * 3) == O.equal_cum(3)
    assert O.quantise_fractions([0.5, 0.5]) == O.equal_cum(2)


def test_profile_summary_windows_the_bench_sweeps(tmp_path):
    """tools/summarize_prof.py averages exactly the bench's timed sweeps: the
    sampler's dispatches form one sequence whatever their template arguments
    (the large-K sampler alternates two ring depths), the skipped warm-up /
    burn-in sweeps and whatever follows the timed region (the estimate() side
    figure's launches) stay out."""
    import csv
    import importlib.util
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("sp", os.path.join(root, "tools", "summarize_prof.py"))
    sp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sp)
    # 4 untimed sweeps, 3 timed, then 5 small "side figure" launches; sweep 1
    # and timed sweep 5 use the other instantiation
    names = ["k_sample_big<64, 3, 10, false>"] * 12
    names[1] = names[5] = "k_sample_big<64, 3, 8, false>"
    durs = [100, 90, 80, 70, 60, 50, 40, 1, 1, 1, 1, 1]
    with open(tmp_path / "x_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for i, (n, d) in enumerate(zip(names, durs)):
            w.writerow({"Kernel_Name": n, "Start_Timestamp": 1000 * i, "End_Timestamp": 1000 * i + d})
            w.writerow({"Kernel_Name": "k_apply(int)", "Start_Timestamp": 1000 * i + 500,
                        "End_Timestamp": 1000 * i + 510})
    with open(tmp_path / "x_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Dispatch_Id", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (n, d) in enumerate(zip(names, durs)):
            for half in (0.5, 0.5):          # a counter reported per XCD-like slice
                w.writerow({"Kernel_Name": n, "Dispatch_Id": 2 * i, "Counter_Name": "WRITE_SIZE",
                            "Counter_Value": d * half})
    out = tmp_path / "s.json"
    sp.main(str(tmp_path), str(out), 4, 1, 3)
    s = json.load(open(out))
    k10, k8 = "k_sample_big<64, 3, 10, false>", "k_sample_big<64, 3, 8, false>"
    assert s["kernels"][k10]["calls"] == 2 and s["kernels"][k10]["avg_ns"] == 50   # sweeps 4, 6
    assert s["kernels"][k8]["calls"] == 1 and s["kernels"][k8]["avg_ns"] == 50     # sweep 5
    assert s["counters"][k10]["WRITE_SIZE"]["avg_per_dispatch"] == 50
    assert s["kernels"]["k_apply"]["calls"] == 3


def test_kernel_code_hashes_cover_the_samplers(lib):
    """bench.py matches PMC records to the machine code of one kernel family
    (ldagibbssampling_amd/codeobj.py): every sampler family is found in the
    library's gfx950 code object, none holds a PC-relative reference (whose
    immediate would move with the layout), and the hashes of two families
    differ while one family's hash is reproducible."""
    from ldagibbssampling_amd import codeobj
    ks = codeobj.kernels(codeobj.device_code_object(capi.LIB_PATH))
    for fam, arg in (("k_sample", 8), ("k_sample", 16), ("k_sample_big", 64), ("k_sample_big", 32),
                     ("k_sample_quarter", None), ("k_sample_sparse", 8)):
        pre = codeobj.mangled_prefix(fam, arg)
        names = [k for k in ks if k.startswith(pre)]
        assert names, pre
        assert all(codeobj.pc_relative_free(ks[k][0]) for k in names), pre
        assert all(len(ks[k][1]) == 64 for k in names), pre        # the kernel descriptor
    h8 = codeobj.family_sha256(capi.LIB_PATH, "k_sample", 8)
    assert h8 == codeobj.family_sha256(capi.LIB_PATH, "k_sample", 8)
    assert h8 != codeobj.family_sha256(capi.LIB_PATH, "k_sample", 16)
    assert codeobj.family_of("k_sample_big<64, 2, 12, false>") == ("k_sample_big", 64)
    assert codeobj.family_of("k_sample_quarter<8, 4, false>") == ("k_sample_quarter", 8)


def test_cpu_baseline_sample_matches_the_workload_shape():
    """bench.py's cpu_baseline times cpu_mallet on a sample whose word types
    hold the workload's tokens per type (the vocabulary folded, VERDICT r5 weak
    #7) and reports the draw phase apart from Mallet's per-worker count
    rebuild and its merge."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from ldagibbssampling_amd.corpus import synthetic_lda
    c = synthetic_lda(num_docs=4000, num_types=1000, num_topics=16, doc_len=20, seed=3)
    r = bench.cpu_baseline(c, 16, 1.6, 0.01, budget_s=0.3, threads=2, runs=1)
    assert r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
    assert "folded onto 500 types" in r["sample"]          # 1000 x 2000 / 4000
    assert "(80 in the full corpus, 80 here)" in r["sample"]  # tokens per type kept
    assert 0.0 <= r["merge_share"] < 1.0 and 0.0 <= r["build_share"] < 1.0
    assert r["draw_rate"] >= r["sampling_rate"] > 0
    assert r["doc_sample"]["docs"] == 4000 and r["doc_sample"]["value"] > 0
