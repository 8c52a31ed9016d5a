"""CPU checks of the ParallelTopicModel host mirror (liblda_topic_model.so):
header <-> binding <-> exports, Mallet's number renderings, the reference's
ingest pipe, and loud errors without a GPU.  Sampling itself is covered by
tests/test_topic_model_gpu.py."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from ldagibbssampling_amd import capi, topic_model as tm

HEADER = os.path.join(os.path.dirname(capi.HEADER_PATH), "lda_topic_model.h")


def declared():
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    return sorted(set(re.findall(r"\b(ldatm_[a-z_0-9]+)\s*\(", text)))


@pytest.fixture(scope="module")
def L():
    return tm.load_tm()


def test_header_binding_exports_agree(L):
    assert declared() == sorted(tm.TM_SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", tm.TM_LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (ldatm_\w+)", out))
    assert set(declared()) <= exported
    # the mirror sits above the sampler ABI: it links liblda_mi355x.so and RCCL
    dyn = subprocess.run(["readelf", "-d", tm.TM_LIB_PATH], capture_output=True, text=True).stdout
    assert "liblda_mi355x.so" in dyn and "librccl.so" in dyn


@pytest.mark.parametrize("x,java", [
    (1.0, "1.0"), (100.0, "100.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"),
    (9999999.0, "9999999.0"), (123456789.0, "1.23456789E8"), (0.1 + 0.2, "0.30000000000000004"),
    (0.6308917995984609, "0.6308917995984609"), (0.0010402955565968202, "0.0010402955565968202"),
    (-2.5e-5, "-2.5E-5"), (0.0, "0.0"), (-0.0, "-0.0"), (1.5e300, "1.5E300"),
    (float("nan"), "NaN"), (float("inf"), "Infinity"),
])
def test_java_double_to_string(L, x, java):
    assert tm.format_double(x, 0) == java


@pytest.mark.parametrize("x,fmt", [
    (0.00868, "0.00868"), (2.0, "2"), (0.123456, "0.12346"), (1234.56789, "1,234.56789"),
    (1234567.0, "1,234,567"), (-7.123456789, "-7.12346"), (0.1, "0.1"), (5e-324, "0"),
    (0.000015, "0.00002"), (0.000025, "0.00003"),   # HALF_EVEN on the exact binary value
    (0.125, "0.125"), (2.5e-6, "0"),
])
def test_mallet_number_format(L, x, fmt):
    assert tm.format_double(x, 1) == fmt


def test_format_errors_are_loud(L):
    with pytest.raises(capi.LdaError):
        tm.format_double(1.0, 7)


def test_instance_list_from_inverse_docs():
    text = "t1\tFoo/Bar.java\tbaz.java\n t2\tfoo/bar.java\n\tBAZ.java\tnew.java\n"
    il = tm.InstanceList.fromInverseDocs(text)
    a = il.getDataAlphabet()
    assert a.toArray() == ["foo/bar.java", "baz.java", "new.java"]
    assert [list(i.data) for i in il] == [[0, 1], [0], [1, 2]]
    assert [i.target for i in il] == ["t1", " t2", ""]
    # a second list over the same (growing) alphabet, as updateModel does
    il2 = tm.InstanceList.fromInverseDocs("t9\tnew.java\tzzz.java\n", alphabet=a)
    assert a.size() == 4 and list(il2[0].data) == [2, 3]
    # inference-style: no growth, unknown tokens dropped
    il3 = tm.InstanceList.fromInverseDocs("t9\tqqq.java\tbaz.java\n", alphabet=a, grow=False)
    assert a.size() == 4 and list(il3[0].data) == [1]


def test_model_options_without_gpu(L):
    """Creating a model and setting options is host-only; the first use of
    the GPU (estimate) fails loudly when there is none."""
    m = tm.ParallelTopicModel(20, 10.0, 0.01)
    m.setOptimizeInterval(20)
    m.setNumThreads(4)
    m.setNumIterations(5)
    m.setTopicDisplay(0, 0)
    assert m.alphaSum == 10.0 and m.beta == 0.01 and np.allclose(m.alpha, 0.5)
    with pytest.raises(capi.LdaError):
        m.setNumThreads(0)
    with pytest.raises(capi.LdaError):
        tm.ParallelTopicModel(5000, 1.0, 0.01)
    il = tm.InstanceList.fromInverseDocs("a\tx\ty\nb\ty\tz\n")
    m.addInstances(il)
    import torch
    if not torch.cuda.is_available():
        with pytest.raises(capi.LdaError):
            m.estimate()


def test_checkpoint_round_trip_without_gpu(L, tmp_path):
    """save()/load() of a model that has not sampled yet is host-only."""
    il = tm.InstanceList.fromInverseDocs("a\tx\ty\tz\nb\ty\tz\nc\tq\n")
    m = tm.ParallelTopicModel(7, 3.5, 0.02)
    m.setOptimizeInterval(20)
    m.setBurninPeriod(50)
    m.setRandomSeed(11)
    m.addInstances(il)
    p = tmp_path / "model.ldatm"
    m.save(str(p))
    r = tm.ParallelTopicModel.load(str(p))
    assert r._shape() == m._shape() == (7, 4, 3, 6)
    np.testing.assert_array_equal(r.alpha, m.alpha)
    assert r.beta == 0.02 and r.alphaSum == 3.5
    bad = tmp_path / "bad.ldatm"
    bad.write_bytes(b"not a checkpoint")
    with pytest.raises(capi.LdaError):
        tm.ParallelTopicModel.load(str(bad))
    trunc = tmp_path / "trunc.ldatm"
    trunc.write_bytes(p.read_bytes()[:60])
    with pytest.raises(capi.LdaError):
        tm.ParallelTopicModel.load(str(trunc))
    # a v3 file (round 4) still carries the alpha-statistics histograms after
    # max_doc_len; v4 files drop them (estimate() starts them empty) and v3
    # files load with them skipped
    raw = p.read_bytes()
    assert raw[:8] == b"LDATM\x00v4"
    # the last 16 bytes: max_doc_len (-1 before the first estimate), warm
    # parts, warm sweeps, staleness (int32); a v3 file with sized histograms
    assert int(np.frombuffer(raw[-16:-12], np.int32)[0]) == -1
    max_len = 3
    dl = np.arange(max_len + 1, dtype=np.int32)
    td = np.arange(7 * (max_len + 1), dtype=np.int32)
    hist = (np.int64(dl.size).tobytes() + dl.tobytes() + np.int64(td.size).tobytes() + td.tobytes())
    body = raw[8:-16] + np.int32(max_len).tobytes()
    v3 = tmp_path / "v3.ldatm"
    v3.write_bytes(b"LDATM\x00v3" + body + hist + raw[-12:])
    r3 = tm.ParallelTopicModel.load(str(v3))
    assert r3._shape() == m._shape()
    np.testing.assert_array_equal(r3.alpha, m.alpha)
    bad3 = tmp_path / "bad3.ldatm"             # histograms of the wrong shape
    bad3.write_bytes(b"LDATM\x00v3" + body + hist[:8 + 4 * dl.size] + np.int64(1).tobytes()
                     + td[:1].tobytes() + raw[-12:])
    with pytest.raises(capi.LdaError):
        tm.ParallelTopicModel.load(str(bad3))


def test_shard_plan():
    """setNumThreads -> GPU shards (ldatm_plan_shards): capped by the devices
    and the documents, and one GPU when the sweep is shorter than the
    exchange (the reference's C1 corpus with setNumThreads(4))."""
    from ldagibbssampling_amd.topic_model import plan_shards
    # C1 at src/cmu_ron's K = 500 and src/cmu's K = 100, 8 GPUs visible
    assert plan_shards(4, 8, 16_000, 5_000, 500, 2_000) == 1
    assert plan_shards(4, 8, 16_000, 5_000, 100, 2_000) == 1
    # C4 (2e9 tokens, V = 100k, K = 512): every GPU asked for
    assert plan_shards(4, 8, 2_000_000_000, 100_000, 512, 10_000_000) == 4
    assert plan_shards(8, 8, 2_000_000_000, 100_000, 512, 10_000_000) == 8
    assert plan_shards(8, 2, 2_000_000_000, 100_000, 512, 10_000_000) == 2
    # never more shards than documents, at least one
    assert plan_shards(4, 8, 2_000_000_000, 100_000, 512, 3) == 3
    assert plan_shards(0, 8, 10, 10, 10, 0) == 1
    # C2 (2e7 tokens, V = 50k, K = 128): worth two GPUs or more
    assert plan_shards(4, 8, 20_000_000, 50_000, 128, 100_000) >= 2
