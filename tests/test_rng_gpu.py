"""The device RNG against rocRAND: every uniform the
kernels draw is word 0 of Philox4x32-10 with counter {global token index lo,
hi, sweep, stream} and the seed as key; lda_philox_draws returns those words
from the library's own device code, tests/native/philox_vs_rocrand.hip
compares them with rocRAND's philox4x32_10 engine on the same GPU (token
indices past 2^31, 2^32 and 2^61, every stream, sweeps up to 2^32 - 1, six
seeds), and the oracle's Philox (pinned by the Random123 KAT) is checked
against the library's draws here."""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROG = os.path.join(ROOT, "tests", "native", "bin", "philox_vs_rocrand")


def test_device_philox_equals_rocrand():
    assert os.path.exists(PROG), "build() compiles tests/native/bin/philox_vs_rocrand"
    r = subprocess.run([PROG], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["mismatches"] == 0 and out["checked"] > 100000


def test_device_philox_equals_oracle(oracle):
    from ldagibbssampling_amd import capi
    L = capi.load()
    g = np.concatenate([np.arange(2000), (1 << 32) + np.arange(100), [(1 << 31) - 1, 1 << 40]])
    g = g.astype(np.int64)
    for seed, c2, c3 in ((42, 0, 0), (7, 13, 1), (2**63 + 5, 2**32 - 1, 2)):
        out = np.zeros(len(g), np.uint32)
        assert L.lda_philox_draws(seed, c2, c3, g.ctypes.data, len(g), out.ctypes.data) == 0
        ref = [oracle.draw(seed, int(t), c2, c3) for t in g]
        np.testing.assert_array_equal(out, np.array(ref, np.uint32))
