#!/usr/bin/env python3
"""Write profiles/rNN/traffic_k{K}.json (what bench.py reports as
roofline.traffic) from the rocprofv3 summaries of one profile run.

  make_traffic.py <summary_dir> <kernel> <tokens_per_launch> <workload> <out.json> [K]

summary_dir holds summary_kt.json (--kernel-trace --stats), summary_fetch.json
(--pmc FETCH_SIZE) and summary_write.json (--pmc WRITE_SIZE), each its own
rocprofv3 pass over the same bench command (tools/profile.sh).  Bytes follow
MI355X_MICROARCH.md §HBM for gfx950: FETCH_SIZE/WRITE_SIZE are KiB, and
FETCH_SIZE's bytes per byte read depend on the access width, so each sampler
kernel's FETCH is divided by the factor measured on known bytes of its own
pattern (tools/fetch_calib.hip -> profiles/rNN/fetch_calib.json).
When the SQ passes (summary_sq.json / summary_lds.json / summary_grbm.json)
are there too, the per-token instruction mix and the effective clock are
recorded as well: bench.py's issue-bound roofline reads them.
"""
import json
import os
import sys


def lib_sha256(path):
    import hashlib
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _ctr(d, name, kernel, counter):
    p = os.path.join(d, f"summary_{name}.json")
    if not os.path.exists(p):
        return None
    c = json.load(open(p))["counters"].get(kernel, {}).get(counter)
    return c["avg_per_dispatch"] if c else None


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_src_sha256():
    """sha256 of the kernel sources (lda_kernels.hip + lda_kernels.h): the
    counters belong to the machine code built from exactly these."""
    import hashlib
    h = hashlib.sha256()
    for f in ("lda_kernels.hip", "lda_kernels.h"):
        with open(os.path.join(ROOT, "ldagibbssampling_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def access_pattern(kernel):
    """The calibrated load pattern (tools/fetch_calib.hip) of a sampler kernel:
    its word rows are 16 B per lane at C >= 8, 4 B per lane at C = 2, and 4 B
    per lane in 256 B rounds for the large-K sparse sampler."""
    if kernel.startswith("k_sample_big") or kernel.startswith("k_sample_sparse_big"):
        return "k_round4"
    if (kernel.startswith("k_sample<8") or kernel.startswith("k_sample<16")
            or kernel.startswith("k_sample_quarter<8")):     # quarter, K <= 128: uint4 per lane
        return "k_row16"
    if kernel.startswith("k_sample<2") or kernel.startswith("k_sample_quarter<2"):
        return "k_row4x2"
    return None


def fetch_factor(pattern):
    """FETCH_SIZE bytes per byte read for this pattern, from the newest
    profiles/rNN/fetch_calib.json; the guide's 1/2 for 16 B/lane streams when
    no calibration covers it."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "fetch_calib.json")))[::-1]:
        c = json.load(open(path))
        if pattern and pattern in c and c[pattern].get("fetch_over_read"):
            return c[pattern]["fetch_over_read"], os.path.relpath(path, ROOT) + ":" + pattern
    return 0.5, "MI355X_MICROARCH.md §HBM (16 B/lane stream)"


def main(d, kernel, tokens, workload, out, K=None, burnin=None):
    kt = json.load(open(os.path.join(d, "summary_kt.json")))
    fe = json.load(open(os.path.join(d, "summary_fetch.json")))["counters"][kernel]["FETCH_SIZE"]
    wr = json.load(open(os.path.join(d, "summary_write.json")))["counters"][kernel]["WRITE_SIZE"]
    pat = access_pattern(kernel)
    ff, fsrc = fetch_factor(pat)
    t = {
        "workload": workload,
        "kernel": kernel,
        "tokens_per_launch": int(tokens),
        "avg_ns_kernel_trace": kt["kernels"][kernel]["avg_ns"],
        "FETCH_SIZE_KiB": fe["avg_per_dispatch"],
        "WRITE_SIZE_KiB": wr["avg_per_dispatch"],
        "hbm_bytes_per_launch": (fe["avg_per_dispatch"] / ff + wr["avg_per_dispatch"]) * 1024,
        "hbm_bytes_per_launch_uncorrected": (fe["avg_per_dispatch"] + wr["avg_per_dispatch"]) * 1024,
        "access_pattern": pat,
        "fetch_size_per_byte_read": ff,
        "correction": f"bytes = (FETCH_SIZE / {ff:.4f} + WRITE_SIZE) * 1024, the FETCH factor "
                      f"calibrated on known bytes of this access pattern ({fsrc}); FETCH_SIZE also "
                      "counts Infinity-Cache hits",
        "source": f"tools/profile.sh passes summarised in {d}",
    }
    tcc = os.path.join(d, "summary_tcc.json")
    if os.path.exists(tcc):
        c = json.load(open(tcc))["counters"].get(kernel, {})
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            h, m = c["TCC_HIT_sum"]["avg_per_dispatch"], c["TCC_MISS_sum"]["avg_per_dispatch"]
            t["l2_hit_rate"] = h / (h + m) if h + m else None
    t["bytes_per_token"] = t["hbm_bytes_per_launch"] / t["tokens_per_launch"]
    if K is not None:
        t["num_topics"] = int(K)
    if burnin is not None and int(burnin) > 0:
        # the profiled command's --burnin (bench.py matches a line's window on it)
        t["burnin"] = int(burnin)
    # instruction mix per token (wave-instructions: SQ_INSTS_* sum over all waves)
    mix = {}
    for name, counter in (("sq", "SQ_INSTS_VALU"), ("lds", "SQ_INSTS_SALU"), ("lds", "SQ_INSTS_LDS"),
                          ("lds", "SQ_INSTS_SMEM"), ("sq", "SQ_WAVE_CYCLES"), ("sq", "SQ_WAIT_ANY"),
                          ("sq", "SQ_WAIT_INST_ANY"), ("sq", "SQ_ACTIVE_INST_ANY")):
        v = _ctr(d, name, kernel, counter)
        if v is not None:
            mix[counter] = v / float(tokens)
    if mix:
        t["per_token"] = mix
    g = _ctr(d, "grbm", kernel, "GRBM_GUI_ACTIVE")
    if g is not None:
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles (MI355X_MICROARCH.md, DVFS item)
        t["effective_clock_ghz"] = g / 8.0 / (t["avg_ns_kernel_trace"])
    # the library these counters belong to: bench.py uses the file only for it
    lib = os.environ.get("LDA_MI355X_LIB") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ldagibbssampling_amd", "lib",
        "liblda_mi355x.so")
    t["lib_sha256"] = lib_sha256(lib)
    t["kernel_src_sha256"] = kernel_src_sha256()
    # the machine code of this kernel family (every instantiation's text and
    # descriptor, ldagibbssampling_amd/codeobj.py): what bench.py matches on,
    # so an edit to another kernel does not orphan this record
    sys.path.insert(0, ROOT)
    from ldagibbssampling_amd import codeobj
    fam, arg = codeobj.family_of(kernel)
    if fam in ("k_sample_half", "k_sample_quarter"):
        arg = None       # bench.py matches these over all their instantiations
    t["kernel_family"] = codeobj.mangled_prefix(fam, arg)
    t["kernel_code_sha256"] = codeobj.family_sha256(lib, fam, arg)
    with open(out, "w") as f:
        json.dump(t, f, indent=1)
    print(json.dumps(t, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:8])
