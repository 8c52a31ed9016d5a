#!/usr/bin/env python3
"""Benchmark: Gibbs tokens sampled/sec at K=512 (BASELINE.json metric).

Workload (one "step" = one full Gibbs sweep over the corpus = sample kernel
+ [RCCL all-reduce of the nw/nwsum exchange buffer when N > 1] + apply):
  config C4 of BASELINE.json, the whole corpus (10M docs x 200 tokens = 2e9
  tokens, V=100k, K=512), drawn as 8 blocks of 1.25M documents; with N GPUs
  rank r holds blocks [8r/N, 8(r+1)/N) (AD-LDA document shards), so every N
  runs the same corpus (strong scaling: N=1 is all of C4 on one MI355X, N=8
  is BASELINE's 8-GPU C4).  --config c4shard keeps 1.25M docs per GPU (weak
  scaling, the round-2 headline).
Synthetic corpus: LDA generative process, drawn on the GPU.

Prints ONE JSON line (rank 0).  value = tokens sampled by all ranks per
second of the max-over-ranks wall time of the K timed sweeps.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c1|c2|c3|c5]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: docs per GPU, doc length, V, K, description
    # c1: BASELINE configs[0], the reference's own scale (changelist-shaped
    # inverse_docs corpus; K=20, alphaSum 10 as src/cmu, 100 sweeps)
    "c1": dict(docs=2_000, doc_len=None, V=5_000, K=20, alpha_sum=10.0, steps=100,
               desc="C1: changelist-shaped corpus, 2000 docs x Poisson(8) tok, Zipf(1.1) over 5000 paths, K=20"),
    # the same corpus at the reference's own training settings
    "c1cmu": dict(docs=2_000, doc_len=None, V=5_000, K=100, alpha_sum=10.0, beta=0.001, steps=100,
                  desc="C1 corpus at src/cmu/TrainAndPredict.java:259 settings: K=100, alphaSum 10, beta 0.001"),
    "c1ron": dict(docs=2_000, doc_len=None, V=5_000, K=500, alpha_sum=100.0, beta=1.0, steps=100,
                  desc="C1 corpus at src/cmu_ron/TrainAndPredict.java:160 settings: K=500, alphaSum 100, beta 1"),
    # the headline: the whole C4 corpus, 8 blocks of 1.25M docs split over the ranks
    "c4": dict(docs=10_000_000, blocks=8, doc_len=200, V=100_000, K=512, scaling="strong",
               desc="C4: 10M docs x 200 tok (2e9 tokens), V=100k, K=512, documents split over the GPUs"),
    "c4shard": dict(docs=1_250_000, doc_len=200, V=100_000, K=512,
                    desc="C4 shard: 1.25M docs x 200 tok per GPU, V=100k, K=512 (weak scaling)"),
    "c2": dict(docs=100_000, doc_len=200, V=50_000, K=128, desc="C2: 100k docs x 200 tok, V=50k, K=128"),
    "c3": dict(docs=100_000, doc_len=200, V=50_000, K=1024, desc="C3: 100k docs x 200 tok, V=50k, K=1024"),
    "c5": dict(docs=1_250_000, doc_len=200, V=262_144, K=4096, sampler="sparse",
               desc="C5 shard: 1.25M docs x 200 tok per GPU, V=262144, K=4096, sparse sampler"),
}
HBM_PEAK_GBS = 8000.0   # MI355X spec (MI355X_MICROARCH.md: 8.0 TB/s)


def bytes_per_token(K: int) -> int:
    """SURVEY.md §8d fixed contract: 4K (int32 nw row gather) + 4 (word id)
    + 4 (z read) + 4 (z write) + 4 (amortised nw/nwsum delta updates)."""
    return 4 * K + 16


def encoding_bytes_per_token(Kp: int) -> int:
    """Bytes the shipped dense encoding needs per token: the word's 16-bit row
    over the Kp padded topics (2 Kp), word id, z read, z write and the
    amortised delta (4 each) — the contract's terms with 2-byte cells."""
    return 2 * Kp + 16


def _newest(pattern):
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", pattern)))[::-1]


def pmc_record(tokens_per_launch: int, kernel_prefix: str, K: int, burnin: int = 0, C: int = None):
    """The newest committed rocprofv3 summary (profiles/rNN/traffic_*.json,
    tools/make_traffic.py over separate FETCH_SIZE / WRITE_SIZE / SQ passes of
    this same command) measured on the machine code loaded now, for this
    workload, kernel and burn-in (a file without "burnin" profiled the
    command without one: rows, change rates and bytes per token move with the
    sweep window); (None, None) otherwise.

    "The machine code loaded now" is the kernel family's own code
    (`kernel_code_sha256`: the text and descriptor of every instantiation of
    e.g. k_sample<8, ...> in the loaded library's gfx950 code object,
    ldagibbssampling_amd/codeobj.py), so editing one kernel leaves the other
    kernels' records valid (the whole-file source hash
    had orphaned the unchanged dense kernel's record).  Records written
    before round 6 carry only the library's sha256, which still matches."""
    import hashlib
    from ldagibbssampling_amd import capi, codeobj
    lib = os.environ.get("LDA_MI355X_LIB") or capi.LIB_PATH
    with open(lib, "rb") as f:
        lib_sha = hashlib.sha256(f.read()).hexdigest()
    fam = kernel_prefix.rstrip("<")
    try:
        code_sha = codeobj.family_sha256(lib, fam, C)
    except (OSError, ValueError):
        code_sha = None
    for path in _newest("traffic_*.json"):
        with open(path) as f:
            t = json.load(f)
        same_code = t.get("lib_sha256") == lib_sha or (
            code_sha is not None and t.get("kernel_code_sha256") == code_sha
            and t.get("kernel_family") == codeobj.mangled_prefix(fam, C))
        if (t.get("tokens_per_launch") == tokens_per_launch and same_code
                and t.get("kernel", "").startswith(kernel_prefix)
                and t.get("num_topics", K) == K and t.get("burnin", 0) == burnin):
            return t, os.path.relpath(path, ROOT)
    return None, None


def issue_roofline(rec, tokens_per_s_kernel: float):
    """Instruction-issue bound of the sampler: its measured VALU and SALU
    wave-instructions per token (SQ_INSTS_VALU / SQ_INSTS_SALU of the PMC
    record) times the kernel's token rate, against the chip's measured issue
    peaks (tools/issue_peak.hip: independent s_add / v_add chains at 32 waves
    per CU, profiles/rNN/issue_peak.json).  frac = the larger of the two."""
    if not rec or "per_token" not in rec:
        return None
    peaks = _newest("issue_peak.json")
    if not peaks:
        return None
    with open(peaks[0]) as f:
        pk = json.load(f)
    pt = rec["per_token"]
    out = {"peaks_source": os.path.relpath(peaks[0], ROOT), "unit": "wave-instructions/s"}
    for kind, ctr, peak in (("valu", "SQ_INSTS_VALU", pk["valu_per_s"]),
                            ("salu", "SQ_INSTS_SALU", pk["salu_per_s"])):
        if ctr in pt:
            ach = pt[ctr] * tokens_per_s_kernel
            out[kind] = {"per_token": pt[ctr], "achieved": ach, "peak": peak, "frac": ach / peak}
    parts = [(v["frac"], k) for k, v in out.items() if isinstance(v, dict)]
    if not parts:
        return None
    out["frac"], out["binding"] = max(parts)
    if "SQ_INSTS_LDS" in pt:
        out["lds_per_token"] = pt["SQ_INSTS_LDS"]
    for c in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if c in pt:
            out.setdefault("quad_cycles_per_token", {})[c] = pt[c]
    if "effective_clock_ghz" in rec:
        out["effective_clock_ghz"] = rec["effective_clock_ghz"]
    return out


def stream_copy_gbs(device: int, nbytes: int = 2 << 30, reps: int = 10) -> float:
    """Measured device-to-device copy rate (read + write bytes / s) on this
    box: SURVEY.md §8d's "measured stream-copy peak" beside the 8 TB/s spec."""
    import torch
    x = torch.empty(nbytes // 4, dtype=torch.int32, device=f"cuda:{device}")
    y = torch.empty_like(x)
    y.copy_(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del x, y
    torch.cuda.empty_cache()
    return gbs


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_share() -> int:
    """The host cores this job may use: OMP_NUM_THREADS where the box sets it
    (the GPU box gives each GPU a 16-core share of a 256-CPU host), else the
    CPUs in this process's affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_baseline(corpus, K, alpha_sum, beta, budget_s=15.0, threads=4, runs=3):
    """cpu_mallet (oracle/, the Mallet 2.0.7 SparseLDA restatement) timed on a
    bounded sample of the same workload on this host's cores (SURVEY.md §8d,
    BASELINE.md: T = 1 and T = nproc): `threads` workers (the reference's
    setNumThreads(4)), a single thread, and every core of this job's CPU share.
    Each leg is `runs` separate timed runs of ~budget_s / runs seconds, worker
    t pinned to the t-th CPU of the job's affinity mask; a leg reports the
    median and the spread (min, max) of its runs, and the multi-thread legs the
    split of their time between the workers' sampling and Mallet's
    single-threaded sumTypeTopicCounts merge (the share that caps their
    speed-up over one thread)."""
    from oracle import oracle as O
    O.build()

    def timed(sub, V, T, budget, max_sweeps):
        m = O.MalletModel(K, alpha_sum, beta, V, sub.doc_off, sub.words, seed=1, num_threads=T)
        m.set_pin_threads(True)
        m.estimate(2)                                    # warm-up sweeps
        m.timing(reset=True)
        t0 = time.perf_counter()
        sweeps = 0
        while True:
            m.estimate(1)
            sweeps += 1
            if time.perf_counter() - t0 >= budget or sweeps >= max_sweeps:
                break
        dt = time.perf_counter() - t0
        ts, tm = m.timing()
        tb = m.build_time()
        n = sub.num_tokens * sweeps
        return n / dt, sweeps, tm / dt, n / ts, n / max(ts - tb, 1e-12), tb / ts

    def leg(sub, V, T, budget, max_sweeps, nruns=runs):
        r = [timed(sub, V, T, budget / nruns, max_sweeps) for _ in range(nruns)]
        v = sorted(x[0] for x in r)
        return {"median": float(np.median(v)), "min": v[0], "max": v[-1], "runs": nruns,
                "sweeps": [x[1] for x in r], "merge_share": float(np.median([x[2] for x in r])),
                # the workers' phase alone (sampling + Mallet's per-worker
                # buildLocalTypeTopicCounts), without the single-threaded merge
                "sampling_rate": float(np.median([x[3] for x in r])),
                # the draws alone: the workers' phase less Mallet's per-worker
                # buildLocalTypeTopicCounts (each T > 1 worker re-inserts its
                # documents' tokens into count-sorted rows every sweep)
                "draw_rate": float(np.median([x[4] for x in r])),
                "build_share": float(np.median([x[5] for x in r]))}

    # (1) the shape-matched sample: Mallet's cost per
    # token grows with the word's row (its nonzero topics) and its merge with
    # V x row length, so a 20k-document slice over the full vocabulary (~40
    # tokens per word type against the workload's N / V) runs short rows and
    # an inflated merge.  Here the first `nd` documents keep their lengths and
    # topic mixtures and the vocabulary is folded onto Vs = V * nd / D types
    # (w -> w mod Vs), so a word type holds the workload's tokens per type
    # (C4: 2e9 / 1e5 = 20000) and its rows fill as they do at full scale.
    nd = min(corpus.num_docs, 2_000)
    vs = max(1, int(round(corpus.num_types * nd / corpus.num_docs)))
    shaped = corpus.subset(np.arange(nd))
    from ldagibbssampling_amd.corpus import Corpus
    shaped = Corpus(shaped.doc_off, np.ascontiguousarray(shaped.words % vs, dtype=np.int32), vs)
    s4 = leg(shaped, vs, threads, budget_s, 40)
    s1 = leg(shaped, vs, 1, budget_s / 2, 20)
    tn = cpu_share()
    sn = leg(shaped, vs, tn, budget_s / 2, 40)
    # (2) rounds 2-5's sample, for continuity: the first 20k documents over
    # the full vocabulary, one run per leg
    ndocs = min(corpus.num_docs, 20_000)
    sub = corpus.subset(np.arange(ndocs))
    l4 = leg(sub, corpus.num_types, threads, budget_s / 3, 50, nruns=1)
    l1 = leg(sub, corpus.num_types, 1, budget_s / 3, 20, nruns=1)
    return {
        "value": s4["median"],
        "unit": "tokens/s",
        "cores": threads,
        "kind": "port",
        "spread": [s4["min"], s4["max"]],
        "merge_share": s4["merge_share"],
        "sampling_rate": s4["sampling_rate"],
        "t1_value": s1["median"],
        "t1_spread": [s1["min"], s1["max"]],
        "t1_sampling_rate": s1["sampling_rate"],
        "tnproc_value": sn["median"],
        "tnproc_spread": [sn["min"], sn["max"]],
        "tnproc_merge_share": sn["merge_share"],
        "tnproc_sampling_rate": sn["sampling_rate"],
        "tnproc_cores": tn,
        "sampling_speedup_4_over_1": s4["sampling_rate"] / s1["sampling_rate"],
        "draw_rate": s4["draw_rate"],
        "t1_draw_rate": s1["draw_rate"],
        "draw_speedup_4_over_1": s4["draw_rate"] / s1["draw_rate"],
        "build_share": s4["build_share"],
        "why_4_threads_scale_weakly": (
            "Mallet's multi-thread sweep does work a single thread does not: after its draws every "
            "worker rebuilds its local typeTopicCounts from its own documents "
            "(buildLocalTypeTopicCounts: a linear search and re-sort in the count-sorted row per "
            "token; build_share of the workers' phase), then one thread merges them "
            "(sumTypeTopicCounts, merge_share of the wall time); the draws alone scale by "
            "draw_speedup_4_over_1"),
        "sample": (f"cpu_mallet (Mallet 2.0.7 SparseLDA restatement, oracle/lda_oracle.c), "
                   f"{threads} threads (= setNumThreads(4), src/cmu_ron/TrainAndPredict.java:164), "
                   f"shape-matched sample: the first {nd} docs ({shaped.num_tokens} tokens) of this "
                   f"workload with the vocabulary folded onto {vs} types (w mod {vs}), so that a type "
                   f"holds the workload's tokens per type ({corpus.num_tokens / max(corpus.num_types, 1):.0f}"
                   f" in the full corpus, {shaped.num_tokens / vs:.0f} here) and rows reach their "
                   f"full-scale length; each leg {runs} runs (2 warm-up sweeps, then timed sweeps: "
                   f"{s4['sweeps']} / 1 thread {s1['sweeps']} / {tn} threads {sn['sweeps']}), median "
                   f"with [min, max] spread, worker t pinned to the t-th CPU of the job's affinity mask; "
                   f"merge_share = the fraction of the timed wall time in Mallet's single-threaded "
                   f"sumTypeTopicCounts merge; sampling_rate = tokens per second of the workers' phase "
                   f"alone; tnproc: {tn} threads = this job's CPU share (OMP_NUM_THREADS, else the "
                   f"affinity mask); host {_cpu_model()}, {os.cpu_count()} logical CPUs visible"),
        "doc_sample": {
            "docs": ndocs, "tokens": sub.num_tokens, "num_types": corpus.num_types,
            "value": l4["median"], "merge_share": l4["merge_share"],
            "sampling_rate": l4["sampling_rate"], "t1_value": l1["median"],
            "t1_sampling_rate": l1["sampling_rate"],
            "note": "rounds 2-5's sample (first 20k docs over the full vocabulary: short rows, "
                    "V-sized merge), one run per leg, kept for continuity",
        },
    }


SIDE_WORKLOADS = {
    # the C4 shard (block 0 of C4) and C2 (BASELINE configs[1]: K = 128, the
    # reference's K <= 128 regime, src/cmu/TrainAndPredict.java:259 K = 100)
    "c4": dict(docs=1_250_000, V=100_000, K=512,
               desc="C4 shard (block 0 of C4: 1.25M docs x 200 tok, V=100k, K=512), one GPU"),
    "c2": dict(docs=100_000, V=50_000, K=128, desc="C2 (100k docs x 200 tok, V=50k, K=128), one GPU"),
}


def estimate_side_figure(device: int, iters: int = 100, burnin: int = 50, workload: str = "c4"):
    """What the drop-in delivers: the native
    ParallelTopicModel (liblda_topic_model.so, the host mirror the JNI shim
    drives) running estimate() on the C4 shard (block 0 of the C4 corpus:
    1.25M docs x 200 tokens, V = 100k, K = 512, alphaSum 51.2, beta 0.01)
    with the reference's setNumThreads(4) (its staleness schedule, one GPU
    shard) and its defaults -- the 4 x 50 warm start (sweeps 0..49 in 4
    sequential parts), LL/token every 10 iterations -- and setOptimizeInterval(20) with
    burn-in `burnin` (Mallet's default 200 would put no optimisation inside
    100 iterations; 50 gives 3: iterations 60, 80, 100).  Timed: the
    estimate() call of `iters` iterations, after an estimate() of 0
    iterations that builds the shard (upload, Philox init, counts; Mallet
    does that work in addInstances).  Never `value`."""
    import ctypes as C
    from ldagibbssampling_amd.corpus import synthetic_lda_torch
    from ldagibbssampling_amd.topic_model import _check, load_tm
    L = load_tm()
    wl = SIDE_WORKLOADS[workload]
    K, V = wl["K"], wl["V"]
    c = synthetic_lda_torch(wl["docs"], V, K, doc_len=200, seed=20261015, doc_seed=20261015,
                            device=f"cuda:{device}")
    h = C.c_void_p()
    _check(L.ldatm_create(C.byref(h), K, 0.1 * K, 0.01), "ldatm_create")
    try:
        _check(L.ldatm_set_alphabet(h, V, None), "ldatm_set_alphabet")
        off = np.ascontiguousarray(c.doc_off, np.int64)
        words = np.ascontiguousarray(c.words, np.int32)
        _check(L.ldatm_add_instances(h, c.num_docs, off, words.ctypes.data, None), "ldatm_add_instances")
        _check(L.ldatm_set_random_seed(h, 1), "ldatm_set_random_seed")
        _check(L.ldatm_set_topic_display(h, 0, 0), "ldatm_set_topic_display")
        _check(L.ldatm_set_optimize_interval(h, 20), "ldatm_set_optimize_interval")
        _check(L.ldatm_set_burnin_period(h, burnin), "ldatm_set_burnin_period")
        # the reference's setNumThreads(4) (src/cmu_ron/TrainAndPredict.java:164):
        # its staleness schedule; the shard stays on this one GPU
        _check(L.ldatm_set_num_threads(h, 4), "ldatm_set_num_threads")
        _check(L.ldatm_set_devices(h, 1, (C.c_int32 * 1)(device)), "ldatm_set_devices")
        _check(L.ldatm_set_num_iterations(h, 0), "ldatm_set_num_iterations")
        t0 = time.perf_counter()
        _check(L.ldatm_estimate(h), "ldatm_estimate (shard build)")
        t_build = time.perf_counter() - t0
        _check(L.ldatm_set_num_iterations(h, iters), "ldatm_set_num_iterations")
        t0 = time.perf_counter()
        _check(L.ldatm_estimate(h), "ldatm_estimate")
        dt = time.perf_counter() - t0
        a = np.zeros(K)
        asum, b = C.c_double(), C.c_double()
        _check(L.ldatm_get_hyper(h, a.ctypes.data, C.byref(asum), C.byref(b)), "ldatm_get_hyper")
    finally:
        L.ldatm_destroy(h)
    n = int(c.num_tokens)
    return {
        "tokens_per_s": n * iters / dt,
        "unit": "tokens/s",
        "seconds": dt,
        "iterations": iters,
        "tokens": n,
        "shard_build_s": t_build,
        "workload": wl["desc"],
        "count_update": os.environ.get("LDA_RECOUNT", "auto (default)"),
        "settings": (f"native ParallelTopicModel.estimate(): setNumThreads(4) (one GPU shard; "
                     f"sweeps with 4 threads' staleness), warm start 4 x 50 (default), LL/token "
                     f"every 10, setOptimizeInterval(20), setBurninPeriod({burnin}) -> "
                     f"{len([i for i in range(1, iters + 1) if i > burnin and i % 20 == 0])} "
                     f"optimisations"),
        "learned_alpha_sum": asum.value,
        "learned_beta": b.value,
    }


def dropin_schedule(args, sampler, trainer, world, device, tokens_all):
    """What the Java drop-in runs per sweep: the native
    ParallelTopicModel's default schedule past its warm start -- Mallet's
    setNumThreads(4) staleness (src/cmu_ron/TrainAndPredict.java:164),
    lda_staleness_schedule(4): two sequential parts per sweep, each sampled,
    exchanged across the ranks (N > 1) and applied before the next -- timed
    over --dropin-steps sweeps after the main timed region (1 untimed warm-up
    sweep), barrier + synchronize on both sides, max over ranks.  The parts
    are cut in the whole corpus's global token order (every rank passes the
    same corpus range), as the shard group does.  Never `value`."""
    import torch
    import torch.distributed as dist
    from ldagibbssampling_amd.sampler import staleness_schedule
    if args.config.startswith("c1") and world > 1:
        return None            # c1 shards are separate corpora (token_base = rank << 32)
    parts, fr = staleness_schedule(4)
    sampler.set_sequential_sweeps(parts, fr, 0, tokens_all)
    try:
        n_ex0 = len(trainer._sent)
        trainer.sweep(1)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        trainer.sweep(args.dropin_steps)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{device}")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        ks = sampler.sample_times(args.dropin_steps * parts)
        out = {
            "tokens_per_s": tokens_all * args.dropin_steps / dt,
            "ms_per_sweep": 1e3 * dt / args.dropin_steps,
            "sweeps": args.dropin_steps,
            "parts_per_sweep": parts,
            "part_fractions": [float(x) for x in fr],
            "exchanges_per_sweep": parts if trainer.exchange else 0,
            "sampler_ms_per_sweep": float(np.sum(ks)) / args.dropin_steps,
            "escape_counts_read": len(trainer._sent) - n_ex0 if trainer.exchange else 0,
            "schedule": "lda_staleness_schedule(4): Mallet's setNumThreads(4) mean live fraction "
                        "1/8, two sequential parts, each exchanged and applied before the next",
        }
        if trainer.exchange and trainer.time_reduce:
            out["collective_ms_per_sweep"] = trainer.reduce_ms(args.dropin_steps * parts) * parts
        return out
    finally:
        sampler.set_sequential_sweeps(1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed sweeps (default 10; 100 for c1)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0,
                    help="override docs per GPU (per block for a blocked config)")
    ap.add_argument("--sampler", default=None, choices=["dense", "sparse"],
                    help="draw kernel (default: dense, sparse for c5)")
    ap.add_argument("--burnin", type=int, default=0,
                    help="extra untimed sweeps before the warm-up (steady-state measurement)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tokens-per-range", type=int, default=0,
                    help="work-queue granule (0 = the library's default)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse several ranks on one GPU)")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-estimate", action="store_true",
                    help="skip the side figure: ParallelTopicModel.estimate() on the C4 shard "
                         "(N=1, c4 / c4shard only)")
    ap.add_argument("--exchange-parts", type=int, default=None,
                    help="N > 1: split every sweep into P parts whose all-reduces overlap the "
                         "next part's sampling (default 1: DESIGN.md §5)")
    ap.add_argument("--exchange-cells", type=int, default=None, choices=[2, 4],
                    help="N > 1: cells per packed exchange word (lda_set_exchange_cells: 4 halves "
                         "the bytes, more escapes; default: ADLDATrainer's choice, 4 for K > 1024; "
                         "DESIGN.md §5)")
    ap.add_argument("--int32-exchange", action="store_true",
                    help="N > 1: all-reduce the int32 exchange buffer instead of the compact "
                         "packed form (A/B)")
    ap.add_argument("--force-exchange", action="store_true",
                    help="N = 1: run the exchange anyway (an RCCL process group of one rank: the "
                         "pack, the in-place all-reduce, the all-gather and the unpack, whose sum "
                         "is the identity) to price the exchange's on-GPU cost; never the default")
    ap.add_argument("--dropin-steps", type=int, default=5,
                    help="after the timed region, time this many sweeps under the Java drop-in's "
                         "default schedule (Mallet's 4-thread staleness: two sequential parts, "
                         "each exchanged when N > 1; DESIGN.md §2, §5); 0 = skip")
    ap.add_argument("--reserve-cus", type=int, default=-1,
                    help="split sweeps: CUs' worth of sampler blocks left free for RCCL (-1: the library default, 1/32 of the CUs)")
    args = ap.parse_args()
    if os.environ.get("LDA_BENCH_STACKS"):
        # diagnostics: every rank dumps its Python stacks every N s to stderr
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["LDA_BENCH_STACKS"]), repeat=True)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    ndev = torch.cuda.device_count()
    device = local_rank % ndev                 # == local_rank with one GPU per rank
    torch.cuda.set_device(device)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
    elif args.force_exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            with socket.socket() as so:
                so.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(so.getsockname()[1])
        dist.init_process_group(args.backend, rank=0, world_size=1,
                                device_id=torch.device("cuda", device) if args.backend == "nccl" else None)

    from ldagibbssampling_amd.corpus import synthetic_lda_torch
    from ldagibbssampling_amd.distributed import ADLDATrainer
    from ldagibbssampling_amd.sampler import GibbsSampler

    cfg = CONFIGS[args.config]
    if args.sampler is None:
        args.sampler = cfg.get("sampler", "dense")
    if args.steps is None:
        args.steps = cfg.get("steps", 10)
    K, V, L = cfg["K"], cfg["V"], cfg["doc_len"]
    docs = args.docs or cfg["docs"]
    alpha_sum, beta = cfg.get("alpha_sum", 0.1 * K), cfg.get("beta", 0.01)
    t_gen = time.perf_counter()
    token_base = None
    blocks_info = None
    if cfg.get("blocks"):
        # one corpus for every N: block b is drawn with doc_seed 20261015 + b
        # (the topics, phi, from one seed); rank r takes a contiguous run of blocks
        nb = cfg["blocks"]
        total_docs = args.docs * nb if args.docs else cfg["docs"]
        if nb % world:
            nb = world            # N not dividing 8: N blocks (a different draw, noted in config)
        per_block = total_docs // nb
        b0, b1 = rank * nb // world, (rank + 1) * nb // world
        parts = [synthetic_lda_torch(per_block, V, K, doc_len=L, seed=20261015, doc_seed=20261015 + b,
                                     device=f"cuda:{device}") for b in range(b0, b1)]
        from ldagibbssampling_amd.corpus import Corpus
        offs = [parts[0].doc_off]
        for c_ in parts[1:]:
            offs.append(c_.doc_off[1:] + offs[-1][-1])
        corpus = Corpus(np.concatenate(offs), np.concatenate([c_.words for c_ in parts]), V)
        del parts
        docs = corpus.num_docs
        token_base = b0 * per_block * L
        blocks_info = {"blocks": nb, "docs_per_block": per_block, "doc_seeds": "20261015 + block",
                       "rank0_blocks": [0, nb // world]}
    elif args.config.startswith("c1"):
        from ldagibbssampling_amd.corpus import synthetic_changelists
        corpus = synthetic_changelists(num_docs=docs, num_types=V, seed=20261015 + rank)
        V = corpus.num_types          # the alphabet: paths seen in this shard
    else:
        # one corpus: the topics (phi) are shared by every shard, the documents
        # are drawn per rank (rank 0 == the N=1 workload)
        corpus = synthetic_lda_torch(docs, V, K, doc_len=L, seed=20261015,
                                     doc_seed=20261015 + rank, device=f"cuda:{device}")
    t_gen = time.perf_counter() - t_gen
    n_local = corpus.num_tokens
    sampler = GibbsSampler(K, V, corpus.doc_off, corpus.words, np.full(K, alpha_sum / K), beta,
                           seed=1, device=device,
                           # unique Philox counters per rank (c1 shards differ in size)
                           token_base=(token_base if token_base is not None else
                                       (rank << 32) if args.config.startswith("c1") else rank * n_local),
                           tokens_per_range=args.tokens_per_range, sampler=args.sampler)
    # one non-default stream carries the sampler kernels and (as torch's
    # current stream) orders the all-reduce behind them: no host sync per sweep.
    # (handle 0 = the legacy default stream would mean "the context's own
    # stream" to lda_set_stream, which the collective would not wait for)
    stream = torch.cuda.Stream(device=device)
    torch.cuda.set_stream(stream)
    sampler.set_stream(stream.cuda_stream)
    # AD-LDA: sample; all-reduce (SUM) of every rank's int32 nw/nwsum delta; apply.
    # --exchange-parts P > 1 splits the sweep so that part i's all-reduce
    # overlaps part i+1's sampling; the default is one blocking collective per
    # sweep (C4: 205 MB against a 35 ms sweep).
    if args.exchange_parts is None:
        args.exchange_parts = 1
    if args.exchange_parts > 1:
        sampler.set_exchange_parts(args.exchange_parts, args.reserve_cus)
    trainer = ADLDATrainer(sampler, sync_before_reduce=False, time_reduce=True,
                           compact=not args.int32_exchange,
                           exchange=True if args.force_exchange else None,
                           cells_per_word=args.exchange_cells)
    trainer.init_counts()

    def step():
        trainer.sweep(1)

    for _ in range(args.burnin + args.warmup):
        step()
    torch.cuda.synchronize()
    nnz0 = sampler.row_stats() if args.sampler == "sparse" and rank == 0 else None
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-launch duration of the sampler kernel over the timed region: HIP
    # events recorded around every launch on the sampler's stream, read back
    # after the closing synchronize (no host sync inside the timed loop)
    parts = sampler.exchange_parts
    ks = sampler.sample_times(args.steps * parts)
    nnz1 = sampler.row_stats() if nnz0 is not None else None
    assert len(ks) == min(args.steps * parts, 256)
    # a split sweep is `parts` launches: the sampler's time per sweep is their sum
    kern_ms = float(np.mean(ks)) * parts
    # the dense samplers' recount kernel after each launch of a recounting
    # sweep (lda_set_count_update: AUTO recounts the first sweeps of a small
    # corpus); the delta sweeps launch none
    rc = sampler.recount_times(args.steps * parts)
    n_rc = int((rc > 0).sum())
    recount_ms = float(rc[rc > 0].mean()) * parts if n_rc else None
    count_mode = sampler.count_update()
    copy_gbs = stream_copy_gbs(device) if rank == 0 else None

    # every rank's replica of nw / nwsum must be identical after the timed
    # region (lda_counts_checksum + the LL's word part, MIN == MAX over the
    # ranks), and the ranks' own timed-region seconds travel with the line
    replicas = trainer.replica_check(seconds=elapsed)
    t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{device}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    nt = torch.tensor([n_local], dtype=torch.int64, device=f"cuda:{device}")
    if world > 1:
        dist.all_reduce(nt, op=dist.ReduceOp.SUM)
    tokens_all = int(nt.item())
    total_tokens = tokens_all * args.steps
    value = total_tokens / elapsed
    ll = trainer.log_likelihood()
    dropin = None
    if args.dropin_steps > 0:
        # a side figure: an error raised identically on every rank (the same
        # call sequence everywhere) is reported in the line instead of
        # dropping the main measurement above
        try:
            dropin = dropin_schedule(args, sampler, trainer, world, device, tokens_all)
        except Exception as e:  # noqa: BLE001
            print(f"dropin_schedule failed: {e!r}", file=sys.stderr)
            dropin = {"error": repr(e)}

    if rank == 0:
        bpt = bytes_per_token(K)
        kname = (("k_sample_big" if K > 1024 else "k_sample_sparse")
                 if args.sampler == "sparse" else "k_sample")
        if args.sampler != "sparse" and sampler.Kp <= 128:
            # K <= 128 picks its dense kernel as lda_create does (LDA_DENSE_HALF:
            # unset/2 quarter-wave, 1 half-wave, 0 full-wave k_sample<C>)
            hv = os.environ.get("LDA_DENSE_HALF", "2")[:1]
            kname = {"0": "k_sample", "1": "k_sample_half"}.get(hv, "k_sample_quarter")
        if nnz0 is not None:
            # the sparse samplers read 4 B per nonzero entry of the token's word
            # row (token-weighted mean over the timed region's snapshots) + 16 B
            mean_nnz = 0.5 * (nnz0 + nnz1)
            enc = 4.0 * mean_nnz + 16.0
            enc_model = (f"4 B per nonzero (count, topic) entry of the word's row (mean "
                         f"{mean_nnz:.1f} entries, lda_row_stats) + word + z read + z write + "
                         f"amortised delta (4 each)")
        else:
            enc = float(encoding_bytes_per_token(sampler.Kp))
            enc_model = (f"16-bit row over Kp={sampler.Kp} topics (2 Kp) + word + z read + z write "
                         f"+ amortised delta (4 each)")
        achieved = n_local * enc / (kern_ms * 1e-3) / 1e9          # GB/s, shipped encoding
        # the family's first template argument is C = Kp / 64 for the full-wave
        # kernels; the half / quarter-wave ones are matched over all their
        # instantiations
        farg = None if kname in ("k_sample_half", "k_sample_quarter") else sampler.Kp // 64
        rec, rec_src = pmc_record(n_local, kname + "<", K, args.burnin, C=farg)
        traffic_gb = rec["hbm_bytes_per_launch"] / 1e9 if rec else None
        tok_s_kernel = n_local / (kern_ms * 1e-3)
        # what binds the sampler.  The dense rows of a table that
        # fits the 256 MB Infinity Cache (2 V Kp bytes: C4 102 MB) are a random
        # gather from that cache, and a 2 MB table runs only 3% faster: the
        # token is bound by the gather plus its instruction issue / dependency
        # chain (issue.frac), not by HBM.  The C5 sparse rows (4 GB) stream
        # from HBM.  achieved / peak stay the memory path's bytes against the
        # HBM spec peak (the Infinity Cache has no published bandwidth).
        if args.sampler != "sparse" and 2 * V * sampler.Kp <= 256 << 20:
            bound = "infinity-cache-gather+issue"
            bound_detail = (f"16-bit rows {2 * V * sampler.Kp / 1e6:.0f} MB <= 256 MB Infinity "
                            "Cache: random-row gather from the cache plus the token's issue / "
                            "dependency chain; frac is against the HBM spec peak")
        else:
            bound = "hbm"
            bound_detail = ("word rows streamed from HBM (table larger than the Infinity Cache) "
                            "plus the token's dependency chain")
        coll = None
        if trainer.exchange:
            xb = trainer.exchange_bytes()
            nbytes = xb["allreduce_bytes"] + xb["allgather_bytes"]
            rs = replicas.get("rank_seconds") or []
            int32_bytes = 4 * (V * sampler.Kp + sampler.Kp)
            # modelled time of one exchange at N = 8 on one ring over xGMI links of
            # ~153 GB/s (the per-link figure; RCCL's several rings only cut it):
            # all-reduce 2 (W-1)/W M, all-gather (W-1)/W of the W lists
            link = 153e9
            model8 = (2 * 7 / 8 * xb["allreduce_bytes"] + 7 / 8 * xb["allgather_bytes"] * 8 / world) / link
            coll = {"op": ((f"compact exchange (lda_exchange_pack: {sampler.exchange_cells} cells per int32 word + escape "
                            "lists): all_reduce(SUM, int32) of the packed words + all_gather of the "
                            "escape lists" + (" at their used length (after a MAX all_reduce of the "
                                              "counts; none gathered when no rank has one)"
                                              if trainer.escape_lists == "used" else
                                              " at their full capacity")
                            if trainer.compact else
                            "all_reduce(SUM, int32) of the nw/nwsum delta")
                           + (", once per sweep" if parts == 1 else
                              f", for each of {parts} sweep parts, part i's overlapping part "
                              f"i+1's sampling")),
                    "compact": trainer.compact,
                    "cells_per_word": sampler.exchange_cells if trainer.compact else None,
                    "exchange_parts": parts,
                    "reserve_cus": args.reserve_cus if parts > 1 else 0,
                    "bytes_per_sweep": nbytes * parts,
                    "allreduce_bytes_per_part": xb["allreduce_bytes"],
                    "allgather_bytes_per_part": xb["allgather_bytes"],
                    "allgather_capacity_bytes_per_part": xb.get("allgather_capacity_bytes"),
                    "escape_lists": xb.get("escape_lists", "none (int32 exchange)"),
                    "escape_count_max": xb.get("escape_count_max"),
                    "replicas_agree": replicas["replicas_agree"],
                    "counts_checksum": replicas["counts_checksum"],
                    "world_size": replicas["world_size"],
                    "ranks_counted": replicas["ranks_counted"],
                    "rank_ms_per_sweep": [1e3 * x / args.steps for x in rs],
                    "int32_bytes_per_sweep": int32_bytes * parts,
                    "ring_bytes_per_rank_per_sweep": 2 * (world - 1) * xb["allreduce_bytes"] * parts // world,
                    "modelled_n8_ms_per_sweep": model8 * parts * 1e3,
                    "model": "one ring, 153 GB/s per xGMI link, N = 8, bytes as above",
                    # parts == 1: the whole collective; > 1: the exposed tail after
                    # the last part's sampling
                    "ms_per_sweep": trainer.reduce_ms(args.steps),
                    "ms_kind": "collective" if parts == 1 else "exposed (after the last part)"}
            if world == 1:
                coll["forced_one_rank"] = ("--force-exchange: one RCCL rank, so ms_per_sweep is the "
                                           "pack + unpack kernels and RCCL's one-rank calls, not a "
                                           "transfer")
        result = {
            "metric": f"Gibbs tokens sampled/sec at K={K}",
            "value": value,
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "burnin": args.burnin,
            "sampler": args.sampler,
            "ms_per_step": elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": cfg.get("scaling", "weak"),
            "vs_baseline": None,
            "dtype": "fp32 weights / int32 counts",
            "data": ("synthetic (changelist-shaped inverse_docs corpus, SURVEY.md §8d; corpus.synthetic_changelists)"
                     if args.config.startswith("c1") else
                     "synthetic (LDA generative process, SURVEY.md §8d; phi~Dir(0.01), theta~Dir(0.1))"),
            "config": {
                "workload": cfg["desc"],
                "docs_per_gpu": docs,
                "doc_len": L,
                "tokens_per_gpu": n_local,
                "tokens_all_gpus": tokens_all,
                "corpus_blocks": blocks_info,
                "num_types": V,
                "num_topics": K,
                "alpha_sum": alpha_sum,
                "beta": beta,
                "parallelism": f"dp{world} (AD-LDA doc shards, "
                               f"{'RCCL' if args.backend == 'nccl' else 'gloo'} all-reduce of int32 delta)",
            },
            "roofline": {
                "bound": bound,
                "bound_detail": bound_detail,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic_gb,
                "bytes_per_token": enc,
                "bytes_model": enc_model,
                "kernel_ms_timed_region": kern_ms,
                "count_update": {"mode": count_mode[0], "recount_sweeps": count_mode[1],
                                 "timed_launches_recounted": n_rc,
                                 "model": "recount: the sampler writes z, k_recount rebuilds the "
                                          "shard's rows from a word-sorted token index; delta: "
                                          "device atomics per changed token"},
                "recount_ms_timed_region": recount_ms,
                "measured_copy_gbs": copy_gbs,
                # the bandwidth the kernel really moves (PMC bytes / its time)
                "traffic_gbs": (traffic_gb / (kern_ms * 1e-3)) if traffic_gb else None,
                "traffic_frac": (traffic_gb / (kern_ms * 1e-3) / HBM_PEAK_GBS) if traffic_gb else None,
                "traffic_unit": "GB per launch (rocprofv3 PMC, gfx950-corrected)",
                "traffic_source": rec_src,
                # SURVEY.md §8d's fixed contract B(K) = 4K + 16 (int32 rows), which
                # the kernel does not read (it reads the lossless 16-bit rows):
                # kept as an equivalent rate, not as a fraction of any peak
                "survey_contract": {
                    "bytes_per_token": bpt,
                    "gb_per_launch": n_local * bpt / 1e9,
                    "equivalent_gbs": n_local * bpt / (kern_ms * 1e-3) / 1e9,
                    "note": "SURVEY §8d's int32-row bytes at the measured launch time; the "
                            "kernel reads bytes_per_token above, so this rate is not a "
                            "bandwidth it moves",
                },
                "kernel": f"{kname}<C={sampler.Kp // 64}> avg {kern_ms:.3f} ms/launch over "
                          f"{n_local} tokens",
                "issue": issue_roofline(rec, tok_s_kernel),
                # what the kernel actually hits: the dense rows are
                # a random-row gather that the 256 MB Infinity Cache largely holds
                # (C4: 102 MB of 16-bit rows), so "hbm" names the memory path's
                # roofline, not HBM-resident bytes; the issue fraction is the other
                # ceiling the token's dependency chain runs into
                "ceiling": ("random-row gather of the word rows (Infinity-Cache resident when "
                            "they fit: 2 V Kp bytes <= 256 MB) + instruction issue / dependency "
                            "chain; see issue.frac" if args.sampler != "sparse" else
                            "streamed nonzero entries of long rows + scalar issue; see issue.frac"),
            },
            "collective": coll,
            "dropin_schedule": dropin,
            "ll_per_token": ll / tokens_all,
            "corpus_gen_s": t_gen,
        }
        if nnz0 is not None:
            result["roofline"]["mean_row_nnz"] = [nnz0, nnz1]
        if world == 1 and not args.no_estimate and args.config in ("c4", "c4shard", "c2") and not args.docs:
            result["estimate_side"] = estimate_side_figure(device, workload="c2" if args.config == "c2" else "c4")
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(corpus, K, alpha_sum, beta, args.cpu_budget)
        print(json.dumps(result), flush=True)
    sampler.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
