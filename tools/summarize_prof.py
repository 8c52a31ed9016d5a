#!/usr/bin/env python3
"""Condense rocprofv3 CSV output into small per-kernel summaries.

  summarize_prof.py <prof_dir> <out.json> [skip_sweeps] [dispatches_per_sweep] [keep_sweeps]

skip_sweeps: leave out each kernel's dispatches of the first `skip_sweeps`
sweeps (in dispatch order), so that a profile of a bench command describes
the bench's own timed sweeps (skip_sweeps = --burnin + --warmup of that
command, tools/profile.sh).  dispatches_per_sweep (default 1): how many
launches of a kernel one sweep makes -- the sampler launches once per part
with --exchange-parts P (the skip had not been scaled, so split
profiles kept near-init launches).  The summary records both.
keep_sweeps (default 0 = all): keep only the next `keep_sweeps` sweeps'
dispatches after the skipped ones -- the bench's --steps -- so work the
bench command does after its timed region (the estimate() side figure) does
not enter the averages.  The sampler kernels (k_sample*) are counted as ONE
sequence in dispatch order, whatever their template arguments: the large-K
sampler switches between two instantiations (ring depths) from sweep to
sweep, and a per-name count would skip the wrong sweeps.

Reads every *_kernel_stats.csv, *_kernel_trace.csv and
*_counter_collection.csv under prof_dir and writes, per kernel name:
  - dispatch count, average / min / max duration (kernel trace),
  - per counter: number of dispatches and the average value per dispatch.
HBM traffic per dispatch (MI355X_MICROARCH.md §HBM, gfx950 corrections):
  FETCH_SIZE and WRITE_SIZE are in KiB; FETCH_SIZE reads half the bytes of a
  16 B/lane coalesced stream, so hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024
  for kernels whose reads are 16 B/lane (the sampler's row gather).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.strip('"')
    if "k_sample" in name:
        # keep the template arguments
        i = name.find("k_sample")
        return name[i:].split("(")[0]
    for key in ("k_apply", "k_prepare_topics", "k_count", "k_init_z", "k_doc_topics",
                "k_ll_docs", "k_ll_words", "k_infer_init"):
        if key in name:
            return key
    return name.split("(")[0][:80]


def window(items, skip, keep):
    """items: (order key, name, value); the kept (name, value) pairs: per
    name, the dispatches past the first `skip` (and at most `keep`, 0 = all);
    the sampler kernels form one sequence.  A name with nothing left keeps
    all its dispatches (a kernel that runs only before the window)."""
    out = defaultdict(list)
    samp = sorted((o, n, v) for o, n, v in items if n.startswith("k_sample"))
    rest = defaultdict(list)
    for o, n, v in items:
        if not n.startswith("k_sample"):
            rest[n].append((o, v))
    end = skip + keep if keep else None
    sel = samp[skip:end]
    for _, n, v in sel:
        out[n].append(v)
    for n in {n for _, n, _ in samp} - set(out):
        out[n] = [v for o, nn, v in samp if nn == n]
    for n, vs in rest.items():
        vs = [v for _, v in sorted(vs)]
        out[n] = vs[skip:end] or vs
    return out


def main(prof_dir, out_path, skip=0, per_sweep=1, keep=0):
    skip_sweeps, per_sweep, keep_sweeps = int(skip), max(1, int(per_sweep)), int(keep)
    skip, keep = skip_sweeps * per_sweep, keep_sweeps * per_sweep
    out = {"kernels": {}, "counters": {}, "skipped_sweeps": skip_sweeps,
           "dispatches_per_sweep": per_sweep, "skipped_dispatches_per_kernel": skip,
           "kept_sweeps": keep_sweeps}
    for path in glob.glob(os.path.join(prof_dir, "**", "*_kernel_trace.csv"), recursive=True):
        items = []
        with open(path) as f:
            for row in csv.DictReader(f):
                dur = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
                items.append((int(row["Start_Timestamp"]), short(row["Kernel_Name"]), dur))
        for k, v in window(items, skip, keep).items():
            v.sort()
            out["kernels"][k] = {
                "calls": len(v),
                "avg_ns": sum(v) / len(v),
                "min_ns": v[0],
                "max_ns": v[-1],
                "median_ns": v[len(v) // 2],
            }
    for path in glob.glob(os.path.join(prof_dir, "**", "*_kernel_stats.csv"), recursive=True):
        with open(path) as f:
            out["kernel_stats_csv"] = list(csv.DictReader(f))[:40]
    for path in glob.glob(os.path.join(prof_dir, "**", "*_counter_collection.csv"), recursive=True):
        agg = defaultdict(lambda: defaultdict(list))
        with open(path) as f:
            for row in csv.DictReader(f):
                agg[short(row["Kernel_Name"])][row["Counter_Name"]].append(
                    (int(row.get("Dispatch_Id", 0) or 0), float(row["Counter_Value"])))
        by_counter = defaultdict(list)
        for k, ctrs in agg.items():
            for c, vals in ctrs.items():
                per_dispatch = defaultdict(float)
                for disp, v in vals:
                    per_dispatch[disp] += v
                by_counter[c] += [(i, k, x) for i, x in per_dispatch.items()]
        for c, items in by_counter.items():
            for k, xs in window(items, skip, keep).items():
                d = out["counters"].setdefault(k, {})
                d[c] = {"dispatches": len(xs), "avg_per_dispatch": sum(xs) / len(xs),
                        "min": min(xs), "max": max(xs)}
    for k, ctrs in out["counters"].items():
        if "FETCH_SIZE" in ctrs and "WRITE_SIZE" in ctrs:
            ctrs["hbm_bytes_per_dispatch_corrected"] = (
                2 * ctrs["FETCH_SIZE"]["avg_per_dispatch"] + ctrs["WRITE_SIZE"]["avg_per_dispatch"]) * 1024
            ctrs["hbm_bytes_per_dispatch_raw"] = (
                ctrs["FETCH_SIZE"]["avg_per_dispatch"] + ctrs["WRITE_SIZE"]["avg_per_dispatch"]) * 1024
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:6])
