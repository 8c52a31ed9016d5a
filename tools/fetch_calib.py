#!/usr/bin/env python3
"""Join tools/bin/fetch_calib's known byte counts with the rocprofv3
FETCH_SIZE / WRITE_SIZE summaries of the same program (tools/gpu_calib.sh):

  fetch_calib.py <known.json> <summary_fetch.json> <summary_write.json> <out.json>

For each pattern: FETCH_SIZE bytes (KiB * 1024, one dispatch) over the bytes
the kernel reads, and WRITE_SIZE bytes over the bytes it writes.  The ratio
is the factor make_traffic.py divides by for a kernel with that access
pattern (MI355X_MICROARCH.md §HBM: other access widths are uncalibrated)."""
import json
import sys


def main(known_p, fetch_p, write_p, out_p):
    known = json.loads(open(known_p).read().strip().splitlines()[-1])
    fe = json.load(open(fetch_p))["counters"]
    wr = json.load(open(write_p))["counters"]
    out = {}
    for k, kb in known.items():
        f = fe.get(k, {}).get("FETCH_SIZE", {}).get("avg_per_dispatch")
        w = wr.get(k, {}).get("WRITE_SIZE", {}).get("avg_per_dispatch")
        rec = {"known": kb, "fetch_bytes": f * 1024 if f is not None else None,
               "write_bytes": w * 1024 if w is not None else None}
        # random patterns: every request counts (a line requested twice over a
        # 4 GiB buffer has long left L2 and the 256 MiB Infinity Cache, so it
        # is fetched again); read_distinct_expected is kept for reference
        rd = kb.get("read") or kb.get("read_requested")
        if rd and f is not None:
            rec["fetch_over_read"] = f * 1024 / rd
        if kb.get("write") and w is not None:
            rec["write_over_written"] = w * 1024 / kb["write"]
        if kb.get("atomics") and f is not None and w is not None:
            rec["fetch_bytes_per_atomic"] = f * 1024 / kb["atomics"]
            rec["write_bytes_per_atomic"] = w * 1024 / kb["atomics"]
        out[k] = rec
    with open(out_p, "w") as fo:
        json.dump(out, fo, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
