#!/usr/bin/env python3
"""Print the sampler kernel's counters from a tools/profile.sh summary dir."""
import glob, json, os, sys
d = sys.argv[1]
tok = float(sys.argv[2]) if len(sys.argv) > 2 else 2.5e8
ctr = {}
for f in glob.glob(os.path.join(d, "summary_*.json")):
    j = json.load(open(f))
    for k, v in j.get("counters", {}).items():
        if k.startswith("k_sample"):
            for c, x in v.items():
                if isinstance(x, dict):
                    ctr[(k, c)] = x["avg_per_dispatch"]
    for k, v in j.get("kernels", {}).items():
        if k.startswith("k_sample"):
            print("kernel", k, "avg ms %.3f" % (v["avg_ns"] / 1e6), "calls", v["calls"])
ks = sorted({k for k, _ in ctr})
for k in ks:
    g = lambda c: ctr.get((k, c))
    print("==", k)
    for (kk, c), v in sorted(ctr.items()):
        if kk == k:
            print("  %-40s %.4g   per token %.4g" % (c, v, v / tok))
    if g("FETCH_SIZE") and g("WRITE_SIZE"):
        print("  hbm bytes/launch (2*FETCH+WRITE)*1024 = %.4g GB; per token %.1f B" % (
            (2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024 / 1e9, (2 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024 / tok))
    if g("SQ_ACCUM_PREV_HIRES") and g("SQ_INSTS_VMEM_RD"):
        print("  avg VMEM latency ~ ACCUM_PREV_HIRES/INSTS_VMEM_RD = %.0f cycles" % (g("SQ_ACCUM_PREV_HIRES") / g("SQ_INSTS_VMEM_RD")))
    if g("SQ_WAVE_CYCLES"):
        w = g("SQ_WAVE_CYCLES")
        print("  wait_any %.2f wait_inst %.2f active %.2f valu_active %.2f" % (
            g("SQ_WAIT_ANY") / w, g("SQ_WAIT_INST_ANY") / w, g("SQ_ACTIVE_INST_ANY") / w, g("SQ_ACTIVE_INST_VALU") / w))
    if g("TCC_EA0_RDREQ_sum") and g("TCC_EA0_RDREQ_DRAM_sum"):
        print("  EA read reqs: dram fraction %.3f" % (g("TCC_EA0_RDREQ_DRAM_sum") / g("TCC_EA0_RDREQ_sum")))
    if g("TCC_HIT_sum"):
        print("  L2 hit rate %.3f" % (g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum"))))
    if g("TCC_EA0_RDREQ_LEVEL_sum") and g("TCC_EA0_RDREQ_sum"):
        print("  EA read latency ~ LEVEL/RDREQ = %.0f cycles" % (g("TCC_EA0_RDREQ_LEVEL_sum") / g("TCC_EA0_RDREQ_sum")))
