"""Summarize a rocprofv3 profile directory (scripts/profile.sh output) into JSON.

    python scripts/pmc_summary.py gpurun_out/prof_TAG KERNEL_SUBSTR > profiles/...json

Per-dispatch counter values of the named kernel are summed over XCD/SE
instances, then averaged over dispatches.  HBM traffic follows the
MI355X_MICROARCH.md HBM section: FETCH_SIZE/WRITE_SIZE are KiB of L2<->fabric
traffic; gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, and
profiles/r02_calib/calib.json measured the same 0.5x for the 1-byte loads this
decoder issues (WRITE_SIZE exact for 1/8/16-byte stores), so the per-launch
figure is 2 x FETCH_SIZE + WRITE_SIZE; the raw read count is kept beside it.
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, kname = sys.argv[1], sys.argv[2]
    out = {"profile_dir": d, "kernel": kname, "counters": {}}
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "pmc_counter_collection.csv"))):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        per = collections.defaultdict(list)
        for (disp, c), v in agg.items():
            per[c].append(v)
        for c, v in per.items():
            out["counters"][c] = sum(v) / len(v)
    bs = os.path.join(d, "binary.sha256")
    if os.path.exists(bs):
        out["binary"] = "liblzmagpu.so sha256 " + open(bs).read().split()[0][:16]
    ks = os.path.join(d, "kt", "kt_kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            if kname in r["Name"]:
                out["kernel_avg_ns"] = float(r["AverageNs"])
                out["kernel_calls"] = int(r["Calls"])
    c = out["counters"]
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd, wr = c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        out["hbm_read_bytes_raw"] = rd
        out["hbm_read_bytes_x2"] = 2 * rd
        out["hbm_write_bytes"] = wr
        out["hbm_bytes_per_launch"] = 2 * rd + wr
        out["hbm_bytes_per_launch_raw"] = rd + wr
        if "kernel_avg_ns" in out:
            out["hbm_GBps"] = (2 * rd + wr) / out["kernel_avg_ns"]
    if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
        out["wait_any_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
        out["active_inst_frac"] = c.get("SQ_ACTIVE_INST_ANY", 0) / c["SQ_WAVE_CYCLES"]
    if "GRBM_GUI_ACTIVE" in c and "kernel_avg_ns" in out:
        out["effective_clock_GHz"] = c["GRBM_GUI_ACTIVE"] / 8 / out["kernel_avg_ns"]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
