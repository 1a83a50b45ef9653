"""Summarise scripts/traffic_calib.sh: counter bytes / true bytes per access shape.

    python scripts/traffic_calib.py gpurun_out/calib > profiles/r02_calib/calib.json
"""
import collections
import csv
import glob
import json
import os
import sys

BYTES = 4096 * 32 * 256 * 8  # kW x lanes x groups (traffic_calib.hip)


def counter(d, name):
    f = glob.glob(os.path.join(d, "**", "pmc_counter_collection.csv"), recursive=True)
    if not f:
        return None
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == name:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = sorted(per.items(), key=lambda kv: int(kv[0]))[2:]  # skip the 2 warm-up launches
    return sum(x for _, x in v) / len(v) * 1024 if v else None  # KiB -> bytes


def main():
    root = sys.argv[1]
    out = {"true_bytes_per_launch": BYTES, "shapes": {}}
    for k in ("st1", "st8u", "st16", "ld1", "ld16"):
        fs = counter(os.path.join(root, f"{k}_FETCH_SIZE"), "FETCH_SIZE")
        ws = counter(os.path.join(root, f"{k}_WRITE_SIZE"), "WRITE_SIZE")
        ns = None
        for f in glob.glob(os.path.join(root, f"{k}_kt", "**", "kt_kernel_stats.csv"),
                           recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Name"].startswith(k):
                    ns = float(r["AverageNs"])
        out["shapes"][k] = {"FETCH_SIZE_bytes": fs, "WRITE_SIZE_bytes": ws,
                            "fetch_per_true_byte": fs / BYTES if fs is not None else None,
                            "write_per_true_byte": ws / BYTES if ws is not None else None,
                            "kernel_avg_ns": ns,
                            "GBps_true": BYTES / ns if ns else None}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
