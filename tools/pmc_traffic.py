#!/usr/bin/env python3
"""Turn a rocprofv3 `--pmc FETCH_SIZE` counter CSV into the per-launch HBM
traffic JSON that bench.py reads for `roofline.traffic`.

    python tools/pmc_traffic.py <counter_collection.csv> <config> <kernel tag> <out.json>

FETCH_SIZE is reported in KiB; on gfx950 it counts exactly half of the bytes of
a wide (16 B/lane) coalesced streaming read (MI355X_MICROARCH.md, HBM
section), so bytes = FETCH_SIZE x 1024 x 2.  Averaged over every
pech_crc32c_main dispatch in the file.
"""
import csv
import json
import sys


def main():
    path, cfg, tag, out = sys.argv[1:5]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"] in ("pech_crc32c_main", "pech_crc32c_main_copy") and r["Counter_Name"] == "FETCH_SIZE"]
    if not vals:
        raise SystemExit("no pech_crc32c_main FETCH_SIZE rows")
    kib = sum(vals) / len(vals)
    res = {"config": cfg, "kernel": tag, "dispatches": len(vals), "fetch_size_kib_per_launch": round(kib, 1),
           "hbm_bytes_per_launch": int(kib * 1024 * 2),
           "correction": "x2: gfx950 FETCH_SIZE reports half of wide streaming-read bytes (MI355X_MICROARCH.md)",
           "source": path}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
