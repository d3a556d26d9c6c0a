#!/usr/bin/env python3
"""Turn rocprofv3 `--pmc FETCH_SIZE` (and optionally `--pmc WRITE_SIZE`)
counter CSVs into the per-launch HBM traffic JSON that bench.py reads for
`roofline.traffic`.

    python tools/pmc_traffic.py <fetch counter_collection.csv> <config> <kernel tag> <out.json> [<write csv>]

FETCH_SIZE/WRITE_SIZE are reported in KiB.  On gfx950 FETCH_SIZE counts
exactly half of the bytes of a wide (16 B/lane) coalesced streaming read, and
WRITE_SIZE reads the bytes exactly for 16-B-per-lane streaming stores
(MI355X_MICROARCH.md, HBM section): bytes = FETCH x 1024 x 2 + WRITE x 1024.
Averaged over every dispatch of the config's main kernel (main / main_copy / direct / flat / flatg; one of them per run).
"""
import csv
import json
import sys

KERNELS = ("pech_crc32c_main", "pech_crc32c_main_copy", "pech_crc32c_direct", "pech_crc32c_direct_copy", "pech_crc32c_flat",
           "pech_crc32c_flat_il", "pech_crc32c_flatg")


def per_launch_kib(path, counter):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Kernel_Name"] in KERNELS and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {KERNELS} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    path, cfg, tag, out = sys.argv[1:5]
    fetch, nd = per_launch_kib(path, "FETCH_SIZE")
    res = {"config": cfg, "kernel": tag, "dispatches": nd, "fetch_size_kib_per_launch": round(fetch, 1),
           "read_bytes_per_launch": int(fetch * 1024 * 2)}
    total = res["read_bytes_per_launch"]
    src = [path]
    if len(sys.argv) > 5:
        write, _ = per_launch_kib(sys.argv[5], "WRITE_SIZE")
        res["write_size_kib_per_launch"] = round(write, 1)
        res["write_bytes_per_launch"] = int(write * 1024)
        total += res["write_bytes_per_launch"]
        src.append(sys.argv[5])
    res["hbm_bytes_per_launch"] = total
    res["correction"] = "FETCH_SIZE x2 (gfx950 reports half of wide streaming-read bytes), WRITE_SIZE x1 " \
                        "(MI355X_MICROARCH.md)"
    res["source"] = src
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
