#!/usr/bin/env python3
"""Shrink rocprofv3 outputs under a directory after their summaries are
taken (gpurun copies back at most 64 MiB of gpurun_out/): counter-collection
CSVs keep the header and the first dispatches of each pech kernel, kernel
traces are dropped (the stats CSV beside them stays)."""
import csv
import os
import sys


def trim(path, keep=40):
    rows = list(csv.reader(open(path)))
    if not rows:
        return
    hdr, body = rows[0], rows[1:]
    ki = hdr.index("Kernel_Name") if "Kernel_Name" in hdr else None
    seen, out = {}, []
    for r in body:
        name = r[ki] if ki is not None else ""
        if name.startswith("pech_crc32c") and seen.get(name, 0) < keep:
            seen[name] = seen.get(name, 0) + 1
            out.append(r)
    w = csv.writer(open(path, "w", newline=""))
    w.writerow(hdr)
    w.writerows(out)


for root in sys.argv[1:]:
    for d, _, files in os.walk(root):
        for f in files:
            p = os.path.join(d, f)
            if f.endswith("counter_collection.csv"):
                trim(p)
            elif f.endswith("kernel_trace.csv"):
                os.remove(p)
