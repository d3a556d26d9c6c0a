#!/usr/bin/env python3
"""Per-dispatch averages of rocprofv3 counter CSVs for pech_crc32c_main, and
the derived busy fractions (SQ counters are summed over the chip; cycles
per SQ: GRBM_GUI_ACTIVE / 8 XCDs, per MI355X_MICROARCH.md)."""
import csv
import json
import os
import sys
from collections import defaultdict


def main():
    acc = defaultdict(list)
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            if r["Kernel_Name"] == os.environ.get("PECH_PMC_KERNEL", "pech_crc32c_main"):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    out = {"per_dispatch": {k: round(v, 1) for k, v in sorted(avg.items())}}
    g = avg.get("GRBM_GUI_ACTIVE")
    if g:
        cyc = g / 8.0  # per XCD
        out["gpu_cycles_per_xcd"] = round(cyc)
        cus = 256
        for name in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_BUSY_CYCLES"):
            if name in avg:
                out[name + "_per_cu_cycle"] = round(avg[name] / (cyc * cus), 4)
    if "SQ_LDS_BANK_CONFLICT" in avg and "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"]:
        out["lds_bank_conflict_frac"] = round(avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"], 4)
    if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
        out["wait_inst_frac_of_wave_cycles"] = round(avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"], 4)
        out["wait_any_frac_of_wave_cycles"] = round(avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
