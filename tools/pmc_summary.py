"""Fold rocprofv3 PMC passes into profiles/pmc_traffic*.json (read by bench.py).

    python tools/pmc_summary.py FETCH_CSV WRITE_CSV KERNEL_SUBSTR TOTAL_STEPS OUT [KERNEL_SHORT]

FETCH_SIZE / WRITE_SIZE come from separate passes (they do not fit one TCC pass on
gfx950); both are reported in KiB.  Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE
under-reports wide coalesced streaming reads by exactly 2x on gfx950, so it is doubled;
WRITE_SIZE is exact for 16-B/lane streaming stores.  TOTAL_STEPS = the filter steps all
profiled launches of the kernel cover together (warm-up + timed run of bench.py), so
bytes_per_step = sum over those launches / TOTAL_STEPS (for the resident kernel this
includes each launch's entry / exit state traffic).
"""
import csv
import json
import sys

import numpy as np


def per_launch(path, counter, kern):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
         if kern in r["Kernel_Name"] and r["Counter_Name"] == counter]
    if not v:
        raise SystemExit(f"no {counter} rows for kernel '{kern}' in {path}")
    return np.array(v) * 1024.0  # KiB -> bytes


def main():
    fetch_csv, write_csv, kern = sys.argv[1], sys.argv[2], sys.argv[3]
    steps = float(sys.argv[4])
    out = sys.argv[5]
    short = sys.argv[6] if len(sys.argv) > 6 else ("k_resident" if "k_resident" in kern else "k_step")
    f = per_launch(fetch_csv, "FETCH_SIZE", kern)
    w = per_launch(write_csv, "WRITE_SIZE", kern)
    tot = float(2 * f.sum() + w.sum())
    d = {
        "kernel": kern,
        "kernel_short": short,
        "launches": [int(f.size), int(w.size)],
        "total_steps": steps,
        "fetch_bytes_raw_total": float(f.sum()),
        "fetch_bytes_total_x2": float(2 * f.sum()),
        "write_bytes_total": float(w.sum()),
        "bytes_per_step": tot / steps,
        "source": f"rocprofv3 --pmc FETCH_SIZE ({fetch_csv}) and --pmc WRITE_SIZE ({write_csv}); "
                  "KiB->B, FETCH doubled per the gfx950 rule; summed over the kernel's launches / filter steps",
    }
    with open(out, "w") as fh:
        json.dump(d, fh, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
