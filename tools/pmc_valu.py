"""VALU issue floor of a kernel from a rocprofv3 --pmc SQ_INSTS_VALU ... database.

usage: python tools/pmc_valu.py <results.db> <workload> <kernel_short> <steps_per_launch> <simds> [out.json]

SQ_INSTS_VALU counts wave-level vector instructions (per-SE values, summed here over the
SEs of a dispatch).  On gfx950 a wave issues one VALU instruction every 2 cycles
(MI355X_MICROARCH.md: 32 lanes/cycle), so the issue floor of a filter step is
    insts_per_step * 2 / simds / 2.4 GHz
with `simds` the SIMDs the launch occupies (k_resident: 4 per resident workgroup; k_step:
all 1024).  Transcendentals issue slower than that, so this is a lower bound on VALU time.
The largest dispatch of the kernel is taken (the timed launch of bench.py)."""
import collections
import json
import sqlite3
import sys

db, workload, kshort, steps, simds = sys.argv[1], sys.argv[2], sys.argv[3], float(sys.argv[4]), int(sys.argv[5])
out = sys.argv[6] if len(sys.argv) > 6 else None
c = sqlite3.connect(db)
rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                 "group by dispatch_id, counter_name").fetchall()
per = collections.defaultdict(dict)
names = {}
for d, k, cn, v in rows:
    if kshort in k:
        per[d][cn] = v
        names[d] = k
if not per:
    sys.exit(f"no dispatch of {kshort} in {db}")
disp = list(per)
if steps > 1:  # multi-step launch: the biggest one is the timed run
    disp = [max(per, key=lambda d: per[d].get("SQ_INSTS_VALU", 0.0))]
valu = sum(per[d]["SQ_INSTS_VALU"] for d in disp) / len(disp) / steps
salu = sum(per[d].get("SQ_INSTS_SALU", 0.0) for d in disp) / len(disp) / steps
lds = sum(per[d].get("SQ_INSTS_LDS", 0.0) for d in disp) / len(disp) / steps
floor_us = valu * 2.0 / simds / 2.4e9 * 1e6
res = {"workload": workload, "kernel": names[disp[0]], "kernel_short": kshort, "dispatches_used": len(disp),
       "steps_per_launch": steps, "valu_insts_per_step": valu, "salu_insts_per_step": salu,
       "lds_insts_per_step": lds, "simds": simds, "issue_floor_us_per_step": floor_us,
       "source": f"rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES "
                 f"({workload}); 2 cycles per wave VALU issue, 2.4 GHz"}
print(json.dumps(res, indent=1))
if out:
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
