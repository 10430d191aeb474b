"""Fold the PMC passes of tools/gpu_pmc_all.sh / gpu_pmc.sh into profiles/pmc_*.json (read by bench.py)
and copy the raw counter files under profiles/<round>/pmc/.

    python tools/pmc_fold.py gpurun_out/<pmc dir> <round, e.g. r05> [name=K,W ...]

(name=K,W overrides the bench line's timed steps K and warm-up W the profiled run used.)

Per workload: FETCH_SIZE / WRITE_SIZE per launch of the bench line's dominant kernel (separate
passes, tools/pmc_summary.py: KiB -> B, FETCH doubled on gfx950), summed over its launches and
divided by the filter steps the profiled bench run covers (STEPS below); the SQ issue counters
through tools/pmc_valu.py."""
import csv
import glob
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
D = sys.argv[1]
RND = sys.argv[2] if len(sys.argv) > 2 else "r05"
OUT = os.path.join(REPO, "profiles", RND, "pmc")
os.makedirs(OUT, exist_ok=True)

# filter steps the profiled bench run covers: the warm-up W and the timed K, plus (nx > 4 with the
# covariance) a second K-step window for the step kernels' own time, or (LEDH) a second W + K run
STEPS = {"l96": lambda K, W: W + 2 * K, "mat": lambda K, W: W + 2 * K, "ledh": lambda K, W: 2 * (W + K),
         "ledh_mat": lambda K, W: 2 * (W + K)}
# name: (bench steps K, warm-up W, kernel substring, kernel_short, steps per launch for pmc_valu, SIMDs)
LINES = {
    "sv": (20, 5, "k_resident<float, 1, 1", "k_resident", 20, None),
    "sv64": (20, 3, "k_step_stream<1, 0, 0>", "k_step_stream", 1, 1024),
    "sv_fp64": (20, 5, "k_step<double, 1, 1", "k_step", 1, 1024),
    "l96": (50, 5, "k_step_grp<float, 40, 10", "k_step_grp", 1, 1024),
    "mat": (40, 4, "k_step_grp<float, 16, 25", "k_step_grp", 1, 1024),
    "ledh": (200, 20, "k_ledh_fused", "k_ledh_fused", 1, 628),  # 157 one-wave-per-SIMD workgroups
    "ledh_mat": (10, 2, "k_flow_wave_lr", "k_flow_wave_lr", 1, 500),  # one 64-lane workgroup per particle
}
for arg in sys.argv[3:]:  # name=K,W
    nm, kw = arg.split("=")
    k_, w_ = (int(v) for v in kw.split(","))
    LINES[nm] = (k_, w_) + LINES[nm][2:]
OUTNAME = {"sv": "pmc_traffic.json"}


def first(pattern):
    g = sorted(glob.glob(pattern, recursive=True))
    return g[0] if g else None


def launches(path, counter, kern):
    return sum(1 for r in csv.DictReader(open(path)) if kern in r["Kernel_Name"] and r["Counter_Name"] == counter)


for name, (K, W, kern, short, spl, simds) in LINES.items():
    fcsv = first(f"{D}/{name}_FETCH_SIZE/**/*counter_collection.csv")
    wcsv = first(f"{D}/{name}_WRITE_SIZE/**/*counter_collection.csv")
    if not (fcsv and wcsv):
        print(f"{name}: no traffic passes under {D}")
        continue
    dst_f = os.path.join(OUT, f"{name}_FETCH_SIZE_counter_collection.csv")
    dst_w = os.path.join(OUT, f"{name}_WRITE_SIZE_counter_collection.csv")
    shutil.copy(fcsv, dst_f)
    shutil.copy(wcsv, dst_w)
    n = launches(dst_f, "FETCH_SIZE", kern)
    steps = STEPS.get(name, lambda K, W: W + K)(K, W)
    print(f"{name}: {n} launches of {kern}, {steps} filter steps")
    rel_f, rel_w = os.path.relpath(dst_f, REPO), os.path.relpath(dst_w, REPO)
    out = os.path.join(REPO, "profiles", OUTNAME.get(name, f"pmc_traffic_{name}.json"))
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_summary.py"), rel_f, rel_w, kern, str(steps), out,
                    short], check=True, cwd=REPO, stdout=subprocess.DEVNULL)
    db = first(f"{D}/{name}_issue/**/*results.db")
    if db:
        # per-dispatch counter sums exported as CSV (the rocpd database itself is ~5 MB)
        import sqlite3
        c = sqlite3.connect(db)
        rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value) from counters_collection "
                         "group by dispatch_id, counter_name order by dispatch_id").fetchall()
        dst_csv = os.path.join(OUT, f"{name}_issue_counters.csv")
        with open(dst_csv, "w", newline="") as fh:
            wr = csv.writer(fh)
            wr.writerow(["dispatch_id", "kernel_name", "counter_name", "value"])
            wr.writerows(rows)
        # the resident kernel occupies 4 SIMDs per workgroup of its grid: pmc_valu takes the grid's SIMDs
        sim = simds if simds else int(os.environ.get("PF_RES_SIMDS", "980"))
        outj = os.path.join(REPO, "profiles", f"pmc_valu_{name}.json")
        subprocess.run([sys.executable, os.path.join(REPO, "tools", "pmc_valu.py"), db, name, short, str(spl), str(sim),
                        outj], check=True, cwd=REPO, stdout=subprocess.DEVNULL)
        import json
        d = json.load(open(outj))
        d["source"] = (f"rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES "
                       f"({name}); 2 cycles per wave VALU issue, 2.4 GHz; per-dispatch sums in "
                       f"{os.path.relpath(dst_csv, REPO)} (tools/gpu_pmc_all.sh, tools/pmc_fold.py)")
        json.dump(d, open(outj, "w"), indent=1)
    st = first(f"{D}/{name}_stats/**/*results.db")
    if st:  # rocprofv3 --kernel-trace --stats of the same line: per-kernel statistics (tools/rocpd_stats.py)
        subprocess.run([sys.executable, os.path.join(REPO, "tools", "rocpd_stats.py"), st,
                        os.path.join(OUT, f"{name}_kernel_stats.csv")], check=True, cwd=REPO, stdout=subprocess.DEVNULL)
print(f"folded into profiles/pmc_*.json; raw files under profiles/{RND}/pmc/")
