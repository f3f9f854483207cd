"""Summarize the PMC passes of scripts/gpu_pmc.sh for one kernel into profiles/<round>_pmc_<kernel>.json.

HBM traffic per launch = FETCH_SIZE + WRITE_SIZE (rocprofv3 derived counters, KiB).  Per
/opt/skills/guides/MI355X_MICROARCH.md (HBM section) FETCH_SIZE counts 64 B per 128-B request of
wide coalesced reads (x2 correction) and is uncalibrated for other widths; this kernel's traffic is
scratch (spill) traffic of 4-byte-per-lane accesses, so the raw value is reported next to the x2
figure and bench.py uses the raw (lower) one.
"""
import csv
import glob
import json
import os
import sys


def main(pmc_dir, kernel, out_path, note, items=65536, bytes_per_item=188):
    vals = {}
    for f in sorted(glob.glob(os.path.join(pmc_dir, "*.csv")) + glob.glob(os.path.join(pmc_dir, "p*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    waves = avg.get("SQ_WAVES", 0)
    out = {"kernel": kernel, "note": note, "counters_per_launch": avg}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        out["hbm_bytes_per_launch_raw"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        out["hbm_bytes_per_launch_fetch_x2"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        # algorithmic input per launch: pk 48 + sig 96 + root 32 + offset 8 + status 4 = 188 B per item
        out["traffic_ratio"] = out["hbm_bytes_per_launch_raw"] / (items * bytes_per_item)
    if waves:
        out["valu_insts_per_wave"] = avg.get("SQ_INSTS_VALU", 0) / waves
        cyc = max(avg.get("SQ_WAVE_CYCLES", 1), 1)
        out["wait_any_frac"] = avg.get("SQ_WAIT_ANY", 0) / cyc
        # fraction of resident-wave cycles with a VALU instruction in flight; one wave per SIMD here, so this is
        # the SIMD's VALU busy fraction (SQ_ACTIVE_INST_VALU and SQ_WAVE_CYCLES are both per-wave sums)
        out["valu_util"] = avg.get("SQ_ACTIVE_INST_VALU", 0) / cyc
    json.dump(out, open(out_path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else "",
         int(sys.argv[5]) if len(sys.argv) > 5 else 65536)
