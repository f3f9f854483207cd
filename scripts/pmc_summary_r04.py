"""Per-kernel summary of one workload's rocprofv3 --pmc passes (scripts/gpu_pmc_r04.sh): averages per launch and the
derived figures the roofline uses.

* VALU instructions per wave (SQ_INSTS_VALU / SQ_WAVES) and, when the box lists them, the integer-VALU counts
  (SQ_INSTS_VALU_INT32 / _INT64) per wave: the measured multiply-add stream beside the algorithmic unit;
* valu_util = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (one wave per SIMD: the SIMD's VALU busy fraction);
* wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on memory: here scratch);
* HBM-side bytes per launch = FETCH_SIZE + WRITE_SIZE (KiB counters; MI355X_MICROARCH.md: FETCH_SIZE reads half the
  bytes of wide streaming reads, uncalibrated for this kernel's 16-B scratch accesses, so raw and x2 are both given);
* effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (the counter run's own timestamps; profiled runs clock
  lower than unprofiled ones, MI355X_MICROARCH.md DVFS note).
"""
import csv
import glob
import json
import os
import sys


def main(pmc_dir):
    per = {}
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].strip()
            per.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                per[k].setdefault("_duration_ns", []).append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
                per[k].setdefault("_scratch_B", []).append(float(r["Scratch_Size"]))
    out = {}
    for k, vals in per.items():
        avg = {c: sum(v) / len(v) for c, v in vals.items()}
        d = {"launches_seen": max(len(v) for v in vals.values()), "counters_per_launch": avg}
        waves = avg.get("SQ_WAVES", 0)
        if waves:
            d["valu_insts_per_wave"] = avg.get("SQ_INSTS_VALU", 0) / waves if "SQ_INSTS_VALU" in avg else None
            for c in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if c in avg:
                    d[c.lower() + "_per_wave"] = avg[c] / waves
        cyc = avg.get("SQ_WAVE_CYCLES")
        if cyc:
            d["valu_util"] = avg.get("SQ_ACTIVE_INST_VALU", 0) / cyc if "SQ_ACTIVE_INST_VALU" in avg else None
            d["wait_any_frac"] = avg.get("SQ_WAIT_ANY", 0) / cyc if "SQ_WAIT_ANY" in avg else None
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            d["hbm_bytes_per_launch_raw"] = (avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
            d["hbm_bytes_per_launch_fetch_x2"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
        if "_duration_ns" in avg and avg["_duration_ns"] > 0 and "GRBM_GUI_ACTIVE" in avg:
            d["duration_ms_profiled"] = avg["_duration_ns"] / 1e6
            d["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / avg["_duration_ns"]
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg and avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"] > 0:
            d["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        out[k] = d
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
