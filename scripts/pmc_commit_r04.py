"""Condense the round-4 PMC passes (gpurun_out/pmc_<wl>/summary.json, scripts/gpu_pmc_r04.sh) into the committed
profiles: profiles/r04/pmc_<wl>.json (per kernel: VALU and integer-VALU instructions per wave, VALU utilisation,
wait fraction, HBM bytes per launch, L2 hit rate) and profiles/r04/pmc_verify.json (k_verify_fused in the form
bench.py's roofline reads, with the commit the counters were taken at).

Run:  python3 scripts/pmc_commit_r04.py <git rev of the profiled build> [round dir, default r04] [input prefix, default
      pmc_ (gpurun_out/pmc_<wl>); round 5: r05 pmc5_ (scripts/gpu_pmc_r05.sh)]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = ("valu_insts_per_wave", "sq_insts_valu_int64_per_wave", "sq_insts_valu_int32_per_wave",
        "sq_insts_lds_per_wave", "sq_insts_salu_per_wave", "valu_util", "wait_any_frac", "hbm_bytes_per_launch_raw",
        "hbm_bytes_per_launch_fetch_x2", "l2_hit_rate", "duration_ms_profiled", "effective_clock_ghz",
        "launches_seen")
C2_ITEMS = 65536  # scripts/gpu_pmc_r04.sh WL=c2: the default bench, 65,536 Verify per launch
IN_BYTES_PER_VERIFY = 188  # pk 48 + sig 96 + message 32 + offsets 8 + status 4


def main(rev, rnd="r04", prefix="pmc_"):
    os.makedirs(os.path.join(ROOT, "profiles", rnd), exist_ok=True)
    for wl in ("c2", "c3", "c4"):
        src = os.path.join(ROOT, "gpurun_out", prefix + wl, "summary.json")
        if not os.path.exists(src):
            continue
        d = json.load(open(src))
        script = {"r04": "scripts/gpu_pmc_r04.sh", "r05": "scripts/gpu_pmc_r05.sh"}.get(rnd, "scripts/gpu_pmc.sh")
        out = {"taken_at": rev, "workload": wl, "source": "%s WL=%s" % (script, wl), "kernels": {}}
        for k, v in sorted(d.items()):
            if isinstance(v, dict) and v.get("valu_insts_per_wave"):
                out["kernels"][k] = {kk: (round(v[kk], 4) if isinstance(v.get(kk), float) else v.get(kk))
                                     for kk in KEYS if kk in v}
        with open(os.path.join(ROOT, "profiles", rnd, "pmc_%s.json" % wl), "w") as f:
            json.dump(out, f, indent=1)
        if wl == "c2" and "k_verify_fused" in d:
            v = d["k_verify_fused"]
            hbm = v.get("hbm_bytes_per_launch_raw")
            ver = {"kernel": "k_verify_fused", "taken_at": rev,
                   "note": "rocprofv3 --pmc passes over the default bench's C2 step at this commit "
                           "(%s WL=c2); FETCH_SIZE + WRITE_SIZE in KiB x 1024" % script,
                   "counters_per_launch": v.get("counters_per_launch"),
                   "hbm_bytes_per_launch_raw": hbm,
                   "hbm_bytes_per_launch_fetch_x2": v.get("hbm_bytes_per_launch_fetch_x2"),
                   "traffic_ratio": hbm / (C2_ITEMS * IN_BYTES_PER_VERIFY) if hbm else None,
                   "valu_insts_per_wave": v.get("valu_insts_per_wave"),
                   "int64_valu_insts_per_wave": v.get("sq_insts_valu_int64_per_wave"),
                   "int32_valu_insts_per_wave": v.get("sq_insts_valu_int32_per_wave"),
                   "wait_any_frac": v.get("wait_any_frac"), "valu_util": v.get("valu_util")}
            with open(os.path.join(ROOT, "profiles", rnd, "pmc_verify.json"), "w") as f:
                json.dump(ver, f, indent=1)
        print("wrote profiles/%s/pmc_%s.json (%d kernels)" % (rnd, wl, len(out["kernels"])))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "unknown", *(sys.argv[2:4]))
