"""Print the headline fields of a bench.py JSON line (scripts/gpu.sh)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print("C2 %.0f/s frac %s kernel %s ms  build %s" % (d["value"], r.get("frac"), r.get("kernel_avg_ms"),
                                                  (d.get("build_src_sha") or "")[:16]))
if d.get("threshold_aggregates_per_s"):
    print("C3 %s one call, %s two streams" % (d["threshold_aggregates_per_s"],
                                             d.get("threshold_aggregates_per_s_two_streams")))
if d.get("drop_in_latency"):
    lat = d["drop_in_latency"]
    print("n=1 p50 %s ms p90 %s ms" % (lat.get("p50_ms"), lat.get("p90_ms")))
if d.get("full_slot_mix"):
    c5 = d["full_slot_mix"]
    print("C5 %s ms/slot  failed-batch-check %s  amortized %s  table %s" % (
        c5.get("ms_per_slot"), c5.get("failed_batch_check_ms_per_slot"), c5.get("auto_mode_amortized_ms_per_slot"),
        c5.get("ms_per_slot_pubshare_table")))
for k, v in (d.get("rlc_batch_verify") or {}).items():
    if isinstance(v, dict) and "ms_per_batch" in v:
        print("RLC %s %s ms  fallback items %s  windows failed %s  kernels %s  table %s/s" % (
            k, v.get("ms_per_batch"), v.get("items_fallback"), v.get("windows_failed"), v.get("kernel_avg_ms"),
            v.get("verified_partial_sigs_per_s_pubshare_table")))
if d.get("cpu_baseline"):
    print("cpu", d["cpu_baseline"])
