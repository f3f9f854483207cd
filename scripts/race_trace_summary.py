"""Summarize a scripts/race_trace.py run under rocprofv3 --kernel-trace: per block of calls (replicas 1/8/1/8/2/4), the
host-side latency and the n = 1 path's kernel durations (the prep and whichever check ran: octet or sixteen-lane).
Usage: python scripts/race_trace_summary.py <trace dir with host.jsonl and run_kernel_trace.csv> <out.json> <note>"""
import csv
import json
import statistics
import sys


def main(d, out, note):
    host = [json.loads(line) for line in open(d + "/host.jsonl")]
    rows = sorted(csv.DictReader(open(d + "/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))

    def durs(tag):
        return [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if tag in r["Kernel_Name"]]

    prep = durs("k_verify_prep8")
    check = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows
             if "k_verify_pair_lq8" in r["Kernel_Name"] or "k_verify_pair_lq16" in r["Kernel_Name"]]
    names = sorted({r["Kernel_Name"].split("(")[0].split("::")[-1] for r in rows if "k_verify_pair_lq" in r["Kernel_Name"]})
    k = sum(b["calls"] for b in host)
    off_c, off_p = len(check) - k, len(prep) - k
    at = 0
    for b in host:
        c = check[off_c + at:off_c + at + b["calls"]]
        p = prep[off_p + at:off_p + at + b["calls"]]
        at += b["calls"]
        b["kernel_trace"] = {"check_p50_ms": round(statistics.median(c), 3), "check_min_ms": round(min(c), 3),
                             "check_max_ms": round(max(c), 3), "prep_p50_ms": round(statistics.median(p), 3),
                             "prep_min_ms": round(min(p), 3), "prep_max_ms": round(max(p), 3)}
        print(b["replicas"], b["p50_ms"], b["kernel_trace"])
    json.dump({"what": note, "check_kernels": names, "blocks": host}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
