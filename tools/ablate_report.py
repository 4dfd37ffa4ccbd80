"""Summarise tools/traffic_ablate.sh output: PMC calibration factors and the
per-variant k_fill FETCH_SIZE / WRITE_SIZE (KB per dispatch) and durations.
usage: python tools/ablate_report.py gpurun_out/TAG > profiles/...json"""
import csv
import glob
import json
import os
import sys


def counters(d, counter, ksub):
    vals = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and ksub in r["Kernel_Name"]:
                key = r.get("Dispatch_Id") or r.get("Correlation_Id")
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals, key=lambda x: int(x))]


def kernel_ms(d, ksub):
    for f in glob.glob(os.path.join(d, "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if ksub in r["Name"]:
                return float(r["AverageNs"]) / 1e6
    return None


def main():
    base = sys.argv[1]
    out = {"calibration": {}, "variants": {}}
    # pmc_calib: one dispatch per pattern, in pattern order; bytes are 1 GiB except pattern 3 (256 MiB)
    truth = [2 ** 30, 2 ** 30, 2 ** 30, 2 ** 28, 2 ** 30, 2 ** 30]
    names = ["dword_store_256B_rows", "byte_store_64B_rows", "dword_load_all_lanes",
             "dword_load_one_lane_in_four", "vec16_store", "vec16_load"]
    f = counters(os.path.join(base, "calib_FETCH_SIZE"), "FETCH_SIZE", "k_")
    w = counters(os.path.join(base, "calib_WRITE_SIZE"), "WRITE_SIZE", "k_")
    for i, nm in enumerate(names):
        out["calibration"][nm] = {"bytes": truth[i], "fetch_size_bytes": f[i] * 1024 if i < len(f) else None,
                                  "write_size_bytes": w[i] * 1024 if i < len(w) else None}
    for v in ("default", "nomatch", "notrace", "nostore"):
        fe = counters(os.path.join(base, v + "_FETCH_SIZE"), "FETCH_SIZE", "k_fill")
        wr = counters(os.path.join(base, v + "_WRITE_SIZE"), "WRITE_SIZE", "k_fill")
        out["variants"][v] = {"fetch_size_kb": sum(fe) / len(fe) if fe else None,
                              "write_size_kb": sum(wr) / len(wr) if wr else None,
                              "k_fill_ms": kernel_ms(os.path.join(base, v + "_trace"), "k_fill")}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
