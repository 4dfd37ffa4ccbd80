"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV (one step
starts at each k_plan): start, duration and gap of every dispatch."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_plan" in r["Kernel_Name"]]
for s, e in zip(idx[-3:-1], idx[-2:]):
    t0, prev = int(rows[s]["Start_Timestamp"]), None
    for r in rows[s:e + 1]:
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print("%-44s start %8.2f dur %8.2f gap %6.2f" % (r["Kernel_Name"][:44], (a - t0) / 1e3, (b - a) / 1e3,
                                                        (a - prev) / 1e3 if prev else 0))
        prev = b
    print()
