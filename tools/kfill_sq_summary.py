"""k_fill's SQ counters on the headline batch (tools/pmc_kfill.sh: passes kf1 and kf2
of `bench.py --steps 3 --warmup 1`), summed per dispatch and averaged over the
k_fill dispatches, with VALU lane-instructions per in-band cell.
usage: python tools/kfill_sq_summary.py gpurun_out/TAG [OUT.json]"""
import collections
import csv
import glob
import json
import os
import sys

IN_BAND_CELLS_C3 = 4333039596  # in-band cells of the C3 batch (bench.py c3 workload)


def main():
    d = sys.argv[1]
    tot = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for sub in ("kf1", "kf2"):
        for f in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "k_fill" not in r["Kernel_Name"]:
                    continue
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((sub, r["Dispatch_Id"]))
    per = {k: int(round(v / len(disp[k]))) for k, v in sorted(tot.items())}
    out = {
        "kernel": "k_fill",
        "workload": "C3 (1M x 150 bp, band 31), one launch",
        "dispatches": max(len(s) for s in disp.values()) if disp else 0,
        "counters_per_launch": per,
        "in_band_cells_per_launch": IN_BAND_CELLS_C3,
        "valu_lane_instructions_per_in_band_cell": round(per.get("SQ_INSTS_VALU", 0) * 64 / IN_BAND_CELLS_C3, 2),
        "wait_any_per_wave_cycle": round(per.get("SQ_WAIT_ANY", 0) / max(1, per.get("SQ_WAVE_CYCLES", 1)), 3),
        "note": "SQ_INSTS_VALU counts wave64 instructions; x64 lanes / in-band cells = lane instructions per "
                "cell over the whole kernel (fill steps, masked skew steps, ring staging, traceback sweep). "
                "SQ_*_CYCLES / WAIT counters are quad-cycles (MI355X_MICROARCH.md).",
    }
    s = json.dumps(out, indent=1)
    print(s)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")


if __name__ == "__main__":
    main()
