"""The stage-3 pass side line of bench.py alone (bench.measure_stage3), for
quick GPU iterations: python tools/s3_bench.py [PATHS] [REPS]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    paths = int(sys.argv[1]) if len(sys.argv) > 1 else 7424
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    print(json.dumps(bench.measure_stage3(paths=paths, reps=reps)), flush=True)
