"""bench.py's C4 transcript line alone (bench.measure_c4_transcripts), for GPU
iterations: python tools/c4t_bench.py [TRANSCRIPTS] [--no-cpu]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 50_000
    print(json.dumps(bench.measure_c4_transcripts(n, cpu="--no-cpu" not in sys.argv)), flush=True)
