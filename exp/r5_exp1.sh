# round-5 experiment: k_fill wave cap on the slices, stage-3 host profiles
O=gpurun_out/${1:-r5e1}; mkdir -p $O
for m in 0 4 3; do
  GSNAPDP_FILL_MIN_TASKS=$m timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices_$m.json 2> $O/slices_$m.err || exit 1
done
GSNAPDP_S3_PROFILE=1 timeout -k 10 300 python tools/c4t_bench.py 50000 --no-cpu > $O/c4t.json 2> $O/c4t.err || exit 1
GSNAPDP_S3_PROFILE=1 timeout -k 10 300 python -c "import json,bench; print(json.dumps(bench.measure_stage3_compute(cpu=False)))" > $O/s3c.json 2> $O/s3c.err || exit 1
