# stage-3 lines at 14 / 15 / 16 host threads (GSNAPDP_S3_THREADS), GPU legs only
O=gpurun_out/${1:-r5t}; mkdir -p $O
for th in 16 15 14 16; do
  GSNAPDP_S3_THREADS=$th timeout -k 10 300 python -c "import json,bench; print(json.dumps({'s3p': bench.measure_stage3(), 's3c': bench.measure_stage3_compute(cpu=False), 'c4t': bench.measure_c4_transcripts(50000, cpu=False)}))" > $O/t$th.json 2> $O/t$th.err || exit 1
  python -c "import json; d=json.load(open('$O/t$th.json')); print($th, d['s3p']['value'], d['s3c']['value'], d['c4t']['value'])"
done
