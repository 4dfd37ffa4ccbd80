# record the C4 transcript pass's rounds (10k paths) for host replay (tools/s3_record_c4.py)
O=gpurun_out/c4rec; mkdir -p $O
GSNAPDP_S3_RECORD=$O timeout -k 10 300 python tools/s3_record_c4.py $O 10000 --gpu > $O/rec.txt 2>&1 || exit 1
du -sh $O
