# k_fill class partition (GSNAPDP_FILL_PARTITION): GPU suite with it on, then C3 and 125k per setting, alternating
O=gpurun_out/${1:-r5pt}; mkdir -p $O
GSNAPDP_FILL_PARTITION=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  for p in 0 1; do
    GSNAPDP_FILL_PARTITION=$p ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/p${p}_$i.json 2>&1 || exit 1
    GSNAPDP_FILL_PARTITION=$p ABLATE_READS=125000 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/p${p}125_$i.json 2>&1 || exit 1
  done
done
for f in $O/p*.json; do echo "$f $(tail -n1 $f)"; done
