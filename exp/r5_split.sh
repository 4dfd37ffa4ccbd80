# k_fill class split (GSNAPDP_FILL_SPLIT / _W): GPU suite on the default, then C3 1M and 125k per setting
O=gpurun_out/${1:-r5sp}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  for cfg in "-1 5" "0 5" "1 5" "1 4" "-1 3"; do
    set -- $cfg
    GSNAPDP_FILL_SPLIT=$1 GSNAPDP_FILL_SPLIT_W=$2 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > "$O/s$1_w$2_$i.json" 2>&1 || exit 1
    GSNAPDP_FILL_SPLIT=$1 GSNAPDP_FILL_SPLIT_W=$2 ABLATE_READS=125000 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > "$O/s$1_w$2_125k_$i.json" 2>&1 || exit 1
  done
done
for f in $O/s*.json; do echo "$f $(tail -n1 $f)"; done
