# C4 probability mode: the outcome's site probabilities reused from the tables (current) vs re-evaluated (gpuexp/oldgg)
O=gpurun_out/${1:-r5g1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ggap or gband or c4 or stage3 or dropin" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/cur_$i.txt 2>&1 || exit 1
  GSNAPDP_LIB=gpuexp/oldgg/libgsnapdp.so timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/old_$i.txt 2>&1 || exit 1
  GSNAPDP_GBAND_PROB=1 timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/curband_$i.txt 2>&1 || exit 1
done
for f in $O/*_[12].txt; do echo "$f $(tail -n1 $f)"; done
