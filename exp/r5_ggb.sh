# C4 probability mode: the bridge's site probabilities loaded four columns at a time (gpuexp/ggb) vs the product
O=gpurun_out/${1:-r5gb}; mkdir -p $O
GSNAPDP_LIB=gpuexp/ggb/libgsnapdp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ggap or gband or c4 or stage3" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/cur_$i.txt 2>&1 || exit 1
  GSNAPDP_LIB=gpuexp/ggb/libgsnapdp.so timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/ggb_$i.txt 2>&1 || exit 1
done
for f in $O/*_[12].txt; do echo "$f $(tail -n1 $f)"; done
