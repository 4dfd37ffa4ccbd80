# k_fill with the traceback sweep in its own function (GSNAPDP_TB_NOINLINE: own register allocation), prefetch 1 / 2
O=gpurun_out/${1:-r5n}; mkdir -p $O
GSNAPDP_LIB=gpuexp/tbni/libgsnapdp.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "c3 or parity or c2 or end or sj" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2; do
  for v in prod tbni tbni2; do
    L=""; [ $v != prod ] && L=gpuexp/$v/libgsnapdp.so
    GSNAPDP_LIB=$L ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/${v}_$i.json 2>&1 || exit 1
    GSNAPDP_LIB=$L ABLATE_READS=125000 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/${v}125_$i.json 2>&1 || exit 1
  done
done
for f in $O/*_[12].json; do echo "$f $(tail -n1 $f)"; done
