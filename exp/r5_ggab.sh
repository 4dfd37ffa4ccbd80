# C4 probability mode: k_ggap without one phase each (timing only; wrong results)
O=gpurun_out/${1:-r5ga}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/prod_$i.txt 2>&1 || exit 1
  for v in NOFILL NOBRIDGE NOTRACE NOPROB; do
    GSNAPDP_LIB=gpuexp/gg_$v/libgsnapdp.so timeout -k 10 300 python3 tools/ablate_ggap.py prob > $O/${v}_$i.txt 2>&1 || exit 1
  done
done
for f in $O/*_[12].txt; do echo "$f $(tail -n1 $f)"; done
