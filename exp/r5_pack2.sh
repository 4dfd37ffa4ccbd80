# packed k_fill pairs with contiguous task chunks (gpuexp/pack2), unpacked with chunks (gpuexp/blk), product
O=gpurun_out/${1:-r5p2}; mkdir -p $O
GSNAPDP_LIB=gpuexp/pack2/libgsnapdp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_pack2.txt 2>&1 || { tail -30 $O/pytest_pack2.txt; exit 1; }
tail -1 $O/pytest_pack2.txt
for i in 1 2; do
  for v in prod pack2 blk; do
    L=""; [ $v != prod ] && L=gpuexp/$v/libgsnapdp.so
    GSNAPDP_LIB=$L ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/${v}_$i.json 2>&1 || exit 1
    GSNAPDP_LIB=$L ABLATE_READS=125000 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/${v}125_$i.json 2>&1 || exit 1
  done
done
for f in $O/*_[12].json; do echo "$f $(tail -n1 $f)"; done
