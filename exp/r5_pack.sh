# packed k_fill pairs (gpuexp/pack): GPU suite, then C3 / 125k k_fill times beside the product, alternating
O=gpurun_out/${1:-r5p1}; mkdir -p $O
GSNAPDP_LIB=gpuexp/pack/libgsnapdp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_pack.txt 2>&1 || { tail -30 $O/pytest_pack.txt; exit 1; }
tail -1 $O/pytest_pack.txt
for i in 1 2; do
  ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/prod_$i.json 2>&1 || exit 1
  GSNAPDP_LIB=gpuexp/pack/libgsnapdp.so ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/pack_$i.json 2>&1 || exit 1
  ABLATE_READS=125000 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/prod125_$i.json 2>&1 || exit 1
  ABLATE_READS=125000 GSNAPDP_LIB=gpuexp/pack/libgsnapdp.so ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/pack125_$i.json 2>&1 || exit 1
done
tail -qn1 $O/prod_*.json $O/pack_*.json $O/prod125_*.json $O/pack125_*.json
