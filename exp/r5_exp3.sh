# round-5 experiment: VALU issue rates; traceback prefetch distance 2 / 3 on the slices
O=gpurun_out/${1:-r5e3}; mkdir -p $O
timeout -k 10 120 gpuexp/valu_rate5 > $O/valu_rate5.txt 2>&1 || exit 1
for v in ahead2 ahead3; do
  GSNAPDP_LIB=gpuexp/$v/libgsnapdp.so timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices_$v.json 2> $O/slices_$v.err || exit 1
done
timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices_prod.json 2> $O/slices_prod.err || exit 1
timeout -k 10 400 python tools/l2sort_probe.py 30 > $O/l2sort.json 2> $O/l2sort.err || exit 1
bash tools/r5_rec.sh
