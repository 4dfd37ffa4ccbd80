O=gpurun_out/r5abl2; mkdir -p $O
timeout -k 10 120 gpuexp/valu_rate5 > $O/valu_rate5.txt 2>&1 || exit 1
run() { GSNAPDP_LIB=$2 ABLATE_C3=1 ABLATE_STEPS=20 timeout -k 10 300 python3 tools/ablate.py > $O/$1.json 2>$O/$1.err || exit 1; cat $O/$1.json; }
run prod0 ""
for v in fillonly permfill permbits; do run $v gpuexp/$v/libgsnapdp.so; done
run prod1 ""
GSNAPDP_LIB=gpuexp/permbits/libgsnapdp.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_permbits.txt 2>&1; tail -3 $O/pytest_permbits.txt
