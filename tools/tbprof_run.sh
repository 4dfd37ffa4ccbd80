O=gpurun_out/tbprof; mkdir -p $O
GSNAPDP_LIB=gpuexp/tbprof/libgsnapdp.so ABLATE_C3=1 ABLATE_STEPS=3 timeout -k 10 300 python -u tools/ablate.py > $O/c3.txt 2>&1
GSNAPDP_LIB=gpuexp/tbprof/libgsnapdp.so ABLATE_STEPS=3 timeout -k 10 300 python -u tools/ablate.py > $O/c2.txt 2>&1
bash tools/quick_round.sh r3i
