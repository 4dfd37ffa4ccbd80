# round-5 experiment: slices with the product k_fill and the no-traceback variant (timing only)
O=gpurun_out/${1:-r5e2}; mkdir -p $O
timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices_prod.json 2> $O/slices_prod.err || exit 1
GSNAPDP_LIB=gpuexp/notrace/libgsnapdp.so timeout -k 10 300 python bench.py --no-cpu --no-c4 --no-c5 --no-extra --no-c4t --steps 100 > $O/slices_notrace.json 2> $O/slices_notrace.err
tail -3 $O/slices_notrace.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
GSNAPDP_LIB=gpuexp/notrace/libgsnapdp.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $O/kf_notrace -o run -- python3 bench.py $B > /dev/null 2> $O/kf_notrace.err || exit 1
