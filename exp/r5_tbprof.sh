# k_fill cycle split (TB_PROF build: fill_group / trace_batch / whole-wave s_memtime sums) at 1M and 125k
O=gpurun_out/${1:-r5tb}; mkdir -p $O
export GSNAPDP_LIB=$GRAFT_REPO_ROOT/gpuexp/tbprof/libgsnapdp.so
ABLATE_C3=1 ABLATE_STEPS=3 timeout -k 10 300 python3 tools/ablate.py > $O/tb1m.json 2> $O/tb1m.err || exit 1
ABLATE_C3=1 ABLATE_READS=125000 ABLATE_STEPS=3 timeout -k 10 300 python3 tools/ablate.py > $O/tb125.json 2> $O/tb125.err || exit 1
grep tb_prof $O/tb1m.err | tail -2; grep tb_prof $O/tb125.err | tail -2
