set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/sq; mkdir -p $O
for v in cur cur_notrace; do
GSNAPDP_LIB=exp/$v/libgsnapdp.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-c4 --no-c5 --no-extra > /dev/null 2> $O/$v.err
done
