# SQ counters of k_fill, product vs packed pairs (gpuexp/pack)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r5pm}; mkdir -p $O
B="--steps 3 --warmup 1 --no-cpu --no-side --no-steady"
for v in blk pack2; do
  L=gpuexp/$v/libgsnapdp.so
  GSNAPDP_LIB=$L timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d $O/${v}1 -o run -- python3 bench.py $B > /dev/null 2> $O/${v}1.err || exit 1
  GSNAPDP_LIB=$L timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS --output-format csv -d $O/${v}2 -o run -- python3 bench.py $B > /dev/null 2> $O/${v}2.err || exit 1
done
