#!/bin/bash
# k_fill scratch-traffic ablation and PMC calibration (run under gpurun).
#   bash tools/traffic_ablate.sh TAG   -> gpurun_out/TAG/{calib,VARIANT}_{fetch,write,trace}
# Variants: default and exp/{nomatch,notrace,nostore}/libgsnapdp.so (tools/build_variant.sh).
set -e
TAG=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$TAG; mkdir -p $O
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $O/calib_$C -o run -- ./exp/pmc_calib > $O/calib.txt 2> $O/calib_$C.err
done
for V in default nomatch notrace nostore; do
  if [ $V = default ]; then L=""; else L=exp/$V/libgsnapdp.so; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    GSNAPDP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/${V}_$C -o run -- python3 tools/traffic_ablate.py 3 > $O/${V}_$C.out 2> $O/${V}_$C.err
  done
  GSNAPDP_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${V}_trace -o run -- python3 tools/traffic_ablate.py 10 > $O/${V}_trace.out 2> $O/${V}_trace.err
done
echo done
