#!/bin/bash
# Like build_variant.sh but without the make step (the other product objects as
# they stand in lib/): several variants can compile at once.
# usage: [SRC=kernels] bash tools/build_variant_fast.sh NAME [-DFLAG ...]
set -e
NAME=$1; shift
SRC=${SRC:-kernels}
cd "$(dirname "$0")/../gmap-gsnap_amd"
REST="lib/gsnapdp_micro.o lib/gsnapdp_gather.o lib/gsnapdp_gwin.o lib/gsnapdp_host.o lib/gsnapdp_stage3.o lib/gsnapdp_stage3_exec.o lib/gsnapdp_stage3_compute.o lib/gsnapdp_iit.o lib/gsnapdp_scan.o"
O=../gpuexp/$NAME; mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function "$@" \
  -c csrc/gsnapdp_$SRC.hip -o $O/gsnapdp_$SRC.o
OBJS="$REST"
for s in kernels ggap gband; do
  if [ $s = $SRC ]; then OBJS="$OBJS $O/gsnapdp_$s.o"; else OBJS="$OBJS lib/gsnapdp_$s.o"; fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,-Bsymbolic -o $O/libgsnapdp.so $OBJS
