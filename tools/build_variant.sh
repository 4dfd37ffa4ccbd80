#!/bin/bash
# Diagnostics: build libgsnapdp.so with extra -D flags on one kernel source into gpuexp/NAME/ (git-ignored; it travels with gpurun: delete it after the experiment).
# usage: [SRC=ggap|gband|kernels] bash tools/build_variant.sh NAME [-DFLAG ...]
#        then GSNAPDP_LIB=gpuexp/NAME/libgsnapdp.so python tools/ablate.py (or ablate_ggap.py)
set -e
NAME=$1; shift
SRC=${SRC:-kernels}
cd "$(dirname "$0")/../gmap-gsnap_amd"
REST="lib/gsnapdp_micro.o lib/gsnapdp_gather.o lib/gsnapdp_gwin.o lib/gsnapdp_host.o lib/gsnapdp_stage3.o lib/gsnapdp_stage3_exec.o lib/gsnapdp_stage3_compute.o lib/gsnapdp_iit.o lib/gsnapdp_scan.o"
make -s lib/gsnapdp_kernels.o lib/gsnapdp_ggap.o lib/gsnapdp_gband.o $REST
O=../gpuexp/$NAME; mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function "$@" \
  -c csrc/gsnapdp_$SRC.hip -o $O/gsnapdp_$SRC.o
OBJS="$REST"
for s in kernels ggap gband; do
  if [ $s = $SRC ]; then OBJS="$OBJS $O/gsnapdp_$s.o"; else OBJS="$OBJS lib/gsnapdp_$s.o"; fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -Wl,-Bsymbolic -o $O/libgsnapdp.so $OBJS
