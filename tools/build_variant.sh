#!/bin/bash
# Diagnostics: build libgsnapdp.so with extra -D flags on gsnapdp_kernels.hip into exp/NAME/.
# usage: bash tools/build_variant.sh NAME [-DFLAG ...]; then GSNAPDP_LIB=exp/NAME/libgsnapdp.so python tools/ablate.py
set -e
NAME=$1; shift
cd "$(dirname "$0")/../gmap-gsnap_amd"
make -s lib/gsnapdp_ggap.o lib/gsnapdp_micro.o lib/gsnapdp_host.o
O=../exp/$NAME; mkdir -p $O
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function "$@" \
  -c csrc/gsnapdp_kernels.hip -o $O/gsnapdp_kernels.o
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $O/libgsnapdp.so $O/gsnapdp_kernels.o \
  lib/gsnapdp_ggap.o lib/gsnapdp_micro.o lib/gsnapdp_host.o
