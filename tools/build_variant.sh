#!/bin/bash
# A/B builds: liborbgpu.so with one source file compiled with extra flags, into build/var/NAME/.
#   tools/build_variant.sh NAME SOURCE.hip "-DFLAG=..."   (run `make` first for the other objects)
# On the GPU box a variant is tried by copying it over orb-slam3_byzyh_amd/lib/liborbgpu.so
# (tools/var_ab.sh).
set -eu
NAME=$1; SRCF=$2; FLAGS=${3:-}
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Iinclude -Iorb-slam3_byzyh_amd/csrc -w"
mkdir -p vars/$NAME
base=$(basename $SRCF .hip)
case $SRCF in */*) SP=$SRCF;; *) SP=orb-slam3_byzyh_amd/csrc/$SRCF;; esac
/opt/rocm/bin/hipcc $HIPFLAGS $FLAGS -c $SP -o vars/$NAME/$base.o
objs=""
for o in build/obj/*.o; do [ "$(basename $o .o)" = "$base" ] || objs="$objs $o"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o vars/$NAME/liborbgpu.so $objs vars/$NAME/$base.o
echo built vars/$NAME/liborbgpu.so
