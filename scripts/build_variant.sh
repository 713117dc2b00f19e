#!/bin/bash
# Build an experimental R=7 plain-FMA bilateral library variant into /root/repo/variants/<name>.so
# usage: build_variant.sh <name> <extra hipcc flags...>
set -e
name=$1; shift
cd "$(dirname "$0")/../various_image_processings_amd/csrc"
mkdir -p ../../variants /tmp/var_$name
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-slp-vectorize -I../../include -I. $*"
hipcc $F -DVIP_ONLY_R7 -DVIP_BIL_FMA -c vip_bilateral.hip -o /tmp/var_$name/b.o
hipcc $F -DVIP_ONLY_R7 -DVIP_BIL_JOINT -DVIP_BIL_FMA -c vip_bilateral.hip -o /tmp/var_$name/bj.o
hipcc $F -DVIP_ONLY_R7 -c vip_bilateral.hip -o /tmp/var_$name/bm.o
hipcc $F -DVIP_ONLY_R7 -DVIP_BIL_JOINT -c vip_bilateral.hip -o /tmp/var_$name/bjm.o
hipcc $F -DVIP_ONLY_R7 -DVIP_ADA_FMA -c vip_adaptive.hip -o /tmp/var_$name/a.o
hipcc $F -DVIP_ONLY_R7 -c vip_adaptive.hip -o /tmp/var_$name/am.o
# the texture, C ABI and C++ API objects of the in-place CMake build (__graft_entry__.build())
O=../../build/cmake/CMakeFiles
hipcc --offload-arch=gfx950 -shared -o ../../variants/$name.so /tmp/var_$name/*.o \
  $(ls $O/vip_{texture,capi,stencil_rt}.dir/various_image_processings_amd/csrc/*.o $O/vip_hip.dir/various_image_processings_amd/csrc/*.o)
echo built variants/$name.so
