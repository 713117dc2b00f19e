#!/bin/bash
# Build a libvip variant with an alternative texture build into /root/repo/variants/<name>.so
# usage: build_texture_variant.sh <name> <extra hipcc flags...>   (e.g. -DVIP_GF_TH=32)
set -e
name=$1; shift
cd "$(dirname "$0")/../various_image_processings_amd/csrc"
mkdir -p ../../variants /tmp/tvar_$name
F="--offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-slp-vectorize -I../../include -I. $*"
hipcc $F -c vip_texture.hip -o /tmp/tvar_$name/t.o
# every other object from the in-place CMake build (__graft_entry__.build())
O=../../build/cmake/CMakeFiles
hipcc --offload-arch=gfx950 -shared -o ../../variants/$name.so /tmp/tvar_$name/t.o \
  $(ls $O/vip_{bil,ada,capi,stencil_rt}*.dir/various_image_processings_amd/csrc/*.o $O/vip_hip.dir/various_image_processings_amd/csrc/*.o)
echo built variants/$name.so
