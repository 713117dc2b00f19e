#!/bin/bash
# Build a libvip variant in which ONE CMake object target is recompiled with extra flags and
# every other object comes from the in-place CMake build (__graft_entry__.build()):
#   build_object_variant.sh <name> <target> <source> <flags...>  -> variants/<name>.so
# e.g. build_object_variant.sh jbf_ablcvt vip_bil_joint_fma vip_bilateral.hip -DVIP_BIL_JOINT -DVIP_BIL_FMA -DVIP_ABL_CVT
# (the target's own -D definitions must be repeated: CMakeLists.txt vip_variant lines)
set -e
name=$1; target=$2; src=$3; shift 3
cd "$(dirname "$0")/../various_image_processings_amd/csrc"
mkdir -p ../../variants /tmp/ovar_$name
hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off -fno-slp-vectorize -I../../include -I. "$@" \
  -c $src -o /tmp/ovar_$name/v.o
O=../../build/cmake/CMakeFiles
others=$(ls $O/vip_{bil,ada,texture,capi,stencil_rt}*.dir/various_image_processings_amd/csrc/*.o | grep -v "/$target.dir/")
hipcc --offload-arch=gfx950 -shared -o ../../variants/$name.so /tmp/ovar_$name/v.o $others
echo built variants/$name.so
