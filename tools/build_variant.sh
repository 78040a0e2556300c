#!/bin/bash
# Build an A/B variant of libdruidgpu.so with extra -D flags: tools/build_variant.sh NAME -DFOO ...
set -e
name=$1; shift
cd "$(dirname "$0")/../incubator-druid_amd/csrc"
out=../lib/variants/$name
mkdir -p $out/obj
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wno-unused-value -Wno-unused-result -I../../include $*"
$H -c -x hip dg_lz4.hip -o $out/obj/dg_lz4.o &
$H -c -x hip dg_kernels.hip -o $out/obj/dg_kernels.o &
$H -c -x hip dg_sort.hip -o $out/obj/dg_sort.o &
$H -c dg_engine.cpp -o $out/obj/dg_engine.o &
$H -c dg_segment.cpp -o $out/obj/dg_segment.o &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libdruidgpu.so $out/obj/*.o
echo "$out/libdruidgpu.so"
