#!/bin/bash
# Per-kernel resources of one HIP source (gfx950 device code object): scratch, VGPRs, LDS.
# usage: tools/kernel_resources.sh incubator-druid_amd/csrc/dg_sort.hip [name-filter]
set -eu
src=$1
out=/tmp/kres_$$.co
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$(dirname "$0")/../include" -x hip --offload-device-only --no-gpu-bundle-output -c "$src" -o "$out"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$out" | grep -E "^ +\.name:|\.private_segment_fixed_size|\.vgpr_count|\.group_segment_fixed_size|\.agpr_count" \
  | awk '/\.group_segment_fixed_size/{lds=$2} /\.name:/{name=$2} /\.private_segment_fixed_size/{scr=$2} /\.vgpr_count/{printf "%-60s lds=%-6s scratch=%-5s vgpr=%s\n", substr(name,1,60), lds, scr, $2}' \
  | grep -E "${2:-.}" || true
rm -f "$out"
