#!/bin/bash
# Register / scratch footprint of the step kernels in a built object (no GPU needed):
#   scripts/kernel_resources.sh [build/obj/hip_step.hip.o]
set -e
B=/opt/rocm/lib/llvm/bin
objs=${@:-$(ls build/obj/hip_step.hip.part*.o | grep -v part0)}
tmp=$(mktemp -d)
for obj in $objs; do
  $B/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fatbin "$obj"
  $B/clang-offload-bundler --unbundle --type=o --input=$tmp/fatbin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/co
  $B/llvm-readelf --notes $tmp/co | grep -E '^\s+\.name:|\.vgpr_count|\.sgpr_count|\.private_segment_fixed_size|\.vgpr_spill_count|\.agpr_count' \
    | awk '/\.name:/{if(n)print n, r; n=$2; r=""; next} {r=r" "$1$2} END{print n, r}' | grep step_kernel | c++filt || true
done
rm -rf $tmp
