#!/bin/bash
# gfx950 disassembly of a built HIP object (no GPU needed): scripts/disasm.sh [obj] > out.s
set -e
B=/opt/rocm/lib/llvm/bin
objs=${@:-$(ls build/obj/hip_step.hip.part*.o | grep -v part0)}
tmp=$(mktemp -d)
for obj in $objs; do
  $B/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fatbin "$obj"
  $B/clang-offload-bundler --unbundle --type=o --input=$tmp/fatbin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/co
  $B/llvm-objdump -d --mcpu=gfx950 $tmp/co
done
rm -rf $tmp
