#!/bin/bash
# VGPR / SGPR / scratch / spills of every kernel in built objects or .so
# files: tools/kernel_regs.sh libsrtp_amd/build/srtp_icm_nr10_km2.o ...
B=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
for f in "$@"; do
  $B/llvm-objcopy -O binary --only-section=.hip_fatbin "$f" $t/fb.bin &&
  $B/clang-offload-bundler --type=o --input=$t/fb.bin \
      --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$t/k.co --unbundle &&
  $B/llvm-readelf --notes $t/k.co | grep -E "^ +\.(name|vgpr_count|sgpr_count|private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count|group_segment_fixed_size):" |
  awk '/\.name:/{if(n)print line; n=$2; line=n} !/\.name:/{line=line" "$1$2}END{print line}' | grep "k_"
done
rm -rf $t
