#!/bin/bash
# Register / spill / LDS report of single conv_fast instantiations without the full library build
# (the launch tables instantiate every tile: ~10 min). usage: tools/kernel_regs.sh "<template args>" ...
# e.g. tools/kernel_regs.sh "_Float16, 256, 224, 64, 4, 2, 4, 1, true, true, false, true"
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
{
  echo '#define PC_FAST_KERNEL_ONLY'
  echo "#include \"$ROOT/person_capture_amd/csrc/pc_conv_fast.hip\""
  i=0
  for a in "$@"; do
    echo "template __global__ void pc::conv_fast<$a>(pc::ConvParams);"
    i=$((i + 1))
  done
} > "$T/k.hip"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only --no-gpu-bundle-output -c "$T/k.hip" -o "$T/k.co" \
  -I"$ROOT/person_capture_amd/csrc"
/opt/rocm/lib/llvm/bin/llvm-readelf --notes "$T/k.co" | python3 -c '
import re, sys
t = sys.stdin.read()
for b in t.split(".name:")[1:]:
    name = b.split("\n")[0].strip()
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", b) or [None, None])[1]
    if "conv_fast" in name:
        print(name, "vgpr", g("vgpr_count"), "agpr", g("agpr_count"), "spill", g("vgpr_spill_count"), "lds", g("group_segment_fixed_size"))
'
rm -rf "$T"
