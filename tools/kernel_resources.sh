#!/bin/bash
# VGPR / SGPR / LDS / spill figures of the kernels of one built object (default build/trellis64.o;
# gfx950 code object from its .hip_fatbin section).  Usage: tools/kernel_resources.sh [regex] [lib]
RE=${1:-.}
LIB=${2:-$(dirname "$0")/../consistent-viterbi_amd/csrc/build/trellis64.o}
T=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "$LIB" /dev/null
TGT=$($L/clang-offload-bundler --list --type=o --input=$T/fb.bin | grep gfx950 | head -1)
$L/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=$TGT --output=$T/k.co
$L/llvm-readelf --notes $T/k.co | python3 -c '
import re, sys
rx = re.compile(sys.argv[1])
cur = {}
out = []
for line in sys.stdin:
    m = re.match(r"[\s-]+\.(\w+):\s+(.*)", line)
    if not m: continue
    k, v = m.groups()
    cur["agpr" if k == "agpr_count" else k] = v
    if k == "wavefront_size":
        if "name" in cur: out.append(cur)
        cur = {}
for c in out:
    if rx.search(c.get("name", "")):
        g = c.get
        print("vgpr %s agpr %s sgpr %s lds %s spill v%s s%s  %s" % (g("vgpr_count"), g("agpr"), g("sgpr_count"),
              g("group_segment_fixed_size"), g("vgpr_spill_count"), g("sgpr_spill_count"), c["name"]))
' "$RE"
rm -rf $T
