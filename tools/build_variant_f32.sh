#!/bin/bash
# Build a variant of libcviterbi.so into tools/_ab/lib_<name>.so with extra flags for trellis.o
# only (the f32 kernels; the other objects are reused).  Usage: tools/build_variant_f32.sh <name> "<flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/consistent-viterbi_amd/csrc
name=$1; shift
B=build_v_$name
rm -rf $C/$B && mkdir -p $C/$B $R/tools/_ab
cp -p $C/build/*.o $C/$B/
rm -f $C/$B/trellis.o
make -s -C $C BUILD=$B OUT=$R/tools/_ab/lib_$name.so TRFLAGS="$*"
rm -rf $C/$B
echo "built tools/_ab/lib_$name.so"
