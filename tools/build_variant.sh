#!/bin/bash
# Build a variant of libcviterbi.so into tools/_ab/lib_<name>.so for tools/ab_lib.sh /
# tools/ab_small.sh: the in-tree objects are reused, only trellis64.o (and chain.o) are rebuilt
# with the extra flags.  Usage: tools/build_variant.sh <name> "<extra T64 flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/consistent-viterbi_amd/csrc
name=$1; shift
B=build_v_$name
rm -rf $C/$B && mkdir -p $C/$B
cp -p $C/build/*.o $C/$B/
rm -f $C/$B/trellis64.o $C/$B/chain.o
make -s -C $C BUILD=$B OUT=$R/tools/_ab/lib_$name.so T64FLAGS="-fno-honor-nans $*"
rm -rf $C/$B
echo "built tools/_ab/lib_$name.so"
