#!/bin/bash
# Build a variant of libcviterbi.so with extra fit.o flags into tools/_ab/lib_<name>.so (the
# in-tree objects are reused, only fit.o is rebuilt).  Usage: tools/build_fit_variant.sh <name> "<flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/consistent-viterbi_amd/csrc
name=$1; shift
B=build_f_$name
rm -rf $C/$B && mkdir -p $C/$B $R/tools/_ab
cp -p $C/build/*.o $C/$B/
rm -f $C/$B/fit.o
make -s -C $C BUILD=$B OUT=$R/tools/_ab/lib_$name.so FITFLAGS="$*"
rm -rf $C/$B
echo "built tools/_ab/lib_$name.so"
