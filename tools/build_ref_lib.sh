#!/bin/bash
# Build libcviterbi.so of a git revision (default HEAD) into tools/_ab/lib_<name>.so for
# interleaved A/B runs on one box (CV_LIB_PATH=...): a throwaway worktree under /tmp.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
rev=${1:-HEAD}; name=${2:-ref}
W=/tmp/cv_wt_$name
rm -rf $W; git -C $R worktree prune
git -C $R worktree add -f --detach $W $rev > /dev/null
mkdir -p $W/consistent-viterbi_amd/csrc/build
cp -p $R/consistent-viterbi_amd/csrc/build/*.o $W/consistent-viterbi_amd/csrc/build/ 2>/dev/null || true
touch $W/consistent-viterbi_amd/csrc/*.cpp $W/consistent-viterbi_amd/csrc/kernels/*.hip
make -s -j8 -C $W/consistent-viterbi_amd/csrc > /dev/null
mkdir -p $R/tools/_ab
cp $W/consistent-viterbi_amd/cviterbi/libcviterbi.so $R/tools/_ab/lib_$name.so
git -C $R worktree remove --force $W
echo "built tools/_ab/lib_$name.so from $(git -C $R rev-parse --short $rev)"
