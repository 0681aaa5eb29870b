#!/bin/bash
# Build libolpe.so of a git revision into diag/<name>/ for same-box A/B runs
# (tools/ab_libs.sh <name>).  usage: tools/build_rev.sh <rev> <name> [extra hipcc flags]
rev=$1; name=$2; shift 2
tmp=$(mktemp -d)
mkdir -p $tmp/olpefit_amd/csrc $tmp/include
for f in $(git ls-tree --name-only -r $rev olpefit_amd/csrc include); do git show $rev:$f > $tmp/$f; done
mkdir -p diag/$name
# the revision's sources (olpe_csv.cpp from its introduction on)
srcs="$tmp/olpefit_amd/csrc/olpe.hip $tmp/olpefit_amd/csrc/olpe_comm.hip"
[ -f $tmp/olpefit_amd/csrc/olpe_csv.cpp ] && srcs="$srcs $tmp/olpefit_amd/csrc/olpe_csv.cpp"
[ -f $tmp/olpefit_amd/csrc/olpe_moments.hip ] && srcs="$srcs $tmp/olpefit_amd/csrc/olpe_moments.hip"
/opt/rocm/bin/hipcc $(python -m olpefit_amd.build --print-flags) "$@" \
  -o diag/$name/libolpe.so $srcs -lrccl
rm -rf $tmp
