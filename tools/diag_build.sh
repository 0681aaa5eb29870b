#!/bin/bash
# Build a diagnostic libolpe variant into /root/repo/diag/<name>/libolpe.so (never the
# product library).  usage: tools/diag_build.sh <name> <extra hipcc flags...>
#
# The diagnostic hooks (-DOLPE_DIAG_TIMING, _SPAN, _FALLBACK, _RING8, _HCONST, _DWCONST,
# _HSMEM[_PW/_HALF/_ROT]) are not in the product sources (verdict r05 item 4): they live
# in tools/diag/diag_hooks.patch, applied here to a copy of the sources, so the product
# tree carries no diagnostic code and no build of it can pick one up by accident.
set -euo pipefail
name=$1; shift
repo=$(cd "$(dirname "$0")/.." && pwd)
src=$(mktemp -d)
trap 'rm -rf "$src"' EXIT
mkdir -p "$src/olpefit_amd" "$src/include"
cp -r "$repo/olpefit_amd/csrc" "$src/olpefit_amd/"
cp "$repo/include/olpe.h" "$src/include/"
patch -p1 -s -d "$src" < "$repo/tools/diag/diag_hooks.patch"
mkdir -p "$repo/diag/$name"
c="$src/olpefit_amd/csrc"
/opt/rocm/bin/hipcc $(cd "$repo" && python -m olpefit_amd.build --print-flags) \
  "$@" -o "$repo/diag/$name/libolpe.so" "$c/olpe.hip" "$c/olpe_comm.hip" \
  "$c/olpe_moments.hip" "$c/olpe_csv.cpp" -lrccl
