#!/bin/bash
# Build a diagnostic libolpe variant into /root/repo/diag/<name>/libolpe.so (never the
# product library).  usage: tools/diag_build.sh <name> <extra hipcc flags...>
name=$1; shift
mkdir -p diag/$name
/opt/rocm/bin/hipcc $(python -m olpefit_amd.build --print-flags) \
  "$@" -o diag/$name/libolpe.so olpefit_amd/csrc/olpe.hip olpefit_amd/csrc/olpe_comm.hip \
  olpefit_amd/csrc/olpe_moments.hip olpefit_amd/csrc/olpe_csv.cpp -lrccl
