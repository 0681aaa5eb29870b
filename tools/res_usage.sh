#!/bin/bash
# VGPRs and scratch bytes per lane of every sampler kernel instantiation (device-only
# compile, no library written):  tools/res_usage.sh [source dir, default the tree]
#   columns: NSRC NT LDS_IMG WPB FAST  v=VGPRs s=scratch
root=${1:-$(cd "$(dirname "$0")/.." && pwd)}
out=$(mktemp)
(cd "$root" && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off \
  -mllvm -disable-machine-licm --cuda-device-only -c -o /dev/null olpefit_amd/csrc/olpe.hip \
  -Rpass-analysis=kernel-resource-usage) > "$out" 2>&1
grep -E "Function Name|VGPRs:|ScratchSize" "$out" | paste - - - | grep gibbs |
  sed -E 's/.*kernelILi([0-9])ELi([0-9]+)ELb([01])ELi([0-9]+)ELb([01]).*VGPRs: ([0-9]+).*lane\]: ([0-9]+).*/\1 \2 \3 \4 \5 v=\6 s=\7/'
rm -f "$out"
