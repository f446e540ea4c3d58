#!/bin/bash
# Local (no GPU) ISA statistics of one kernel instance: registers, spills, instruction mix.
# Usage: tools/isa_stats.sh <source.hip> <mangled-kernel-name-regex>
set -e
src=$1; pat=$2
out=/tmp/isa_$(basename $src .hip)
mkdir -p $out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -Itools/isa $ISAFLAGS -O3 -ffp-contract=off -fno-slp-vectorize -std=c++17 -Wno-unused-result \
  -Iinclude -Iuhsdr_amd/csrc --offload-device-only -S -o $out/k.s $src -Rpass-analysis=kernel-resource-usage 2> $out/res.txt
name=$(grep -o "^${pat}[^:]*:" $out/k.s | head -1 | tr -d :)
echo "kernel: $name"
grep -A9 "Function Name: $name " $out/res.txt | grep -E "VGPRs:|SGPRs Spill|VGPRs Spill|Occupancy|TotalSGPRs|Scratch" | sed 's/.*remark: *//; s/ \[-Rpass.*//'
awk -v n="$name:" '$1==n{f=1} f{print} f&&/s_endpgm/{exit}' $out/k.s > $out/one.s
echo "lines $(wc -l < $out/one.s)  VALU $(grep -cE '^\s+v_' $out/one.s)  readlane $(grep -c v_readlane $out/one.s)  writelane $(grep -c v_writelane $out/one.s)  SALU $(grep -cE '^\s+s_' $out/one.s)  branches $(grep -cE 's_cbranch' $out/one.s)  saveexec $(grep -c saveexec $out/one.s)  blocks $(grep -c '^.LBB' $out/one.s)"
