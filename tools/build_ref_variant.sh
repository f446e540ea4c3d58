#!/bin/bash
# Build a P48-only libuhsdr_amd variant from the sources of a git revision (A/B against the
# working tree on one box): tools/build_ref_variant.sh <rev> <tag> [extra hipcc flags]
set -e
rev=$1; tag=$2; shift 2
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
if [ "$rev" = . ]; then mkdir -p "$tmp/uhsdr_amd" && cp -r uhsdr_amd/csrc "$tmp/uhsdr_amd/" && cp -r include "$tmp/"
else git archive "$rev" uhsdr_amd/csrc include | tar -x -C "$tmp"; fi
mkdir -p uhsdr_amd/lib/variants "$tmp/obj"
for f in "$tmp"/uhsdr_amd/csrc/*.hip; do
  [ "$(basename $f)" = uhsdr_cmsis.hip ] && continue
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -ffp-contract=off -fno-slp-vectorize -std=c++17 -Wno-unused-result \
      -I"$(pwd)/tools/isa" "$@" -I"$tmp/include" -I"$tmp/uhsdr_amd/csrc" -c "$f" -o "$tmp/obj/$(basename $f .hip).o" &
done
for f in "$tmp"/uhsdr_amd/csrc/*.c; do
  gcc -O2 -fPIC -ffp-contract=off -std=gnu11 -I"$tmp/include" -I"$tmp/uhsdr_amd/csrc" -c "$f" -o "$tmp/obj/$(basename $f .c).o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o uhsdr_amd/lib/variants/libuhsdr_amd_$tag.so "$tmp"/obj/*.o -lm
rm -rf "$tmp"
echo "uhsdr_amd/lib/variants/libuhsdr_amd_$tag.so"
