#!/bin/bash
# Resource usage (VGPRs, SGPR spills, scratch) of the gfx950 kernels in one built object.
#   tools/kres.sh uhsdr_amd/build/uhsdr_rx.o [name-regex]
set -e
obj=${1:-uhsdr_amd/build/uhsdr_rx.o}
pat=${2:-.}
tmp=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fat.bin "$obj"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$tmp/fat.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $tmp/k.co > $tmp/notes.txt
python3 - "$tmp/notes.txt" "$pat" <<'EOF'
import re, sys
txt = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
rows, cur = [], {}
for line in txt.splitlines():
    m = re.match(r"\s+\.(name|private_segment_fixed_size|vgpr_count|sgpr_spill_count|vgpr_spill_count):\s+(\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "name":
        cur = {"name": v}
        rows.append(cur)
    else:
        cur[k] = v
print(f"{'kernel':72s} {'vgpr':>5s} {'sspill':>6s} {'vspill':>6s} {'scratch':>7s}")
for r in rows:
    if pat.search(r["name"]):
        print(f"{r['name'][:72]:72s} {r.get('vgpr_count','?'):>5s} {r.get('sgpr_spill_count','?'):>6s} "
              f"{r.get('vgpr_spill_count','?'):>6s} {r.get('private_segment_fixed_size','?'):>7s}")
EOF
rm -rf $tmp
