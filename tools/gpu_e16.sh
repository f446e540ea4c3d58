#!/bin/bash
# tx_voice2 tests + TX line; C2 A/B of the rx_back lattice form (packed vs scalar VGPR coefficients)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_e14.sh || exit 1
V=uhsdr_amd/lib/variants
WL=c2 bash tools/gpu_lib_ab.sh e16 "cur|UHSDR_LIB=$V/libuhsdr_amd_cur.so|" "lats|UHSDR_LIB=$V/libuhsdr_amd_lats.so|" "cur2|UHSDR_LIB=$V/libuhsdr_amd_cur.so|" "lats2|UHSDR_LIB=$V/libuhsdr_amd_lats.so|"
