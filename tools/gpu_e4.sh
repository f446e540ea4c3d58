set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
V=uhsdr_amd/lib/variants
UHSDR_LIB=$V/libuhsdr_amd_dec2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_paths.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "(test_device_path_matches_oracle and p48_) or call_granularity or full_batch or (north_star_batch and 48) or test_device_matches_reference_firmware and p48_usb" > gpurun_out/e4_pytest.log 2>&1 || { tail -40 gpurun_out/e4_pytest.log; exit 1; }
tail -2 gpurun_out/e4_pytest.log
bash tools/gpu_lib_ab.sh e4 "base|UHSDR_LIB=$V/libuhsdr_amd_base.so|--schedule fused" "dec2|UHSDR_LIB=$V/libuhsdr_amd_dec2.so|--schedule fused" "basefma|UHSDR_LIB=$V/libuhsdr_amd_base.so|--schedule fused --precision fma" "dec2fma|UHSDR_LIB=$V/libuhsdr_amd_dec2.so|--schedule fused --precision fma" "base2|UHSDR_LIB=$V/libuhsdr_amd_base.so|--schedule fused" "dec2b|UHSDR_LIB=$V/libuhsdr_amd_dec2.so|--schedule fused"
