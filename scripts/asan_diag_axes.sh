R=$(pwd)
mkdir -p gpurun_out/asan_diag
python3 -c "
import sys; sys.path.insert(0,'tests'); import oracle_lib as O
O.gen_ods(32, 5).tofile('gpurun_out/asan_diag/ods.bin')"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:protect_shadow_gap=0
for t in 1 2 16; do
  timeout -k 5 120 tests/abi_client/rsmt2d_axes_asan cda $R/celestia-app_amd/cda/libcda_asan.so extend 32 $t 1 gpurun_out/asan_diag/ods.bin gpurun_out/asan_diag > gpurun_out/asan_diag/t$t.log 2>&1
  echo "threads $t rc=$?"; head -c 300 gpurun_out/asan_diag/t$t.log; echo
done
timeout -k 5 120 tests/abi_client/rsmt2d_axes_asan cda $R/celestia-app_amd/cda/libcda_asan.so single 32 3 gpurun_out/asan_diag/ods.bin > gpurun_out/asan_diag/single.log 2>&1
echo "single rc=$?"; head -c 300 gpurun_out/asan_diag/single.log
exit 0
