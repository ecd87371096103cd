#!/bin/bash
# Host-side AddressSanitizer run (no GPU): the C-ABI library's host code (icrc_capi.cpp,
# icrc_ring.cpp, protocol.cpp, icrc_tables.cpp) rebuilt with -fsanitize=address (hipcc: -Xarch_host only, the
# device code is the product's own objects), loaded by the CPU test suite through ICRC_AMD_LIB.
# GPU sanitizers are not available on the pool; this covers the PacketWriter / header writer /
# table builder / engine error paths the CPU tests drive.
set -eu
cd "$(dirname "$0")/.."
B=/tmp/icrc_asan; mkdir -p $B
CLX=/opt/rocm/lib/llvm/bin/clang++
RT=$($CLX -print-file-name=libclang_rt.asan-x86_64.so)
make -s -C open-rdma-driver_amd _build/icrc_kernels.o _build/icrc_oct.o _build/icrc_ring_kernel.o
cp open-rdma-driver_amd/_build/icrc_kernels.o open-rdma-driver_amd/_build/icrc_oct.o open-rdma-driver_amd/_build/icrc_ring_kernel.o $B/
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -Iinclude \
  -Iopen-rdma-driver_amd/csrc -c open-rdma-driver_amd/csrc/icrc_capi.cpp -o $B/icrc_capi.o
for f in protocol icrc_tables icrc_ring; do
  $CLX -O1 -g -std=c++17 -fPIC -fsanitize=address -Iinclude -Iopen-rdma-driver_amd/csrc \
    -c open-rdma-driver_amd/csrc/$f.cpp -o $B/$f.o
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -fsanitize=address -fno-gpu-sanitize -shared-libsan -o $B/libicrc_amd.so \
  $B/icrc_kernels.o $B/icrc_oct.o $B/icrc_ring_kernel.o $B/icrc_capi.o $B/protocol.o $B/icrc_tables.o $B/icrc_ring.o
LD_LIBRARY_PATH=$(dirname "$RT") LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:replace_intrin=0 \
  ICRC_AMD_LIB=$B/libicrc_amd.so python3 -c "import sys; sys.path.insert(0, 'open-rdma-driver_amd'); import icrc_amd; print('library:', icrc_amd.LIB_PATH)"
LD_LIBRARY_PATH=$(dirname "$RT") LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:replace_intrin=0 \
  ICRC_AMD_LIB=$B/libicrc_amd.so python3 -m pytest tests/test_capi_host.py tests/test_oracle.py tests/test_golden.py -q -m "not gpu"
