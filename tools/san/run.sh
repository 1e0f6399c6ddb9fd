#!/bin/bash
# Sanitizer runs of the host C++ (CPU only, this container or any host):
#   1. ASan + UBSan: the CPU tests that drive the native host code (SBOM decoder, bbolt walker,
#      wire encoder, ignore / VEX compilers, DB flattener, C-ABI) against libtrivy_amd_san.so
#   2. libFuzzer + ASan + UBSan over the untrusted-input decoders (CycloneDX, bbolt), seeded
#      from the reference's own SBOM / bolt fixtures (tests/golden)
#   3. TSan: the worker pool, the parallel wire encoder and the SBOM decoder's host threads,
#      1 thread against 8 (tools/san/tsan_host.cpp)
# Logs: profiles/r06/san/ (OUT=...).  The fuzzers are built without ASan's global-variable
# instrumentation (-asan-globals=0): with -fsanitize=fuzzer this clang registers identical
# string literals of one module twice and aborts on a false "ODR violation / misaligned global"
# before the first input; heap, stack and UBSan checks are unaffected.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${OUT:-$R/profiles/r06/san}
FUZZ_S=${FUZZ_S:-60}
mkdir -p $OUT
LLVM=/opt/rocm/lib/llvm
RT=$(ls -d $LLVM/lib/clang/*/lib/linux | head -1)
CXX=$LLVM/bin/clang++
CS=$R/trivy_amd/csrc
make -s -C $CS -j8 san
# 1. the CPU tests on the sanitizer build
cd $R
LD_PRELOAD=$RT/libclang_rt.asan-x86_64.so \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
TVM_LIB_PATH=$R/trivy_amd/libtrivy_amd_san.so TVM_HOST_THREADS=8 \
  timeout -k 10 1200 python -m pytest -q -m "not gpu" -p no:cacheprovider \
  tests/test_sbom_native.py tests/test_bbolt.py tests/test_wire_host.py tests/test_ignore_host.py \
  tests/test_vex_host.py tests/test_db_host.py tests/test_capi.py tests/test_libver_host.py tests/test_verkey_host.py \
  tests/test_fastdeb_host.py tests/test_sbom.py > $OUT/asan_ubsan_tests.log 2>&1
tail -3 $OUT/asan_ubsan_tests.log
# 2. fuzzers
B=$(mktemp -d)
FZ="-O1 -g -std=c++17 -fsanitize=fuzzer,address,undefined -fno-sanitize-recover=all -mllvm -asan-globals=0 -I$CS"
$CXX $FZ -o $B/fuzz_sbom $R/tools/san/fuzz_sbom.cpp $CS/sbom.cpp -lpthread
$CXX $FZ -o $B/fuzz_bbolt $R/tools/san/fuzz_bbolt.cpp $CS/bbolt.cpp -lpthread
mkdir -p $B/c_sbom $B/c_bbolt
cp $R/tests/golden/sbom/*.json $B/c_sbom/ 2>/dev/null || true
find $R/tests/golden -name "*.db" -exec cp {} $B/c_bbolt/ \;
ASAN_OPTIONS=detect_leaks=1 timeout -k 10 $((FUZZ_S + 60)) $B/fuzz_sbom -max_total_time=$FUZZ_S -max_len=262144 \
  -rss_limit_mb=4096 $B/c_sbom > $OUT/fuzz_sbom.log 2>&1
tail -2 $OUT/fuzz_sbom.log
ASAN_OPTIONS=detect_leaks=1 timeout -k 10 $((FUZZ_S + 60)) $B/fuzz_bbolt -max_total_time=$FUZZ_S -max_len=1048576 \
  -rss_limit_mb=4096 $B/c_bbolt > $OUT/fuzz_bbolt.log 2>&1
tail -2 $OUT/fuzz_bbolt.log
# 3. TSan
# (hipcc: engine.h carries device code; the sanitizer applies to the host side only)
/opt/rocm/bin/hipcc -O1 -g -std=c++17 --offload-arch=gfx950 -Xarch_host -fsanitize=thread -x hip -I$CS \
  -o $B/tsan_host $R/tools/san/tsan_host.cpp $CS/wire.cpp $CS/sbom.cpp $CS/hostbatch.cpp -lpthread
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 timeout -k 10 600 $B/tsan_host > $OUT/tsan_host.log 2>&1
tail -3 $OUT/tsan_host.log
rm -rf $B
echo "sanitizer runs clean"
