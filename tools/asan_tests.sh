#!/usr/bin/env bash
# The host code under AddressSanitizer + UndefinedBehaviorSanitizer, CPU only:
# builds `make asan` (the library's host translation units — planner, engine, the threaded
# text loader — and the oracle, with clang's ASan + UBSan; the HIP kernels' objects unchanged),
# then runs the CPU tests that drive that code through the C-ABI with the sanitized libraries
# in place of the normal ones (MVG_LIB, MVG_ORACLE_LIB). Any ASan report or UBSan finding
# aborts the run (halt_on_error, -fno-sanitize-recover). Python itself is not instrumented, so
# the ASan runtime is preloaded; leak detection is off (the interpreter's own allocations).
# Usage: tools/asan_tests.sh [log]   (default log: profiles/r06/asan_host_tests.log)
set -euo pipefail
REPO="$(cd "$(dirname "$0")/.." && pwd)"
LOG="${1:-$REPO/profiles/r06/asan_host_tests.log}"
mkdir -p "$(dirname "$LOG")"
make -s -C "$REPO" asan
RT="$(/opt/rocm/lib/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)"
cd "$REPO"
{
  echo "# tools/asan_tests.sh — $(date -u +%Y-%m-%dT%H:%M:%SZ)"
  echo "# MVG_LIB=build/asan/libmatvec_gpu.so MVG_ORACLE_LIB=build/asan/liboracle.so LD_PRELOAD=$RT"
  echo "# flags: $(make -s -C "$REPO" -pn asan 2>/dev/null | grep '^SANFLAGS :=' | head -1)"
} > "$LOG"
# ranks started by mpiexec inside the tests (the real reference, oracle/_ref) are not ours:
# they get neither the runtime nor the sanitized libraries
set +e
env MVG_LIB="$REPO/build/asan/libmatvec_gpu.so" MVG_ORACLE_LIB="$REPO/build/asan/liboracle.so" MVG_NO_TORCH=1 \
    ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:detect_odr_violation=0" \
    UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1" \
    LD_PRELOAD="$RT" \
    python -m pytest tests/test_capi_host.py tests/test_oracle_golden.py tests/test_cpuset.py tests/test_single_process_exchange.py \
        -q -p no:cacheprovider -m "not gpu" -k "not ref_runner" >> "$LOG" 2>&1
rc=$?
echo "# exit $rc" >> "$LOG"
tail -3 "$LOG"
exit $rc
