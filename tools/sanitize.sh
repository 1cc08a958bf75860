#!/bin/bash
# Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, no GPU):
#   * oracle/*.c (the CPU restatement)                      -> oracle/_asan/liboracle.so
#   * the tx_host RLP decoder and the host builds of the device field headers (secp256k1_fe9.cuh with
#     its column forms and fe9_pow_pm3_4, modinv30.cuh, bn254_fe9.cuh) through tests/native/*.cpp,
#     rebuilt with the sanitizer flags by tests/conftest.py build_native when GSV_SANITIZE=1, and the
#     trie-plan emulator (tests/native/plan_emu.cpp)
# and runs the CPU tests that exercise them with the sanitizer runtimes preloaded into Python.
#   bash tools/sanitize.sh [pytest args] > profiles/rNN/sanitize.log 2>&1
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/oracle" asan
ASAN=$(gcc -print-file-name=libasan.so)
UBSAN=$(gcc -print-file-name=libubsan.so)
cd "$R"
export GSV_SANITIZE=1 GSV_ORACLE_LIB="$R/oracle/_asan/liboracle.so"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$ASAN:$UBSAN${LD_PRELOAD:+:$LD_PRELOAD}" python -m pytest -q -p no:cacheprovider \
    tests/test_oracle.py tests/test_tx_host.py tests/test_fe9.py tests/test_bn9.py tests/test_configs_cpu.py \
    tests/test_plan_emu.py tests/test_recover_twist.py tests/test_asm_emulated.py \
    -m "not gpu" "$@"
