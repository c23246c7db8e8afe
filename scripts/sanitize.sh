#!/usr/bin/env bash
# CPU sanitizer pass (no GPU): AddressSanitizer + UndefinedBehaviorSanitizer over
#   1. libcda's host planners (celestia-app_amd/csrc/plan.cpp, the same TU libcda links) driven by
#      tests/san/plan_check.cpp against naive restatements;
#   2. the C oracle (make -C oracle SAN=1) under the whole CPU test suite, with the gcc sanitizer runtimes
#      preloaded into python and CDA_ORACLE_LIB pointing at the sanitized build.
# Usage: scripts/sanitize.sh [log]   (default profiles/r03_sanitizers.log)
set -euo pipefail
cd "$(dirname "$0")/.."
LOG=${1:-profiles/r03_sanitizers.log}
mkdir -p "$(dirname "$LOG")" build_san
SANF="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer"
export ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{
  echo "== $(date -u) sanitizer pass ($(gcc --version | head -1))"
  echo "== 1. host planners: g++ $SANF plan.cpp + tests/san/plan_check.cpp"
  g++ -std=c++17 -O1 -g -Wall -Wextra $SANF -o build_san/plan_check tests/san/plan_check.cpp \
    celestia-app_amd/csrc/plan.cpp
  ./build_san/plan_check
  echo "== 2. oracle under the CPU suite: make -C oracle SAN=1; pytest -m 'not gpu'"
  make -s -C oracle SAN=1
  LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
    CDA_ORACLE_LIB="$PWD/oracle/_san/liboracle.so" \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider 2>&1
  echo "== sanitizer pass clean"
} 2>&1 | tee "$LOG"
