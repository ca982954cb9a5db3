#!/usr/bin/env bash
# Host sanitizer run (SURVEY.md §5 "Race detection / sanitizers"): the C oracle built with
# -fsanitize=address,undefined (make asan), preloaded into the CPU test suite's Python processes
# (libasan must come first in a process whose interpreter is not instrumented).  Any ASan report or
# UBSan runtime error aborts the offending test (-fno-sanitize-recover), so a green suite is a clean run.
#   oracle/run_sanitized.sh [pytest args]     (default: the whole CPU suite, -m "not gpu")
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
make -s -C "$here" asan
export RTKV_ORACLE_LIB="$here/_build_asan/librtkv_oracle.so"
export LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)${LD_PRELOAD:+:$LD_PRELOAD}"
# CPython and its extensions keep objects alive at exit (not leaks of the oracle); halt on any error
export ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:allocator_may_return_null=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
cd "$here/.."
if [ $# -eq 0 ]; then set -- tests -m "not gpu" -q -x -p no:cacheprovider; fi
exec python -m pytest "$@"
