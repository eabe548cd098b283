#!/bin/bash
# Host AddressSanitizer + UBSan run of the CPU test suite (SURVEY §5 "race detection /
# sanitizers"): the C++ runtime (config reader, NetConfig, IO, metrics, checkpoint PODs) and the
# CXN* C ABI are rebuilt with -fsanitize=address,undefined into cxxnet_amd/_native_asan and the
# suite runs against them.  Host only: GPU ASan is not available on this pool.
set -o pipefail
cd "$(dirname "$0")/.."
python -m cxxnet_amd.build --asan || exit 1
export CXXNET_NATIVE_DIR=$PWD/cxxnet_amd/_native_asan
export LD_PRELOAD="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libubsan.so)"
# leak checking off: CPython and torch keep allocations alive until exit by design
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
python -m pytest tests/ -x -q -m "not gpu" -p no:cacheprovider "$@"
