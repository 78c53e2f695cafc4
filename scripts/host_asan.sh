#!/bin/bash
# CPU AddressSanitizer/UBSan run of the host-native C++ library
# (csrc/host/*.cpp): builds build/_sq_host_asan.so and runs the host-native
# test modules against it (the in-tree _sq_host.so is left untouched).
set -e
cd "$(dirname "$0")/.."
lib=$(python -m sq_learn_amd._build --host-sanitize address,undefined | tail -1)
export SQ_HOST_LIB="$lib"
# sanitizer runtimes appended to any preload already in the environment
export LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD:}$(g++ -print-file-name=libasan.so):$(g++ -print-file-name=libubsan.so)"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:verify_asan_link_order=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
if [ $# -eq 0 ]; then
  set -- tests/test_host_native_cpu.py tests/test_tree_ensemble_cpu.py tests/test_sgd_cpu.py \
         tests/test_svm_libsvm_cpu.py tests/test_structured_ward_cpu.py tests/test_linear_model_cpu.py \
         tests/test_tron_cpu.py tests/test_manifold_cpu.py
fi
# -s: sanitizer reports go to the terminal, not into pytest's fd capture
exec python -m pytest -q -x -s -m "not gpu" -p no:xdist "$@"
