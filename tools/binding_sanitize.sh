#!/usr/bin/env bash
# binding_sanitize.sh -- the binding harness (oracle/_ref/binding_exec) built
# with a host sanitizer, run by tests/test_gpu_binding_exec.py on the GPU box.
# Host code only: the binding, the hand-off (consumer, copy threads, lease
# counts), the reference's ThreadPool and the test doubles are instrumented;
# libaqz_gpu.so and the HIP runtime are not (no GPU sanitizer).
#   bash tools/binding_sanitize.sh build        (here: needs /root/reference)
#   bash tools/binding_sanitize.sh run [thread|address]   (GPU box)
set -euo pipefail
cd "$(dirname "$0")/.."
REF=/root/reference
OUT=oracle/_ref/san
if [ "${1:-build}" = build ]; then
  mkdir -p "$OUT"
  SRCS="$REF/src/streaming/downsampler.cpp $REF/src/streaming/array.dimensions.cpp
        $REF/src/streaming/zarr.common.cpp $REF/src/streaming/thread.pool.cpp
        $REF/src/streaming/blosc.compression.params.cpp $REF/src/logger/logger.cpp"
  INC="-Itests/native -Iinclude -Iintegration -Ioracle/_ref/include -I$REF/include
       -I$REF/src/streaming -I$REF/src/logger -idirafter /opt/conda/include"
  for san in thread address; do
    # non-PIE: gcc's TSan rejects a PIE mapped high by this kernel's ASLR
    g++ -O1 -g -fno-omit-frame-pointer -fsanitize=$san -no-pie -std=c++20 -ffp-contract=off -pthread -w \
      -o "$OUT/binding_exec_$san" tests/native/binding_exec.cpp $SRCS $INC \
      -Loracle/_ref/lib -lblosc -lzstd -Lacquire-zarr_amd -laqz_gpu \
      -Wl,-rpath,'$ORIGIN/../lib' -Wl,-rpath,'$ORIGIN/../../../acquire-zarr_amd' \
      -Wl,-rpath,/opt/rocm/lib &
  done
  wait
  ls -la "$OUT"
else
  san=${2:-thread}
  export TSAN_OPTIONS="halt_on_error=1 exitcode=66 second_deadlock_stack=1 suppressions=$PWD/tools/tsan.supp"
  export ASAN_OPTIONS="halt_on_error=1 exitcode=66 detect_leaks=1 protect_shadow_gap=0"
  export LSAN_OPTIONS="exitcode=66 suppressions=$PWD/tools/lsan.supp"
  # ASLR off for the harness (setarch -R execs it before it touches the
  # GPU): gcc's TSan rejects libraries mapped below its high-memory range
  # a stalled harness writes where it is every 10 s (and so keeps the run
  # from looking silent until pytest's own limit ends it)
  export BINDING_EXEC_PROGRESS="$PWD/gpurun_out/binding_progress_$san.txt"
  BINDING_EXEC_PREFIX="setarch $(uname -m) -R" BINDING_EXEC="$OUT/binding_exec_$san" timeout -k 10 900 python3 -u -m pytest -x -v \
    --timeout 300 --timeout-method thread tests/test_gpu_binding_exec.py ${3:+-k "$3"} \
    > "gpurun_out/binding_$san.log" 2>&1
fi
