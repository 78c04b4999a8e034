#!/usr/bin/env bash
# binding_mutants.sh -- does tests/test_gpu_binding_exec.py catch a broken
# binding?  Builds oracle/_ref/mut/binding_exec_<name> from mutated copies of
# integration/multiscale.array.gpu.cpp (one deliberate bug each), then, on
# the GPU box (`bash tools/binding_mutants.sh run`), runs the test file
# against each with BINDING_EXEC=<mutant>: every mutant must FAIL.
#   bash tools/binding_mutants.sh build     (here: needs /root/reference)
#   bash tools/binding_mutants.sh run       (GPU box: prints one line a mutant)
set -euo pipefail
cd "$(dirname "$0")/.."
REF=/root/reference
OUT=oracle/_ref/mut
declare -A MUT=(
  # the frame id the reference's counters carry is not mirrored
  [last_id]='s/        last_successful_frame_id_ = ledger_.last_successful_frame_id;//'
  # total bytes not mirrored: should_rollover_ reads a stale frame count
  [total_bytes]='s/        total_bytes_written_ = ledger_.total_bytes_written;//'
  # rollover without the zarr.json rewrite
  [no_metadata]='s/        CHECK(write_metadata_());//'
  # chunk bytes to the neighbouring internal index
  [internal]='s/ok = shard->write_chunk(internal_idx, buffer);/ok = shard->write_chunk(internal_idx ^ 1u, buffer);/'
  # no frame-order check
  [order]='s/        if (frame_id != handoff_->frames_accepted())/        if (false)/'
  # the lease released before the copy out of the pinned buffer
  [lease]='s/                const std::vector<uint8_t> buffer(bytes, bytes + nbytes);/                lease.release(); std::this_thread::sleep_for(std::chrono::milliseconds(2)); const std::vector<uint8_t> buffer(bytes, bytes + nbytes);/'
)
if [ "${1:-build}" = build ]; then
  mkdir -p "$OUT/obj" "$OUT/src"
  SRCS="$REF/src/streaming/downsampler.cpp $REF/src/streaming/array.dimensions.cpp
        $REF/src/streaming/zarr.common.cpp $REF/src/streaming/thread.pool.cpp
        $REF/src/streaming/blosc.compression.params.cpp $REF/src/logger/logger.cpp"
  INC="-Itests/native -Iinclude -Ioracle/_ref/include -I$REF/include -I$REF/src/streaming
       -I$REF/src/logger -idirafter /opt/conda/include"
  for s in $SRCS; do
    o="$OUT/obj/$(basename "$s" .cpp).o"
    [ -f "$o" ] || g++ -O2 -std=c++20 -ffp-contract=off -pthread -w -c $INC "$s" -o "$o" &
  done
  wait
  for m in "${!MUT[@]}"; do
    sed "${MUT[$m]}" integration/multiscale.array.gpu.cpp > "$OUT/src/multiscale.array.gpu.cpp"
    if cmp -s "$OUT/src/multiscale.array.gpu.cpp" integration/multiscale.array.gpu.cpp; then
      echo "mutant $m: pattern not found" >&2; exit 1
    fi
    cp integration/aqz_handoff.hh "$OUT/src/"
    g++ -O2 -std=c++20 -ffp-contract=off -pthread -w -o "$OUT/binding_exec_$m" \
      tests/native/binding_exec.cpp "$OUT"/obj/*.o -I"$OUT/src" $INC \
      -Loracle/_ref/lib -lblosc -lzstd -Lacquire-zarr_amd -laqz_gpu \
      -Wl,-rpath,'$ORIGIN/../lib' -Wl,-rpath,'$ORIGIN/../../../acquire-zarr_amd' \
      -Wl,-rpath,/opt/rocm/lib
    echo "built $OUT/binding_exec_$m"
  done
  rm -rf "$OUT/src"
else
  for m in $(ls "$OUT" | sed -n 's/^binding_exec_//p'); do
    if BINDING_EXEC="$OUT/binding_exec_$m" timeout -k 10 300 python -u -m pytest -x -q \
         --timeout 120 --timeout-method thread tests/test_gpu_binding_exec.py \
         > "gpurun_out/mutant_$m.log" 2>&1; then
      echo "{\"mutant\": \"$m\", \"caught\": false}"
    else
      rc=$?
      # a time limit is not a catch: stop here
      [ $rc -eq 124 ] || [ $rc -eq 137 ] && { echo "mutant $m: time limit"; exit 1; }
      echo "{\"mutant\": \"$m\", \"caught\": true, \"first_failure\": \"$(grep -m1 -o 'FAILED [^ ]*' "gpurun_out/mutant_$m.log" || true)\"}"
    fi
  done
fi
