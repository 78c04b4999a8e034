// aqz_hostsplit.hh -- the level-0 tile split on the host, for a raw
// hand-off.
//
// The level-0 split is a pure rearrangement of the frame's bytes.  When the
// frames start in host memory and the chunk layers go back to host memory
// raw, splitting level 0 on the device costs PCIe twice (H2D of the frame,
// D2H of its chunks) for bytes the host already holds; splitting it where
// the bytes are leaves the device the pyramid (H2D 1x, D2H 1/3x).  The loop
// is Array::write_frame_to_chunks_ (array.cpp:537-619) with
// Chunk::write_tile_rows (chunk.cpp:17-58): tile t of a frame goes to chunk
// t + tile_group_offset(frame), its rows at chunk_internal_offset(frame) +
// r * tile_cols * bpp, ragged padding left as it is (zero), has_data set
// when a copied byte is nonzero.  Split by rows so several threads share a
// frame (the reference splits by tiles under OpenMP, array.cpp:575).
#pragma once

#include "aqz_geometry.hh"

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace aqz {

// Where one frame's rows go (storage order = acquisition order: no XY
// transposition; ArrayDimensions::needs_xy_transposition() is refused).
struct SplitGeom
{
    uint32_t W = 0, H = 0, tw = 0, th = 0, ntx = 0;
    uint32_t bpp = 0;
    uint64_t bpc = 0;      // bytes per chunk
    uint32_t group = 0;    // chunk of tile 0 (tile_group_offset)
    uint64_t internal = 0; // byte offset of the frame inside its chunks
};

// frame_id: the level-0 frame id in acquisition order (frames_written_ of
// the array); transposed to storage order here as array.cpp:557-561 does.
SplitGeom split_geom(const ArrayDimensions& ad, uint64_t frame_id);

// Rows [row_begin, row_end) of one frame into the packed chunks
// [chunk0, chunk0 + n_chunks) at dst (chunk c at (c - chunk0) * bpc).
// has_data[c - chunk0] becomes 1 once a copied byte of chunk c is nonzero
// (never cleared here).  frame_copy (optional): the same rows are also
// copied there (a frame-sized buffer; the hand-off's pinned batch), in the
// same pass.  Threads may split disjoint rows of the same frame into the
// same chunks at once.  Stores are streaming (nontemporal) and fenced before
// return.  Throws Error(1) when a tile's chunk lies outside the range.
void split_rows(const SplitGeom& g, const uint8_t* frame, uint32_t row_begin,
                uint32_t row_end, uint8_t* dst, uint32_t chunk0, uint32_t n_chunks,
                uint8_t* has_data, uint8_t* frame_copy = nullptr);

// A fixed set of worker threads (pinned to `cpus`) plus the caller running
// n tasks of fn(i), i in [0, n); returns when all have run.  The first
// exception a task throws is rethrown to the caller.
class SplitPool
{
  public:
    explicit SplitPool(unsigned workers, std::vector<int> cpus = {});
    ~SplitPool();
    SplitPool(const SplitPool&) = delete;
    SplitPool& operator=(const SplitPool&) = delete;
    void run(size_t n, const std::function<void(size_t)>& fn);
    unsigned threads() const { return unsigned(threads_.size()) + 1; }

  private:
    void work();
    void drain();

    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable go_, done_;
    uint64_t gen_ = 0;
    unsigned busy_ = 0;
    bool stop_ = false;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0, next_ = 0;
    std::exception_ptr err_;
};

} // namespace aqz
