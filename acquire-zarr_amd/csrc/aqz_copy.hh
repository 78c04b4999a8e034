// aqz_copy.hh -- parallel host memcpy for the ingestion path.
//
// ZarrStream_append copies the caller's frame before it returns
// (src/streaming/frame.queue.cpp:37-39); here that one copy lands directly in
// the stage's pinned staging buffer, from which the H2D DMA reads.  A single
// thread's memcpy (~10 GB/s) would cap the pipeline well below PCIe, so the
// copy is split over a few persistent workers plus the calling thread.
#pragma once

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <thread>
#include <vector>

namespace aqz {

class CopyPool
{
  public:
    explicit CopyPool(unsigned workers);
    ~CopyPool();
    CopyPool(const CopyPool&) = delete;
    CopyPool& operator=(const CopyPool&) = delete;

    // dst[0, n) = src[0, n); returns when every piece is done
    void copy(void* dst, const void* src, size_t n);
    unsigned workers() const { return unsigned(threads_.size()); }

  private:
    void run(unsigned id);
    void piece(size_t i);

    std::vector<std::thread> threads_;
    std::mutex mu_;
    std::condition_variable go_, done_;
    uint64_t gen_ = 0;
    unsigned pending_ = 0;
    bool stop_ = false;
    uint8_t* dst_ = nullptr;
    const uint8_t* src_ = nullptr;
    size_t n_ = 0, pieces_ = 0;
};

} // namespace aqz
