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

// NUMA placement of the host threads that feed one GPU (one
// host thread group per GPU, pinned to the GPU's NUMA node).  The CPUs of
// the NUMA node of PCI device `bus_id` ("dddd:bb:dd.f"), intersected with
// this process's affinity; empty when unknown (no sysfs entry, node -1).
std::vector<int> numa_cpus_for_pci(const char* bus_id, int* node = nullptr);
// Pins the calling thread to `cpus` (no-op when empty).
void pin_current_thread(const std::vector<int>& cpus);

class CopyPool
{
  public:
    explicit CopyPool(unsigned workers, std::vector<int> cpus = {});
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
