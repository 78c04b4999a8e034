// aqz_hostzstd.hh -- the zstd codecs of Chunk::compress_and_take_buffer
// (chunk.cpp:78-106): blosc1 frames with the zstd codec
// (zarr::compress_in_place -> blosc_compress_ctx(..., "zstd", ...),
// zarr.common.cpp:106-140) and plain zstd frames (ZSTD_compress at the
// settings' level, zarr.common.cpp:142-166).
//
// Split of the work: the GPU shuffles (byte or bit) every block of a
// resident chunk layer in HBM and one D2H brings the shuffled layer to
// pinned host memory; a pool of host threads runs zstd, one task per chunk
// with data, and the frames leave in shard-major order.  zstd comes from the
// system's libzstd.so.1, loaded at first use (dlopen: the library keeps no
// hard dependency; without it these codecs report
// AQZ_STATUS_NOT_YET_IMPLEMENTED).
//
// Parity is at the decoded level, as for blosc-lz4: any blosc1 / zstd
// decoder returns the chunk bytes exactly.  The blosc frames differ from
// c-blosc's in the block size (kZstdBlock; the header records it) and in not
// splitting blocks into typesize streams (the header's "don't split" flag
// says so; zstd matches across the byte planes of a shuffled block).
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace aqz {

// blosc-zstd block size (bytes, rounded down to whole pixels)
constexpr uint32_t kZstdBlock = 256 * 1024;

// libzstd.so.1, resolved once.
struct ZstdLib
{
    size_t (*compress_bound)(size_t) = nullptr;
    unsigned (*is_error)(size_t) = nullptr;
    void* (*create_cctx)() = nullptr;
    size_t (*free_cctx)(void*) = nullptr;
    size_t (*compress_cctx)(void*, void*, size_t, const void*, size_t, int) = nullptr;
    int (*max_clevel)() = nullptr;
    bool ok = false;
    static const ZstdLib& get();
};

// A fixed pool of host worker threads running queued tasks.
class TaskPool
{
  public:
    // cpus: pin every worker there (empty = no pinning)
    explicit TaskPool(unsigned workers, std::vector<int> cpus = {});
    ~TaskPool();
    TaskPool(const TaskPool&) = delete;
    TaskPool& operator=(const TaskPool&) = delete;
    void push(std::function<void()> task);
    unsigned workers() const { return unsigned(threads_.size()); }

  private:
    void run();
    std::vector<std::thread> threads_;
    std::deque<std::function<void()>> q_;
    std::mutex mu_;
    std::condition_variable cv_;
    bool stop_ = false;
};

// The blosc1 block geometry of a blosc-zstd frame.
struct ZstdBloscGeom
{
    uint32_t nbytes, typesize, blocksize, nblocks;
};
ZstdBloscGeom make_zstd_blosc_geom(uint32_t nbytes, uint32_t typesize);

// One layer's host compression.  Inputs: the chunks (packed at bpc; for
// blosc-zstd with a shuffle, every block already shuffled on the device)
// and has_data bytes, both in pinned memory the D2H fills.  Outputs: one
// frame per chunk in its own region of `tmp`, its size in `fsize` (0 = no
// data: skipped) and the frame offsets in output order.
struct HostLayerJob
{
    int32_t codec = 0;   // 2 blosc-zstd, 3 zstd
    int32_t clevel = 1;
    int32_t shuffle = 0; // blosc: 0 none, 1 byte, 2 bit
    uint32_t typesize = 1;
    uint64_t bpc = 0;
    uint32_t n_chunks = 0;
    const uint8_t* chunks = nullptr;
    const uint8_t* has_data = nullptr;
    std::vector<uint32_t> order;   // output position -> chunk
    uint64_t frame_cap = 0;        // bytes of one chunk's region in tmp
    std::vector<uint8_t> tmp;
    std::vector<uint64_t> fsize;
    std::vector<uint64_t> offsets; // n_chunks + 1, output order

    std::atomic<uint32_t> remaining{ 0 };
    std::mutex mu;
    std::condition_variable cv;
    bool done = true;
    int32_t status = 0; // 0 ok, else an AQZ status code
    void wait();
    bool finished()
    {
        std::lock_guard<std::mutex> lk(mu);
        return done;
    }
    // frames in output order -> dst (offsets[n_chunks] bytes)
    void gather(uint8_t* dst) const;
};

// Compresses every chunk with data on the pool; `ready` (run by a pool
// worker first) waits for the D2H that fills the inputs.  Returns at once;
// HostLayerJob::wait() returns when the frames and offsets are complete.
void host_zstd_compress(TaskPool& pool, const std::shared_ptr<HostLayerJob>& job,
                        std::function<void()> ready);

} // namespace aqz
