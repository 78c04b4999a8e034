#include "aqz_hostsplit.hh"
#include "aqz_copy.hh"

#include <immintrin.h>

#include <atomic>
#include <cstdlib>
#include <cstring>

namespace aqz {

SplitGeom
split_geom(const ArrayDimensions& ad, uint64_t frame_id)
{
    if (ad.needs_xy_transposition())
        throw Error(9, "the host split takes storage rows = acquisition rows "
                       "(no XY-transposed storage order)");
    SplitGeom g;
    const Dim& x = ad.width_dim();
    const Dim& y = ad.height_dim();
    g.W = x.array_size_px;
    g.H = y.array_size_px;
    g.tw = x.chunk_size_px;
    g.th = y.chunk_size_px;
    if (g.tw == 0 || g.th == 0)
        throw Error(9, "zero tile size");
    g.ntx = parts_along(g.W, g.tw);
    g.bpp = uint32_t(bytes_of_type(ad.dtype()));
    g.bpc = ad.bytes_per_chunk();
    // array.cpp:557-566: the storage-order frame id, then its chunk group
    // and its offset inside every chunk of the group
    const uint64_t fid = ad.transpose_frame_id(frame_id);
    g.group = ad.tile_group_offset(fid);
    g.internal = ad.chunk_internal_offset(fid);
    return g;
}

namespace {

// any nonzero byte in [p, p + n) (Chunk::write_tile_rows' any_of, chunk.cpp:
// 41-52, over the bytes just copied)
bool
any_nonzero(const uint8_t* p, size_t n)
{
    size_t i = 0;
    for (; i + 32 <= n; i += 32) {
        uint64_t a, b, c, d;
        std::memcpy(&a, p + i, 8);
        std::memcpy(&b, p + i + 8, 8);
        std::memcpy(&c, p + i + 16, 8);
        std::memcpy(&d, p + i + 24, 8);
        if (a | b | c | d)
            return true;
    }
    for (; i < n; ++i)
        if (p[i])
            return true;
    return false;
}

// Streaming (nontemporal) copy: the split's destinations -- a chunk layer
// of hundreds of MiB, a pinned batch the DMA reads -- are not read back by
// this core soon, so the stores skip the read-for-ownership and the caches
// (tools/split_probe.cpp on the GPU host: the split 1.4-2.4x, copy + split
// 1.2-2.7x the plain memcpy rate).  The caller fences (_mm_sfence) before
// another thread reads the bytes.
__attribute__((target("avx2"))) void
stream_copy_avx2(uint8_t* d, const uint8_t* s, size_t n)
{
    size_t i = 0;
    // head: plain stores up to the first 32-byte boundary of d
    const size_t head = std::min(n, size_t((32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31));
    std::memcpy(d, s, head);
    i = head;
    for (; i + 128 <= n; i += 128) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
        const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
        const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
    }
    for (; i + 32 <= n; i += 32)
        _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i),
                            _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i)));
    std::memcpy(d + i, s + i, n - i);
}

// AQZ_SPLIT_NT=0: plain memcpy stores (A/B)
const bool kStream = __builtin_cpu_supports("avx2") &&
                     !(std::getenv("AQZ_SPLIT_NT") && std::atoi(std::getenv("AQZ_SPLIT_NT")) == 0);

inline void
stream_copy(uint8_t* d, const uint8_t* s, size_t n)
{
    if (kStream && n >= 128)
        stream_copy_avx2(d, s, n);
    else
        std::memcpy(d, s, n);
}

} // namespace

void
split_rows(const SplitGeom& g, const uint8_t* frame, uint32_t row_begin, uint32_t row_end,
           uint8_t* dst, uint32_t chunk0, uint32_t n_chunks, uint8_t* has_data,
           uint8_t* frame_copy)
{
    row_end = std::min(row_end, g.H);
    if (row_begin >= row_end)
        return;
    const size_t src_stride = size_t(g.W) * g.bpp;
    const size_t tile_row = size_t(g.tw) * g.bpp;
    // every tile row the rows touch must map into [chunk0, chunk0 + n_chunks)
    const uint64_t c_first = uint64_t(g.group) + uint64_t(row_begin / g.th) * g.ntx;
    const uint64_t c_last = uint64_t(g.group) + uint64_t((row_end - 1) / g.th) * g.ntx + g.ntx;
    if (c_first < chunk0 || c_last > uint64_t(chunk0) + n_chunks)
        throw Error(1, "the frame's tiles lie outside the destination's chunks");
    // blocks of 16 rows (64 KiB of a 2048-px u16 frame): the block is copied
    // (frame_copy) and then split while its rows are in this core's cache
    constexpr uint32_t kBlock = 16;
    for (uint32_t r0 = row_begin; r0 < row_end; r0 += kBlock) {
        const uint32_t r1 = std::min(row_end, r0 + kBlock);
        if (frame_copy)
            stream_copy(frame_copy + size_t(r0) * src_stride, frame + size_t(r0) * src_stride,
                        size_t(r1 - r0) * src_stride);
        for (uint32_t r = r0; r < r1; ++r) {
            const uint32_t ty = r / g.th;
            const uint64_t dst_row = g.internal + uint64_t(r % g.th) * tile_row;
            const uint8_t* src = frame + size_t(r) * src_stride;
            const uint32_t c_row = g.group + ty * g.ntx - chunk0;
            for (uint32_t tx = 0; tx < g.ntx; ++tx) {
                const uint32_t col = tx * g.tw;
                const size_t n = size_t(std::min(g.tw, g.W - col)) * g.bpp;
                const uint32_t c = c_row + tx;
                const uint8_t* s = src + size_t(col) * g.bpp;
                stream_copy(dst + uint64_t(c) * g.bpc + dst_row, s, n);
                // has_data: a relaxed byte flag (threads of disjoint rows may
                // set the same chunk's); once set, the scan is skipped
                std::atomic_ref<uint8_t> h(has_data[c]);
                if (!h.load(std::memory_order_relaxed) && any_nonzero(s, n))
                    h.store(1, std::memory_order_relaxed);
            }
        }
    }
    _mm_sfence(); // the streaming stores are visible before the caller signals
}

SplitPool::SplitPool(unsigned workers, std::vector<int> cpus)
{
    for (unsigned i = 0; i < workers; ++i)
        threads_.emplace_back([this, cpus] {
            pin_current_thread(cpus);
            work();
        });
}

SplitPool::~SplitPool()
{
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    go_.notify_all();
    for (auto& t : threads_)
        t.join();
}

// take tasks until none is left (the lock is dropped while one runs)
void
SplitPool::drain()
{
    std::unique_lock<std::mutex> lk(mu_);
    while (next_ < n_) {
        const size_t i = next_++;
        lk.unlock();
        try {
            (*fn_)(i);
        } catch (...) {
            lk.lock();
            if (!err_)
                err_ = std::current_exception();
            next_ = n_; // no new tasks after a failure
            continue;
        }
        lk.lock();
    }
}

void
SplitPool::work()
{
    uint64_t seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu_);
            go_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_)
                return;
            seen = gen_;
        }
        drain();
        std::lock_guard<std::mutex> g(mu_);
        if (--busy_ == 0)
            done_.notify_one();
    }
}

void
SplitPool::run(size_t n, const std::function<void(size_t)>& fn)
{
    if (n == 0)
        return;
    if (threads_.empty() || n == 1) {
        for (size_t i = 0; i < n; ++i)
            fn(i);
        return;
    }
    {
        std::lock_guard<std::mutex> g(mu_);
        fn_ = &fn;
        n_ = n;
        next_ = 0;
        err_ = nullptr;
        busy_ = unsigned(threads_.size());
        ++gen_;
    }
    go_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
    if (err_)
        std::rethrow_exception(err_);
}

} // namespace aqz
