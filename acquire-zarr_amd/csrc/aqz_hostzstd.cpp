// aqz_hostzstd.cpp -- see aqz_hostzstd.hh.
#include "aqz_hostzstd.hh"

#include "aqz_copy.hh"

#include <dlfcn.h>

#include <algorithm>
#include <cstring>

namespace aqz {

const ZstdLib&
ZstdLib::get()
{
    static const ZstdLib lib = [] {
        ZstdLib z;
        void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h)
            return z;
        z.compress_bound = reinterpret_cast<size_t (*)(size_t)>(dlsym(h, "ZSTD_compressBound"));
        z.is_error = reinterpret_cast<unsigned (*)(size_t)>(dlsym(h, "ZSTD_isError"));
        z.create_cctx = reinterpret_cast<void* (*)()>(dlsym(h, "ZSTD_createCCtx"));
        z.free_cctx = reinterpret_cast<size_t (*)(void*)>(dlsym(h, "ZSTD_freeCCtx"));
        z.compress_cctx = reinterpret_cast<size_t (*)(void*, void*, size_t, const void*,
                                                      size_t, int)>(
          dlsym(h, "ZSTD_compressCCtx"));
        z.max_clevel = reinterpret_cast<int (*)()>(dlsym(h, "ZSTD_maxCLevel"));
        z.ok = z.compress_bound && z.is_error && z.create_cctx && z.free_cctx &&
               z.compress_cctx && z.max_clevel;
        return z;
    }();
    return lib;
}

// ---- task pool ---------------------------------------------------------------
TaskPool::TaskPool(unsigned workers, std::vector<int> cpus)
{
    for (unsigned i = 0; i < std::max(1u, workers); ++i)
        threads_.emplace_back([this, cpus] {
            pin_current_thread(cpus);
            run();
        });
}

TaskPool::~TaskPool()
{
    {
        std::lock_guard<std::mutex> g(mu_);
        stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : threads_)
        t.join();
}

void
TaskPool::push(std::function<void()> task)
{
    {
        std::lock_guard<std::mutex> g(mu_);
        q_.push_back(std::move(task));
    }
    cv_.notify_one();
}

void
TaskPool::run()
{
    for (;;) {
        std::function<void()> t;
        {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
            if (q_.empty())
                return; // stop_ and drained
            t = std::move(q_.front());
            q_.pop_front();
        }
        t();
    }
}

// ---- frames ------------------------------------------------------------------
ZstdBloscGeom
make_zstd_blosc_geom(uint32_t nbytes, uint32_t typesize)
{
    ZstdBloscGeom g{ nbytes, typesize, 0, 0 };
    uint32_t bs = std::min(kZstdBlock, nbytes);
    bs -= bs % typesize;
    if (bs == 0)
        bs = nbytes;
    g.blocksize = bs;
    g.nblocks = bs ? (nbytes + bs - 1) / bs : 0;
    return g;
}

namespace {

void
put32(uint8_t* d, uint32_t v)
{
    d[0] = uint8_t(v);
    d[1] = uint8_t(v >> 8);
    d[2] = uint8_t(v >> 16);
    d[3] = uint8_t(v >> 24);
}

// Inverse of the device's block shuffle (c-blosc 1.x byte shuffle /
// bitshuffle of one block), for a chunk stored as a memcpyed frame.
void
unshuffle_block(int sh, uint32_t ts, const uint8_t* src, uint8_t* dst, uint32_t n)
{
    const uint32_t ne = n / ts;
    if (sh == 1 && ts > 1) {
        for (uint32_t j = 0; j < ts; ++j)
            for (uint32_t i = 0; i < ne; ++i)
                dst[i * ts + j] = src[j * ne + i];
        std::memcpy(dst + ne * ts, src + ne * ts, n - ne * ts);
    } else if (sh == 2 && ne % 8 == 0 && ne * ts == n) {
        const uint32_t row = ne / 8;
        std::memset(dst, 0, n);
        for (uint32_t r = 0; r < 8 * ts; ++r) {
            const uint32_t j = r >> 3, b = r & 7u;
            for (uint32_t m = 0; m < row; ++m) {
                const uint8_t v = src[r * row + m];
                for (uint32_t k = 0; k < 8; ++k)
                    dst[(8 * m + k) * ts + j] |= uint8_t(((v >> k) & 1u) << b);
            }
        }
    } else {
        std::memcpy(dst, src, n);
    }
}

// c-blosc 1.x's zstd level for a blosc clevel (zstd_wrap_compress): it
// reassigns clevel = clevel < 9 ? 2 * clevel - 1 : ZSTD_maxCLevel() and only
// then tests `clevel == 8`, which the odd or maximal value never is -- so the
// effective map is 2c - 1 for c < 9 and the maximum level for 9.
int
blosc_zstd_level(const ZstdLib& z, int clevel)
{
    return clevel < 9 ? clevel * 2 - 1 : z.max_clevel();
}

struct CCtx
{
    void* p = nullptr;
    ~CCtx()
    {
        if (p)
            ZstdLib::get().free_cctx(p);
    }
};

void*
thread_cctx()
{
    thread_local CCtx c;
    if (!c.p)
        c.p = ZstdLib::get().create_cctx();
    return c.p;
}

// One chunk -> its frame in job.tmp; returns the frame bytes (0 on error).
uint64_t
compress_chunk(HostLayerJob& job, uint32_t c)
{
    const ZstdLib& z = ZstdLib::get();
    const uint8_t* src = job.chunks + uint64_t(c) * job.bpc;
    uint8_t* out = job.tmp.data() + uint64_t(c) * job.frame_cap;
    void* cctx = thread_cctx();
    if (!cctx)
        return 0;
    if (job.codec == 3) {
        const size_t n = z.compress_cctx(cctx, out, job.frame_cap, src, job.bpc, job.clevel);
        return z.is_error(n) ? 0 : n;
    }
    // blosc1 frame: header, block starts, one (csize, bytes) record per block
    const ZstdBloscGeom g = make_zstd_blosc_geom(uint32_t(job.bpc), job.typesize);
    const int level = blosc_zstd_level(z, job.clevel);
    uint64_t pos = 16 + 4ull * g.nblocks;
    bool memcpyed = job.clevel == 0;
    for (uint32_t j = 0; j < g.nblocks && !memcpyed; ++j) {
        const uint32_t len = std::min(g.blocksize, g.nbytes - j * g.blocksize);
        put32(out + 16 + 4 * j, uint32_t(pos));
        uint8_t* rec = out + pos + 4;
        const uint64_t room = job.frame_cap - pos - 4;
        size_t n = z.compress_cctx(cctx, rec, room, src + uint64_t(j) * g.blocksize, len, level);
        if (z.is_error(n) || n >= len) { // stored raw: csize == block bytes
            std::memcpy(rec, src + uint64_t(j) * g.blocksize, len);
            n = len;
        }
        put32(out + pos, uint32_t(n));
        pos += 4 + n;
        if (pos > uint64_t(g.nbytes) + 16)
            memcpyed = true; // blosc's rule: never larger than a plain copy
    }
    if (memcpyed) {
        for (uint32_t j = 0; j < g.nblocks; ++j) {
            const uint32_t len = std::min(g.blocksize, g.nbytes - j * g.blocksize);
            unshuffle_block(job.shuffle, job.typesize, src + uint64_t(j) * g.blocksize,
                            out + 16 + uint64_t(j) * g.blocksize, len);
        }
        pos = uint64_t(g.nbytes) + 16;
    }
    out[0] = 2; // BLOSC_VERSION_FORMAT
    out[1] = 1; // BLOSC_ZSTD_VERSION_FORMAT
    out[2] = uint8_t(4u << 5 | 0x10u | (job.shuffle == 1 ? 0x1u : 0u) |
                     (job.shuffle == 2 ? 0x4u : 0u) | (memcpyed ? 0x2u : 0u));
    out[3] = uint8_t(job.typesize);
    put32(out + 4, g.nbytes);
    put32(out + 8, g.blocksize);
    put32(out + 12, uint32_t(pos));
    return pos;
}

void
finish(HostLayerJob& job)
{
    uint64_t at = 0;
    for (uint32_t i = 0; i < job.n_chunks; ++i) {
        job.offsets[i] = at;
        at += job.fsize[job.order[i]];
    }
    job.offsets[job.n_chunks] = at;
    std::lock_guard<std::mutex> g(job.mu);
    job.done = true;
    job.cv.notify_all();
}

} // namespace

void
HostLayerJob::wait()
{
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
}

void
HostLayerJob::gather(uint8_t* dst) const
{
    for (uint32_t i = 0; i < n_chunks; ++i) {
        const uint32_t c = order[i];
        if (fsize[c])
            std::memcpy(dst + offsets[i], tmp.data() + uint64_t(c) * frame_cap, fsize[c]);
    }
}

void
host_zstd_compress(TaskPool& pool, const std::shared_ptr<HostLayerJob>& job,
                   std::function<void()> ready)
{
    {
        std::lock_guard<std::mutex> g(job->mu);
        job->done = false;
        job->status = 0;
    }
    job->fsize.assign(job->n_chunks, 0);
    job->offsets.assign(size_t(job->n_chunks) + 1, 0);
    pool.push([&pool, job, ready = std::move(ready)] {
        ready();
        std::vector<uint32_t> todo;
        for (uint32_t c = 0; c < job->n_chunks; ++c)
            if (job->has_data[c])
                todo.push_back(c);
        if (todo.empty()) {
            finish(*job);
            return;
        }
        job->remaining.store(uint32_t(todo.size()));
        for (uint32_t c : todo)
            pool.push([job, c] {
                const uint64_t n = compress_chunk(*job, c);
                if (n == 0) {
                    std::lock_guard<std::mutex> g(job->mu);
                    job->status = 8; // ZarrStatusCode_CompressionError
                }
                job->fsize[c] = n;
                if (job->remaining.fetch_sub(1) == 1)
                    finish(*job);
            });
    });
}

} // namespace aqz
