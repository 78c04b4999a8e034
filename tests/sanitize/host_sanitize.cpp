// Host-side sanitizer driver (SURVEY §5 "Race detection / sanitizers").
// Built with -fsanitize=address,undefined by tests/test_sanitize_cpu.py
// together with the product's pure-host sources (aqz_geometry.cpp: the
// ArrayDimensions / level-rule restatement that drives kernel addressing;
// aqz_copy.cpp: the staging copy pool; aqz_hostsplit.cpp: the host split of
// level 0 and its pool; aqz_hostzstd.cpp: the host zstd pool and frame
// writer) and the CPU oracle (oracle/aqz_oracle.c,
// aqz_codec_oracle.c).  It drives them hard -- random geometries, a copy pool
// under concurrent use, host zstd jobs from several threads -- and
// cross-checks product against oracle, so ASan/UBSan see every path.  Exit
// status 0 = clean (the sanitizers abort on the first report).
#include "aqz_copy.hh"
#include "aqz_geometry.hh"
#include "aqz_hostsplit.hh"
#include "aqz_hostzstd.hh"

extern "C" {
#include "aqz_oracle.h"
}

#include <dlfcn.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <random>
#include <thread>
#include <vector>

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

using namespace aqz;

static std::vector<Dim>
random_dims(std::mt19937& rng)
{
    auto r = [&](int lo, int hi) { return int(rng() % uint32_t(hi - lo + 1)) + lo; };
    const int nd = r(3, 5);
    std::vector<Dim> d;
    d.push_back(Dim{ kTime, uint32_t(r(0, 2) * 4), uint32_t(r(1, 5)), uint32_t(r(1, 2)) });
    for (int i = 0; i < nd - 3; ++i)
        d.push_back(Dim{ r(0, 2), uint32_t(r(1, 6)), uint32_t(r(1, 3)), uint32_t(r(1, 2)) });
    d.push_back(Dim{ kSpace, uint32_t(r(1, 80)), uint32_t(r(1, 11)), uint32_t(r(1, 2)) });
    d.push_back(Dim{ kSpace, uint32_t(r(1, 80)), uint32_t(r(1, 11)), uint32_t(r(1, 2)) });
    return d;
}

static void
geometry(std::mt19937& rng)
{
    for (int it = 0; it < 400; ++it) {
        const auto dims = random_dims(rng);
        const int dtype = int(rng() % 10);
        std::vector<or_dim> od;
        for (const Dim& x : dims)
            od.push_back(or_dim{ x.type, x.array_size_px, x.chunk_size_px, x.shard_size_chunks });
        const int n = int(od.size());
        ArrayDimensions a(dims, dtype);
        CHECK(a.bytes_per_chunk() == or_bytes_per_chunk(od.data(), n, dtype));
        CHECK(a.number_of_chunks_in_memory() == or_number_of_chunks_in_memory(od.data(), n));
        CHECK(a.frames_per_chunk_layer() == or_frames_per_chunk_layer(od.data(), n));
        for (uint64_t f = 0; f < 60; ++f) {
            CHECK(a.tile_group_offset(f) == or_tile_group_offset(od.data(), n, f));
            CHECK(a.chunk_internal_offset(f) == or_chunk_internal_offset(od.data(), n, dtype, f));
        }
        const uint32_t nc = std::min<uint32_t>(200, a.chunks_per_shard() * a.number_of_shards());
        for (uint32_t c = 0; c < nc; ++c) {
            CHECK(a.shard_index_for_chunk(c) == or_shard_index_for_chunk(od.data(), n, c));
            CHECK(a.shard_internal_index(c) == or_shard_internal_index(od.data(), n, c));
        }
        (void)a.supports_dim1_banding();
        (void)a.frames_per_dim1_band();
        const uint32_t ml = rng() % 4;
        const auto lv = make_pyramid_levels(a.dims(), ml);
        int nl = 0;
        std::vector<or_dim> out(size_t(OR_MAX_LEVELS) * n);
        CHECK(or_make_levels(od.data(), n, ml, &nl, out.data(), OR_MAX_LEVELS) == 0);
        CHECK(int(lv.size()) == nl);
        for (int l = 0; l < nl; ++l)
            for (int i = 0; i < n; ++i)
                CHECK(lv[l][i].array_size_px == out[size_t(l) * n + i].array_size_px);
    }
}

// the oracle's cascade on random frames (the checker itself under ASan)
static void
oracle_cascade(std::mt19937& rng)
{
    for (int it = 0; it < 40; ++it) {
        const uint32_t h = 1 + rng() % 70, w = 1 + rng() % 70;
        const int dtype = int(rng() % 10), method = int(rng() % 4);
        or_dim dims[4] = { { OR_TIME, 0, 1, 1 }, { OR_SPACE, 1 + rng() % 6, 1 + rng() % 3, 1 },
                           { OR_SPACE, h, 1 + rng() % 9, 1 }, { OR_SPACE, w, 1 + rng() % 9, 1 } };
        or_downsampler* ds = or_ds_create(dims, 4, dtype, method, 0);
        CHECK(ds);
        const size_t fb = size_t(h) * w * or_bytes_of_type(dtype);
        std::vector<uint8_t> frame(fb), out(fb);
        for (int f = 0; f < 12; ++f) {
            or_fill_splitmix(frame.data(), fb, rng());
            CHECK(or_ds_add_frame(ds, frame.data(), fb) == 0);
            for (int l = 1; l < or_ds_n_levels(ds); ++l) {
                size_t nb = 0;
                (void)or_ds_take_frame(ds, l, out.data(), out.size(), &nb);
            }
        }
        or_ds_destroy(ds);
        // the tile split of one frame into its layer
        const int n = 4;
        const uint64_t bpc = or_bytes_per_chunk(dims, n, dtype);
        const uint32_t nch = or_number_of_chunks_in_memory(dims, n);
        std::vector<uint8_t> layer(bpc * nch), has(nch);
        for (uint64_t fid = 0; fid < or_frames_per_chunk_layer(dims, n); ++fid)
            or_write_frame_to_chunks(dims, n, dtype, fid, frame.data(), layer.data(), has.data());
    }
}

static void
copy_pool()
{
    CopyPool pool(6);
    std::vector<std::thread> users;
    // the pool serves one caller at a time (the consumer thread); several
    // rounds of sizes around the split threshold
    for (size_t n : { size_t(1), size_t(4095), size_t(8) << 20, (size_t(8) << 20) + 7,
                      size_t(33) << 20 }) {
        std::vector<uint8_t> a(n), b(n, 0);
        for (size_t i = 0; i < n; ++i)
            a[i] = uint8_t(i * 131 + 7);
        pool.copy(b.data(), a.data(), n);
        CHECK(std::memcmp(a.data(), b.data(), n) == 0);
    }
}

// the host split of level 0 (aqz_hostsplit.cpp): random geometries, every
// frame of a layer split in row ranges by a SplitPool (threads sharing a
// frame's chunks and has_data flags), with the batch copy in the same pass;
// the layer and flags equal the oracle's, the copy equals the frames
static void
host_split(std::mt19937& rng)
{
    SplitPool pool(5);
    for (int it = 0; it < 60; ++it) {
        const uint32_t h = 1 + rng() % 90, w = 1 + rng() % 90;
        const int dtype = int(rng() % 10);
        const std::vector<Dim> dims = { Dim{ kTime, 0, 1 + rng() % 3, 1 },
                                        Dim{ kSpace, 1 + rng() % 5, 1 + rng() % 3, 1 },
                                        Dim{ kSpace, h, 1 + rng() % 17, 1 },
                                        Dim{ kSpace, w, 1 + rng() % 17, 1 } };
        std::vector<or_dim> od;
        for (const Dim& x : dims)
            od.push_back(or_dim{ x.type, x.array_size_px, x.chunk_size_px, x.shard_size_chunks });
        ArrayDimensions a(dims, dtype);
        const uint64_t F = a.frames_per_chunk_layer(), bpc = a.bytes_per_chunk();
        const uint32_t nch = a.number_of_chunks_in_memory();
        const size_t fb = size_t(h) * w * or_bytes_of_type(dtype);
        std::vector<uint8_t> frames(F * fb), copy(F * fb, 0), layer(bpc * nch, 0),
          has(nch, 0), olayer(bpc * nch, 0), ohas(nch, 0);
        or_fill_splitmix(frames.data(), frames.size(), rng());
        if (F > 1)
            std::memset(frames.data(), 0, fb); // a frame without data
        const uint32_t rows = 1 + rng() % 7;
        const uint32_t per_frame = (h + rows - 1) / rows;
        pool.run(size_t(F) * per_frame, [&](size_t i) {
            const uint64_t f = i / per_frame;
            const uint32_t r0 = uint32_t(i % per_frame) * rows;
            split_rows(split_geom(a, f), frames.data() + f * fb, r0, std::min(h, r0 + rows),
                       layer.data(), 0, nch, has.data(), copy.data() + f * fb);
        });
        for (uint64_t f = 0; f < F; ++f)
            or_write_frame_to_chunks(od.data(), int(od.size()), dtype, f, frames.data() + f * fb,
                                     olayer.data(), ohas.data());
        CHECK(layer == olayer);
        CHECK(has == ohas);
        CHECK(copy == frames);
    }
    // a task that throws reaches the caller, and the pool stays usable
    bool threw = false;
    try {
        pool.run(8, [](size_t i) {
            if (i == 3)
                throw Error(1, "task 3");
        });
    } catch (const Error&) {
        threw = true;
    }
    CHECK(threw);
    std::atomic<int> n{ 0 };
    pool.run(100, [&](size_t) { ++n; });
    CHECK(n == 100);
}

using zdec_t = size_t (*)(void*, size_t, const void*, size_t);
using ziserr_t = unsigned (*)(size_t);

static void
host_zstd()
{
    const ZstdLib& z = ZstdLib::get();
    if (!z.ok) {
        std::fprintf(stderr, "libzstd.so.1 absent: host zstd not exercised\n");
        return;
    }
    void* h = dlopen("libzstd.so.1", RTLD_NOW);
    auto dec = reinterpret_cast<zdec_t>(dlsym(h, "ZSTD_decompress"));
    auto iserr = reinterpret_cast<ziserr_t>(dlsym(h, "ZSTD_isError"));
    TaskPool pool(5);
    std::mt19937 rng(7);
    // several layers in flight at once (the stage's ring slots)
    std::vector<std::shared_ptr<HostLayerJob>> jobs;
    std::vector<std::vector<uint8_t>> ins, hds;
    for (int k = 0; k < 6; ++k) {
        auto j = std::make_shared<HostLayerJob>();
        j->codec = (k % 3 == 2) ? 3 : 2;
        j->clevel = (k == 1) ? 0 : 5;
        j->shuffle = k % 3;
        j->typesize = (k % 2) ? 2 : 4;
        j->bpc = 300000 + 1000 * k + (k % 2) * 2;
        j->n_chunks = 5;
        ins.emplace_back(j->bpc * j->n_chunks);
        hds.emplace_back(j->n_chunks, 1);
        hds.back()[3] = 0;
        auto& in = ins.back();
        for (size_t i = 0; i < in.size(); ++i) // half smooth, half random
            in[i] = (i / 4096) % 2 ? uint8_t(rng()) : uint8_t(i / 64);
        j->chunks = in.data();
        j->has_data = hds.back().data();
        for (uint32_t c = 0; c < j->n_chunks; ++c)
            j->order.push_back(j->n_chunks - 1 - c);
        const ZstdBloscGeom g = make_zstd_blosc_geom(uint32_t(j->bpc), j->typesize);
        j->frame_cap = std::max<uint64_t>(z.compress_bound(j->bpc), j->bpc + 16 + 8ull * g.nblocks + 64);
        j->tmp.resize(j->frame_cap * j->n_chunks);
        host_zstd_compress(pool, j, [] {});
        jobs.push_back(j);
    }
    for (size_t k = 0; k < jobs.size(); ++k) {
        HostLayerJob& j = *jobs[k];
        j.wait();
        CHECK(j.status == 0);
        std::vector<uint8_t> all(j.offsets[j.n_chunks] + 1);
        j.gather(all.data());
        for (uint32_t i = 0; i < j.n_chunks; ++i) {
            const uint32_t c = j.order[i];
            const uint64_t o = j.offsets[i], nb = j.offsets[i + 1] - o;
            if (!j.has_data[c]) {
                CHECK(nb == 0);
                continue;
            }
            const uint8_t* src = j.chunks + uint64_t(c) * j.bpc;
            std::vector<uint8_t> out(j.bpc);
            if (j.codec == 3) {
                const size_t r = dec(out.data(), out.size(), all.data() + o, nb);
                CHECK(!iserr(r) && r == j.bpc);
                CHECK(std::memcmp(out.data(), src, j.bpc) == 0);
                continue;
            }
            // blosc1 frame: header + per-block records; memcpyed frames hold
            // the unshuffled bytes, others the (pre-shuffled) blocks
            const uint8_t* f = all.data() + o;
            uint32_t nbytes, bs, cbytes;
            std::memcpy(&nbytes, f + 4, 4);
            std::memcpy(&bs, f + 8, 4);
            std::memcpy(&cbytes, f + 12, 4);
            CHECK(nbytes == j.bpc && cbytes == nb && (f[2] >> 5) == 4);
            if (f[2] & 0x2)
                continue; // memcpyed: unshuffled copy of the chunk
            const uint32_t nblocks = (nbytes + bs - 1) / bs;
            for (uint32_t b = 0; b < nblocks; ++b) {
                uint32_t start, cs;
                std::memcpy(&start, f + 16 + 4 * b, 4);
                std::memcpy(&cs, f + start, 4);
                const uint32_t len = std::min(bs, nbytes - b * bs);
                if (cs == len) {
                    CHECK(std::memcmp(f + start + 4, src + uint64_t(b) * bs, len) == 0);
                } else {
                    const size_t r = dec(out.data(), len, f + start + 4, cs);
                    CHECK(!iserr(r) && r == len);
                    CHECK(std::memcmp(out.data(), src + uint64_t(b) * bs, len) == 0);
                }
            }
        }
    }
}

int
main()
{
    std::mt19937 rng(2024);
    geometry(rng);
    oracle_cascade(rng);
    copy_pool();
    host_split(rng);
    host_zstd();
    std::printf("host sanitizer driver: clean\n");
    return 0;
}
