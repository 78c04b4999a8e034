// stream_to_filesystem.cpp -- the whole multiscale path through the C ABI
// (include/aqz_gpu.h), from a host frame buffer to Zarr v3 shard files:
//
//   host frames --H2D--> aqz stage (level-0 tile split + pyramid + tile split
//   of every level, on the GPU) --> [device blosc1-lz4 compression] --D2H-->
//   shard files written by a pool of writer threads (pwrite), each shard
//   ending in its index table + CRC-32C.
//
// This is what the reference's consumer thread does for a multiscale array
// (MultiscaleArray::write_frame, multiscale.array.cpp:57-74, 291-325; chunk
// jobs array.cpp:664-760; Shard::write_chunk / write_table_,
// shard.cpp:53-166), with the pixel work and the compression on the device.
// Shard paths follow the reference: <out>/<level>/c/<append shard>/<shard
// coordinates...> (Array::data_root_, array.cpp:130-135; construct_data_paths,
// sink.cpp:47-100).  zarr.json metadata is not written (out of scope).
//
//   stream_to_filesystem OUT_DIR [--config c1|c2|c3] [--frames N]
//       [--ring R] [--codec raw|lz4|blosc-zstd|zstd] [--shuffle 0|1|2]
//       [--source pinned|pageable]
//       [--seed S] [--writers K] [--pattern random|camera] [--no-write]
//
// Frames are a splitmix64 byte stream (seed S; the same stream as the test
// oracle's synthetic_frames) or, with --pattern camera, a compressible
// camera-like signal (1000 + 200 sin(i/977) + noise); R distinct frames are
// appended cyclically.  Prints
// one JSON line with the end-to-end rate.
#include "aqz_gpu.h"
#include "aqz_gpu_bench.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

[[noreturn]] void
die(const char* what, aqz_status s = 0)
{
    std::fprintf(stderr, "stream_to_filesystem: %s (%s)%s%s\n", what, aqz_status_message(s),
                 s ? ": " : "", s ? aqz_last_error() : "");
    std::exit(1);
}

void
check(aqz_status s, const char* what)
{
    if (s != AQZ_STATUS_SUCCESS)
        die(what, s);
}

void
fill_splitmix(uint8_t* p, size_t n, uint64_t seed)
{
    uint64_t s = seed;
    size_t i = 0;
    auto next = [&] {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    for (; i + 8 <= n; i += 8) {
        const uint64_t v = next();
        std::memcpy(p + i, &v, 8);
    }
    if (i < n) {
        const uint64_t v = next();
        std::memcpy(p + i, &v, n - i);
    }
}

// smooth background + noise of about 30 counts (the bench's camera-like
// payload), as pixels of bpp bytes
void
fill_camera(uint8_t* p, size_t n, uint32_t bpp, uint64_t seed)
{
    std::vector<uint8_t> noise(n / bpp * 4);
    fill_splitmix(noise.data(), noise.size(), seed);
    for (size_t i = 0; i < n / bpp; ++i) {
        int sum = 0; // sum of 4 uniform bytes: mean 510, sd ~148
        for (int k = 0; k < 4; ++k)
            sum += noise[4 * i + k];
        double v = 1000.0 + 200.0 * std::sin(double(i) / 977.0) + (sum - 510) * (30.0 / 148.0);
        if (bpp == 1)
            v /= 8.0;
        const uint32_t u = uint32_t(std::clamp(v, 0.0, 65535.0));
        std::memcpy(p + i * bpp, &u, bpp); // little endian
    }
}

void
mkdirs(const std::string& path)
{
    for (size_t i = 1; i <= path.size(); ++i)
        if (i == path.size() || path[i] == '/')
            ::mkdir(path.substr(0, i).c_str(), 0755);
}

// A fixed pool of writer threads (the reference's ThreadPool running chunk
// jobs, thread.pool.cpp; here the jobs are pwrites of whole shard runs).
class Writers
{
  public:
    explicit Writers(int n)
    {
        for (int i = 0; i < n; ++i)
            th_.emplace_back([this] { loop(); });
    }
    ~Writers()
    {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_)
            t.join();
    }
    void push(std::function<void()> job)
    {
        {
            std::lock_guard<std::mutex> g(m_);
            q_.push_back(std::move(job));
            ++pending_;
        }
        cv_.notify_one();
    }
    void drain()
    {
        std::unique_lock<std::mutex> g(m_);
        done_cv_.wait(g, [this] { return pending_ == 0; });
    }

  private:
    void loop()
    {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [this] { return stop_ || !q_.empty(); });
                if (q_.empty())
                    return;
                job = std::move(q_.front());
                q_.pop_front();
            }
            job();
            {
                std::lock_guard<std::mutex> g(m_);
                if (--pending_ == 0)
                    done_cv_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::deque<std::function<void()>> q_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    size_t pending_ = 0;
    bool stop_ = false;
};

void
pwrite_all(int fd, const uint8_t* p, size_t n, uint64_t off)
{
    while (n > 0) {
        const ssize_t w = ::pwrite(fd, p, n, off_t(off));
        if (w <= 0)
            die("pwrite failed");
        p += w;
        n -= size_t(w);
        off += uint64_t(w);
    }
}

// One append-dimension shard row of one level: n_shards open files, their
// running offsets and (offset, extent) tables (zarr::Shard, shard.cpp:13-166).
struct ShardRow
{
    int64_t row = -1;
    std::vector<int> fd;
    std::vector<uint64_t> end;
    std::vector<std::vector<uint64_t>> off, ext;
};

struct Level
{
    uint32_t index = 0;
    aqz_level_layout lay{};
    std::vector<aqz_dimension> dims; // storage order
    uint32_t cps = 1, n_shards = 1, lps = 1;
    std::vector<uint32_t> shard_of, internal0; // raw mode: per chunk of a layer
    std::vector<uint32_t> shards_along;        // dims 1..n-1
    ShardRow sr;
    uint64_t handed = 0;
};

struct Buffer
{
    uint8_t* p = nullptr;
    size_t cap = 0;
    uint8_t* has = nullptr;
    std::atomic<int> busy{ 0 }; // writer jobs still reading it
};

struct Job
{
    Level* L;
    uint64_t layer;
    Buffer* buf;
    int stage; // 0: compressing, 1: D2H issued
};

} // namespace

int
main(int argc, char** argv)
{
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s OUT_DIR [--config c1|c2|c3] [--frames N] [--ring R] "
                             "[--codec raw|lz4|blosc-zstd|zstd] [--shuffle 0|1|2] "
                             "[--source pinned|pageable] [--seed S] [--writers K] "
                             "[--no-write]\n",
                     argv[0]);
        return 2;
    }
    std::string out = argv[1], config = "c1", codec = "lz4", source = "pinned";
    std::string pattern = "random";
    uint64_t n_frames = 256, ring = 0, seed = 7;
    int shuffle = 1, n_writers = 8;
    bool write = true;
    for (int i = 2; i < argc; ++i) {
        const std::string a = argv[i];
        auto val = [&] {
            if (i + 1 >= argc)
                die("missing value");
            return std::string(argv[++i]);
        };
        if (a == "--config")
            config = val();
        else if (a == "--frames")
            n_frames = std::stoull(val());
        else if (a == "--ring")
            ring = std::stoull(val());
        else if (a == "--codec")
            codec = val();
        else if (a == "--shuffle")
            shuffle = std::stoi(val());
        else if (a == "--source")
            source = val();
        else if (a == "--seed")
            seed = std::stoull(val());
        else if (a == "--writers")
            n_writers = std::stoi(val());
        else if (a == "--pattern")
            pattern = val();
        else if (a == "--no-write")
            write = false;
        else
            die("unknown argument");
    }

    // BASELINE.json configs (t unbounded, y, x): configs[0] (c1), [1] (c2), [2] (c3)
    std::vector<aqz_dimension> dims;
    int32_t dtype = AQZ_DTYPE_UINT16;
    uint32_t force_levels = 0, batch = 64;
    if (config == "c1") {
        dims = { { AQZ_DIM_TIME, 0, 64, 1 }, { AQZ_DIM_SPACE, 512, 128, 2 },
                 { AQZ_DIM_SPACE, 512, 128, 2 } };
    } else if (config == "c2") {
        dims = { { AQZ_DIM_TIME, 0, 64, 1 }, { AQZ_DIM_SPACE, 2048, 256, 4 },
                 { AQZ_DIM_SPACE, 2048, 256, 4 } };
        force_levels = 5;
    } else if (config == "c3") {
        dims = { { AQZ_DIM_TIME, 0, 32, 1 }, { AQZ_DIM_SPACE, 4096, 128, 8 },
                 { AQZ_DIM_SPACE, 4096, 128, 8 } };
        dtype = AQZ_DTYPE_UINT8;
        batch = 32;
    } else {
        die("unknown config");
    }
    int32_t codec_id = AQZ_CODEC_NONE;
    if (codec == "lz4")
        codec_id = AQZ_CODEC_BLOSC_LZ4;
    else if (codec == "blosc-zstd")
        codec_id = AQZ_CODEC_BLOSC_ZSTD;
    else if (codec == "zstd")
        codec_id = AQZ_CODEC_ZSTD;
    else if (codec != "raw")
        die("unknown codec");
    const bool compress = codec_id != AQZ_CODEC_NONE;
    aqz_array_desc desc{ dims.data(), dims.size(), dtype, 1, AQZ_METHOD_MEAN, 0, nullptr, 0 };
    // this writer emits sharded Zarr v3 arrays only (every dimension has a
    // shard size); an unsharded array stores each chunk as its own file with
    // no index table, which is not implemented here
    for (const aqz_dimension& d : dims)
        if (d.shard_size_chunks == 0)
            die("unsharded arrays are not supported by this example");
    aqz_stage_options opt{};
    opt.layer_slots = 3;
    opt.max_batch_frames = batch;
    // c2: BASELINE's 5 levels at 256-px chunks (the bench-only extension)
    aqz_stage_bench_options bopt{};
    bopt.force_levels = force_levels;
    aqz_stage* st = nullptr;
    check(aqz_stage_create_bench(&desc, &opt, &bopt, &st), "aqz_stage_create");

    const uint32_t nl = aqz_stage_n_levels(st);
    std::vector<Level> lv(nl);
    for (uint32_t l = 0; l < nl; ++l) {
        Level& L = lv[l];
        L.index = l;
        check(aqz_stage_level_layout(st, l, &L.lay), "layout");
        L.dims.resize(16);
        size_t nd = 0;
        check(aqz_stage_level_dims(st, l, L.dims.data(), L.dims.size(), &nd), "level_dims");
        L.dims.resize(nd);
        check(aqz_stage_shard_geometry(st, l, &L.cps, &L.n_shards, &L.lps), "shard_geometry");
        for (size_t i = 1; i < nd; ++i) {
            const aqz_dimension& d = L.dims[i];
            const uint32_t chunks = (d.array_size_px + d.chunk_size_px - 1) / d.chunk_size_px;
            const uint32_t s = std::max<uint32_t>(1, d.shard_size_chunks);
            L.shards_along.push_back((chunks + s - 1) / s);
        }
        aqz_dims* ad = nullptr;
        check(aqz_dims_create(L.dims.data(), nd, dtype, nullptr, &ad), "aqz_dims_create");
        for (uint32_t c = 0; c < L.lay.chunks_per_layer; ++c) {
            L.shard_of.push_back(aqz_dims_shard_index_for_chunk(ad, c));
            L.internal0.push_back(aqz_dims_shard_internal_index(ad, c));
        }
        aqz_dims_destroy(ad);
    }
    const uint64_t fbytes = lv[0].lay.frame_bytes;
    if (ring == 0)
        ring = std::min<uint64_t>(n_frames, 2 * uint64_t(batch));

    // the host frame buffer (a camera's DMA ring when pinned)
    uint8_t* src = nullptr;
    std::vector<uint8_t> pageable;
    if (source == "pinned") {
        check(aqz_host_alloc(ring * fbytes, reinterpret_cast<void**>(&src)), "aqz_host_alloc");
    } else {
        pageable.resize(ring * fbytes);
        src = pageable.data();
    }
    if (pattern == "camera")
        fill_camera(src, ring * fbytes, dtype == AQZ_DTYPE_UINT8 ? 1 : 2, seed);
    else
        fill_splitmix(src, ring * fbytes, seed);
    const int32_t mem = source == "pinned" ? AQZ_MEM_HOST_PINNED : AQZ_MEM_HOST;

    // hand-off buffers: 4 per level, rotated
    constexpr int kBufs = 4;
    std::vector<std::vector<Buffer>> bufs(nl);
    for (uint32_t l = 0; l < nl; ++l) {
        bufs[l] = std::vector<Buffer>(kBufs);
        const size_t layer_bytes = lv[l].lay.bytes_per_chunk * lv[l].lay.chunks_per_layer;
        for (Buffer& b : bufs[l]) {
            // + per-chunk frame overhead (blosc header + block table, or a
            // zstd frame's block headers: < 0.5% of the chunk)
            b.cap = layer_bytes + layer_bytes / 128 +
                    (64 + 1024) * size_t(lv[l].lay.chunks_per_layer) + 4096;
            check(aqz_host_alloc(b.cap, reinterpret_cast<void**>(&b.p)), "aqz_host_alloc");
            check(aqz_host_alloc(lv[l].lay.chunks_per_layer, reinterpret_cast<void**>(&b.has)),
                  "aqz_host_alloc");
        }
    }

    Writers writers(n_writers);
    std::atomic<uint64_t> bytes_written{ 0 };

    auto close_row = [&](Level& L) {
        if (L.sr.row < 0)
            return;
        writers.drain(); // every run of the row has landed
        for (uint32_t s = 0; s < L.n_shards; ++s) {
            std::vector<uint8_t> tab(aqz_shard_table_bytes(L.cps));
            check(aqz_shard_table(L.sr.off[s].data(), L.sr.ext[s].data(), L.cps, tab.data(),
                                  tab.size()),
                  "aqz_shard_table");
            if (write) {
                pwrite_all(L.sr.fd[s], tab.data(), tab.size(), L.sr.end[s]);
                ::close(L.sr.fd[s]);
            }
            bytes_written += tab.size();
        }
        L.sr = ShardRow{};
    };
    auto open_row = [&](Level& L, int64_t row) {
        if (L.sr.row == row)
            return;
        close_row(L);
        L.sr.row = row;
        L.sr.fd.assign(L.n_shards, -1);
        L.sr.end.assign(L.n_shards, 0);
        L.sr.off.assign(L.n_shards, std::vector<uint64_t>(L.cps, UINT64_MAX));
        L.sr.ext.assign(L.n_shards, std::vector<uint64_t>(L.cps, UINT64_MAX));
        if (!write)
            return;
        for (uint32_t s = 0; s < L.n_shards; ++s) {
            // shard s -> coordinates over dims 1..n-1, row-major
            std::vector<uint32_t> co(L.shards_along.size());
            uint32_t r = s;
            for (size_t i = co.size(); i-- > 0;) {
                co[i] = r % L.shards_along[i];
                r /= L.shards_along[i];
            }
            std::string dir = out + "/" + std::to_string(L.index) + "/c/" + std::to_string(row);
            for (size_t i = 0; i + 1 < co.size(); ++i)
                dir += "/" + std::to_string(co[i]);
            mkdirs(dir);
            const std::string path = dir + "/" + std::to_string(co.back());
            L.sr.fd[s] = ::open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
            if (L.sr.fd[s] < 0)
                die("open shard");
        }
    };
    // the runs of one handed-off layer: (shard, internal, offset in buf, bytes)
    struct Run
    {
        uint32_t shard, internal;
        uint64_t off, n;
    };
    auto write_layer = [&](Level& L, uint64_t layer, Buffer* b, const std::vector<Run>& runs) {
        open_row(L, int64_t(layer / L.lps));
        // consecutive runs of one shard are one contiguous pwrite
        size_t i = 0;
        while (i < runs.size()) {
            const uint32_t s = runs[i].shard;
            const uint64_t o0 = runs[i].off, f0 = L.sr.end[s];
            uint64_t n = 0;
            size_t j = i;
            for (; j < runs.size() && runs[j].shard == s && runs[j].off == o0 + n; ++j) {
                L.sr.off[s][runs[j].internal] = f0 + n;
                L.sr.ext[s][runs[j].internal] = runs[j].n;
                n += runs[j].n;
            }
            L.sr.end[s] += n;
            bytes_written += n;
            if (write && n) {
                const int fd = L.sr.fd[s];
                const uint8_t* p = b->p + o0;
                b->busy.fetch_add(1);
                writers.push([fd, p, n, f0, b] {
                    pwrite_all(fd, p, n, f0);
                    b->busy.fetch_sub(1);
                });
            }
            i = j;
        }
        if ((layer + 1) % L.lps == 0)
            close_row(L);
    };

    std::deque<Job> jobs;
    std::vector<int> next_buf(nl, 0);
    auto take_buffer = [&](uint32_t l) {
        Buffer* b = &bufs[l][size_t(next_buf[l]++ % kBufs)];
        while (b->busy.load() != 0)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        return b;
    };
    // blosc codecs at clevel 5, plain zstd at level 3 (the settings' levels)
    const aqz_compression comp{ codec_id, codec_id == AQZ_CODEC_ZSTD ? 3 : 5,
                                codec_id == AQZ_CODEC_ZSTD ? 0 : shuffle };

    // completed layers of every level -> compression or raw D2H
    auto hand_off = [&](bool final) {
        for (Level& L : lv) {
            const uint64_t fw = aqz_stage_frames_written(st, L.index);
            uint64_t done = fw / L.lay.frames_per_layer;
            if (final && fw % L.lay.frames_per_layer)
                ++done; // the zero-filled partial last layer
            for (; L.handed < done; ++L.handed) {
                Buffer* b = take_buffer(L.index);
                if (compress) {
                    check(aqz_stage_compress_layer(st, L.index, L.handed, &comp), "compress");
                    jobs.push_back({ &L, L.handed, b, 0 });
                } else {
                    check(aqz_stage_copy_layer_async(
                            st, L.index, L.handed, b->p, b->cap, b->has,
                            L.lay.chunks_per_layer),
                          "copy_layer_async");
                    jobs.push_back({ &L, L.handed, b, 1 });
                }
            }
        }
    };
    // compressed layers: entries + D2H; copies issued earlier: write out
    auto advance = [&](bool all) {
        std::vector<Job> landed;
        if (all || !jobs.empty()) {
            // copies issued before this point complete together
            bool any_copy = false;
            for (const Job& j : jobs)
                any_copy |= j.stage == 1;
            if (any_copy)
                check(aqz_stage_wait_copies(st), "wait_copies");
        }
        std::deque<Job> keep;
        for (Job& j : jobs) {
            if (j.stage == 1) {
                landed.push_back(j);
                continue;
            }
            // compression done -> its frames go D2H now
            check(aqz_stage_copy_compressed_async(st, j.L->index, j.layer, j.buf->p, j.buf->cap),
                  "copy_compressed_async");
            j.stage = 1;
            keep.push_back(j);
        }
        jobs.swap(keep);
        for (const Job& j : landed) {
            Level& L = *j.L;
            std::vector<Run> runs;
            if (compress) {
                std::vector<aqz_chunk_entry> ent(L.lay.chunks_per_layer);
                check(aqz_stage_compressed_entries(st, L.index, j.layer, ent.data(), ent.size()),
                      "compressed_entries");
                for (const aqz_chunk_entry& e : ent)
                    if (e.nbytes)
                        runs.push_back({ e.shard, e.internal, e.offset, e.nbytes });
            } else {
                // raw chunks in shard-major order; chunks without data are
                // skipped (array.cpp:713-720)
                std::vector<uint32_t> order(L.lay.chunks_per_layer);
                for (uint32_t c = 0; c < order.size(); ++c)
                    order[c] = c;
                std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b2) {
                    return L.shard_of[a] != L.shard_of[b2] ? L.shard_of[a] < L.shard_of[b2]
                                                           : L.internal0[a] < L.internal0[b2];
                });
                const uint32_t stride = L.cps / L.lps, cl = uint32_t(j.layer % L.lps);
                for (uint32_t c : order)
                    if (j.buf->has[c])
                        runs.push_back({ L.shard_of[c], L.internal0[c] + cl * stride,
                                         uint64_t(c) * L.lay.bytes_per_chunk,
                                         L.lay.bytes_per_chunk });
            }
            write_layer(L, j.layer, j.buf, runs);
        }
    };

    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t f = 0; f < n_frames;) {
        const uint64_t n = std::min<uint64_t>({ uint64_t(batch), n_frames - f, ring - f % ring });
        // Back-pressure of a camera DMA ring: frames f..f+n-1 go into ring
        // slots last used by frames f-ring..f+n-1-ring, which a pinned source
        // hands to the stage asynchronously.  The camera may write those
        // slots only once the stage has read them (aqz_stage_frames_consumed);
        // here the slots keep their synthetic contents, but the wait is the
        // one a real producer needs.  (A pageable source is copied before
        // aqz_stage_append returns.)
        if (mem == AQZ_MEM_HOST_PINNED && f + n > ring)
            while (aqz_stage_frames_consumed(st) < f + n - ring)
                std::this_thread::yield();
        check(aqz_stage_append(st, src + (f % ring) * fbytes, n, mem), "append");
        f += n;
        advance(false);
        hand_off(false);
    }
    check(aqz_stage_finalize(st), "finalize");
    hand_off(true);
    while (!jobs.empty())
        advance(true);
    for (Level& L : lv)
        close_row(L);
    writers.drain();
    const double el =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();

    const double in_bytes = double(n_frames) * double(fbytes);
    std::printf("{\"metric\": \"end-to-end input GB/s, host frames -> H2D -> multiscale stage -> "
                "%s -> D2H -> shard files\", \"value\": %.3f, \"unit\": \"GB/s\", "
                "\"frames\": %llu, \"seconds\": %.3f, \"levels\": %u, \"config\": \"%s\", "
                "\"source\": \"%s\", \"codec\": \"%s\", \"shuffle\": %d, "
                "\"bytes_to_sink\": %llu, \"sink_bytes_per_input_byte\": %.4f, "
                "\"writers\": %d, \"write\": %s, \"pattern\": \"%s\"}\n",
                codec_id == AQZ_CODEC_BLOSC_LZ4    ? "device blosc-lz4"
                : codec_id == AQZ_CODEC_BLOSC_ZSTD ? "blosc-zstd"
                : codec_id == AQZ_CODEC_ZSTD       ? "zstd"
                                                   : "raw chunks",
                in_bytes / el / 1e9,
                static_cast<unsigned long long>(n_frames), el, nl, config.c_str(),
                source.c_str(), codec.c_str(), shuffle,
                static_cast<unsigned long long>(bytes_written.load()),
                double(bytes_written.load()) / in_bytes, n_writers, write ? "true" : "false",
                pattern.c_str());

    for (auto& v : bufs)
        for (Buffer& b : v) {
            aqz_host_free(b.p);
            aqz_host_free(b.has);
        }
    if (source == "pinned")
        aqz_host_free(src);
    aqz_stage_destroy(st);
    return 0;
}
