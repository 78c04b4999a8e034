// handoff_replay -- runs the reference-side binding's hand-off
// (integration/aqz_handoff.hh, the code GpuMultiscaleArray drives) over the C
// ABI with a recording sink in place of zarr::GpuArray, so the binding's
// batching, asynchronous appends, device compression, ticketed D2H hand-off
// and frame-order commits run on the GPU without the reference library.
// The sink does what GpuArray::write_unit does per chunk -- the bytes copied
// out of the pinned hand-off buffer into a vector by a pool thread holding
// the unit's lease (Shard::write_chunk takes a vector, shard.hh:38) -- and,
// instead of a shard write, records them.
//
//   handoff_replay JOB OUT      (OUT "-": record nothing, time only)
//
// JOB (little endian, written by tests/test_gpu_handoff.py):
//   "AQZ2", u32 ndims, ndims x {i32 type, u32 size, u32 chunk, u32 shard},
//   i32 dtype, i32 method, u32 batch, u32 host_slots, i32 device,
//   i32 codec, i32 clevel, i32 shuffle, u32 copy_threads, u32 pool_threads,
//   u32 synth (0: frames follow; 1: camera-like u16/u8 frames made here;
//   2: random bytes made here), u32 placement_tries, u32 z_slabs (>= 2: that
//   many stages, z slab r of every stack each, assembled by
//   aqz_stage_import_frames), u64 n_frames,
//   u64 frame_bytes, [n_frames frames].
// OUT: "AQZ4", u32 n_levels, then per level {u64 n, n x {u64 layer,
//   u32 chunk (0xffffffff: a shard's ragged padding), u32 append-shard row,
//   u32 shard, u32 internal, u64 nbytes, nbytes bytes}, u64 n_rollovers,
//   n_rollovers x u64 frames committed at the rollover}: every chunk the
//   router handed to the recording writer (nbytes 0: skipped, no data).
// Every unit runs through aqz_binding::ShardRouter (integration/
// aqz_handoff.hh), the code GpuArray runs, over aqz_dims.
// stdout: one JSON line per unit and a final summary; exit 0 only if every
// check held: units contiguous in frame order per level, only a level's
// last layer incomplete, every frame committed, the router's layer the
// unit's layer inside its shard row, every compressed entry's shard and
// internal index equal to the map's.
#include "aqz_gpu.h"
#include "aqz_handoff.hh"
#include "synth_frames.hh"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

namespace {

// a minimal stand-in for zarr::ThreadPool (thread.pool.hh): FIFO jobs
class Pool
{
  public:
    explicit Pool(unsigned n)
    {
        for (unsigned i = 0; i < n; ++i)
            t_.emplace_back([this] { run(); });
    }
    ~Pool()
    {
        drain();
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : t_)
            t.join();
    }
    void push(std::function<void()> f)
    {
        if (t_.empty()) {
            f();
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push(std::move(f));
            ++pending_;
        }
        cv_.notify_one();
    }
    void drain()
    {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
    }

  private:
    void run()
    {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty())
                    return;
                f = std::move(q_.front());
                q_.pop();
            }
            f();
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0)
                done_cv_.notify_all();
        }
    }
    std::vector<std::thread> t_;
    std::queue<std::function<void()>> q_;
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    size_t pending_ = 0;
    bool stop_ = false;
};

constexpr uint32_t kPadding = 0xffffffffu; // Record::chunk of a ragged-padding skip

struct Record
{
    uint64_t layer;
    uint32_t chunk, append, shard, internal;
    std::vector<uint8_t> bytes;
};

// One level: the shipped router (aqz_binding::ShardRouter, what GpuArray
// runs) over aqz_dims, writing into a recorder in place of the shards.
// zarr::Array's counters as the reference advances them, frame by frame:
// the tail of Array::write_frame (array.cpp:196-199) and, for an array with
// dim-1 banding, flush_completed_bands_ (:882-905).  The replay checks the
// binding's ArrayLedger against it after every complete unit.
struct RefCounters
{
    uint64_t total = 0, last_id = 0;
    uint32_t flushed = 0;
    void frame(uint64_t bpf, uint64_t F, bool banded, uint64_t fpb)
    {
        last_id = total / bpf; // frame_id == frames_written_() (checked above it)
        total += bpf;
        if (!banded)
            return;
        const uint64_t in_layer = (total / bpf) % F;
        if (in_layer == 0)
            flushed = 0;
        else if (in_layer % fpb == 0)
            flushed = std::max<uint32_t>(flushed, uint32_t(in_layer / fpb));
    }
};

struct LevelState final : aqz_binding::ShardWriter
{
    uint64_t F = 0, bpc = 0, committed = 0;
    uint64_t frame_bytes = 0, fpb = 0;
    bool banded = false;
    aqz_binding::ArrayLedger ledger; // what GpuArray::commit_unit runs
    RefCounters ref;
    uint32_t n_chunks = 0;
    bool incomplete_seen = false;
    uint64_t incomplete_layer = 0;
    aqz_dims* dims = nullptr;
    std::unique_ptr<aqz_binding::DimsShardMap> map;
    std::unique_ptr<aqz_binding::ShardRouter> router;
    uint32_t append = 0;   // append-dimension shard rows rolled over so far
    uint64_t layer = 0;    // the unit being routed
    std::vector<uint64_t> rollovers; // frames committed at each rollover
    Pool* pool = nullptr;
    bool record = true;
    std::atomic<uint64_t>* chunk_bytes = nullptr;
    std::mutex mu;
    std::vector<Record> rec;

    // GpuArray::dispatch_bytes_job_: the copy out of the pinned buffer on a
    // pool thread that holds the lease
    void write_chunk(uint32_t shard, uint32_t internal, uint32_t chunk, const uint8_t* p,
                     size_t n, const aqz_binding::Lease& lease) override
    {
        *chunk_bytes += n;
        pool->push([this, ly = layer, local = chunk % n_chunks, a = append, shard, internal,
                    p, n, lease = aqz_binding::Lease(lease)]() mutable {
            std::vector<uint8_t> v(p, p + n);
            lease.release();
            if (record) {
                std::lock_guard<std::mutex> lk(mu);
                rec.push_back(Record{ ly, local, a, shard, internal, std::move(v) });
            }
        });
    }
    void skip_chunk(uint32_t shard, uint32_t internal, uint32_t chunk) override
    {
        if (!record)
            return;
        std::lock_guard<std::mutex> lk(mu);
        rec.push_back(Record{ layer, chunk == kPadding ? kPadding : chunk % n_chunks, append,
                              shard, internal, {} });
    }
    // Array::should_rollover_ (array.cpp:924-937): frames written a
    // multiple of append chunk x append shard x the intermediate extents =
    // frames per chunk layer x chunk layers per shard
    bool should_rollover() override
    {
        return committed % (F * map->layers_per_shard()) == 0;
    }
    void rollover() override
    {
        rollovers.push_back(committed);
        ++append;
    }
};

struct RecordingSink final : aqz_binding::HandoffSink
{
    std::vector<std::unique_ptr<LevelState>> lv;
    bool quiet = false;
    std::atomic<bool> ok{ true };
    std::atomic<uint64_t> units{ 0 }, chunk_bytes{ 0 };

    aqz_status unit(aqz_binding::Unit& u) override
    {
        LevelState& L = *lv.at(u.level);
        // frame order: a unit starts where the level's last one ended, and
        // only the last layer's units may be incomplete (close)
        if (L.incomplete_seen && (u.complete || u.layer != L.incomplete_layer))
            ok = false;
        if (!u.complete) {
            L.incomplete_seen = true;
            L.incomplete_layer = u.layer;
        } else if (u.frames == 0) {
            ok = false;
        }
        if (u.frames ? L.committed != u.first : (u.complete || u.first < L.committed))
            ok = false;
        // the router's layer is the unit's layer inside its shard row
        if (L.router->current_layer() != u.layer % L.map->layers_per_shard())
            ok = false;
        if (!quiet)
            printf("{\"level\": %u, \"layer\": %llu, \"band\": %u, \"first\": %llu, "
                   "\"frames\": %llu, \"complete\": %s, \"compressed\": %s}\n",
                   u.level, (unsigned long long)u.layer, u.band,
                   (unsigned long long)L.committed, (unsigned long long)u.frames,
                   u.complete ? "true" : "false", u.entries ? "true" : "false");
        ++units;
        L.layer = u.layer;
        const aqz_status s = L.router->route(u, L);
        if (s != AQZ_STATUS_SUCCESS) {
            ok = false;
            return s;
        }
        // GpuArray::commit_unit: the frames are counted (the shipped
        // ArrayLedger), then the layer advance or rollover
        if (!L.ledger.commit(u, L.frame_bytes, 0))
            ok = false;
        L.committed = L.ledger.frames_written(L.frame_bytes);
        for (uint64_t i = 0; i < u.frames; ++i)
            L.ref.frame(L.frame_bytes, L.F, L.banded, L.fpb);
        if (u.complete && (L.ledger.total_bytes_written != L.ref.total ||
                           (u.frames && L.ledger.last_successful_frame_id != L.ref.last_id) ||
                           L.ledger.flushed_band_count != L.ref.flushed ||
                           L.ledger.bytes_to_flush != 0)) {
            fprintf(stderr, "level %u layer %llu band %u: counters differ from Array's: total "
                            "%llu/%llu last %llu/%llu bands %u/%u\n",
                    u.level, (unsigned long long)u.layer, u.band,
                    (unsigned long long)L.ledger.total_bytes_written,
                    (unsigned long long)L.ref.total,
                    (unsigned long long)L.ledger.last_successful_frame_id,
                    (unsigned long long)L.ref.last_id, L.ledger.flushed_band_count,
                    L.ref.flushed);
            ok = false;
        }
        L.router->commit(u, L);
        return AQZ_STATUS_SUCCESS;
    }
};

template<typename T>
bool
rd(FILE* f, T* v, size_t n = 1)
{
    return fread(v, sizeof(T), n, f) == n;
}


} // namespace

int
main(int argc, char** argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: handoff_replay JOB OUT\n");
        return 2;
    }
    FILE* f = fopen(argv[1], "rb");
    if (!f)
        return 2;
    char magic[4];
    uint32_t nd = 0;
    if (!rd(f, magic, 4) || memcmp(magic, "AQZ2", 4) || !rd(f, &nd) || nd > 16)
        return 2;
    std::vector<aqz_dimension> dims(nd);
    for (auto& d : dims)
        if (!rd(f, &d.type) || !rd(f, &d.array_size_px) || !rd(f, &d.chunk_size_px) ||
            !rd(f, &d.shard_size_chunks))
            return 2;
    int32_t dtype, method, device, codec, clevel, shuffle;
    uint32_t batch, slots, copy_threads, pool_threads, synth, tries, n_slabs;
    uint64_t n_frames, fbytes;
    if (!rd(f, &dtype) || !rd(f, &method) || !rd(f, &batch) || !rd(f, &slots) ||
        !rd(f, &device) || !rd(f, &codec) || !rd(f, &clevel) || !rd(f, &shuffle) ||
        !rd(f, &copy_threads) || !rd(f, &pool_threads) || !rd(f, &synth) || !rd(f, &tries) ||
        !rd(f, &n_slabs) || !rd(f, &n_frames) || !rd(f, &fbytes))
        return 2;
    std::vector<uint8_t> frames;
    uint32_t R = 0;
    if (synth == 0) {
        frames.resize(n_frames * fbytes);
        if (!rd(f, frames.data(), frames.size()))
            return 2;
        R = uint32_t(n_frames);
    } else {
        R = uint32_t(std::min<uint64_t>(n_frames, 8));
        frames = aqz_test::synth_frames(synth, dtype, fbytes, R);
    }
    fclose(f);
    const bool record = std::strcmp(argv[2], "-") != 0;

    aqz_array_desc desc{ dims.data(), dims.size(), dtype, 1, method, 0, nullptr, device };
    // level 0 split on the host for a raw hand-off, as the binding ships it
    // (aqz_binding::level0_on_host_for); AQZ_REPLAY_LEVEL0=device|host
    // forces one side
    const aqz_compression comp{ codec, clevel, shuffle };
    bool level0_host = aqz_binding::level0_on_host_for(desc, comp);
    if (const char* e = std::getenv("AQZ_REPLAY_LEVEL0"))
        level0_host = std::strcmp(e, "host") == 0;
    aqz_stage_options opt{};
    opt.max_batch_frames = batch;
    opt.layer_slots = 2;
    opt.placement_tries = tries;
    opt.level0_split_on_host = level0_host ? 1u : 0u;
    aqz_stage* st = nullptr;
    if (aqz_stage_create(&desc, &opt, &st) != AQZ_STATUS_SUCCESS) {
        fprintf(stderr, "aqz_stage_create: %s\n", aqz_last_error());
        return 1;
    }
    // z slabs: stage r owns planes [begin_r, end_r) of every stack
    // (GpuMultiscaleArray with AQZ_Z_SLABS, here all on `device`)
    std::vector<aqz_stage*> stages{ st };
    aqz_binding::SlabPlan plan;
    if (n_slabs > 1) {
        const uint32_t nl0 = aqz_stage_n_levels(st);
        aqz_dimension d0[16], dl[16];
        size_t n0 = 0, n1 = 0;
        aqz_stage_level_dims(st, 0, d0, 16, &n0);
        aqz_stage_level_dims(st, nl0 - 1, dl, 16, &n1);
        const uint32_t Z = d0[n0 - 3].array_size_px;
        plan = aqz_binding::plan_z_slabs(Z, n_slabs, Z / dl[n1 - 3].array_size_px);
        if (plan.begin.size() != n_slabs) {
            fprintf(stderr, "no z-slab plan for %u planes over %u stages\n", Z, n_slabs);
            return 1;
        }
        aqz_stage_destroy(st);
        stages.clear();
        for (uint32_t r = 0; r < n_slabs; ++r) {
            aqz_stage_options o = opt;
            o.z_slab_begin = plan.begin[r];
            o.z_slab_end = plan.end[r];
            aqz_stage* s = nullptr;
            if (aqz_stage_create(&desc, &o, &s) != AQZ_STATUS_SUCCESS) {
                fprintf(stderr, "aqz_stage_create (slab %u): %s\n", r, aqz_last_error());
                return 1;
            }
            stages.push_back(s);
        }
        st = stages[0];
    }
    const uint32_t nl = aqz_stage_n_levels(st);
    RecordingSink sink;
    sink.quiet = !record;
    Pool pool(pool_threads);
    for (uint32_t l = 0; l < nl; ++l) {
        auto L = std::make_unique<LevelState>();
        aqz_level_layout lay{};
        aqz_stage_level_layout(st, l, &lay);
        L->F = lay.frames_per_layer;
        L->bpc = lay.bytes_per_chunk;
        L->n_chunks = lay.chunks_per_layer;
        L->frame_bytes = lay.frame_bytes;
        {
            int32_t banded = 0;
            uint32_t nb = 1, cpb = 0;
            uint64_t fpb = 0;
            aqz_stage_band_geometry(st, l, &banded, &nb, &fpb, &cpb);
            L->banded = banded != 0;
            L->fpb = fpb ? fpb : L->F;
        }
        std::vector<aqz_dimension> ld(16);
        size_t n = 0;
        aqz_stage_level_dims(st, l, ld.data(), ld.size(), &n);
        if (aqz_dims_create(ld.data(), n, dtype, nullptr, &L->dims) != AQZ_STATUS_SUCCESS)
            return 1;
        L->map = std::make_unique<aqz_binding::DimsShardMap>(L->dims);
        L->router = std::make_unique<aqz_binding::ShardRouter>(*L->map);
        L->pool = &pool;
        L->record = record;
        L->chunk_bytes = &sink.chunk_bytes;
        sink.lv.push_back(std::move(L));
    }
    int rc = 0;
    double seconds = 0;
    uint64_t host_bytes = 0, device_bytes = 0, est_host = 0, est_device = 0;
    aqz_binding::Handoff::Stats hs{};
    {
        aqz_binding::HandoffOptions ho;
        ho.batch_frames = batch;
        ho.host_slots = slots;
        ho.copy_threads = copy_threads;
        ho.comp = comp;
        ho.level0_on_host = level0_host;
        aqz_binding::Handoff h(stages, plan, fbytes, ho, sink);
        if (h.status() != AQZ_STATUS_SUCCESS) {
            fprintf(stderr, "handoff: %s\n", aqz_last_error());
            return 1;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t i = 0; i < n_frames; ++i)
            if (h.write_frame(frames.data() + (i % R) * fbytes) != AQZ_STATUS_SUCCESS) {
                fprintf(stderr, "write_frame %llu: %s\n", (unsigned long long)i,
                        aqz_last_error());
                return 1;
            }
        if (h.close() != AQZ_STATUS_SUCCESS) {
            fprintf(stderr, "close: %s\n", aqz_last_error());
            return 1;
        }
        pool.drain(); // the writer jobs (Array::close_ waits on write_counter_)
        seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        hs = h.stats();
        // what the drop-in holds now (every compressed slot in use) against
        // its estimate (aqz_binding::estimate_memory)
        host_bytes = h.host_bytes();
        for (aqz_stage* s : stages) {
            aqz_memory_usage m{};
            aqz_stage_memory_usage(s, &m);
            host_bytes += m.pinned_bytes;
            device_bytes += m.device_bytes;
        }
        aqz_binding::MemoryEstimate est{};
        if (aqz_binding::estimate_memory(desc, opt, ho, uint32_t(stages.size()), &est) !=
            AQZ_STATUS_SUCCESS) {
            fprintf(stderr, "estimate_memory: %s\n", aqz_last_error());
            return 1;
        }
        est_host = est.host_bytes;
        est_device = est.device_bytes;
    }
    for (uint32_t l = 0; l < nl && n_slabs <= 1; ++l)
        if (sink.lv[l]->committed != aqz_stage_frames_written(st, l)) {
            fprintf(stderr, "level %u: committed %llu of %llu frames\n", l,
                    (unsigned long long)sink.lv[l]->committed,
                    (unsigned long long)aqz_stage_frames_written(st, l));
            rc = 1;
        }
    if (!sink.ok)
        rc = 1;
    const double in = double(n_frames) * double(fbytes);
    printf("{\"summary\": true, \"ok\": %s, \"units\": %llu, \"tickets\": %llu, "
           "\"frames\": %llu, \"seconds\": %.4f, \"input_gbs\": %.3f, "
           "\"sink_bytes_per_input_byte\": %.4f, \"codec\": %d, \"clevel\": %d, "
           "\"shuffle\": %d, \"device\": %d, \"batch\": %u, \"copy_threads\": %u, "
           "\"pool_threads\": %u, \"host_bytes\": %llu, \"device_bytes\": %llu, "
           "\"estimate_host_bytes\": %llu, \"estimate_device_bytes\": %llu, "
           "\"level0_split\": \"%s\", \"consumer_s\": {\"write_frame\": %.4f, "
           "\"wait_consumed\": %.4f, \"copy\": %.4f, \"slot_wait\": %.4f, \"append\": %.4f, "
           "\"sink\": %.4f}}\n",
           rc == 0 ? "true" : "false", (unsigned long long)sink.units.load(),
           (unsigned long long)aqz_stage_last_ticket(stages.back()), (unsigned long long)n_frames,
           seconds, in / seconds / 1e9, double(sink.chunk_bytes.load()) / in, codec, clevel,
           shuffle, device, batch, copy_threads, pool_threads, (unsigned long long)host_bytes,
           (unsigned long long)device_bytes, (unsigned long long)est_host,
           (unsigned long long)est_device, level0_host ? "host" : "device",
           hs.write_frame_ns * 1e-9, hs.wait_consumed_ns * 1e-9, hs.copy_ns * 1e-9,
           hs.slot_wait_ns * 1e-9, hs.append_ns * 1e-9, hs.sink_ns * 1e-9);
    for (aqz_stage* s : stages)
        aqz_stage_destroy(s);
    for (auto& L : sink.lv)
        aqz_dims_destroy(L->dims);
    if (!record)
        return rc;

    FILE* o = fopen(argv[2], "wb");
    if (!o)
        return 2;
    fwrite("AQZ4", 1, 4, o);
    fwrite(&nl, 4, 1, o);
    for (auto& L : sink.lv) {
        const uint64_t n = L->rec.size();
        fwrite(&n, 8, 1, o);
        for (const Record& r : L->rec) {
            const uint64_t nb = r.bytes.size();
            fwrite(&r.layer, 8, 1, o);
            fwrite(&r.chunk, 4, 1, o);
            fwrite(&r.append, 4, 1, o);
            fwrite(&r.shard, 4, 1, o);
            fwrite(&r.internal, 4, 1, o);
            fwrite(&nb, 8, 1, o);
            fwrite(r.bytes.data(), 1, nb, o);
        }
        const uint64_t nr = L->rollovers.size();
        fwrite(&nr, 8, 1, o);
        fwrite(L->rollovers.data(), 8, nr, o);
    }
    fclose(o);
    return rc;
}
