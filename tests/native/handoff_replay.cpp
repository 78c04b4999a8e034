// handoff_replay -- runs the reference-side binding's hand-off
// (integration/aqz_handoff.hh, the code GpuMultiscaleArray drives) over the C
// ABI with a recording sink in place of zarr::GpuArray, so the binding's
// batching, asynchronous appends, ticketed D2H hand-off and frame-order
// commits run on the GPU without the reference library.
//
//   handoff_replay JOB OUT
//
// JOB (little endian, written by tests/test_gpu_handoff.py):
//   "AQZJ", u32 ndims, ndims x {i32 type, u32 size, u32 chunk, u32 shard},
//   i32 dtype, i32 method, u32 batch, u32 host_slots, u64 n_frames,
//   u64 frame_bytes, n_frames frames.
// OUT: "AQZO", u32 n_levels, then per level {u64 n_layers, u64 layer_bytes,
//   u32 n_chunks, then per layer {u64 layer, layer bytes, has_data bytes}}.
// stdout: one JSON line per commit and a final summary; exit 0 only if every
// check held (commits contiguous in frame order per level, flush = false
// only on a level's last unit, every frame committed).
#include "aqz_gpu.h"
#include "aqz_handoff.hh"

#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

namespace {

struct LevelStore
{
    uint64_t F = 0, bpc = 0;
    uint32_t n_chunks = 0;
    uint64_t committed = 0;
    bool closed = false; // a flush = false commit was seen
    std::map<uint64_t, std::pair<std::vector<uint8_t>, std::vector<uint8_t>>> layers;
};

struct RecordingSink final : aqz_binding::HandoffSink
{
    std::vector<LevelStore> lv;
    bool ok = true;
    uint64_t installs = 0;

    void install(uint32_t level, const uint8_t* chunks, const uint8_t* has, uint32_t c0,
                 uint32_t n) override
    {
        LevelStore& L = lv.at(level);
        const uint64_t layer = L.committed / L.F;
        auto& [buf, hd] = L.layers[layer];
        if (buf.empty()) {
            buf.assign(L.bpc * L.n_chunks, 0);
            hd.assign(L.n_chunks, 0);
        }
        if (c0 + n > L.n_chunks) {
            ok = false;
            return;
        }
        std::memcpy(buf.data() + c0 * L.bpc, chunks, n * L.bpc);
        std::memcpy(hd.data() + c0, has, n);
        ++installs;
    }

    aqz_status commit(uint32_t level, uint64_t frames, bool flush) override
    {
        LevelStore& L = lv.at(level);
        if (L.closed || frames == 0)
            ok = false; // nothing may follow the partial last unit
        printf("{\"level\": %u, \"first\": %llu, \"frames\": %llu, \"flush\": %s}\n", level,
               (unsigned long long)L.committed, (unsigned long long)frames,
               flush ? "true" : "false");
        L.committed += frames;
        if (!flush)
            L.closed = true;
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
    if (!rd(f, magic, 4) || memcmp(magic, "AQZJ", 4) || !rd(f, &nd) || nd > 16)
        return 2;
    std::vector<aqz_dimension> dims(nd);
    for (auto& d : dims)
        if (!rd(f, &d.type) || !rd(f, &d.array_size_px) || !rd(f, &d.chunk_size_px) ||
            !rd(f, &d.shard_size_chunks))
            return 2;
    int32_t dtype, method;
    uint32_t batch, slots;
    uint64_t n_frames, fbytes;
    if (!rd(f, &dtype) || !rd(f, &method) || !rd(f, &batch) || !rd(f, &slots) ||
        !rd(f, &n_frames) || !rd(f, &fbytes))
        return 2;
    std::vector<uint8_t> frames(n_frames * fbytes);
    if (!rd(f, frames.data(), frames.size()))
        return 2;
    fclose(f);

    aqz_array_desc desc{ dims.data(), dims.size(), dtype, 1, method, 0, nullptr, 0 };
    aqz_stage_options opt{};
    opt.max_batch_frames = batch;
    opt.layer_slots = 2;
    aqz_stage* st = nullptr;
    if (aqz_stage_create(&desc, &opt, &st) != AQZ_STATUS_SUCCESS) {
        fprintf(stderr, "aqz_stage_create: %s\n", aqz_last_error());
        return 1;
    }
    const uint32_t nl = aqz_stage_n_levels(st);
    RecordingSink sink;
    sink.lv.resize(nl);
    for (uint32_t l = 0; l < nl; ++l) {
        aqz_level_layout lay{};
        aqz_stage_level_layout(st, l, &lay);
        sink.lv[l].F = lay.frames_per_layer;
        sink.lv[l].bpc = lay.bytes_per_chunk;
        sink.lv[l].n_chunks = lay.chunks_per_layer;
    }
    int rc = 0;
    {
        aqz_binding::Handoff h(st, fbytes, batch, slots, sink);
        if (h.status() != AQZ_STATUS_SUCCESS)
            return 1;
        for (uint64_t i = 0; i < n_frames; ++i)
            if (h.write_frame(frames.data() + i * fbytes) != AQZ_STATUS_SUCCESS) {
                fprintf(stderr, "write_frame %llu: %s\n", (unsigned long long)i,
                        aqz_last_error());
                return 1;
            }
        if (h.close() != AQZ_STATUS_SUCCESS) {
            fprintf(stderr, "close: %s\n", aqz_last_error());
            return 1;
        }
    }
    for (uint32_t l = 0; l < nl; ++l)
        if (sink.lv[l].committed != aqz_stage_frames_written(st, l)) {
            fprintf(stderr, "level %u: committed %llu of %llu frames\n", l,
                    (unsigned long long)sink.lv[l].committed,
                    (unsigned long long)aqz_stage_frames_written(st, l));
            rc = 1;
        }
    if (!sink.ok)
        rc = 1;
    printf("{\"summary\": true, \"ok\": %s, \"installs\": %llu, \"tickets\": %llu}\n",
           rc == 0 ? "true" : "false", (unsigned long long)sink.installs,
           (unsigned long long)aqz_stage_last_ticket(st));
    aqz_stage_destroy(st);

    FILE* o = fopen(argv[2], "wb");
    if (!o)
        return 2;
    fwrite("AQZO", 1, 4, o);
    fwrite(&nl, 4, 1, o);
    for (const LevelStore& L : sink.lv) {
        const uint64_t n = L.layers.size(), lb = L.bpc * L.n_chunks;
        fwrite(&n, 8, 1, o);
        fwrite(&lb, 8, 1, o);
        fwrite(&L.n_chunks, 4, 1, o);
        for (const auto& [layer, bh] : L.layers) {
            fwrite(&layer, 8, 1, o);
            fwrite(bh.first.data(), 1, bh.first.size(), o);
            fwrite(bh.second.data(), 1, bh.second.size(), o);
        }
    }
    fclose(o);
    return rc;
}
