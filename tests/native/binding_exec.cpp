// binding_exec -- TEST INFRASTRUCTURE ONLY.  Runs the shipped drop-in
// binding, integration/multiscale.array.gpu.cpp (GpuMultiscaleArray,
// GpuArray, make_gpu_multiscale_array, gpu_slab_plan,
// estimate_gpu_array_memory), on the GPU: the file is compiled in here
// unchanged, over the test doubles of binding_doubles.hh for the three
// reference classes whose definitions do not build from this image, and
// over the reference's own ArrayConfig, ArrayDimensions, Downsampler,
// ThreadPool and logger (compiled from /root/reference by oracle/Makefile,
// target `binding`, into oracle/_ref/binding_exec).
//
// It does what ZarrStream_s does with a multiscale array: the ArrayConfig
// of make_array_config (zarr.stream.cpp:330-375, with make_compression_
// params :191-208 and make_array_dimensions :210-242), the hook of
// configure_array_ (:1232-1279), write_frame per
// frame with frame ids, and finalize_array at the end.
//
//   binding_exec JOB OUT
//
// JOB: the handoff_replay job ("AQZ2", tests/test_gpu_handoff.py), with
//   batch 0 = the hook (make_gpu_multiscale_array: its defaults) instead of
//   the constructor with (batch, host_slots); z_slabs >= 2 sets AQZ_Z_SLABS
//   (every slab on the visible device(s), as select_device hands them out);
//   frames follow (synth 0), or synth 1 / 2: camera-like / random frames
//   made here (synth_frames.hh, 8 distinct frames round robin).
// OUT: the AQZ4 records of handoff_replay, made from what the shard doubles
//   received: per level, every (append-shard row, shard, internal index)
//   written or skipped, mapped back to (layer, chunk) through the level's
//   ArrayDimensions (chunk 0xffffffff: a shard's ragged padding), and the
//   frame counts at each Array::rollover_.
//   OUT "-": a timing run -- nothing written, chunk sizes only.
// stdout: one JSON summary line; exit 0 only if the binding's calls all
//   returned what the reference's interface promises and no double
//   recorded an error.
#include "binding_doubles.hh"
#include "synth_frames.hh"

// the binding itself, unchanged
#include "multiscale.array.gpu.cpp"

#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <atomic>
#include <thread>
#include <tuple>

namespace {

template<class T>
bool
rd(FILE* f, T* v, size_t n = 1)
{
    return fread(v, sizeof(T), n, f) == n;
}

const char* const kNames[] = { "a", "b", "c", "d", "e", "f", "g", "h" };

std::string
json_str(const std::string& s)
{
    std::string o = "\"";
    for (char c : s)
        o += c == '"' || c == '\\' ? std::string("\\") + c : (c == '\n' ? " " : std::string(1, c));
    return o + "\"";
}

} // namespace

int
main(int argc, char** argv)
{
    using namespace zarr;
    if (argc != 3)
        return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f)
        return 2;
    char magic[4];
    uint32_t nd = 0;
    if (!rd(f, magic, 4) || memcmp(magic, "AQZ2", 4) || !rd(f, &nd) || nd < 3 || nd > 8)
        return 2;
    std::vector<aqz_dimension> jd(nd);
    for (auto& d : jd)
        if (!rd(f, &d.type) || !rd(f, &d.array_size_px) || !rd(f, &d.chunk_size_px) ||
            !rd(f, &d.shard_size_chunks))
            return 2;
    int32_t dtype, method, device, codec, clevel, shuffle;
    uint32_t batch, slots, copy_threads, pool_threads, synth, tries, n_slabs;
    uint64_t n_frames, fbytes;
    if (!rd(f, &dtype) || !rd(f, &method) || !rd(f, &batch) || !rd(f, &slots) ||
        !rd(f, &device) || !rd(f, &codec) || !rd(f, &clevel) || !rd(f, &shuffle) ||
        !rd(f, &copy_threads) || !rd(f, &pool_threads) || !rd(f, &synth) || !rd(f, &tries) ||
        !rd(f, &n_slabs) || !rd(f, &n_frames) || !rd(f, &fbytes) || n_frames == 0)
        return 2;
    // the caller's frame vectors (ZarrStream_s hands write_frame its own)
    std::vector<std::vector<uint8_t>> frames;
    if (synth == 0) {
        frames.assign(n_frames, std::vector<uint8_t>(fbytes));
        for (auto& fr : frames)
            if (!rd(f, fr.data(), fbytes))
                return 2;
    } else {
        const uint32_t R = uint32_t(std::min<uint64_t>(n_frames, 8));
        const std::vector<uint8_t> v = aqz_test::synth_frames(synth, dtype, fbytes, R);
        for (uint32_t i = 0; i < R; ++i)
            frames.emplace_back(v.begin() + i * fbytes, v.begin() + (i + 1) * fbytes);
    }
    fclose(f);
    const bool record = std::strcmp(argv[2], "-") != 0;
    binding_log().keep_bytes = record;
    (void)copy_threads;
    (void)tries;
    if (n_slabs > 1)
        setenv("AQZ_Z_SLABS", std::to_string(n_slabs).c_str(), 1);
    setenv("AQZ_DEVICE", std::to_string(device).c_str(), 0);

    // the ZarrArraySettings a caller configures (zarr.types.h:150-169)
    std::vector<ZarrDimensionProperties> props(nd);
    for (uint32_t i = 0; i < nd; ++i)
        props[i] = ZarrDimensionProperties{ kNames[i],
                                            ZarrDimensionType(jd[i].type),
                                            jd[i].array_size_px,
                                            jd[i].chunk_size_px,
                                            jd[i].shard_size_chunks,
                                            nullptr,
                                            0.0 };
    ZarrCompressionSettings cs{};
    cs.compressor = codec == 0   ? ZarrCompressor_None
                    : codec == 3 ? ZarrCompressor_Zstd
                                 : ZarrCompressor_Blosc1;
    cs.codec = codec == 1 ? ZarrCompressionCodec_BloscLZ4 : ZarrCompressionCodec_BloscZstd;
    cs.level = uint8_t(clevel);
    cs.shuffle = uint8_t(shuffle);
    ZarrArraySettings settings{};
    settings.output_key = nullptr;
    settings.compression_settings = codec ? &cs : nullptr;
    settings.dimensions = props.data();
    settings.dimension_count = nd;
    settings.data_type = ZarrDataType(dtype);
    settings.multiscale = true;
    settings.downsampling_method = ZarrDownsamplingMethod(method);
    settings.max_levels = 0;
    // BINDING_EXEC_ORDER="0,2,1": the array's storage_dimension_order
    std::vector<size_t> order;
    if (const char* o = std::getenv("BINDING_EXEC_ORDER")) {
        for (const char* c = o; *c;) {
            order.push_back(size_t(std::strtoul(c, const_cast<char**>(&c), 10)));
            if (*c == ',')
                ++c;
        }
        if (order.size() != nd)
            return 2;
    }
    settings.storage_dimension_order = order.empty() ? nullptr : order.data();

    // make_array_config (zarr.stream.cpp:330-375)
    std::vector<ZarrDimension> zd;
    for (const auto& p : props)
        zd.emplace_back(p.name, p.type, p.array_size_px, p.chunk_size_px, p.shard_size_chunks,
                        "", 1.0);
    auto dims = std::make_shared<ArrayDimensions>(std::move(zd), settings.data_type, order);
    auto config = std::make_shared<ArrayConfig>(
      "/binding_exec", "", std::nullopt, compression_params_of(settings.compression_settings),
      dims, settings.data_type, std::optional(settings.downsampling_method), 0,
      settings.max_levels);
    auto pool = std::make_shared<ThreadPool>(
      std::max(1u, pool_threads),
      [](const std::string& e) { binding_log().error("thread pool: " + e); });

    std::vector<std::string> failures;
    auto fail = [&](const std::string& s) { failures.push_back(s); };
    // BINDING_EXEC_PROGRESS=file: a line every 10 s (phase, frames written,
    // chunks the shard doubles received), so a stalled run says where it is
    std::atomic<int> phase{ 0 };
    std::atomic<uint64_t> frames_done{ 0 };
    std::atomic<bool> stop_watch{ false };
    std::thread watch;
    if (const char* pf = std::getenv("BINDING_EXEC_PROGRESS")) {
        watch = std::thread([&, path = std::string(pf)] {
            const char* names[] = { "construct", "write_frame", "close", "teardown" };
            for (int k = 1; !stop_watch.load(); ++k) {
                for (int i = 0; i < 100 && !stop_watch.load(); ++i)
                    std::this_thread::sleep_for(std::chrono::milliseconds(100));
                if (stop_watch.load())
                    break;
                size_t chunks = 0;
                {
                    std::lock_guard lk(binding_log().mu);
                    chunks = binding_log().chunks.size();
                }
                if (FILE* w = fopen(path.c_str(), "a")) {
                    fprintf(w, "%s t=%ds phase=%s frames=%llu/%llu chunks=%zu\n", argv[1], 10 * k,
                            names[phase.load()], (unsigned long long)frames_done.load(),
                            (unsigned long long)n_frames, chunks);
                    fclose(w);
                }
            }
        });
    }
    // every return below stops and joins the watchdog first
    struct WatchGuard
    {
        std::atomic<bool>& stop;
        std::thread& t;
        ~WatchGuard()
        {
            stop = true;
            if (t.joinable())
                t.join();
        }
    } watch_guard{ stop_watch, watch };
    const auto t0 = std::chrono::steady_clock::now();
    std::unique_ptr<GpuMultiscaleArrayBase> array;
    bool factory = batch == 0;
    try {
        if (factory) {
            // the hook configure_array_ calls (zarr.stream.cpp:1252-1258)
            array = make_gpu_multiscale_array(config, pool, nullptr, nullptr, settings);
            if (!array) {
                fprintf(stderr, "make_gpu_multiscale_array: nullptr\n");
                return 1;
            }
        } else {
            int32_t n = 0;
            if (aqz_device_count(&n) != AQZ_STATUS_SUCCESS)
                return 1;
            const auto plan = gpu_slab_plan(settings);
            std::vector<int32_t> devs;
            for (size_t r = 0; r < std::max<size_t>(1, plan.begin.size()); ++r)
                devs.push_back(aqz_binding::select_device(n));
            array = std::make_unique<GpuMultiscaleArray>(config, pool, nullptr, nullptr,
                                                         settings, devs, plan, batch, slots);
        }
    } catch (const std::exception& e) {
        fprintf(stderr, "constructing the binding: %s\n", e.what());
        return 1;
    }
    auto* gpu = dynamic_cast<GpuMultiscaleArray*>(array.get());
    if (!gpu)
        return 1;

    // Array::write_frame's refusals (array.cpp:160-189), before any frame
    size_t bw = 7;
    {
        std::vector<uint8_t> short_frame(fbytes - 1);
        if (gpu->write_frame(short_frame, bw, 0) != WriteResult::FrameSizeMismatch || bw != 0)
            fail("a short frame was not refused with FrameSizeMismatch");
        bw = 7;
        if (gpu->write_frame(frames[0], bw, 1) != WriteResult::FrameOutOfOrder || bw != 0)
            fail("frame id 1 first was not refused with FrameOutOfOrder");
    }
    size_t mem_during = 0;
    const auto t_frames = std::chrono::steady_clock::now();
    phase = 1;
    for (uint64_t i = 0; i < n_frames; ++i, frames_done = i) {
        const WriteResult r = gpu->write_frame(frames[i % frames.size()], bw, i);
        if (r != WriteResult::Ok || bw != fbytes) {
            fail("write_frame " + std::to_string(i) + " returned " + std::to_string(int(r)));
            break;
        }
        if (i == n_frames / 2)
            mem_during = gpu->memory_usage();
    }
    // a bounded append dimension, filled: one more frame is out of bounds
    // (array.cpp:176-189) and writes nothing
    const size_t max = gpu->max_bytes();
    bool oob_probed = false;
    if (max > 0 && n_frames * fbytes == max) {
        bw = 7;
        oob_probed = true;
        if (gpu->write_frame(frames[0], bw, n_frames) != WriteResult::OutOfBounds || bw != 0)
            fail("a frame past the bounded append dimension was not refused");
    }
    const size_t mem_end = gpu->memory_usage();
    const size_t dev_mem = gpu->device_memory_usage();
    const aqz_binding::MemoryEstimate est =
      factory ? estimate_gpu_array_memory(settings)
              : estimate_gpu_array_memory(settings, batch, slots);
    // levels: the base's writer configurations (the reference Downsampler)
    std::vector<std::shared_ptr<ArrayDimensions>> level_dims;
    {
        Downsampler ds(std::make_shared<ArrayConfig>("/binding_exec", "/0", std::nullopt,
                                                     config->compression_params, dims,
                                                     config->dtype, std::nullopt, 0, 0),
                       settings.downsampling_method);
        const auto& cfgs = ds.writer_configurations();
        level_dims.resize(cfgs.size());
        for (const auto& [lod, c] : cfgs)
            level_dims[lod] = c->dimensions;
    }
    bool closed = false;
    try {
        phase = 2;
        closed = array->finalize(); // finalize_array -> GpuMultiscaleArray::close_
    } catch (const std::exception& e) {
        fail(std::string("close: ") + e.what());
    }
    if (!closed)
        fail("close_ returned false");
    // close_ has drained every chunk job (Array::close_ waits on
    // write_counter_): the stream's data is in the shards
    const auto t_closed = std::chrono::steady_clock::now();
    const uint64_t group_md = array->group_metadata_writes();
    phase = 3;
    array.reset();
    pool->await_stop();
    stop_watch = true;
    // first write_frame to close_ done: the stream's rate; the one-off
    // costs (stage creation and placement, teardown) apart
    const auto t_end = std::chrono::steady_clock::now();
    const double seconds = std::chrono::duration<double>(t_closed - t_frames).count();
    const double construct_seconds = std::chrono::duration<double>(t_frames - t0).count();
    const double destroy_seconds = std::chrono::duration<double>(t_end - t_closed).count();

    BindingLog& log = binding_log();
    const uint32_t nl = uint32_t(level_dims.size());
    if (log.levels.size() != nl)
        fail("closed levels " + std::to_string(log.levels.size()) + " of " + std::to_string(nl));
    // every shard: finalized once, complete unless it is in the last,
    // partial append-shard row
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, int> ends;
    uint64_t by_countdown = 0, at_close = 0, incomplete = 0;
    for (const auto& e : log.shard_ends) {
        if (++ends[{ e.level, e.append, e.shard }] != 1)
            fail("a shard finalized twice");
        by_countdown += e.by_countdown;
        at_close += !e.by_countdown;
        incomplete += !e.complete;
    }

    // per level: every shard of every completed append-shard row finalized
    // by its countdown, complete; the open row's shards (if any frames
    // reached it) finalized at close
    for (uint32_t l = 0; l < nl && l < log.levels.size(); ++l) {
        const ArrayDimensions& d = *level_dims[l];
        const uint32_t ns = d.number_of_shards();
        const auto& e = log.levels[l];
        uint64_t row_frames = uint64_t(d.final_dim().chunk_size_px) * d.final_dim().shard_size_chunks;
        for (size_t i = 1; i + 2 < d.ndims(); ++i)
            row_frames *= d.at(i).array_size_px;
        const uint64_t rows_done = e.frames_written / row_frames;
        if (e.rollovers.size() != rows_done)
            fail("level " + std::to_string(l) + ": " + std::to_string(e.rollovers.size()) +
                 " rollovers for " + std::to_string(rows_done) + " complete rows");
        const bool open_row = e.frames_written % row_frames != 0;
        for (uint32_t a = 0; a < rows_done + (open_row ? 1 : 0); ++a)
            for (uint32_t sh = 0; sh < ns; ++sh) {
                const BindingLog::ShardEnd* end = nullptr;
                for (const auto& x : log.shard_ends)
                    if (x.level == l && x.append == a && x.shard == sh)
                        end = &x;
                const std::string w = "level " + std::to_string(l) + " row " +
                                      std::to_string(a) + " shard " + std::to_string(sh);
                if (!end)
                    fail(w + ": never finalized");
                else if (a < rows_done && !(end->complete && end->by_countdown))
                    fail(w + ": a completed row's shard did not finish its countdown");
            }
    }

    // the records, mapped back to (layer, chunk)
    std::vector<std::vector<const BindingLog::Chunk*>> per_level(nl);
    for (const auto& c : log.chunks)
        if (c.level < nl)
            per_level[c.level].push_back(&c);
    FILE* o = fopen(record ? argv[2] : "/dev/null", "wb");
    if (!o)
        return 2;
    fwrite("AQZ4", 1, 4, o);
    fwrite(&nl, 4, 1, o);
    for (uint32_t l = 0; l < nl; ++l) {
        const ArrayDimensions& d = *level_dims[l];
        const uint32_t n_mem = d.number_of_chunks_in_memory();
        const uint32_t lps = d.final_dim().shard_size_chunks;
        std::map<std::pair<uint32_t, uint32_t>, uint32_t> inv; // (shard, internal) -> c
        for (uint32_t c = 0; c < lps * n_mem; ++c)
            inv[{ d.shard_index_for_chunk(c), d.shard_internal_index(c) }] = c;
        const uint64_t n = per_level[l].size();
        fwrite(&n, 8, 1, o);
        for (const auto* r : per_level[l]) {
            uint64_t layer = 0;
            uint32_t chunk = 0xffffffffu;
            auto it = inv.find({ r->shard, r->internal });
            if (it != inv.end()) {
                layer = uint64_t(r->append) * lps + it->second / n_mem;
                chunk = it->second % n_mem;
            } else {
                bool found = false;
                for (uint32_t k = 0; k < lps && !found; ++k)
                    for (uint32_t s : d.skipped_internal_indices_for_shard_layer(r->shard, k))
                        if (s == r->internal) {
                            layer = uint64_t(r->append) * lps + k;
                            found = true;
                            break;
                        }
                if (!found)
                    fail("level " + std::to_string(l) + ": internal index " +
                         std::to_string(r->internal) + " of shard " + std::to_string(r->shard) +
                         " is neither a chunk nor padding");
                if (!r->skipped)
                    fail("ragged padding written with bytes");
            }
            const uint64_t nb = r->bytes.size();
            fwrite(&layer, 8, 1, o);
            fwrite(&chunk, 4, 1, o);
            fwrite(&r->append, 4, 1, o);
            fwrite(&r->shard, 4, 1, o);
            fwrite(&r->internal, 4, 1, o);
            fwrite(&nb, 8, 1, o);
            fwrite(r->bytes.data(), 1, nb, o);
        }
        const std::vector<uint64_t>& rolls = log.levels[l].rollovers;
        const uint64_t nr = rolls.size();
        fwrite(&nr, 8, 1, o);
        fwrite(rolls.data(), 8, nr, o);
    }
    fclose(o);

    for (const auto& e : log.errors)
        fail(e);
    uint64_t chunk_bytes = 0;
    for (const auto& c : log.chunks)
        chunk_bytes += c.nbytes;
    std::string lv = "[";
    for (uint32_t l = 0; l < nl; ++l) {
        const auto& e = log.levels[l];
        std::string rolls;
        for (uint64_t r : e.rollovers)
            rolls += (rolls.empty() ? "" : ", ") + std::to_string(r);
        char b[512];
        snprintf(b, sizeof b,
                 "%s{\"level\": %u, \"frames_written\": %llu, \"total_bytes_written\": %llu, "
                 "\"last_frame_id\": %llu, \"bytes_to_flush\": %llu, \"flushed_band_count\": %u, "
                 "\"append_chunk_index\": %u, \"current_layer\": %u, \"metadata_writes\": %llu, "
                 "\"closed\": %s, \"rollovers\": [%s]}",
                 l ? ", " : "", l, (unsigned long long)e.frames_written,
                 (unsigned long long)e.total_bytes_written, (unsigned long long)e.last_frame_id,
                 (unsigned long long)e.bytes_to_flush, e.flushed_band_count,
                 e.append_chunk_index, e.current_layer, (unsigned long long)e.metadata_writes,
                 e.closed ? "true" : "false", rolls.c_str());
        lv += b;
    }
    lv += "]";
    std::string errs = "[";
    for (size_t i = 0; i < failures.size() && i < 8; ++i)
        errs += (i ? ", " : "") + json_str(failures[i]);
    errs += "]";
    printf("{\"summary\": true, \"ok\": %s, \"failures\": %zu, \"errors\": %s, "
           "\"factory\": %s, \"n_levels\": %u, \"frames\": %llu, \"seconds\": %.4f, "
           "\"construct_seconds\": %.4f, \"destroy_seconds\": %.4f, "
           "\"input_gbs\": %.3f, \"sink_bytes_per_input_byte\": %.4f, \"codec\": %d, "
           "\"chunks_recorded\": %zu, \"shards_by_countdown\": %llu, \"shards_at_close\": %llu, "
           "\"shards_incomplete\": %llu, \"group_metadata_writes\": %llu, "
           "\"memory_usage_mid\": %zu, \"memory_usage_end\": %zu, \"device_memory_usage\": %zu, "
           "\"estimate_host_bytes\": %llu, \"estimate_device_bytes\": %llu, "
           "\"max_bytes\": %zu, \"oob_probed\": %s, \"levels\": %s}\n",
           failures.empty() ? "true" : "false", failures.size(), errs.c_str(),
           factory ? "true" : "false", nl, (unsigned long long)n_frames, seconds, construct_seconds, destroy_seconds,
           double(n_frames) * double(fbytes) / seconds / 1e9,
           double(chunk_bytes) / (double(n_frames) * double(fbytes)), codec, log.chunks.size(),
           (unsigned long long)by_countdown, (unsigned long long)at_close,
           (unsigned long long)incomplete, (unsigned long long)group_md, mem_during, mem_end,
           dev_mem, (unsigned long long)est.host_bytes, (unsigned long long)est.device_bytes,
           max, oob_probed ? "true" : "false", lv.c_str());
    return failures.empty() ? 0 : 1;
}
