// aqz_capi.cpp -- extern "C" boundary (include/aqz_gpu.h).  No exception or
// HIP error crosses it: everything maps to a ZarrStatusCode value.
#include "aqz_gpu.h"
#include "aqz_gpu_bench.h"

#include "aqz_engine.hh"

#include <cstring>
#include <new>
#include <string>

using namespace aqz;

struct aqz_dims
{
    std::unique_ptr<ArrayDimensions> ad;
};
struct aqz_downsampler
{
    std::unique_ptr<GpuDownsampler> ds;
    int32_t sticky = AQZ_STATUS_SUCCESS;
};
struct aqz_stage
{
    std::unique_ptr<Stage> st;
    int32_t sticky = AQZ_STATUS_SUCCESS;
};
struct aqz_compressor
{
    std::unique_ptr<Compressor> c;
    int32_t sticky = AQZ_STATUS_SUCCESS;
};

namespace {

thread_local std::string t_last_error;

template<typename F>
aqz_status
guard(F&& f)
{
    try {
        f();
        return AQZ_STATUS_SUCCESS;
    } catch (const Error& e) {
        t_last_error = e.what();
        return e.status;
    } catch (const std::bad_alloc&) {
        t_last_error = "out of memory";
        return AQZ_STATUS_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        t_last_error = e.what();
        return AQZ_STATUS_INTERNAL_ERROR;
    } catch (...) {
        t_last_error = "unknown exception";
        return AQZ_STATUS_INTERNAL_ERROR;
    }
}

// Device/internal errors are sticky on an object, like ZarrStream_s::error_.
template<typename O, typename F>
aqz_status
guard_sticky(O* o, F&& f)
{
    if (!o)
        return AQZ_STATUS_INVALID_ARGUMENT;
    if (o->sticky != AQZ_STATUS_SUCCESS) {
        t_last_error = "object is in a sticky error state from an earlier call";
        return o->sticky;
    }
    const aqz_status s = guard(std::forward<F>(f));
    if (s == AQZ_STATUS_INTERNAL_ERROR || s == AQZ_STATUS_OUT_OF_MEMORY)
        o->sticky = s;
    return s;
}

// A stage's work (and its lazily allocated buffers) belongs to its device,
// whichever device the calling thread had current: one consumer thread may
// drive stages on several GPUs (AQZ_DEVICE round robin, z slabs).
struct DeviceScope
{
    int prev = -1;
    explicit DeviceScope(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess || prev == dev) {
            prev = -1;
            (void)hipGetLastError();
            return;
        }
        (void)hipSetDevice(dev);
    }
    ~DeviceScope()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

template<typename F>
aqz_status
guard_sticky(aqz_stage* o, F&& f)
{
    if (!o || !o->st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    DeviceScope ds(o->st->device());
    return guard_sticky<aqz_stage>(o, std::forward<F>(f));
}

std::vector<Dim>
to_dims(const aqz_dimension* d, size_t n)
{
    if (!d && n)
        throw Error(AQZ_STATUS_INVALID_ARGUMENT, "null dimensions");
    std::vector<Dim> v(n);
    for (size_t i = 0; i < n; ++i)
        v[i] = Dim{ d[i].type, d[i].array_size_px, d[i].chunk_size_px,
                    d[i].shard_size_chunks };
    return v;
}

ArrayDesc
to_desc(const aqz_array_desc* d)
{
    if (!d)
        throw Error(AQZ_STATUS_INVALID_ARGUMENT, "null desc");
    ArrayDesc a;
    a.dims = to_dims(d->dimensions, d->dimension_count);
    a.dtype = d->data_type;
    a.multiscale = d->multiscale != 0;
    a.method = d->downsampling_method;
    a.max_levels = d->max_levels;
    if (d->storage_dimension_order)
        a.storage_order.assign(d->storage_dimension_order,
                               d->storage_dimension_order + d->dimension_count);
    a.device = d->device;
    if (a.dtype < 0 || a.dtype >= AQZ_DTYPE_COUNT)
        throw Error(AQZ_STATUS_INVALID_ARGUMENT, "Invalid data type");
    return a;
}

void
put_dims(const std::vector<Dim>& v, aqz_dimension* out, size_t cap,
         size_t* ndims)
{
    if (ndims)
        *ndims = v.size();
    if (out) {
        if (cap < v.size())
            throw Error(AQZ_STATUS_OVERFLOW, "output too small");
        for (size_t i = 0; i < v.size(); ++i)
            out[i] = aqz_dimension{ v[i].type, v[i].array_size_px,
                                    v[i].chunk_size_px,
                                    v[i].shard_size_chunks };
    }
}

} // namespace

extern "C" {

const char*
aqz_version(void)
{
    return "0.1.0";
}

const char*
aqz_last_error(void)
{
    return t_last_error.c_str();
}

const char*
aqz_status_message(aqz_status s)
{
    // same strings as Zarr_get_status_message (src/streaming/acquire.zarr.cpp)
    switch (s) {
        case 0: return "Success";
        case 1: return "Invalid argument";
        case 2: return "Buffer overflow";
        case 3: return "Invalid index";
        case 4: return "Not yet implemented";
        case 5: return "Internal error";
        case 6: return "Out of memory";
        case 7: return "I/O error";
        case 8: return "Error compressing";
        case 9: return "Invalid settings";
        case 10: return "Refusing to overwrite existing data";
        case 11: return "Data partially written";
        case 12: return "Attempted write beyond array boundary";
        case 13: return "Array key not found";
        default: return "Unknown error";
    }
}

aqz_status
aqz_device_count(int32_t* count)
{
    if (!count)
        return AQZ_STATUS_INVALID_ARGUMENT;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    *count = n;
    return AQZ_STATUS_SUCCESS;
}

// ---- dims ----------------------------------------------------------------
aqz_status
aqz_dims_create(const aqz_dimension* dims, size_t ndims, int32_t data_type,
                const size_t* storage_order, aqz_dims** out)
{
    if (!out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *out = nullptr;
    return guard([&] {
        std::vector<size_t> ord;
        if (storage_order)
            ord.assign(storage_order, storage_order + ndims);
        auto* d = new aqz_dims;
        try {
            d->ad = std::make_unique<ArrayDimensions>(to_dims(dims, ndims),
                                                      data_type, ord);
        } catch (...) {
            delete d;
            throw;
        }
        *out = d;
    });
}

void
aqz_dims_destroy(aqz_dims* d)
{
    delete d;
}

size_t
aqz_dims_ndims(const aqz_dims* d)
{
    return d ? d->ad->ndims() : 0;
}

aqz_status
aqz_dims_get(const aqz_dims* d, size_t i, aqz_dimension* out)
{
    if (!d || !out || i >= d->ad->ndims())
        return AQZ_STATUS_INVALID_ARGUMENT;
    const Dim& x = d->ad->at(i);
    *out = aqz_dimension{ x.type, x.array_size_px, x.chunk_size_px,
                          x.shard_size_chunks };
    return AQZ_STATUS_SUCCESS;
}

uint32_t
aqz_dims_tile_group_offset(const aqz_dims* d, uint64_t fid)
{
    return d->ad->tile_group_offset(fid);
}

uint64_t
aqz_dims_chunk_internal_offset(const aqz_dims* d, uint64_t fid)
{
    return d->ad->chunk_internal_offset(fid);
}

uint32_t
aqz_dims_chunk_lattice_index(const aqz_dims* d, uint64_t fid, uint32_t dim)
{
    try {
        return d->ad->chunk_lattice_index(fid, dim);
    } catch (...) {
        return UINT32_MAX;
    }
}

uint64_t
aqz_dims_transpose_frame_id(const aqz_dims* d, uint64_t fid)
{
    try {
        return d->ad->transpose_frame_id(fid);
    } catch (...) {
        return UINT64_MAX;
    }
}

uint64_t
aqz_dims_bytes_per_chunk(const aqz_dims* d)
{
    return d->ad->bytes_per_chunk();
}

uint32_t
aqz_dims_number_of_chunks_in_memory(const aqz_dims* d)
{
    return d->ad->number_of_chunks_in_memory();
}

uint64_t
aqz_dims_frames_per_chunk_layer(const aqz_dims* d)
{
    return d->ad->frames_per_chunk_layer();
}

uint32_t
aqz_dims_shard_index_for_chunk(const aqz_dims* d, uint32_t c)
{
    try {
        return d->ad->shard_index_for_chunk(c);
    } catch (...) {
        return UINT32_MAX;
    }
}

uint32_t
aqz_dims_shard_internal_index(const aqz_dims* d, uint32_t c)
{
    try {
        return d->ad->shard_internal_index(c);
    } catch (...) {
        return UINT32_MAX;
    }
}

aqz_status
aqz_dims_shard_geometry(const aqz_dims* d, uint32_t* chunks_per_shard, uint32_t* n_shards,
                        uint32_t* layers_per_shard)
{
    if (!d)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        const ArrayDimensions& a = *d->ad;
        if (chunks_per_shard)
            *chunks_per_shard = a.chunks_per_shard();
        if (n_shards)
            *n_shards = a.number_of_shards();
        if (layers_per_shard)
            *layers_per_shard = a.chunk_layers_per_shard();
    });
}

aqz_status
aqz_dims_skipped_internal_indices(const aqz_dims* d, uint32_t shard, uint32_t layer,
                                  uint32_t* out, size_t cap, size_t* n)
{
    if (!d || !n || (cap && !out))
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        const ArrayDimensions& a = *d->ad;
        if (shard >= a.number_of_shards() ||
            layer >= std::max<uint32_t>(1, a.chunk_layers_per_shard()))
            throw Error(AQZ_STATUS_INVALID_ARGUMENT, "shard or layer out of range");
        const auto v = a.skipped_internal_indices_for_shard_layer(shard, layer);
        *n = v.size();
        for (size_t i = 0; i < v.size() && i < cap; ++i)
            out[i] = v[i];
    });
}

aqz_status
aqz_dims_dim1_banding(const aqz_dims* d, int32_t* supported, uint32_t* n_bands,
                      uint64_t* frames_per_band, uint32_t* chunks_per_band)
{
    if (!d)
        return AQZ_STATUS_INVALID_ARGUMENT;
    const ArrayDimensions& a = *d->ad;
    if (supported)
        *supported = a.supports_dim1_banding() ? 1 : 0;
    if (n_bands)
        *n_bands = a.dim1_band_count();
    if (frames_per_band)
        *frames_per_band = a.frames_per_dim1_band();
    if (chunks_per_band)
        *chunks_per_band = a.chunks_per_dim1_band();
    return AQZ_STATUS_SUCCESS;
}

aqz_status
aqz_dims_split_frame_rows(const aqz_dims* d, const void* frame, uint64_t frame_id,
                          uint32_t row_begin, uint32_t row_end, uint32_t chunk0, void* dst,
                          size_t cap, uint8_t* has_data, size_t has_data_cap)
{
    if (!d || !frame || !dst || !has_data)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        const ArrayDimensions& a = *d->ad;
        const uint64_t n = std::min<uint64_t>(cap / a.bytes_per_chunk(), has_data_cap);
        if (n == 0 || chunk0 >= a.number_of_chunks_in_memory())
            throw Error(1, "destination holds no chunk of the layer");
        split_rows(split_geom(a, frame_id), static_cast<const uint8_t*>(frame), row_begin,
                   row_end, static_cast<uint8_t*>(dst), chunk0,
                   uint32_t(std::min<uint64_t>(n, a.number_of_chunks_in_memory() - chunk0)),
                   has_data);
    });
}

aqz_status
aqz_pyramid_levels(const aqz_dimension* dims, size_t ndims, uint32_t max_levels,
                   uint32_t* n_levels, aqz_dimension* out_dims, size_t out_cap)
{
    return guard([&] {
        auto v = to_dims(dims, ndims);
        if (v.size() == 2)
            v.insert(v.begin(), Dim{ kOther, 1, 1, 1 });
        const auto levels = make_pyramid_levels(v, max_levels);
        if (n_levels)
            *n_levels = uint32_t(levels.size());
        if (out_dims) {
            if (out_cap < levels.size() * v.size())
                throw Error(AQZ_STATUS_OVERFLOW, "output too small");
            size_t j = 0;
            for (const auto& l : levels)
                for (const auto& x : l)
                    out_dims[j++] = aqz_dimension{ x.type, x.array_size_px,
                                                   x.chunk_size_px,
                                                   x.shard_size_chunks };
        }
    });
}

// ---- downsampler -------------------------------------------------------------
aqz_status
aqz_downsampler_create(const aqz_array_desc* desc, aqz_downsampler** out)
{
    if (!out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *out = nullptr;
    return guard([&] {
        const ArrayDesc a = to_desc(desc);
        auto* d = new aqz_downsampler;
        try {
            d->ds = std::make_unique<GpuDownsampler>(a);
        } catch (...) {
            delete d;
            throw;
        }
        *out = d;
    });
}

void
aqz_downsampler_destroy(aqz_downsampler* ds)
{
    try {
        delete ds;
    } catch (...) {
    }
}

uint32_t
aqz_downsampler_n_levels(const aqz_downsampler* ds)
{
    return ds ? ds->ds->n_levels() : 0;
}

aqz_status
aqz_downsampler_level_dims(const aqz_downsampler* ds, uint32_t level,
                           aqz_dimension* out, size_t cap, size_t* ndims)
{
    if (!ds)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] { put_dims(ds->ds->level_dims(level), out, cap, ndims); });
}

aqz_status
aqz_downsampler_add_frame(aqz_downsampler* ds, const void* frame, size_t nbytes,
                          int32_t mem)
{
    return guard_sticky(ds, [&] { ds->ds->add_frame(frame, nbytes, mem); });
}

aqz_status
aqz_downsampler_take_frame(aqz_downsampler* ds, uint32_t level, void* dst,
                           size_t cap, int32_t mem, size_t* nbytes,
                           int32_t* found)
{
    return guard_sticky(ds, [&] {
        const bool f = ds->ds->take_frame(level, dst, cap, mem, nbytes);
        if (found)
            *found = f ? 1 : 0;
    });
}

const char*
aqz_downsampler_method_name(const aqz_downsampler* ds)
{
    return ds ? ds->ds->method_name() : "";
}

static void
put_string(const std::string& s, char* buf, size_t cap, size_t* len)
{
    if (len)
        *len = s.size();
    if (buf) {
        if (cap < s.size() + 1)
            throw Error(AQZ_STATUS_OVERFLOW, "buffer too small");
        std::memcpy(buf, s.c_str(), s.size() + 1);
    }
}

aqz_status
aqz_downsampler_metadata_json(const aqz_downsampler* ds, char* buf, size_t cap,
                              size_t* len)
{
    if (!ds)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] { put_string(ds->ds->metadata_json(), buf, cap, len); });
}

const char*
aqz_downsampling_method_name(int32_t method)
{
    try {
        return downsampling_method_name(method);
    } catch (...) {
        return "";
    }
}

aqz_status
aqz_downsampling_metadata_json(int32_t method, char* buf, size_t cap, size_t* len)
{
    return guard([&] { put_string(downsampling_metadata_json(method), buf, cap, len); });
}

// ---- stage ---------------------------------------------------------------------
static void
apply_bench(const aqz_stage_bench_options* bench, StageOptions& o)
{
    if (!bench)
        return;
    o.force_levels = bench->force_levels;
    o.skip_level0_split = o.skip_level0_split || bench->skip_level0_split != 0;
    if (bench->placement_tries)
        o.placement_tries = bench->placement_tries;
    if (bench->placement_reps)
        o.placement_reps = bench->placement_reps;
    o.placement_never_accept = (bench->placement_flags & 1u) != 0;
    o.knobs = bench->knobs;
    if (bench->nt_policy)
        o.nt_mode = bench->nt_policy & 7u;
    o.xcd_rot = bench->xcd_rot;
    o.region_rows_log2 = bench->region_rows_log2;
    o.chunk_pad = bench->chunk_pad_bytes;
    o.ring_malloc_flags = bench->ring_malloc_flags;
    o.ring_spacer = bench->ring_spacer_bytes;
    o.ring_arena = bench->ring_arena_bytes;
    const uint32_t z = bench->zstd_flags;
    o.codec.match = (z & 1u) ? 0 : 1;
    o.codec.far = (z & 2u) ? 0 : 1;
    o.codec.fit = (z & 4u) ? 0 : 1;
    o.codec.phist = (z >> 8) & 0xffu;
    o.codec.parse = (z >> 16) & 0xfu;
    o.codec.vmm = (z >> 20) & 1u;
    o.codec.ranges = (z & (1u << 21)) ? 0 : 1;
}

static void
apply_options(const aqz_stage_options* opt, StageOptions& o)
{
    if (!opt)
        return;
    o.layer_slots = opt->layer_slots;
    o.max_batch_frames = opt->max_batch_frames;
    o.first_frame = opt->first_frame;
    o.z_slab_begin = opt->z_slab_begin;
    o.z_slab_end = opt->z_slab_end;
    o.placement_tries = opt->placement_tries;
    o.level0_on_host = opt->level0_split_on_host != 0;
    o.skip_level0_split = o.skip_level0_split || o.level0_on_host;
}

static aqz_status
create_stage(const aqz_array_desc* desc, const aqz_stage_options* opt,
             const aqz_stage_bench_options* bench, aqz_stage** out)
{
    if (!out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *out = nullptr;
    return guard([&] {
        const ArrayDesc a = to_desc(desc);
        StageOptions o;
        apply_options(opt, o);
        apply_bench(bench, o);
        DeviceScope ds(a.device); // the caller's current device is kept
        auto* s = new aqz_stage;
        try {
            s->st = std::make_unique<Stage>(a, o);
        } catch (...) {
            delete s;
            throw;
        }
        *out = s;
    });
}

aqz_status
aqz_stage_create(const aqz_array_desc* desc, const aqz_stage_options* opt,
                 aqz_stage** out)
{
    return create_stage(desc, opt, nullptr, out);
}

aqz_status
aqz_stage_create_bench(const aqz_array_desc* desc, const aqz_stage_options* opt,
                       const aqz_stage_bench_options* bench, aqz_stage** out)
{
    return create_stage(desc, opt, bench, out);
}

aqz_status
aqz_stage_estimate_memory_bench(const aqz_array_desc* desc, const aqz_stage_options* opt,
                                const aqz_stage_bench_options* bench, aqz_memory_usage* out)
{
    if (!out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        const ArrayDesc a = to_desc(desc);
        StageOptions o;
        apply_options(opt, o);
        apply_bench(bench, o);
        const Footprint f = Stage::estimate_memory(a, o);
        *out = aqz_memory_usage{ f.device, f.pinned };
    });
}

aqz_status
aqz_stage_estimate_memory(const aqz_array_desc* desc, const aqz_stage_options* opt,
                          aqz_memory_usage* out)
{
    return aqz_stage_estimate_memory_bench(desc, opt, nullptr, out);
}

aqz_status
aqz_stage_memory_usage(const aqz_stage* st, aqz_memory_usage* out)
{
    if (!st || !out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        const Footprint f = st->st->memory_usage();
        *out = aqz_memory_usage{ f.device, f.pinned };
    });
}

aqz_status
aqz_stage_wait_stream(aqz_stage* st, void* stream)
{
    return guard_sticky(
      st, [&] { st->st->wait_stream(static_cast<hipStream_t>(stream)); });
}

aqz_status
aqz_stage_band_geometry(const aqz_stage* st, uint32_t level, int32_t* supported,
                        uint32_t* n_bands, uint64_t* frames_per_band,
                        uint32_t* chunks_per_band)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        st->st->band_geometry(level, supported, n_bands, frames_per_band, chunks_per_band);
    });
}

aqz_status
aqz_stage_copy_band_async(aqz_stage* st, uint32_t level, uint64_t layer, uint32_t band,
                          void* dst, size_t cap, uint8_t* has_data, size_t has_data_cap)
{
    return guard_sticky(st, [&] {
        st->st->copy_band_async(level, layer, band, dst, cap, has_data, has_data_cap);
    });
}

void
aqz_stage_destroy(aqz_stage* st)
{
    try {
        if (st && st->st) {
            DeviceScope ds(st->st->device());
            delete st;
        } else {
            delete st;
        }
    } catch (...) {
    }
}

uint32_t
aqz_stage_n_levels(const aqz_stage* st)
{
    return st ? st->st->n_levels() : 0;
}

aqz_status
aqz_stage_level_dims(const aqz_stage* st, uint32_t level, aqz_dimension* out,
                     size_t cap, size_t* ndims)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] { put_dims(st->st->level_dims(level), out, cap, ndims); });
}

aqz_status
aqz_stage_level_layout(const aqz_stage* st, uint32_t level,
                       aqz_level_layout* out)
{
    if (!st || !out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        const LevelLayout l = st->st->layout(level);
        *out = aqz_level_layout{ l.bytes_per_chunk, l.chunks_per_layer,
                                 l.layer_slots,     l.frames_per_layer,
                                 l.frame_bytes,     l.width,
                                 l.height,          l.chunk_pitch };
    });
}

aqz_status
aqz_stage_set_tuning(aqz_stage* st, uint32_t knobs, uint32_t nt)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] { st->st->set_tuning(knobs, nt); });
}

aqz_status
aqz_stage_import_frames(aqz_stage* dst, aqz_stage* src, uint32_t level, uint64_t layer,
                        uint32_t first, uint32_t count)
{
    if (!dst)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard_sticky(dst, [&] {
        dst->st->import_frames(src ? src->st.get() : nullptr, level, layer, first, count);
    });
}

aqz_status
aqz_stage_bind_host_thread(const aqz_stage* st)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] { st->st->bind_host_thread(); });
}

aqz_status
aqz_stage_bench_replace_rings(aqz_stage* st, uint32_t level_mask)
{
    return guard_sticky(st, [&] { st->st->replace_rings(level_mask); });
}

aqz_status
aqz_stage_bench_set_ring_offset(aqz_stage* st, uint64_t offset)
{
    return guard_sticky(st, [&] { st->st->set_ring_offset(offset); });
}

aqz_status
aqz_stage_set_stream(aqz_stage* st, void* stream)
{
    return guard_sticky(
      st, [&] { st->st->set_stream(static_cast<hipStream_t>(stream)); });
}

aqz_status
aqz_stage_append(aqz_stage* st, const void* frames, uint64_t n_frames,
                 int32_t mem)
{
    return guard_sticky(st, [&] {
        if (mem != AQZ_MEM_HOST && mem != AQZ_MEM_DEVICE && mem != AQZ_MEM_HOST_PINNED)
            throw aqz::Error(AQZ_STATUS_INVALID_ARGUMENT, "unknown memory kind");
        st->st->append(frames, n_frames, mem);
    });
}

aqz_status
aqz_stage_synchronize(aqz_stage* st)
{
    return guard_sticky(st, [&] { st->st->synchronize(); });
}

uint64_t
aqz_stage_frames_written(const aqz_stage* st, uint32_t level)
{
    if (!st || level >= st->st->n_levels())
        return 0;
    return st->st->frames_written(level);
}

uint64_t
aqz_stage_frames_consumed(aqz_stage* st)
{
    if (!st || st->sticky != AQZ_STATUS_SUCCESS)
        return 0;
    uint64_t n = 0;
    if (guard_sticky(st, [&] { n = st->st->frames_consumed(); }) != AQZ_STATUS_SUCCESS)
        return 0;
    return n;
}

aqz_status
aqz_stage_wait_consumed(aqz_stage* st, uint64_t frames)
{
    return guard_sticky(st, [&] { st->st->wait_consumed(frames); });
}

uint64_t
aqz_stage_last_ticket(const aqz_stage* st)
{
    return st ? st->st->last_ticket() : 0;
}

uint64_t
aqz_stage_copies_completed(aqz_stage* st)
{
    if (!st || st->sticky != AQZ_STATUS_SUCCESS)
        return 0;
    uint64_t n = 0;
    if (guard_sticky(st, [&] { n = st->st->copies_completed(); }) != AQZ_STATUS_SUCCESS)
        return 0;
    return n;
}

aqz_status
aqz_stage_wait_ticket(aqz_stage* st, uint64_t ticket)
{
    return guard_sticky(st, [&] {
        if (ticket > st->st->last_ticket())
            throw Error(AQZ_STATUS_INVALID_ARGUMENT, "ticket not issued");
        st->st->copies_completed(false, ticket);
    });
}

aqz_status
aqz_stage_copy_layer(aqz_stage* st, uint32_t level, uint64_t layer, void* dst,
                     size_t cap, uint8_t* has_data, size_t has_data_cap,
                     int32_t mem)
{
    return guard_sticky(st, [&] {
        st->st->copy_layer(level, layer, dst, cap, has_data, has_data_cap, mem);
    });
}

aqz_status
aqz_stage_copy_layer_async(aqz_stage* st, uint32_t level, uint64_t layer, void* dst,
                           size_t cap, uint8_t* has_data, size_t has_data_cap)
{
    return guard_sticky(st, [&] {
        st->st->copy_layer_async(level, layer, dst, cap, has_data, has_data_cap);
    });
}

aqz_status
aqz_stage_wait_copies(aqz_stage* st)
{
    return guard_sticky(st, [&] { st->st->wait_copies(); });
}

aqz_status
aqz_host_alloc(size_t bytes, void** out)
{
    if (!out || bytes == 0)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *out = nullptr;
    return hipHostMalloc(out, bytes, hipHostMallocDefault) == hipSuccess
             ? AQZ_STATUS_SUCCESS
             : AQZ_STATUS_OUT_OF_MEMORY;
}

void
aqz_host_free(void* p)
{
    if (p)
        (void)hipHostFree(p);
}

aqz_status
aqz_stage_device_layer(aqz_stage* st, uint32_t level, uint64_t layer,
                       void** chunks, uint32_t** has_data)
{
    return guard_sticky(
      st, [&] { st->st->device_layer(level, layer, chunks, has_data); });
}

aqz_status
aqz_stage_finalize(aqz_stage* st)
{
    return guard_sticky(st, [&] { st->st->finalize(); });
}

// host work only (no GPU call): not sticky, any thread
aqz_status
aqz_stage_split_level0_host(aqz_stage* st, const void* frames, uint64_t n_frames,
                            uint64_t first_frame, uint32_t chunk0, void* dst, size_t cap,
                            uint8_t* has_data, size_t has_data_cap)
{
    if (!st || !st->st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        st->st->split_level0_host(frames, n_frames, first_frame, chunk0, dst, cap, has_data,
                                  has_data_cap);
    });
}

aqz_status
aqz_stage_split_level0_rows(const aqz_stage* st, const void* frame, uint64_t frame_id,
                            uint32_t row_begin, uint32_t row_end, void* frame_copy,
                            uint32_t chunk0, void* dst, size_t cap, uint8_t* has_data,
                            size_t has_data_cap)
{
    if (!st || !st->st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        st->st->split_level0_rows(frame, frame_id, row_begin, row_end, frame_copy, chunk0, dst,
                                  cap, has_data, has_data_cap);
    });
}

aqz_status
aqz_stage_enable_kernel_timing(aqz_stage* st, int32_t enable)
{
    return guard_sticky(st, [&] { st->st->enable_timing(enable != 0); });
}

aqz_status
aqz_stage_kernel_timing(aqz_stage* st, double* total_ms, uint64_t* launches)
{
    return guard_sticky(st, [&] { st->st->timing(total_ms, launches); });
}

aqz_status
aqz_stage_timing_mark(aqz_stage* st, int32_t which)
{
    return guard_sticky(st, [&] { st->st->mark(which); });
}

aqz_status
aqz_stage_timing_elapsed(aqz_stage* st, double* ms)
{
    return guard_sticky(st, [&] {
        const double v = st->st->marked_ms();
        if (ms)
            *ms = v;
    });
}

const char*
aqz_stage_dominant_kernel(const aqz_stage* st)
{
    return st ? st->st->dominant_kernel() : "";
}

uint32_t
aqz_stage_zstd_far_ranges(const aqz_stage* st, uint32_t level)
{
    try {
        return st && st->st ? st->st->zstd_far_ranges(level) : 0;
    } catch (...) {
        return 0;
    }
}

aqz_status
aqz_stage_host_affinity(const aqz_stage* st, int32_t* numa_node, uint32_t* n_cpus)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    if (numa_node)
        *numa_node = st->st->numa_node();
    if (n_cpus)
        *n_cpus = uint32_t(st->st->numa_cpus());
    return AQZ_STATUS_SUCCESS;
}

aqz_status
aqz_stage_placement_report(const aqz_stage* st, aqz_placement_report* out)
{
    if (!st || !out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    const PlacementReport& r = st->st->placement();
    *out = aqz_placement_report{};
    out->n = uint32_t(r.ms.size());
    out->kept = uint32_t(r.kept);
    out->reps = r.reps;
    out->mode = r.mode;
    for (size_t i = 0; i < r.ms.size() && i < 32; ++i)
        out->ms[i] = r.ms[i];
    out->kept_ms_final = r.kept_ms_final;
    out->peak_device_bytes = r.peak_device;
    out->probe_bus_gbs = r.probe_bus_gbs;
    out->expected_ms = r.expected_ms;
    out->alg_bytes = r.alg_bytes;
    out->accepted = r.accepted ? 1u : 0u;
    out->stop = r.stop;
    for (size_t i = 0; i < r.probe_gbs.size() && i < 32; ++i)
        out->probe_gbs[i] = r.probe_gbs[i];
    return AQZ_STATUS_SUCCESS;
}

aqz_status
aqz_stage_placement(const aqz_stage* st, double* ms, size_t cap, size_t* n, uint32_t* kept)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    const auto& v = st->st->placement_ms();
    if (n)
        *n = v.size();
    if (kept)
        *kept = uint32_t(st->st->placement_best());
    for (size_t i = 0; ms && i < v.size() && i < cap; ++i)
        ms[i] = v[i];
    return AQZ_STATUS_SUCCESS;
}

} // extern "C"

// ---- chunk compression ----------------------------------------------------
static Compression
to_compression(const aqz_compression* c)
{
    Compression k;
    k.codec = c->codec;
    k.clevel = c->clevel;
    k.shuffle = c->shuffle;
    return k;
}

aqz_status
aqz_stage_compress_layer(aqz_stage* st, uint32_t level, uint64_t layer,
                         const aqz_compression* comp)
{
    if (!comp)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard_sticky(
      st, [&] { st->st->compress_layer(level, layer, to_compression(comp)); });
}

aqz_status
aqz_stage_compressed_offsets(aqz_stage* st, uint32_t level, uint64_t layer,
                             uint64_t* offsets, size_t n)
{
    if (!offsets)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard_sticky(
      st, [&] { st->st->compressed_offsets(level, layer, offsets, n); });
}

aqz_status
aqz_stage_copy_compressed_async(aqz_stage* st, uint32_t level, uint64_t layer,
                                void* dst, size_t cap)
{
    if (!dst)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard_sticky(
      st, [&] { st->st->copy_compressed_async(level, layer, dst, cap); });
}

aqz_status
aqz_compressor_create(uint64_t chunk_bytes, uint32_t typesize,
                      const aqz_compression* comp, aqz_compressor** out)
{
    if (!comp || !out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *out = nullptr;
    return guard([&] {
        auto h = std::make_unique<aqz_compressor>();
        h->c = std::make_unique<Compressor>(chunk_bytes, typesize, to_compression(comp));
        *out = h.release();
    });
}

void
aqz_compressor_destroy(aqz_compressor* c)
{
    delete c;
}

uint64_t
aqz_compressor_max_bytes(uint64_t chunk_bytes, uint32_t n_chunks)
{
    return Compressor::max_bytes(chunk_bytes, n_chunks);
}

uint64_t
aqz_compressor_scratch_bytes(const aqz_compression* comp, uint64_t chunk_bytes,
                             uint32_t typesize, uint32_t n_chunks)
{
    if (!comp)
        return 0;
    uint64_t n = 0;
    const aqz_status s = guard([&] {
        const Compression c = to_compression(comp);
        Compressor check(chunk_bytes, typesize, c); // validates the settings
        n = Compressor::scratch_bytes(c, chunk_bytes, typesize, n_chunks);
    });
    return s == AQZ_STATUS_SUCCESS ? n : 0;
}

uint32_t
aqz_compressor_blocksize(const aqz_compressor* c)
{
    return c && c->c ? c->c->blocksize() : 0;
}

aqz_status
aqz_compressor_run(aqz_compressor* c, const void* chunks, uint64_t pitch,
                   uint32_t n_chunks, void* dst, size_t dst_cap, uint64_t* offsets,
                   void* stream)
{
    if (!c || !chunks || !dst || !offsets)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard_sticky(c, [&] {
        const uint64_t nb = c->c->chunk_bytes();
        if (pitch < nb)
            throw Error(1, "chunk pitch below the chunk size");
        if (dst_cap < Compressor::max_bytes(nb, n_chunks))
            throw Error(2, "destination below aqz_compressor_max_bytes");
        c->c->run(static_cast<const uint8_t*>(chunks), pitch, n_chunks, nullptr, 0,
                  static_cast<uint8_t*>(dst), offsets, static_cast<hipStream_t>(stream));
    });
}

// ---- shard packing ---------------------------------------------------------
aqz_status
aqz_stage_compression_done(aqz_stage* st, uint32_t level, uint64_t layer, int32_t* done)
{
    if (!done)
        return AQZ_STATUS_INVALID_ARGUMENT;
    *done = 0;
    return guard_sticky(st, [&] { *done = st->st->compression_done(level, layer) ? 1 : 0; });
}

aqz_status
aqz_stage_compressed_entries(aqz_stage* st, uint32_t level, uint64_t layer,
                             aqz_chunk_entry* out, size_t n)
{
    if (!out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    static_assert(sizeof(aqz_chunk_entry) == sizeof(ChunkEntry), "entry layout");
    return guard_sticky(st, [&] {
        st->st->compressed_entries(level, layer, reinterpret_cast<ChunkEntry*>(out), n);
    });
}

aqz_status
aqz_stage_shard_geometry(const aqz_stage* st, uint32_t level, uint32_t* chunks_per_shard,
                         uint32_t* number_of_shards, uint32_t* layers_per_shard)
{
    if (!st)
        return AQZ_STATUS_INVALID_ARGUMENT;
    return guard([&] {
        st->st->shard_geometry(level, chunks_per_shard, number_of_shards, layers_per_shard);
    });
}

size_t
aqz_shard_table_bytes(uint32_t chunks_per_shard)
{
    return size_t(chunks_per_shard) * 16 + 4;
}

aqz_status
aqz_shard_table(const uint64_t* offsets, const uint64_t* extents, uint32_t chunks_per_shard,
                void* out, size_t cap)
{
    if (!offsets || !extents || !out)
        return AQZ_STATUS_INVALID_ARGUMENT;
    if (cap < aqz_shard_table_bytes(chunks_per_shard))
        return AQZ_STATUS_OVERFLOW;
    shard_table(offsets, extents, chunks_per_shard, static_cast<uint8_t*>(out));
    return AQZ_STATUS_SUCCESS;
}

uint32_t
aqz_crc32c(const void* data, size_t n)
{
    return data ? crc32c(static_cast<const uint8_t*>(data), n) : 0;
}
