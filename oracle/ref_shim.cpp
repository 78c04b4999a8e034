// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A C-ABI shim over the *compiled reference* (acquire-zarr sources under
// /root/reference/src/streaming, built by oracle/Makefile into oracle/_ref/).
// It lets the Python tests drive the real zarr::Downsampler,
// ArrayDimensions and zarr::Chunk so the C restatement in aqz_oracle.c (and
// through it the HIP path) is pinned to the reference's own behaviour.
// This file is ours; no reference source is copied into the repo.
#include "array.dimensions.hh"
#include "array.hh"
#include "chunk.hh"
#include "downsampler.hh"
#include "zarr.common.hh"

#include <cstring>
#include <memory>
#include <vector>

extern "C" {
#include "aqz_oracle.h"
}

namespace {
std::vector<ZarrDimension>
to_dims(const or_dim* dims, int ndims)
{
    std::vector<ZarrDimension> v;
    for (int i = 0; i < ndims; ++i) {
        v.emplace_back("d" + std::to_string(i),
                       static_cast<ZarrDimensionType>(dims[i].type),
                       dims[i].array_size_px,
                       dims[i].chunk_size_px,
                       dims[i].shard_size_chunks);
    }
    return v;
}

struct RefDs
{
    std::unique_ptr<zarr::Downsampler> ds;
    int ndims;
};
} // namespace

extern "C" {

void*
ref_ds_create(const or_dim* dims, int ndims, int dtype, int method,
              uint32_t max_levels)
{
    try {
        auto ad = std::make_shared<ArrayDimensions>(
          to_dims(dims, ndims), static_cast<ZarrDataType>(dtype));
        auto cfg = std::make_shared<zarr::ArrayConfig>(
          "", "/0", std::nullopt, std::nullopt, ad,
          static_cast<ZarrDataType>(dtype),
          static_cast<ZarrDownsamplingMethod>(method), 0, max_levels);
        auto* r = new RefDs;
        r->ds = std::make_unique<zarr::Downsampler>(
          cfg, static_cast<ZarrDownsamplingMethod>(method));
        r->ndims = static_cast<int>(ad->ndims());
        return r;
    } catch (...) {
        return nullptr;
    }
}

void
ref_ds_destroy(void* h)
{
    delete static_cast<RefDs*>(h);
}

int
ref_ds_n_levels(void* h)
{
    return static_cast<int>(
      static_cast<RefDs*>(h)->ds->writer_configurations().size());
}

// Fills out[ndims] with level `level`'s dims; returns ndims (after the
// reference's own 2-D phantom prepend) or -1.
int
ref_ds_level_dims(void* h, int level, or_dim* out, int cap)
{
    auto* r = static_cast<RefDs*>(h);
    const auto& cfgs = r->ds->writer_configurations();
    auto it = cfgs.find(level);
    if (it == cfgs.end())
        return -1;
    const auto& d = it->second->dimensions;
    const int n = static_cast<int>(d->ndims());
    if (n > cap)
        return -1;
    for (int i = 0; i < n; ++i) {
        const auto& z = d->at(i);
        out[i].type = z.type;
        out[i].array_size_px = z.array_size_px;
        out[i].chunk_size_px = z.chunk_size_px;
        out[i].shard_size_chunks = z.shard_size_chunks;
    }
    return n;
}

int
ref_ds_add_frame(void* h, const void* frame, size_t nbytes)
{
    try {
        std::vector<uint8_t> f(static_cast<const uint8_t*>(frame),
                               static_cast<const uint8_t*>(frame) + nbytes);
        static_cast<RefDs*>(h)->ds->add_frame(f);
        return 0;
    } catch (...) {
        return -1;
    }
}

int
ref_ds_take_frame(void* h, int level, void* dst, size_t cap, size_t* nbytes)
{
    std::vector<uint8_t> f;
    if (!static_cast<RefDs*>(h)->ds->take_frame(level, f))
        return 0;
    if (nbytes)
        *nbytes = f.size();
    if (dst)
        std::memcpy(dst, f.data(), f.size() < cap ? f.size() : cap);
    return 1;
}

// Downsampler::get_metadata().dump() (downsampler.cpp:440-485) and
// downsampling_method() (:422-438): the OME "metadata" block and "type"
// MultiscaleArray writes into zarr.json (multiscale.array.cpp:271).
// Returns the length; writes at most cap bytes (NUL-terminated if room).
size_t
ref_ds_metadata(void* h, char* buf, size_t cap)
{
    const std::string s = static_cast<RefDs*>(h)->ds->get_metadata().dump();
    if (buf && cap) {
        const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return s.size();
}

size_t
ref_ds_method_name(void* h, char* buf, size_t cap)
{
    const std::string s = static_cast<RefDs*>(h)->ds->downsampling_method();
    if (buf && cap) {
        const size_t n = s.size() < cap - 1 ? s.size() : cap - 1;
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return s.size();
}

// ---- ArrayDimensions ----------------------------------------------------
void*
ref_dims_create(const or_dim* dims, int ndims, int dtype)
{
    try {
        return new ArrayDimensions(to_dims(dims, ndims),
                                   static_cast<ZarrDataType>(dtype));
    } catch (...) {
        return nullptr;
    }
}

void*
ref_dims_create_ordered(const or_dim* dims, int ndims, int dtype,
                        const size_t* order)
{
    try {
        std::vector<size_t> ord(order, order + ndims);
        return new ArrayDimensions(to_dims(dims, ndims),
                                   static_cast<ZarrDataType>(dtype), ord);
    } catch (...) {
        return nullptr;
    }
}

uint64_t
ref_dims_transpose_frame_id(void* h, uint64_t fid)
{
    return static_cast<ArrayDimensions*>(h)->transpose_frame_id(fid);
}

void
ref_dims_destroy(void* h)
{
    delete static_cast<ArrayDimensions*>(h);
}

uint32_t
ref_dims_tile_group_offset(void* h, uint64_t fid)
{
    return static_cast<ArrayDimensions*>(h)->tile_group_offset(fid);
}

uint64_t
ref_dims_chunk_internal_offset(void* h, uint64_t fid)
{
    return static_cast<ArrayDimensions*>(h)->chunk_internal_offset(fid);
}

uint32_t
ref_dims_chunk_lattice_index(void* h, uint64_t fid, uint32_t dim)
{
    return static_cast<ArrayDimensions*>(h)->chunk_lattice_index(fid, dim);
}

uint64_t
ref_dims_bytes_per_chunk(void* h)
{
    return static_cast<ArrayDimensions*>(h)->bytes_per_chunk();
}

uint32_t
ref_dims_number_of_chunks_in_memory(void* h)
{
    return static_cast<ArrayDimensions*>(h)->number_of_chunks_in_memory();
}

uint64_t
ref_dims_frames_per_chunk_layer(void* h)
{
    return static_cast<ArrayDimensions*>(h)->frames_per_chunk_layer();
}

uint32_t
ref_dims_shard_index_for_chunk(void* h, uint32_t c)
{
    return static_cast<ArrayDimensions*>(h)->shard_index_for_chunk(c);
}

uint32_t
ref_dims_shard_internal_index(void* h, uint32_t c)
{
    return static_cast<ArrayDimensions*>(h)->shard_internal_index(c);
}

// dim-1 banding geometry (array.dimensions.cpp:344-373)
void
ref_dims_dim1_banding(void* h, int* supported, uint32_t* n_bands,
                      uint64_t* frames_per_band, uint32_t* chunks_per_band)
{
    auto* d = static_cast<ArrayDimensions*>(h);
    *supported = d->supports_dim1_banding() ? 1 : 0;
    *n_bands = d->dim1_band_count();
    *frames_per_band = d->frames_per_dim1_band();
    *chunks_per_band = d->chunks_per_dim1_band();
}

// shard geometry (array.dimensions.cpp:376-392) and the ragged-padding skip
// list of one shard layer (array.dimensions.cpp:424-453): the count, the
// first min(count, cap) indices into out
void
ref_dims_shard_geometry(void* h, uint32_t* chunks_per_shard, uint32_t* n_shards,
                        uint32_t* layers_per_shard)
{
    auto* d = static_cast<ArrayDimensions*>(h);
    *chunks_per_shard = d->chunks_per_shard();
    *n_shards = d->number_of_shards();
    *layers_per_shard = d->chunk_layers_per_shard();
}

size_t
ref_dims_skipped_internal_indices(void* h, uint32_t shard, uint32_t layer, uint32_t* out,
                                  size_t cap)
{
    const auto v =
      static_cast<ArrayDimensions*>(h)->skipped_internal_indices_for_shard_layer(shard, layer);
    for (size_t i = 0; i < v.size() && i < cap; ++i)
        out[i] = v[i];
    return v.size();
}

// Tile split of one frame into a chunk layer using the reference's own
// ArrayDimensions + zarr::Chunk::write_tile_rows (chunk.cpp:17-58).  The
// driving loop restates array.cpp:537-619 (array.cpp itself needs crc32c,
// absent from the image).  layer/has_data as in or_write_frame_to_chunks.
size_t
ref_write_frame_to_chunks(void* h, int dtype, uint64_t fid, const void* frame,
                          uint8_t* layer, uint8_t* has_data)
{
    auto* dims = static_cast<ArrayDimensions*>(h);
    const size_t bpp = zarr::bytes_of_type(static_cast<ZarrDataType>(dtype));
    const uint32_t W = dims->width_dim().array_size_px;
    const uint32_t tw = dims->width_dim().chunk_size_px;
    const uint32_t H = dims->height_dim().array_size_px;
    const uint32_t th = dims->height_dim().chunk_size_px;
    const size_t bpc = dims->bytes_per_chunk();
    const uint32_t ntx = (W + tw - 1) / tw, nty = (H + th - 1) / th;
    const uint32_t group = dims->tile_group_offset(fid);
    const uint64_t internal = dims->chunk_internal_offset(fid);
    const auto* src = static_cast<const uint8_t*>(frame);
    size_t written = 0;
    for (uint32_t t = 0; t < ntx * nty; ++t) {
        const uint32_t c = t + group;
        zarr::Chunk chunk(bpc, bpp);
        const uint32_t row0 = (t / ntx) * th;
        if (row0 >= H)
            continue;
        const uint32_t n_rows = std::min(th, H - row0);
        const uint32_t col0 = (t % ntx) * tw;
        const uint32_t rw = std::min(col0 + tw, W) - col0;
        chunk.write_tile_rows(internal,
                              src + bpp * (static_cast<size_t>(row0) * W + col0),
                              static_cast<size_t>(W) * bpp,
                              rw * bpp,
                              tw * bpp,
                              n_rows);
        // merge this frame's tile into the caller's layer image
        const auto& buf = chunk.buffer();
        for (uint32_t r = 0; r < n_rows; ++r) {
            std::memcpy(layer + static_cast<uint64_t>(c) * bpc + internal +
                          static_cast<size_t>(r) * tw * bpp,
                        buf.data() + internal + static_cast<size_t>(r) * tw * bpp,
                        rw * bpp);
        }
        if (chunk.has_data())
            has_data[c] = 1;
        written += static_cast<size_t>(rw) * bpp * n_rows;
    }
    return written;
}

// ---- persistent-chunk tile split (CPU baseline timing) -------------------
// Array::write_frame_to_chunks_ (array.cpp:537-619) restated over the
// reference's own ArrayDimensions + zarr::Chunk objects that persist across
// frames of a chunk layer, as in the reference Array (chunks_ vector).
struct RefSplit
{
    std::unique_ptr<ArrayDimensions> dims;
    std::vector<std::unique_ptr<zarr::Chunk>> chunks;
    size_t bpp;
};

void*
ref_split_create(const or_dim* dims, int ndims, int dtype)
{
    try {
        auto* s = new RefSplit;
        s->dims = std::make_unique<ArrayDimensions>(
          to_dims(dims, ndims), static_cast<ZarrDataType>(dtype));
        s->bpp = zarr::bytes_of_type(static_cast<ZarrDataType>(dtype));
        s->chunks.resize(s->dims->number_of_chunks_in_memory());
        return s;
    } catch (...) {
        return nullptr;
    }
}

void
ref_split_destroy(void* h)
{
    delete static_cast<RefSplit*>(h);
}

size_t
ref_split_write(void* h, uint64_t fid, const void* frame)
{
    auto* s = static_cast<RefSplit*>(h);
    auto* dims = s->dims.get();
    const size_t bpp = s->bpp;
    const uint32_t W = dims->width_dim().array_size_px;
    const uint32_t tw = dims->width_dim().chunk_size_px;
    const uint32_t H = dims->height_dim().array_size_px;
    const uint32_t th = dims->height_dim().chunk_size_px;
    const uint32_t ntx = (W + tw - 1) / tw, nty = (H + th - 1) / th;
    const uint32_t group = dims->tile_group_offset(fid);
    const uint64_t internal = dims->chunk_internal_offset(fid);
    const auto* src = static_cast<const uint8_t*>(frame);
    size_t written = 0;
    // the reference's tile loop is OpenMP-parallel (array.cpp:575); each
    // tile owns its chunk, so the lazy allocation below needs no lock here
#pragma omp parallel for schedule(static) reduction(+ : written)
    for (uint32_t t = 0; t < ntx * nty; ++t) {
        auto& chunk = s->chunks[t + group];
        if (!chunk)
            chunk = std::make_unique<zarr::Chunk>(dims->bytes_per_chunk(), bpp);
        const uint32_t row0 = (t / ntx) * th;
        const uint32_t n_rows = std::min(th, H - row0);
        const uint32_t col0 = (t % ntx) * tw;
        const uint32_t rw = std::min(col0 + tw, W) - col0;
        chunk->write_tile_rows(internal,
                               src + bpp * (static_cast<size_t>(row0) * W + col0),
                               static_cast<size_t>(W) * bpp, rw * bpp, tw * bpp,
                               n_rows);
        written += static_cast<size_t>(rw) * bpp * n_rows;
    }
    return written;
}

} // extern "C"
