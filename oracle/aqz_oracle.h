/*
 * aqz_oracle.h -- CPU ORACLE for the multiscale-pyramid + chunk-tile-split
 * hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a from-scratch plain-C restatement of the reference acquire-zarr
 * algorithm (reference @ /root/reference, acquire-zarr 0.8.1).  It exists so
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg can CHECK
 * the HIP product path.  Nothing in acquire-zarr_amd/ links, loads or calls
 * it; the product path has no CPU fallback.
 *
 * Parity pinning: validated against (1) the compiled reference itself
 * (oracle/_ref, built from /root/reference sources by oracle/Makefile) and
 * (2) the reference unit tests' known answers, restated in tests/.
 * Golden vectors generated from the compiled reference live in tests/golden/.
 */
#ifndef AQZ_ORACLE_H
#define AQZ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same numeric values as ZarrDataType / ZarrDownsamplingMethod /
 * ZarrDimensionType (include/zarr.types.h:49-62, 81-97). */
enum { OR_U8 = 0, OR_U16, OR_U32, OR_U64, OR_I8, OR_I16, OR_I32, OR_I64,
       OR_F32, OR_F64, OR_NDTYPES };
enum { OR_DECIMATE = 0, OR_MEAN, OR_MIN, OR_MAX, OR_NMETHODS };
enum { OR_SPACE = 0, OR_CHANNEL, OR_TIME, OR_OTHER };

#define OR_MAX_DIMS 16
#define OR_MAX_LEVELS 32

typedef struct
{
    int32_t type;
    uint32_t array_size_px;
    uint32_t chunk_size_px;
    uint32_t shard_size_chunks;
} or_dim;

size_t or_bytes_of_type(int dtype);

/* ---- a5: one 2x2 level, edge replicate (downsampler.cpp:139-206) ------- */
/* dst must hold ceil(w/2)*ceil(h/2) pixels. */
int or_scale_image(int dtype, int method, const void* src, size_t width,
                   size_t height, void* dst);

/* ---- a6: z-pair reduce dst[i] = f(dst[i], src[i]) (downsampler.cpp:208-246) */
int or_average_two_frames(int dtype, int method, void* dst, const void* src,
                          size_t n_pixels);

/* ---- a1/a2: level geometry (downsampler.cpp:8-37, 494-597) -------------
 * dims are in storage order (slowest first, last two = y, x), ndims >= 3
 * (callers prepend the phantom singleton for 2-D, array.dimensions.cpp:150).
 * Writes n_levels (total, including level 0) and per-level dims into
 * out_dims[level * ndims + i].  Returns 0 on success. */
int or_make_levels(const or_dim* dims, int ndims, uint32_t max_levels,
                   int* n_levels, or_dim* out_dims, int out_cap_levels);

/* ---- a15: ArrayDimensions index math (array.dimensions.cpp:232-326) ---- */
uint32_t or_chunk_lattice_index(const or_dim* dims, int ndims,
                                uint64_t frame_id, int dim_index);
uint32_t or_tile_group_offset(const or_dim* dims, int ndims,
                              uint64_t frame_id);
uint64_t or_chunk_internal_offset(const or_dim* dims, int ndims, int dtype,
                                  uint64_t frame_id);
uint64_t or_bytes_per_chunk(const or_dim* dims, int ndims, int dtype);
uint32_t or_number_of_chunks_in_memory(const or_dim* dims, int ndims);
uint64_t or_frames_per_chunk_layer(const or_dim* dims, int ndims);
uint32_t or_shard_index_for_chunk(const or_dim* dims, int ndims,
                                  uint32_t chunk_index);
uint32_t or_shard_internal_index(const or_dim* dims, int ndims,
                                 uint32_t chunk_index);

/* ---- a12/a14: tile split of one frame into a chunk layer --------------
 * (array.cpp:507-622, chunk.cpp:17-58).  `layer` holds
 * number_of_chunks_in_memory * bytes_per_chunk bytes (chunk c at
 * c*bytes_per_chunk, zero-initialised by the caller like Chunk's ctor,
 * chunk.cpp:8-15); has_data holds one byte per chunk.  `frame_id` is the
 * storage-order frame id (after transpose_frame_id).  Returns bytes copied. */
size_t or_write_frame_to_chunks(const or_dim* dims, int ndims, int dtype,
                                uint64_t frame_id, const void* frame,
                                uint8_t* layer, uint8_t* has_data);

/* ---- a7/a8: the cascade state machine (downsampler.cpp:306-414) ------- */
typedef struct or_downsampler or_downsampler;
or_downsampler* or_ds_create(const or_dim* dims, int ndims, int dtype,
                             int method, uint32_t max_levels);
void or_ds_destroy(or_downsampler* ds);
int or_ds_n_levels(const or_downsampler* ds);
/* level dims, ndims entries */
const or_dim* or_ds_level_dims(const or_downsampler* ds, int level);
int or_ds_add_frame(or_downsampler* ds, const void* frame, size_t nbytes);
/* returns 1 and fills dst (up to cap bytes, *nbytes = frame bytes) if a
 * frame was waiting at `level`, else 0 */
int or_ds_take_frame(or_downsampler* ds, int level, void* dst, size_t cap,
                     size_t* nbytes);

/* ---- synthetic inputs: splitmix64 stream (shared with tests/bench) ---- */
uint64_t or_splitmix64(uint64_t* state);
void or_fill_splitmix(void* dst, size_t nbytes, uint64_t seed);

/* ---- chunk compression / shard index (aqz_codec_oracle.c) ------------- */
typedef struct
{
    uint32_t version, versionlz, flags, typesize;
    uint32_t nbytes, blocksize, cbytes;
} or_blosc_info;

void or_shuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst);
void or_unshuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst);
void or_bitshuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst);
void or_bitunshuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst);
/* decoded bytes (== dsize) or -1 */
long or_lz4_decompress(const uint8_t* src, size_t csize, uint8_t* dst,
                       size_t dsize);
int or_blosc_frame_info(const uint8_t* src, size_t srcsize, or_blosc_info* info);
/* nbytes or < 0; tmp holds one block */
long or_blosc_decompress(const uint8_t* src, size_t srcsize, uint8_t* dst,
                         size_t dstcap, uint8_t* tmp);
uint32_t or_crc32c(const uint8_t* p, size_t n);

#ifdef __cplusplus
}
#endif
#endif
