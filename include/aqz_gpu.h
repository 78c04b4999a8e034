/*
 * aqz_gpu.h -- C ABI of the MI355X-native multiscale-pyramid + chunk-tile
 * stage for acquire-zarr.
 *
 * Plain C, plain pointers and sizes.  Every call returns a status code with
 * the numeric values of ZarrStatusCode (reference include/zarr.types.h:13-31)
 * and never lets a C++ exception or a HIP error cross the boundary (a HIP
 * error maps to AQZ_STATUS_INTERNAL_ERROR and is sticky on the object, like
 * ZarrStream_s::error_, reference src/streaming/zarr.stream.cpp:1442-1449).
 *
 * Objects are not thread-safe: like the reference Downsampler / Array they
 * are driven from one consumer thread (reference zarr.stream.cpp:1683-1684).
 *
 * Which reference interface each entry point replaces is noted per function
 * (paths relative to /root/reference).
 */
#ifndef AQZ_GPU_H
#define AQZ_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (== ZarrStatusCode, include/zarr.types.h:13-31) ---- */
typedef int32_t aqz_status;
#define AQZ_STATUS_SUCCESS 0
#define AQZ_STATUS_INVALID_ARGUMENT 1
#define AQZ_STATUS_OVERFLOW 2
#define AQZ_STATUS_INVALID_INDEX 3
#define AQZ_STATUS_NOT_YET_IMPLEMENTED 4
#define AQZ_STATUS_INTERNAL_ERROR 5
#define AQZ_STATUS_OUT_OF_MEMORY 6
#define AQZ_STATUS_INVALID_SETTINGS 9
#define AQZ_STATUS_WRITE_OUT_OF_BOUNDS 12

/* ---- enums: numeric values of ZarrDataType (zarr.types.h:49-62),
 *      ZarrDimensionType (:81-88), ZarrDownsamplingMethod (:90-97) ------- */
enum
{
    AQZ_DTYPE_UINT8 = 0,
    AQZ_DTYPE_UINT16,
    AQZ_DTYPE_UINT32,
    AQZ_DTYPE_UINT64,
    AQZ_DTYPE_INT8,
    AQZ_DTYPE_INT16,
    AQZ_DTYPE_INT32,
    AQZ_DTYPE_INT64,
    AQZ_DTYPE_FLOAT32,
    AQZ_DTYPE_FLOAT64,
    AQZ_DTYPE_COUNT
};
enum
{
    AQZ_DIM_SPACE = 0,
    AQZ_DIM_CHANNEL,
    AQZ_DIM_TIME,
    AQZ_DIM_OTHER
};
enum
{
    AQZ_METHOD_DECIMATE = 0,
    AQZ_METHOD_MEAN,
    AQZ_METHOD_MIN,
    AQZ_METHOD_MAX,
    AQZ_METHOD_COUNT
};

/* where a frame pointer lives */
enum
{
    AQZ_MEM_HOST = 0,        /* pageable host memory (copied to pinned staging) */
    AQZ_MEM_DEVICE = 1,      /* already resident in this device's HBM */
    AQZ_MEM_HOST_PINNED = 2  /* page-locked host memory (e.g. aqz_host_alloc):
                                DMA'd straight to the device, asynchronously */
};

/* The pixel-geometry subset of ZarrDimensionProperties
 * (zarr.types.h:120-133): name/unit/scale do not affect the data path. */
typedef struct
{
    int32_t type;               /* AQZ_DIM_* */
    uint32_t array_size_px;     /* 0 = unbounded (append dimension only) */
    uint32_t chunk_size_px;
    uint32_t shard_size_chunks;
} aqz_dimension;

/* Mirrors the array part of ZarrArraySettings (zarr.types.h:157-169). */
typedef struct
{
    const aqz_dimension* dimensions; /* acquisition order, slowest first */
    size_t dimension_count;          /* >= 2; last two are Space (y, x) */
    int32_t data_type;               /* AQZ_DTYPE_* */
    int32_t multiscale;              /* bool */
    int32_t downsampling_method;     /* AQZ_METHOD_* */
    uint32_t max_levels;             /* 0 = no limit */
    const size_t* storage_dimension_order; /* NULL = acquisition order */
    int32_t device;                  /* HIP device ordinal */
} aqz_array_desc;

const char* aqz_version(void);
const char* aqz_status_message(aqz_status status);
/* The message of the last failed call on this thread ("" if none): what
 * the reference passes to LOG_ERROR before mapping an exception to a status
 * (src/streaming/zarr.stream.cpp:1704-1719, src/logger/logger.hh). */
const char* aqz_last_error(void);
/* Number of HIP devices visible (0 when no GPU). */
aqz_status aqz_device_count(int32_t* count);

/* ======================================================================
 * Host index math -- ArrayDimensions (src/streaming/array.dimensions.hh:45)
 * Pure host C++; usable without a GPU.
 * ==================================================================== */
typedef struct aqz_dims aqz_dims;

/* ArrayDimensions::ArrayDimensions (array.dimensions.cpp:137-189), including
 * the 2-D phantom-dimension prepend and storage_dimension_order. */
aqz_status aqz_dims_create(const aqz_dimension* dims, size_t ndims,
                           int32_t data_type, const size_t* storage_order,
                           aqz_dims** out);
void aqz_dims_destroy(aqz_dims* d);
size_t aqz_dims_ndims(const aqz_dims* d);
/* storage-order dimension i */
aqz_status aqz_dims_get(const aqz_dims* d, size_t i, aqz_dimension* out);
/* array.dimensions.cpp:264-282 */
uint32_t aqz_dims_tile_group_offset(const aqz_dims* d, uint64_t frame_id);
/* array.dimensions.cpp:284-314 */
uint64_t aqz_dims_chunk_internal_offset(const aqz_dims* d, uint64_t frame_id);
/* array.dimensions.cpp:232-262 */
uint32_t aqz_dims_chunk_lattice_index(const aqz_dims* d, uint64_t frame_id,
                                      uint32_t dim_index);
/* array.dimensions.cpp:602-620 */
uint64_t aqz_dims_transpose_frame_id(const aqz_dims* d, uint64_t frame_id);
uint64_t aqz_dims_bytes_per_chunk(const aqz_dims* d);
uint32_t aqz_dims_number_of_chunks_in_memory(const aqz_dims* d);
uint64_t aqz_dims_frames_per_chunk_layer(const aqz_dims* d);
/* array.dimensions.cpp:393-548 */
uint32_t aqz_dims_shard_index_for_chunk(const aqz_dims* d, uint32_t chunk);
uint32_t aqz_dims_shard_internal_index(const aqz_dims* d, uint32_t chunk);
/* chunks_per_shard, number_of_shards (one append-dimension shard row) and
 * chunk_layers_per_shard (array.dimensions.cpp:376-392); any may be NULL. */
aqz_status aqz_dims_shard_geometry(const aqz_dims* d, uint32_t* chunks_per_shard,
                                   uint32_t* n_shards, uint32_t* layers_per_shard);
/* skipped_internal_indices_for_shard_layer (array.dimensions.cpp:424-453):
 * the internal indices of `shard` that chunk layer `layer` (< layers per
 * shard) leaves unfilled -- ragged padding, skipped so the shard's
 * countdown completes.  Writes min(count, cap) of them to out (may be NULL
 * with cap 0) and the count to *n. */
aqz_status aqz_dims_skipped_internal_indices(const aqz_dims* d, uint32_t shard,
                                             uint32_t layer, uint32_t* out, size_t cap,
                                             size_t* n);
/* supports_dim1_banding, dim1_band_count, frames_per_dim1_band,
 * chunks_per_dim1_band (array.dimensions.cpp:344-373) */
aqz_status aqz_dims_dim1_banding(const aqz_dims* d, int32_t* supported,
                                 uint32_t* n_bands, uint64_t* frames_per_band,
                                 uint32_t* chunks_per_band);

/* Level geometry of the pyramid: Downsampler::make_writer_configurations_
 * (src/streaming/downsampler.cpp:494-597).  dims in storage order; writes the
 * number of levels (including level 0) and, if out_dims != NULL, the dims of
 * every level (n_levels * ndims entries, ndims after the 2-D prepend). */
aqz_status aqz_pyramid_levels(const aqz_dimension* dims, size_t ndims,
                              uint32_t max_levels, uint32_t* n_levels,
                              aqz_dimension* out_dims, size_t out_cap);

/* ======================================================================
 * Downsampler -- drop-in for zarr::Downsampler (src/streaming/downsampler.hh:
 * 12-64): same level geometry, same add/take contract, same cascade state
 * machine (downsampler.cpp:306-414), pixels computed on the GPU.
 * ==================================================================== */
typedef struct aqz_downsampler aqz_downsampler;

/* Downsampler::Downsampler(config, method) (downsampler.cpp:249-304).
 * Invalid dtype/method -> AQZ_STATUS_INVALID_ARGUMENT (the reference throws). */
aqz_status aqz_downsampler_create(const aqz_array_desc* desc,
                                  aqz_downsampler** out);
void aqz_downsampler_destroy(aqz_downsampler* ds);
/* writer_configurations().size() */
uint32_t aqz_downsampler_n_levels(const aqz_downsampler* ds);
/* writer_configurations().at(level)->dimensions (storage order) */
aqz_status aqz_downsampler_level_dims(const aqz_downsampler* ds,
                                      uint32_t level, aqz_dimension* out,
                                      size_t cap, size_t* ndims);
/* Downsampler::add_frame (downsampler.cpp:306-401).  frame is level-0 pixels,
 * nbytes >= width*height*bpp, mem = AQZ_MEM_HOST or AQZ_MEM_DEVICE. */
aqz_status aqz_downsampler_add_frame(aqz_downsampler* ds, const void* frame,
                                     size_t nbytes, int32_t mem);
/* Downsampler::take_frame (downsampler.cpp:403-414): *found = 0 if no frame
 * waits at `level`; otherwise copies it to dst (mem says where dst is). */
aqz_status aqz_downsampler_take_frame(aqz_downsampler* ds, uint32_t level,
                                      void* dst, size_t cap, int32_t mem,
                                      size_t* nbytes, int32_t* found);
/* Downsampler::downsampling_method (downsampler.cpp:422-438):
 * "decimate" | "local_mean" | "local_min" | "local_max" */
const char* aqz_downsampler_method_name(const aqz_downsampler* ds);
/* Downsampler::get_metadata (downsampler.cpp:440-485) as JSON text:
 * byte-identical to the reference's get_metadata().dump(), the block
 * MultiscaleArray embeds in zarr.json (multiscale.array.cpp:271).  With
 * buf == NULL only *len is set; cap must hold *len + 1 bytes. */
aqz_status aqz_downsampler_metadata_json(const aqz_downsampler* ds, char* buf,
                                         size_t cap, size_t* len);
/* The same two, from the method value alone (pure host, no GPU):
 * "" / AQZ_STATUS_INVALID_ARGUMENT for a method outside AQZ_METHOD_*. */
const char* aqz_downsampling_method_name(int32_t method);
aqz_status aqz_downsampling_metadata_json(int32_t method, char* buf, size_t cap,
                                          size_t* len);

/* ======================================================================
 * Stage -- the device-resident hot path of MultiscaleArray::write_frame
 * (src/streaming/multiscale.array.cpp:57-74, 291-325): level-0 tile split
 * (Array::write_frame_to_chunks_, array.cpp:507-622) + pyramid
 * (Downsampler::add_frame) + tile split of every level, written straight
 * into device-resident chunk layers with per-chunk has_data flags
 * (Chunk::write_tile_rows, chunk.cpp:17-58).
 *
 * A "chunk layer" of a level = number_of_chunks_in_memory chunks of
 * bytes_per_chunk bytes, chunk c at c*bytes_per_chunk (the reference's
 * Array::chunks_ vector, array.cpp:575-583), covering frames_per_chunk_layer
 * consecutive frames of that level.  The stage keeps `layer_slots` layers
 * per level resident in HBM as a ring.
 * ==================================================================== */
typedef struct aqz_stage aqz_stage;

typedef struct
{
    uint32_t layer_slots;      /* resident chunk layers per level (>=1; 0 = 2) */
    uint32_t max_batch_frames; /* frames per internal launch (0 = 64) */
    uint64_t first_frame;      /* level-0 frame id of this stage's first
                                  frame (z-slab sharding across GPUs: the
                                  slab's first plane); level k starts at
                                  first_frame * planes_k / planes_0, which
                                  must be exact.  0 = a whole stream. */
    uint32_t z_slab_begin;
    uint32_t z_slab_end;       /* z-slab schedule over a stream of volumes
                                  (BASELINE configs[3]): the stage
                                  receives only planes [begin, end) of every
                                  z stack (the level-0 dim ndims-3; a stack
                                  is one index of the dims before it), in
                                  order.  Frame ids skip the other planes:
                                  after each slab every level's frame id
                                  jumps by planes_k - (end_k - begin_k), so
                                  z pairs (Downsampler::add_frame's
                                  level_frame_count_ % planes,
                                  downsampler.cpp:358-389) and chunk
                                  placement (array.dimensions.cpp:264-314)
                                  stay those of the whole stream.  begin and
                                  end must scale exactly to every level
                                  (multiples of 2^(z-halving levels)); the
                                  first frame is first_frame + begin, with
                                  first_frame a multiple of the stack size.
                                  0, 0 = every plane. */
    uint32_t placement_tries;  /* n > 1: time the chunk-layer rings'
                                  placement on random frames at creation
                                  (aqz_stage_placement_report,
                                  aqz_gpu_bench.h).  Rings of >= 256 MiB in
                                  all are placed in one arena of 2 MiB
                                  virtual-memory pieces, where the fused
                                  kernels run in the fast band on most boxes
                                  (DESIGN.md section 3).  The arena is timed
                                  against the stage's algorithmic bytes at
                                  the rate of a streaming probe of the same
                                  memory; only when it is more than 3% over
                                  that, up to n - 1 fresh arenas follow, each
                                  made while the best is held and freed at
                                  once if slower.  The transient peak (one
                                  batch of random frames and a second ring
                                  set) is in aqz_stage_estimate_memory.
                                  0/1 = none. */
    uint32_t level0_split_on_host; /* 1: the device does not tile-split level
                                  0 (no level-0 ring in HBM); the caller
                                  splits level 0 on the host from the frames
                                  it holds (aqz_stage_split_level0_host /
                                  _rows): a raw hand-off
                                  then moves H2D 1x and D2H 1/3x of the input
                                  instead of D2H 4/3x.  Level-0 hand-off calls
                                  (copy_layer*, copy_band_async,
                                  compress_layer, device_layer,
                                  import_frames) return
                                  AQZ_STATUS_INVALID_ARGUMENT.  Not with an
                                  XY-transposed storage order
                                  (AQZ_STATUS_INVALID_SETTINGS). */
} aqz_stage_options;

typedef struct
{
    uint64_t bytes_per_chunk;
    uint32_t chunks_per_layer;
    uint32_t layer_slots;
    uint64_t frames_per_layer;
    uint64_t frame_bytes;      /* width*height*bpp of this level */
    uint32_t width, height;
    uint64_t chunk_pitch;      /* device bytes from chunk c to chunk c+1 of
                                  a resident layer (>= bytes_per_chunk; the
                                  pad staggers chunks over HBM channels).
                                  Host copies are packed at bytes_per_chunk. */
} aqz_level_layout;

aqz_status aqz_stage_create(const aqz_array_desc* desc,
                            const aqz_stage_options* opt, aqz_stage** out);
void aqz_stage_destroy(aqz_stage* st);
uint32_t aqz_stage_n_levels(const aqz_stage* st);
aqz_status aqz_stage_level_dims(const aqz_stage* st, uint32_t level,
                                aqz_dimension* out, size_t cap, size_t* ndims);
aqz_status aqz_stage_level_layout(const aqz_stage* st, uint32_t level,
                                  aqz_level_layout* out);
/* Run the stage on the HIP stream `stream` (a hipStream_t; NULL = the
 * stage's own stream).  All later work is enqueued there. */
aqz_status aqz_stage_set_stream(aqz_stage* st, void* stream);
/* Make the stage's stream wait for all work enqueued so far on `stream`
 * (a hipStream_t): append device frames produced there without a host
 * synchronisation (e.g. a torch stream that filled them). */
aqz_status aqz_stage_wait_stream(aqz_stage* st, void* stream);
/* Append n_frames full level-0 frames (contiguous, frame after frame).
 * Equivalent to n_frames calls of MultiscaleArray::write_frame.
 *  - AQZ_MEM_HOST: copied into a pinned staging buffer by a few host threads
 *    before return, so the caller may reuse it at once, as with
 *    ZarrStream_append (frame.queue.cpp:37-39);
 *  - AQZ_MEM_HOST_PINNED (a camera's DMA ring) and AQZ_MEM_DEVICE: read
 *    asynchronously; keep the bytes unchanged until aqz_stage_frames_consumed
 *    counts them (or aqz_stage_synchronize returns).
 * The H2D runs on the stage's copy stream and overlaps earlier batches'
 * kernels and hand-off copies. */
aqz_status aqz_stage_append(aqz_stage* st, const void* frames,
                            uint64_t n_frames, int32_t mem);
aqz_status aqz_stage_synchronize(aqz_stage* st);
/* frames written so far to `level` (Array::frames_written_) */
uint64_t aqz_stage_frames_written(const aqz_stage* st, uint32_t level);
/* Level-0 frames appended so far whose source bytes the stage has finished
 * reading (in append order): their source buffers may be reused. */
uint64_t aqz_stage_frames_consumed(aqz_stage* st);
/* Block (on events, no spin) until at least `frames` appended level-0
 * frames have been read: the reference's frame queue hands its buffer back
 * when the consumer pops it (frame.queue.cpp:48-73); a caller that appends
 * pinned batches from a double buffer waits here before refilling one. */
aqz_status aqz_stage_wait_consumed(aqz_stage* st, uint64_t frames);
/* Copy chunk layer `layer` of `level` (must still be resident) to dst
 * (bytes_per_chunk*chunks_per_layer bytes) and its has_data flags (one byte
 * per chunk, 1 = some byte of the chunk is nonzero).  Synchronizes.  Frames
 * of a layer not yet written read as unspecified bytes until the layer is
 * complete or aqz_stage_finalize ran.  mem = where dst lives. */
aqz_status aqz_stage_copy_layer(aqz_stage* st, uint32_t level, uint64_t layer,
                                void* dst, size_t cap, uint8_t* has_data,
                                size_t has_data_cap, int32_t mem);
/* Asynchronous hand-off of a resident chunk layer (outputs D2H
 * straight into host chunk buffers): enqueues, after all work appended so
 * far, a D2H copy of the layer into dst (pinned memory for a real overlap;
 * cap >= bytes_per_chunk * chunks_per_layer) and of its has_data bytes into
 * has_data (NULL to skip), on the stage's hand-off stream.  Returns at once;
 * the ring slot is not rewritten until the copy has finished.  The copies
 * are complete after aqz_stage_wait_copies or aqz_stage_synchronize. */
aqz_status aqz_stage_copy_layer_async(aqz_stage* st, uint32_t level,
                                      uint64_t layer, void* dst, size_t cap,
                                      uint8_t* has_data, size_t has_data_cap);
aqz_status aqz_stage_wait_copies(aqz_stage* st);
/* Hand-off tickets.  Every aqz_stage_copy_layer_async,
 * aqz_stage_copy_band_async and aqz_stage_copy_compressed_async call that
 * succeeds is one ticket, numbered 1, 2, ... in call order;
 * aqz_stage_last_ticket returns the newest.  aqz_stage_copies_completed
 * returns (without blocking) how many tickets have completed -- their
 * destination bytes are in place -- and tickets complete in order.
 * aqz_stage_wait_ticket blocks until ticket `ticket` has completed.  With
 * these a caller installs each handed-off unit into its host chunk buffers
 * (Array::chunks_) when its copy lands, in frame order, and never waits
 * for copies issued after it (cf. the flush in array.cpp:209-219). */
uint64_t aqz_stage_last_ticket(const aqz_stage* st);
uint64_t aqz_stage_copies_completed(aqz_stage* st);
aqz_status aqz_stage_wait_ticket(aqz_stage* st, uint64_t ticket);

/* ---- dim-1 banding ---------------------------------------------------------
 * Array::flush_completed_bands_ (array.cpp:873-908) flushes the chunks of a
 * band of dimension 1 as soon as its frames are written, before the whole
 * chunk layer is: ArrayDimensions::supports_dim1_banding, dim1_band_count,
 * frames_per_dim1_band, chunks_per_dim1_band (array.dimensions.cpp:344-373).
 * Band b of a layer is the contiguous chunk range
 * [b * chunks_per_band, (b + 1) * chunks_per_band). */
aqz_status aqz_stage_band_geometry(const aqz_stage* st, uint32_t level,
                                   int32_t* supported, uint32_t* n_bands,
                                   uint64_t* frames_per_band,
                                   uint32_t* chunks_per_band);
/* Asynchronous hand-off of one complete band of a resident layer, like
 * aqz_stage_copy_layer_async for its chunk range: dst receives
 * chunks_per_band * bytes_per_chunk bytes, has_data (NULL to skip)
 * chunks_per_band flags.  The band must be complete: all its frames
 * written (frames_written(level) >= layer * frames_per_layer +
 * (band + 1) * frames_per_band), or the layer finalized. */
aqz_status aqz_stage_copy_band_async(aqz_stage* st, uint32_t level,
                                     uint64_t layer, uint32_t band, void* dst,
                                     size_t cap, uint8_t* has_data,
                                     size_t has_data_cap);

/* ---- memory accounting ------------------------------------------------------
 * What the stage holds, for ZarrStream_get_current_memory_usage
 * (zarr.stream.cpp:1057-1068) and ZarrStreamSettings_estimate_max_memory_usage
 * (acquire.zarr.cpp:216-314) to include. */
typedef struct
{
    uint64_t device_bytes; /* HBM: chunk-layer rings, has_data words, frame
                              tables, scratch, H2D staging, compressed frames */
    uint64_t pinned_bytes; /* page-locked host memory: host-source staging,
                              compressed-offset read-back */
} aqz_memory_usage;
/* Bytes currently allocated by the stage. */
aqz_status aqz_stage_memory_usage(const aqz_stage* st, aqz_memory_usage* out);
/* Upper bound of what a stage created with (desc, opt) allocates, compressed
 * hand-off excluded (add aqz_compressor_max_bytes per compressed slot and
 * aqz_compressor_scratch_bytes per compressed level).  No GPU needed. */
aqz_status aqz_stage_estimate_memory(const aqz_array_desc* desc,
                                     const aqz_stage_options* opt,
                                     aqz_memory_usage* out);
/* Pin the calling thread to the CPUs of the NUMA node of the stage's device
 * (the CPUs the stage's own host threads run on; no-op when unknown): for a
 * caller's threads that feed the stage or read its hand-off buffers.  The
 * reference pins none of its threads (thread.pool.cpp:6-20). */
aqz_status aqz_stage_bind_host_thread(const aqz_stage* st);
/* Page-locked host memory for frames and hand-off buffers. */
aqz_status aqz_host_alloc(size_t bytes, void** out);
void aqz_host_free(void* p);
/* Device pointers of a resident layer (for device-side consumers).  Chunk c
 * starts at chunks + c * chunk_pitch (aqz_level_layout).  Chunk c has data iff has_data[c] == layer / layer_slots + 1 (the words carry the
 * ring-slot generation, so they are never cleared). */
aqz_status aqz_stage_device_layer(aqz_stage* st, uint32_t level,
                                  uint64_t layer, void** chunks,
                                  uint32_t** has_data);
/* ---- chunk compression on the device ----------------
 * ZarrCompressionSettings (zarr.types.h:112-122) as applied by
 * Chunk::compress_and_take_buffer (chunk.cpp:78-106) ->
 * zarr::compress_in_place (zarr.common.cpp:106-140) -> blosc_compress_ctx.
 * codec: ZarrCompressionCodec values.
 *  - AQZ_CODEC_BLOSC_LZ4: blosc1 frames made on the device (shuffle +
 *    LZ4); clevel 0 stores every chunk as a memcpyed frame, levels 1-9 run
 *    the same GPU match finder.
 *  - AQZ_CODEC_BLOSC_ZSTD: blosc1 frames made on the device: every block
 *    (256 KiB) shuffled, then one zstd frame per block (zarr.common.cpp:
 *    106-140 with "zstd"); blosc clevel 0 stores memcpyed frames.
 *  - AQZ_CODEC_ZSTD: one zstd frame per chunk (ZSTD_compress,
 *    zarr.common.cpp:142-166), made on the device.
 *  The device zstd encoder: Huffman literals (one table per 64 KiB group of
 *  a shuffled block -- per bit plane under bitshuffle at clevel >= 7 -- or
 *  per 256 KiB of unshuffled data), sequence tables fitted per
 *  frame, a greedy LZ parse in 4 KiB units; the level sets how far back
 *  matches reach (zstd level L; blosc clevel c is L = 2c - 1): plain zstd
 *  L 1-2 unit-local, L 3-6 + far candidates from a 2^17-entry table over
 *  the whole chunk, L >= 7 a 2^18-entry table; blosc-zstd with bitshuffle
 *  L >= 3 a 2^15-entry table per block.  Ratios on camera-like and dim u16
 *  data are within ~1% (blosc-zstd) and ~7% (plain zstd L 5) of libzstd
 *  (c-blosc clevel 5 / ZSTD_compress level 5).  With
 *  AQZ_ZSTD_HOST=1 in the environment the zstd codecs run on a host pool
 *  instead (device shuffle, D2H, the system's libzstd.so.1 at the clevel ->
 *  zstd level map of c-blosc; absent library ->
 *  AQZ_STATUS_NOT_YET_IMPLEMENTED), byte for byte what libzstd makes.
 *  Frames decode (any blosc1 / zstd decoder) to the chunk bytes exactly;
 *  their compressed bytes differ from c-blosc's and libzstd's (block size,
 *  match finder, no stream split for blosc-zstd). */
#define AQZ_CODEC_NONE 0
#define AQZ_CODEC_BLOSC_LZ4 1
#define AQZ_CODEC_BLOSC_ZSTD 2
#define AQZ_CODEC_ZSTD 3
typedef struct
{
    int32_t codec;   /* ZarrCompressionCodec */
    int32_t clevel;  /* 0-9 */
    int32_t shuffle; /* 0 none, 1 byte (BLOSC_SHUFFLE), 2 bit (BLOSC_BITSHUFFLE) */
} aqz_compression;

/* Compress resident layer `layer` of `level` into blosc1 frames, one per
 * chunk with data (chunks without data are skipped, like the reference's
 * skip_chunk), back to back in SHARD-MAJOR order: the chunks of shard 0 by
 * shard_internal_index, then shard 1, ... (aqz_stage_compressed_entries
 * lists them), so each shard's frames of the layer are one contiguous run
 * that Shard::write_chunk would append at the shard's file offset.  Runs on the hand-off stream
 * after the kernels that wrote the layer; the slot is not reused until it
 * has been read. */
aqz_status aqz_stage_compress_layer(aqz_stage* st, uint32_t level, uint64_t layer,
                                    const aqz_compression* comp);
/* Waits for that compression.  offsets[i] = start of the i-th frame in
 * output order, offsets[i+1] - offsets[i] its size (0: skipped),
 * offsets[chunks_per_layer] = total bytes.  n >= chunks_per_layer + 1. */
aqz_status aqz_stage_compressed_offsets(aqz_stage* st, uint32_t level,
                                        uint64_t layer, uint64_t* offsets, size_t n);
/* Copy of the layer's frames (total bytes) to dst: host or device,
 * asynchronous, complete after aqz_stage_wait_copies.  With AQZ_ZSTD_HOST=1
 * (zstd frames made on the host) dst is host memory, filled before the
 * call returns. */
aqz_status aqz_stage_copy_compressed_async(aqz_stage* st, uint32_t level,
                                           uint64_t layer, void* dst, size_t cap);
/* *done = 1 once the compression of that layer has finished (no wait): then
 * aqz_stage_compressed_offsets / _entries and aqz_stage_copy_compressed_async
 * do not block the caller.  A consumer thread issues the frames' D2H only
 * for finished layers, as the reference's flush jobs hand a chunk to its
 * shard once compress_and_take_buffer returned (array.cpp:722-736). */
aqz_status aqz_stage_compression_done(aqz_stage* st, uint32_t level, uint64_t layer,
                                      int32_t* done);

/* ---- shard packing -----------------------------------
 * The frames of a compressed layer in output order, with their place in
 * the shards (ArrayDimensions::shard_index_for_chunk / shard_internal_index,
 * array.dimensions.cpp:396-548; the internal index includes the layer's
 * position along the append dimension inside its shard). */
typedef struct
{
    uint32_t chunk;    /* chunk index inside the layer (Array::chunks_ slot) */
    uint32_t shard;    /* shard of the current append-dimension shard row */
    uint32_t internal; /* shard_internal_index */
    uint32_t reserved;
    uint64_t offset;   /* frame start inside the compressed layer */
    uint64_t nbytes;   /* frame bytes; 0 = no data (Shard::skip_chunk) */
} aqz_chunk_entry;
aqz_status aqz_stage_compressed_entries(aqz_stage* st, uint32_t level,
                                        uint64_t layer, aqz_chunk_entry* out,
                                        size_t n);
/* chunks_per_shard, number_of_shards (one append-dimension shard row) and
 * chunk layers per shard (array.dimensions.cpp:376-397) of a level. */
aqz_status aqz_stage_shard_geometry(const aqz_stage* st, uint32_t level,
                                    uint32_t* chunks_per_shard,
                                    uint32_t* number_of_shards,
                                    uint32_t* layers_per_shard);
/* Shard::write_table_ (shard.cpp:145-166): chunks_per_shard (offset,
 * extent) little-endian uint64 pairs -- UINT64_MAX for both when a chunk
 * was never written -- followed by the CRC-32C of those bytes; out holds
 * aqz_shard_table_bytes(chunks_per_shard) bytes.  The table goes at the end
 * of the shard (index_location "end"). */
size_t aqz_shard_table_bytes(uint32_t chunks_per_shard);
aqz_status aqz_shard_table(const uint64_t* offsets, const uint64_t* extents,
                           uint32_t chunks_per_shard, void* out, size_t cap);
uint32_t aqz_crc32c(const void* data, size_t n);

/* Stand-alone compressor (any AQZ_CODEC_*) for device-resident chunk arrays: chunk i of
 * n_chunks at chunks + i * pitch, chunk_bytes each; frames back to back at
 * dst (device, >= aqz_compressor_max_bytes), offsets (device, n_chunks + 1
 * uint64) as above.  Enqueued on `stream` (hipStream_t; NULL = default). */
typedef struct aqz_compressor aqz_compressor;
aqz_status aqz_compressor_create(uint64_t chunk_bytes, uint32_t typesize,
                                 const aqz_compression* comp, aqz_compressor** out);
void aqz_compressor_destroy(aqz_compressor* c);
uint64_t aqz_compressor_max_bytes(uint64_t chunk_bytes, uint32_t n_chunks);
/* Device scratch one compressor (or one level of a stage compressing its
 * layers) allocates to compress n_chunks chunks of chunk_bytes with `comp`
 * (an upper bound; the zstd codecs keep parse units, sequences and per-block
 * state at about 4x the layer).  0 on invalid settings.  No GPU needed. */
uint64_t aqz_compressor_scratch_bytes(const aqz_compression* comp, uint64_t chunk_bytes,
                                      uint32_t typesize, uint32_t n_chunks);
aqz_status aqz_compressor_run(aqz_compressor* c, const void* chunks, uint64_t pitch,
                              uint32_t n_chunks, void* dst, size_t dst_cap,
                              uint64_t* offsets, void* stream);
/* The blosc block size of the frames (recorded in each frame header; 0 for
 * plain zstd). */
uint32_t aqz_compressor_blocksize(const aqz_compressor* c);

/* z-slab assembly of one chunk layer (a volume stream sharded
 * over GPUs by z slabs, aqz_stage_options.z_slab_*): copy the tiles of
 * frames [first, first + count) of `layer` of `level` (frame ids inside the
 * layer) from stage src's resident layer into dst's, with their has_data
 * flags -- over xGMI when the stages' devices differ (peer access is
 * enabled on first use), on dst's stream after all work enqueued so far on
 * src's.  src = NULL zero-fills those frames in dst.  The two stages must
 * have the same array description and options apart from the device and
 * the slab.  The layer becomes resident in dst if it was not; src's ring
 * slot is not rewritten until the copy has read it.  dst then holds the
 * whole layer and hands it off (aqz_stage_copy_*_async,
 * aqz_stage_compress_layer) as if it had written every frame -- the chunk
 * buffers Array::write_frame_to_chunks_ fills (array.cpp:507-622). */
aqz_status aqz_stage_import_frames(aqz_stage* dst, aqz_stage* src, uint32_t level,
                                   uint64_t layer, uint32_t first, uint32_t count);

/* ---- level-0 tile split on the host (aqz_stage_options.
 * level0_split_on_host) ---------------------------------------------------
 * Array::write_frame_to_chunks_ (array.cpp:537-619) with
 * Chunk::write_tile_rows (chunk.cpp:17-58), run by the host on frames it
 * holds: tile t of level-0 frame f goes to chunk t + tile_group_offset(f)
 * of f's chunk layer, its rows at chunk_internal_offset(f) +
 * r * tile_cols * bpp (f transposed to storage order first,
 * array.cpp:557-566); ragged padding is not written; has_data[c] becomes 1
 * once a copied byte of chunk c is nonzero and is never cleared (zero it
 * when a layer starts).  dst holds the packed chunks [chunk0, chunk0 +
 * cap / bytes_per_chunk) of one layer -- the whole layer (chunk0 0), or a
 * dim-1 band (chunk0 = band * chunks_per_band) -- laid out as
 * aqz_stage_copy_layer_async / _band_async would write them; has_data has
 * has_data_cap >= that many bytes.  Every tile of every frame must fall in
 * that range (else AQZ_STATUS_INVALID_ARGUMENT).  Pure host work: no GPU
 * call, any thread. */
/* Frames [first_frame, first_frame + n_frames) (level-0 frame ids, in
 * acquisition order, frame after frame at `frames`; all in one chunk layer,
 * else AQZ_STATUS_INVALID_ARGUMENT), split by the stage's host threads (on
 * the NUMA node of its device). */
aqz_status aqz_stage_split_level0_host(aqz_stage* st, const void* frames, uint64_t n_frames,
                                       uint64_t first_frame, uint32_t chunk0, void* dst,
                                       size_t cap, uint8_t* has_data, size_t has_data_cap);
/* Rows [row_begin, row_end) of one level-0 frame, on the calling thread;
 * several threads may split disjoint rows of one frame at once.  frame_copy
 * (NULL: none): the same rows are also copied to this frame-sized buffer in
 * the same pass -- the hand-off's copy into its pinned batch
 * (ZarrStream_append's one copy, frame.queue.cpp:37-39). */
aqz_status aqz_stage_split_level0_rows(const aqz_stage* st, const void* frame,
                                       uint64_t frame_id, uint32_t row_begin,
                                       uint32_t row_end, void* frame_copy, uint32_t chunk0,
                                       void* dst, size_t cap, uint8_t* has_data,
                                       size_t has_data_cap);
/* The same split over an aqz_dims (the array's acquisition dims with its
 * storage order), no stage and no GPU. */
aqz_status aqz_dims_split_frame_rows(const aqz_dims* d, const void* frame, uint64_t frame_id,
                                     uint32_t row_begin, uint32_t row_end, uint32_t chunk0,
                                     void* dst, size_t cap, uint8_t* has_data,
                                     size_t has_data_cap);

/* Zero the not-yet-written frames of every level's last partial layer so
 * it can be flushed (the reference's lazily zeroed chunks, chunk.cpp:8-15).
 * The unpaired trailing z plane is dropped, as in the reference. */
aqz_status aqz_stage_finalize(aqz_stage* st);

#ifdef __cplusplus
}
#endif
#endif /* AQZ_GPU_H */
