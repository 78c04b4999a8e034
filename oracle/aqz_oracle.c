/*
 * aqz_oracle.c -- CPU ORACLE (test infrastructure only; see aqz_oracle.h).
 *
 * A plain-C restatement of the reference's multiscale downsample and chunk
 * tile split.  Every function cites the reference file:line it follows
 * (paths relative to /root/reference/src/streaming/).
 *
 * Integer semantics (verified against the compiled
 * reference in oracle/_ref): the "overflow-safe" integral overloads of
 * mean4/mean2 (downsampler.cpp:53-62, 114-123) never participate in overload
 * resolution, so the generic `(a+b+c+d)/4` and `(a+b)/2` run for every dtype.
 * 8/16-bit operands promote to int (sum exact, division truncates toward
 * zero); 32/64-bit sums wrap modulo 2^N.  Signed 32/64-bit sums are computed
 * here in the unsigned type and converted back, which is the wrap the
 * reference exhibits without relying on signed-overflow UB.
 */
#include "aqz_oracle.h"

#include <stdlib.h>
#include <string.h>

size_t
or_bytes_of_type(int dtype)
{
    /* zarr.common.cpp:47-70 */
    switch (dtype) {
        case OR_U8:
        case OR_I8:
            return 1;
        case OR_U16:
        case OR_I16:
            return 2;
        case OR_U32:
        case OR_I32:
        case OR_F32:
            return 4;
        case OR_U64:
        case OR_I64:
        case OR_F64:
            return 8;
        default:
            return 0;
    }
}

/* ------------------------------------------------------------------------
 * 2x2 and z-pair reducers (downsampler.cpp:39-137).
 * ---------------------------------------------------------------------- */
#define SMALL_INT_REDUCERS(T, NAME)                                            \
    static T mean4_##NAME(T a, T b, T c, T d)                                  \
    {                                                                          \
        return (T)(((int)a + (int)b + (int)c + (int)d) / 4);                   \
    }                                                                          \
    static T mean2_##NAME(T a, T b) { return (T)(((int)a + (int)b) / 2); }

SMALL_INT_REDUCERS(uint8_t, u8)
SMALL_INT_REDUCERS(uint16_t, u16)
SMALL_INT_REDUCERS(int8_t, i8)
SMALL_INT_REDUCERS(int16_t, i16)

/* 32/64-bit: the sum is computed in the operand type and wraps. */
#define WIDE_INT_REDUCERS(T, U, NAME)                                          \
    static T mean4_##NAME(T a, T b, T c, T d)                                  \
    {                                                                          \
        U s = (U)a + (U)b + (U)c + (U)d;                                       \
        return (T)s / (T)4;                                                    \
    }                                                                          \
    static T mean2_##NAME(T a, T b)                                            \
    {                                                                          \
        U s = (U)a + (U)b;                                                     \
        return (T)s / (T)2;                                                    \
    }

WIDE_INT_REDUCERS(uint32_t, uint32_t, u32)
WIDE_INT_REDUCERS(uint64_t, uint64_t, u64)
WIDE_INT_REDUCERS(int32_t, uint32_t, i32)
WIDE_INT_REDUCERS(int64_t, uint64_t, i64)

/* float: ((a+b)+c)+d, then /4 (downsampler.cpp:46-51) */
static float
mean4_f32(float a, float b, float c, float d)
{
    float s = a + b;
    s = s + c;
    s = s + d;
    return s / 4.0f;
}
static float
mean2_f32(float a, float b)
{
    return (a + b) / 2.0f;
}
static double
mean4_f64(double a, double b, double c, double d)
{
    double s = a + b;
    s = s + c;
    s = s + d;
    return s / 4.0;
}
static double
mean2_f64(double a, double b)
{
    return (a + b) / 2.0;
}

/* Generic per-type bodies.  min4/max4 are compare-select in the order
 * b, c, d with strict comparisons (downsampler.cpp:64-98); min2/max2 are
 * `a < b ? a : b` / `a > b ? a : b` (downsampler.cpp:125-137) where a is the
 * earlier plane. */
#define TYPE_BODIES(T, NAME)                                                   \
    static T reduce4_##NAME(int m, T a, T b, T c, T d)                         \
    {                                                                          \
        T v = a;                                                               \
        switch (m) {                                                           \
            case OR_DECIMATE:                                                  \
                return a;                                                      \
            case OR_MEAN:                                                      \
                return mean4_##NAME(a, b, c, d);                               \
            case OR_MIN:                                                       \
                if (b < v) v = b;                                              \
                if (c < v) v = c;                                              \
                if (d < v) v = d;                                              \
                return v;                                                      \
            default: /* OR_MAX */                                              \
                if (b > v) v = b;                                              \
                if (c > v) v = c;                                              \
                if (d > v) v = d;                                              \
                return v;                                                      \
        }                                                                      \
    }                                                                          \
    static T reduce2_##NAME(int m, T a, T b)                                   \
    {                                                                          \
        switch (m) {                                                           \
            case OR_DECIMATE:                                                  \
                return a;                                                      \
            case OR_MEAN:                                                      \
                return mean2_##NAME(a, b);                                     \
            case OR_MIN:                                                       \
                return a < b ? a : b;                                          \
            default:                                                           \
                return a > b ? a : b;                                          \
        }                                                                      \
    }                                                                          \
    /* scale_image<T>, downsampler.cpp:139-206: w_pad = w + w%2, odd right   \
     * column and bottom row replicate `here` (lines 187-196). */             \
    static void scale_##NAME(int m, const T* src, size_t w, size_t h, T* dst) \
    {                                                                          \
        const size_t w_pad = w + (w % 2), h_pad = h + (h % 2);                 \
        size_t di = 0;                                                         \
        (void)w_pad;                                                           \
        for (size_t row = 0; row < h; row += 2) {                              \
            const int pad_h = (row == h - 1 && h != h_pad);                    \
            for (size_t col = 0; col < w; col += 2) {                          \
                const int pad_w = (col == w - 1 && w != w_pad);                \
                const size_t si = row * w + col;                               \
                const T here = src[si];                                        \
                const T right = src[si + !pad_w];                              \
                const T down = src[si + w * (!pad_h)];                         \
                const T diag = src[si + w * (!pad_h) + (!pad_w)];              \
                dst[di++] = reduce4_##NAME(m, here, right, down, diag);        \
            }                                                                  \
        }                                                                      \
    }                                                                          \
    /* average_two_frames<T>, downsampler.cpp:208-246 */                      \
    static void avg2_##NAME(int m, T* dst, const T* src, size_t n)             \
    {                                                                          \
        for (size_t i = 0; i < n; ++i)                                         \
            dst[i] = reduce2_##NAME(m, dst[i], src[i]);                        \
    }

TYPE_BODIES(uint8_t, u8)
TYPE_BODIES(uint16_t, u16)
TYPE_BODIES(uint32_t, u32)
TYPE_BODIES(uint64_t, u64)
TYPE_BODIES(int8_t, i8)
TYPE_BODIES(int16_t, i16)
TYPE_BODIES(int32_t, i32)
TYPE_BODIES(int64_t, i64)
TYPE_BODIES(float, f32)
TYPE_BODIES(double, f64)

int
or_scale_image(int dtype, int method, const void* src, size_t width,
               size_t height, void* dst)
{
    if (method < 0 || method >= OR_NMETHODS)
        return -1;
#define CASE(ID, T, NAME)                                                      \
    case ID:                                                                   \
        scale_##NAME(method, (const T*)src, width, height, (T*)dst);           \
        return 0;
    switch (dtype) {
        CASE(OR_U8, uint8_t, u8)
        CASE(OR_U16, uint16_t, u16)
        CASE(OR_U32, uint32_t, u32)
        CASE(OR_U64, uint64_t, u64)
        CASE(OR_I8, int8_t, i8)
        CASE(OR_I16, int16_t, i16)
        CASE(OR_I32, int32_t, i32)
        CASE(OR_I64, int64_t, i64)
        CASE(OR_F32, float, f32)
        CASE(OR_F64, double, f64)
        default:
            return -1;
    }
#undef CASE
}

int
or_average_two_frames(int dtype, int method, void* dst, const void* src,
                      size_t n_pixels)
{
    if (method < 0 || method >= OR_NMETHODS)
        return -1;
#define CASE(ID, T, NAME)                                                      \
    case ID:                                                                   \
        avg2_##NAME(method, (T*)dst, (const T*)src, n_pixels);                 \
        return 0;
    switch (dtype) {
        CASE(OR_U8, uint8_t, u8)
        CASE(OR_U16, uint16_t, u16)
        CASE(OR_U32, uint32_t, u32)
        CASE(OR_U64, uint64_t, u64)
        CASE(OR_I8, int8_t, i8)
        CASE(OR_I16, int16_t, i16)
        CASE(OR_I32, int32_t, i32)
        CASE(OR_I64, int64_t, i64)
        CASE(OR_F32, float, f32)
        CASE(OR_F64, double, f64)
        default:
            return -1;
    }
#undef CASE
}

/* ------------------------------------------------------------------------
 * Level geometry (downsampler.cpp:8-37, 494-597)
 * ---------------------------------------------------------------------- */
static uint32_t
bit_width_u32(uint32_t v)
{
    uint32_t n = 0;
    while (v) {
        ++n;
        v >>= 1;
    }
    return n;
}

static uint32_t
ceil_div_u32(uint32_t a, uint32_t b)
{
    return (a + b - 1) / b;
}

static or_dim
downsample_dimension(or_dim d)
{
    /* downsampler.cpp:8-37 */
    or_dim o = d;
    o.array_size_px = (d.array_size_px + (d.array_size_px % 2)) / 2;
    const uint32_t n_chunks = ceil_div_u32(o.array_size_px, d.chunk_size_px);
    o.shard_size_chunks =
      n_chunks < d.shard_size_chunks ? n_chunks : d.shard_size_chunks;
    return o;
}

int
or_make_levels(const or_dim* dims, int ndims, uint32_t max_levels,
               int* n_levels_out, or_dim* out, int out_cap_levels)
{
    if (ndims < 3 || ndims > OR_MAX_DIMS)
        return -1;
    const or_dim* X = &dims[ndims - 1];
    const or_dim* Y = &dims[ndims - 2];
    const or_dim* Z = &dims[ndims - 3];

    /* downsampler.cpp:512-541 */
    const uint32_t ncx = ceil_div_u32(X->array_size_px, X->chunk_size_px);
    const uint32_t nlx = ncx > 1 ? bit_width_u32(ncx - 1) : 0;
    const uint32_t ncy = ceil_div_u32(Y->array_size_px, Y->chunk_size_px);
    const uint32_t nly = ncy > 1 ? bit_width_u32(ncy - 1) : 0;
    uint32_t n_levels = nlx < nly ? nlx : nly;
    if (Z->type == OR_SPACE) {
        const uint32_t ncz = ceil_div_u32(Z->array_size_px, Z->chunk_size_px);
        const uint32_t ndz = ncz > 1 ? bit_width_u32(ncz - 1) : 0;
        n_levels = n_levels > ndz ? n_levels : ndz;
    }
    if (max_levels > 0 && max_levels < n_levels)
        n_levels = max_levels;
    if ((int)n_levels + 1 > out_cap_levels)
        return -2;

    memcpy(out, dims, sizeof(or_dim) * (size_t)ndims);
    for (uint32_t level = 1; level <= n_levels; ++level) {
        const or_dim* prev = &out[(level - 1) * ndims];
        or_dim* cur = &out[level * ndims];
        for (int i = 0; i < ndims - 3; ++i)
            cur[i] = prev[i];
        /* downsampler.cpp:554-561 */
        const or_dim z = prev[ndims - 3];
        if (z.type == OR_SPACE && z.array_size_px > z.chunk_size_px)
            cur[ndims - 3] = downsample_dimension(z);
        else
            cur[ndims - 3] = z;
        /* downsampler.cpp:563-575 */
        const or_dim y = prev[ndims - 2], x = prev[ndims - 1];
        const uint32_t mn =
          y.array_size_px < x.array_size_px ? y.array_size_px : x.array_size_px;
        const uint32_t mx =
          y.chunk_size_px > x.chunk_size_px ? y.chunk_size_px : x.chunk_size_px;
        if (mn > mx) {
            cur[ndims - 2] = downsample_dimension(y);
            cur[ndims - 1] = downsample_dimension(x);
        } else {
            cur[ndims - 2] = y;
            cur[ndims - 1] = x;
        }
    }
    *n_levels_out = (int)n_levels + 1;
    return 0;
}

/* ------------------------------------------------------------------------
 * ArrayDimensions index math (array.dimensions.cpp:137-548)
 * ---------------------------------------------------------------------- */
uint32_t
or_chunk_lattice_index(const or_dim* dims, int ndims, uint64_t frame_id,
                       int dim_index)
{
    /* array.dimensions.cpp:232-262 */
    if (dim_index == 0) {
        uint64_t divisor = dims[0].chunk_size_px;
        for (int i = 1; i < ndims - 2; ++i)
            divisor *= dims[i].array_size_px;
        return (uint32_t)(frame_id / divisor);
    }
    uint64_t mod_div = 1, div_div = 1;
    for (int i = dim_index; i < ndims - 2; ++i) {
        mod_div *= dims[i].array_size_px;
        div_div *= (i == dim_index ? dims[i].chunk_size_px
                                   : dims[i].array_size_px);
    }
    return (uint32_t)((frame_id % mod_div) / div_div);
}

uint32_t
or_tile_group_offset(const or_dim* dims, int ndims, uint64_t frame_id)
{
    /* array.dimensions.cpp:264-282 */
    uint64_t strides[OR_MAX_DIMS];
    strides[ndims - 1] = 1;
    for (int i = ndims - 1; i > 0; --i)
        strides[i - 1] =
          strides[i] * ceil_div_u32(dims[i].array_size_px, dims[i].chunk_size_px);
    uint64_t offset = 0;
    for (int i = ndims - 3; i > 0; --i)
        offset += (uint64_t)or_chunk_lattice_index(dims, ndims, frame_id, i) *
                  strides[i];
    return (uint32_t)offset;
}

uint64_t
or_chunk_internal_offset(const or_dim* dims, int ndims, int dtype,
                         uint64_t frame_id)
{
    /* array.dimensions.cpp:284-314 */
    const uint64_t tile_size = or_bytes_of_type(dtype) *
                               (uint64_t)dims[ndims - 1].chunk_size_px *
                               dims[ndims - 2].chunk_size_px;
    uint64_t array_strides[OR_MAX_DIMS], chunk_strides[OR_MAX_DIMS];
    for (int i = 0; i < ndims - 2; ++i)
        array_strides[i] = chunk_strides[i] = 1;
    uint64_t offset = 0;
    for (int i = ndims - 3; i > 0; --i) {
        const or_dim* d = &dims[i];
        const uint64_t internal_idx = (frame_id / array_strides[i]) %
                                      d->array_size_px % d->chunk_size_px;
        array_strides[i - 1] = array_strides[i] * d->array_size_px;
        chunk_strides[i - 1] = chunk_strides[i] * d->chunk_size_px;
        offset += internal_idx * chunk_strides[i];
    }
    const uint64_t internal_idx =
      (frame_id / array_strides[0]) % dims[0].chunk_size_px;
    offset += internal_idx * chunk_strides[0];
    return offset * tile_size;
}

uint64_t
or_bytes_per_chunk(const or_dim* dims, int ndims, int dtype)
{
    /* array.dimensions.cpp:142, 169-172 */
    uint64_t b = or_bytes_of_type(dtype);
    for (int i = 0; i < ndims; ++i)
        b *= dims[i].chunk_size_px;
    return b;
}

uint32_t
or_number_of_chunks_in_memory(const or_dim* dims, int ndims)
{
    /* array.dimensions.cpp:169-178 */
    uint32_t n = 1;
    for (int i = 1; i < ndims; ++i)
        n *= ceil_div_u32(dims[i].array_size_px, dims[i].chunk_size_px);
    return n;
}

uint64_t
or_frames_per_chunk_layer(const or_dim* dims, int ndims)
{
    /* array.dimensions.cpp:328-336 */
    uint64_t f = dims[0].chunk_size_px;
    for (int i = 1; i + 2 < ndims; ++i)
        f *= dims[i].array_size_px;
    return f;
}

static uint32_t
shards_along(const or_dim* d)
{
    /* zarr.common.cpp:94-104 */
    if (d->shard_size_chunks == 0)
        return 0;
    return ceil_div_u32(ceil_div_u32(d->array_size_px, d->chunk_size_px),
                        d->shard_size_chunks);
}

uint32_t
or_shard_index_for_chunk(const or_dim* dims, int ndims, uint32_t chunk_index)
{
    /* array.dimensions.cpp:461-502 (lattice index of dim 0 stays 0) */
    uint64_t cs[OR_MAX_DIMS];
    uint32_t lat[OR_MAX_DIMS] = { 0 }, ss[OR_MAX_DIMS];
    cs[ndims - 1] = 1;
    for (int i = ndims - 1; i > 0; --i)
        cs[i - 1] =
          cs[i] * ceil_div_u32(dims[i].array_size_px, dims[i].chunk_size_px);
    for (int i = ndims - 1; i > 0; --i)
        lat[i] = (uint32_t)(chunk_index % cs[i - 1] / cs[i]);
    ss[ndims - 1] = 1;
    for (int i = ndims - 1; i > 0; --i)
        ss[i - 1] = ss[i] * shards_along(&dims[i]);
    uint32_t index = 0;
    for (int i = 0; i < ndims; ++i)
        index += (lat[i] / dims[i].shard_size_chunks) * ss[i];
    return index;
}

uint32_t
or_shard_internal_index(const or_dim* dims, int ndims, uint32_t chunk_index)
{
    /* array.dimensions.cpp:504-548 */
    uint64_t cs[OR_MAX_DIMS], lat[OR_MAX_DIMS], is[OR_MAX_DIMS];
    cs[ndims - 1] = 1;
    for (int i = ndims - 1; i > 0; --i)
        cs[i - 1] =
          cs[i] * ceil_div_u32(dims[i].array_size_px, dims[i].chunk_size_px);
    for (int i = ndims - 1; i > 0; --i)
        lat[i] = chunk_index % cs[i - 1] / cs[i];
    lat[0] = chunk_index / cs[0];
    is[ndims - 1] = 1;
    for (int i = ndims - 1; i > 0; --i)
        is[i - 1] = is[i] * dims[i].shard_size_chunks;
    uint64_t index = 0;
    for (int i = 0; i < ndims; ++i)
        index += (lat[i] % dims[i].shard_size_chunks) * is[i];
    return (uint32_t)index;
}

/* ------------------------------------------------------------------------
 * Tile split (array.cpp:537-619 + chunk.cpp:17-58)
 * ---------------------------------------------------------------------- */
size_t
or_write_frame_to_chunks(const or_dim* dims, int ndims, int dtype,
                         uint64_t frame_id, const void* frame, uint8_t* layer,
                         uint8_t* has_data)
{
    const size_t bpp = or_bytes_of_type(dtype);
    const uint32_t W = dims[ndims - 1].array_size_px;
    const uint32_t tw = dims[ndims - 1].chunk_size_px;
    const uint32_t H = dims[ndims - 2].array_size_px;
    const uint32_t th = dims[ndims - 2].chunk_size_px;
    if (tw == 0 || th == 0)
        return 0;
    const uint64_t bpc = or_bytes_per_chunk(dims, ndims, dtype);
    const size_t tile_row_bytes = (size_t)tw * bpp;
    const uint32_t ntx = ceil_div_u32(W, tw), nty = ceil_div_u32(H, th);
    const uint32_t group = or_tile_group_offset(dims, ndims, frame_id);
    const uint64_t internal =
      or_chunk_internal_offset(dims, ndims, dtype, frame_id);
    const uint8_t* src = (const uint8_t*)frame;
    const size_t src_stride = (size_t)W * bpp;
    size_t written = 0;
    for (uint32_t t = 0; t < ntx * nty; ++t) {
        const uint32_t chunk = t + group;
        const uint32_t ty = t / ntx, tx = t % ntx;
        const uint32_t row0 = ty * th;
        if (row0 >= H)
            continue;
        const uint32_t n_rows = th < H - row0 ? th : H - row0;
        const uint32_t col0 = tx * tw;
        const uint32_t region_w = (col0 + tw < W ? col0 + tw : W) - col0;
        const size_t nbytes = (size_t)region_w * bpp;
        const uint8_t* s0 = src + bpp * ((size_t)row0 * W + col0);
        uint8_t* d0 = layer + (uint64_t)chunk * bpc + internal;
        int any = has_data[chunk];
        for (uint32_t r = 0; r < n_rows; ++r) {
            const uint8_t* s = s0 + (size_t)r * src_stride;
            memcpy(d0 + (size_t)r * tile_row_bytes, s, nbytes);
            if (!any) {
                for (size_t b = 0; b < nbytes; ++b)
                    if (s[b]) {
                        any = 1;
                        break;
                    }
            }
        }
        if (any)
            has_data[chunk] = 1;
        written += nbytes * n_rows;
    }
    return written;
}

/* ------------------------------------------------------------------------
 * Cascade state machine (downsampler.cpp:306-414, 599-605)
 * ---------------------------------------------------------------------- */
struct or_downsampler
{
    int dtype, method, ndims, n_levels;
    size_t bpp;
    or_dim dims[OR_MAX_LEVELS * OR_MAX_DIMS];
    uint32_t level_frame_count[OR_MAX_LEVELS];
    uint8_t* partial[OR_MAX_LEVELS];      /* partial_scaled_frames_ */
    uint8_t* downsampled[OR_MAX_LEVELS];  /* downsampled_frames_ */
    size_t downsampled_bytes[OR_MAX_LEVELS];
};

or_downsampler*
or_ds_create(const or_dim* dims, int ndims, int dtype, int method,
             uint32_t max_levels)
{
    if (dtype < 0 || dtype >= OR_NDTYPES || method < 0 ||
        method >= OR_NMETHODS)
        return NULL;
    or_downsampler* ds = (or_downsampler*)calloc(1, sizeof(*ds));
    if (!ds)
        return NULL;
    ds->dtype = dtype;
    ds->method = method;
    ds->ndims = ndims;
    ds->bpp = or_bytes_of_type(dtype);
    if (or_make_levels(dims, ndims, max_levels, &ds->n_levels, ds->dims,
                       OR_MAX_LEVELS) != 0) {
        free(ds);
        return NULL;
    }
    return ds;
}

void
or_ds_destroy(or_downsampler* ds)
{
    if (!ds)
        return;
    for (int i = 0; i < OR_MAX_LEVELS; ++i) {
        free(ds->partial[i]);
        free(ds->downsampled[i]);
    }
    free(ds);
}

int
or_ds_n_levels(const or_downsampler* ds)
{
    return ds->n_levels;
}

const or_dim*
or_ds_level_dims(const or_downsampler* ds, int level)
{
    return &ds->dims[level * ds->ndims];
}

static void
emplace_downsampled(or_downsampler* ds, int level, uint8_t* frame,
                    size_t nbytes)
{
    /* downsampler.cpp:599-605: unordered_map::emplace keeps an existing
     * entry; the level count is bumped regardless. */
    if (ds->downsampled[level] == NULL) {
        ds->downsampled[level] = frame;
        ds->downsampled_bytes[level] = nbytes;
    } else {
        free(frame);
    }
    ++ds->level_frame_count[level];
}

int
or_ds_add_frame(or_downsampler* ds, const void* frame, size_t nbytes)
{
    const int nd = ds->ndims;
    size_t fw = ds->dims[nd - 1].array_size_px;
    size_t fh = ds->dims[nd - 2].array_size_px;
    if (nbytes < fw * fh * ds->bpp)
        return -1;
    ++ds->level_frame_count[0];

    /* current_frame = copy of the input (downsampler.cpp:314) */
    size_t cur_bytes = fw * fh * ds->bpp;
    uint8_t* cur = (uint8_t*)malloc(cur_bytes ? cur_bytes : 1);
    memcpy(cur, frame, cur_bytes);

    for (int level = 1; level < ds->n_levels; ++level) {
        const or_dim* prev = or_ds_level_dims(ds, level - 1);
        const or_dim* next = or_ds_level_dims(ds, level);
        const size_t pw = prev[nd - 1].array_size_px;
        const size_t ph = prev[nd - 2].array_size_px;
        const uint32_t prev_planes = prev[nd - 3].array_size_px;
        const size_t nw = next[nd - 1].array_size_px;
        const size_t nh = next[nd - 2].array_size_px;
        const uint32_t next_planes = next[nd - 3].array_size_px;
        if (pw != fw || ph != fh) {
            free(cur);
            return -2;
        }

        uint8_t* nxt;
        size_t nxt_bytes;
        if (nw < pw || nh < ph) {
            /* scale_fun_ (downsampler.cpp:341-343) */
            const size_t ow = (fw + fw % 2) / 2, oh = (fh + fh % 2) / 2;
            nxt_bytes = ow * oh * ds->bpp;
            nxt = (uint8_t*)malloc(nxt_bytes ? nxt_bytes : 1);
            or_scale_image(ds->dtype, ds->method, cur, fw, fh, nxt);
            fw = ow;
            fh = oh;
        } else {
            nxt_bytes = cur_bytes;
            nxt = (uint8_t*)malloc(nxt_bytes ? nxt_bytes : 1);
            memcpy(nxt, cur, nxt_bytes);
        }
        if (nw != fw || nh != fh) {
            free(nxt);
            free(cur);
            return -3;
        }

        /* downsampler.cpp:358-365 */
        int average_this_frame = next_planes < prev_planes;
        if (prev_planes % 2 != 0 &&
            ds->level_frame_count[level - 1] % prev_planes == 0)
            average_this_frame = 0;

        if (average_this_frame) {
            if (ds->partial[level]) {
                /* swap + average2_fun_(dst=earlier, src=new),
                 * downsampler.cpp:370-385 */
                uint8_t* earlier = ds->partial[level];
                ds->partial[level] = NULL;
                or_average_two_frames(ds->dtype, ds->method, earlier, nxt,
                                      nxt_bytes / ds->bpp);
                free(nxt);
                free(cur);
                cur = (uint8_t*)malloc(nxt_bytes ? nxt_bytes : 1);
                memcpy(cur, earlier, nxt_bytes);
                cur_bytes = nxt_bytes;
                emplace_downsampled(ds, level, earlier, nxt_bytes);
            } else {
                /* store partial and stop the cascade (:386-389) */
                ds->partial[level] = nxt;
                break;
            }
        } else {
            free(cur);
            cur = (uint8_t*)malloc(nxt_bytes ? nxt_bytes : 1);
            memcpy(cur, nxt, nxt_bytes);
            cur_bytes = nxt_bytes;
            emplace_downsampled(ds, level, nxt, nxt_bytes);
        }
    }
    free(cur);
    return 0;
}

int
or_ds_take_frame(or_downsampler* ds, int level, void* dst, size_t cap,
                 size_t* nbytes)
{
    /* downsampler.cpp:403-414 */
    if (level < 0 || level >= OR_MAX_LEVELS || !ds->downsampled[level])
        return 0;
    const size_t n = ds->downsampled_bytes[level];
    if (nbytes)
        *nbytes = n;
    if (dst)
        memcpy(dst, ds->downsampled[level], n < cap ? n : cap);
    free(ds->downsampled[level]);
    ds->downsampled[level] = NULL;
    return 1;
}

/* ------------------------------------------------------------------------
 * splitmix64 synthetic input stream
 * ---------------------------------------------------------------------- */
uint64_t
or_splitmix64(uint64_t* state)
{
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void
or_fill_splitmix(void* dst, size_t nbytes, uint64_t seed)
{
    uint64_t s = seed;
    uint8_t* p = (uint8_t*)dst;
    size_t i = 0;
    for (; i + 8 <= nbytes; i += 8) {
        const uint64_t v = or_splitmix64(&s);
        memcpy(p + i, &v, 8);
    }
    if (i < nbytes) {
        const uint64_t v = or_splitmix64(&s);
        memcpy(p + i, &v, nbytes - i);
    }
}
