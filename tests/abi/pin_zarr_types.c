/* Compiled by tests/test_abi_pin_cpu.py against the reference's public C
 * headers (/root/reference/include): the compiler proves that the numeric
 * values aqz_gpu.h hands across the boundary are the reference's enum
 * values, and that the public structs a drop-in must leave unchanged keep
 * the layout SURVEY.md 8(b) measured (x86-64). */
#include "acquire.zarr.h"
#include "zarr.types.h"

#include "aqz_gpu.h"
#include "aqz_gpu_bench.h"

#include <stddef.h>

#define SAME(a, b) _Static_assert((int)(a) == (int)(b), #a " != " #b)

/* ZarrStatusCode (zarr.types.h:13-31) */
SAME(AQZ_STATUS_SUCCESS, ZarrStatusCode_Success);
SAME(AQZ_STATUS_INVALID_ARGUMENT, ZarrStatusCode_InvalidArgument);
SAME(AQZ_STATUS_OVERFLOW, ZarrStatusCode_Overflow);
SAME(AQZ_STATUS_INVALID_INDEX, ZarrStatusCode_InvalidIndex);
SAME(AQZ_STATUS_NOT_YET_IMPLEMENTED, ZarrStatusCode_NotYetImplemented);
SAME(AQZ_STATUS_INTERNAL_ERROR, ZarrStatusCode_InternalError);
SAME(AQZ_STATUS_OUT_OF_MEMORY, ZarrStatusCode_OutOfMemory);
SAME(AQZ_STATUS_INVALID_SETTINGS, ZarrStatusCode_InvalidSettings);
SAME(AQZ_STATUS_WRITE_OUT_OF_BOUNDS, ZarrStatusCode_WriteOutOfBounds);

/* ZarrDataType (zarr.types.h:49-62) */
SAME(AQZ_DTYPE_UINT8, ZarrDataType_uint8);
SAME(AQZ_DTYPE_UINT16, ZarrDataType_uint16);
SAME(AQZ_DTYPE_UINT32, ZarrDataType_uint32);
SAME(AQZ_DTYPE_UINT64, ZarrDataType_uint64);
SAME(AQZ_DTYPE_INT8, ZarrDataType_int8);
SAME(AQZ_DTYPE_INT16, ZarrDataType_int16);
SAME(AQZ_DTYPE_INT32, ZarrDataType_int32);
SAME(AQZ_DTYPE_INT64, ZarrDataType_int64);
SAME(AQZ_DTYPE_FLOAT32, ZarrDataType_float32);
SAME(AQZ_DTYPE_FLOAT64, ZarrDataType_float64);
SAME(AQZ_DTYPE_COUNT, ZarrDataTypeCount);

/* ZarrDimensionType (zarr.types.h:81-88) */
SAME(AQZ_DIM_SPACE, ZarrDimensionType_Space);
SAME(AQZ_DIM_CHANNEL, ZarrDimensionType_Channel);
SAME(AQZ_DIM_TIME, ZarrDimensionType_Time);
SAME(AQZ_DIM_OTHER, ZarrDimensionType_Other);

/* ZarrDownsamplingMethod (zarr.types.h:90-97) */
SAME(AQZ_METHOD_DECIMATE, ZarrDownsamplingMethod_Decimate);
SAME(AQZ_METHOD_MEAN, ZarrDownsamplingMethod_Mean);
SAME(AQZ_METHOD_MIN, ZarrDownsamplingMethod_Min);
SAME(AQZ_METHOD_MAX, ZarrDownsamplingMethod_Max);
SAME(AQZ_METHOD_COUNT, ZarrDownsamplingMethodCount);

/* ZarrCompressionCodec (zarr.types.h:72-79) */
SAME(AQZ_CODEC_NONE, ZarrCompressionCodec_None);
SAME(AQZ_CODEC_BLOSC_LZ4, ZarrCompressionCodec_BloscLZ4);
SAME(AQZ_CODEC_BLOSC_ZSTD, ZarrCompressionCodec_BloscZstd);
SAME(AQZ_CODEC_ZSTD, ZarrCompressionCodec_Zstd);

/* The public structs stay as they are. */
_Static_assert(sizeof(ZarrStreamSettings) == 56, "ZarrStreamSettings size");
_Static_assert(offsetof(ZarrStreamSettings, arrays) == 32, "ZarrStreamSettings.arrays");
_Static_assert(sizeof(ZarrArraySettings) == 56, "ZarrArraySettings size");
_Static_assert(offsetof(ZarrArraySettings, data_type) == 32, "data_type");
_Static_assert(offsetof(ZarrArraySettings, multiscale) == 36, "multiscale");
_Static_assert(offsetof(ZarrArraySettings, downsampling_method) == 40, "downsampling_method");
_Static_assert(offsetof(ZarrArraySettings, max_levels) == 44, "max_levels");
_Static_assert(offsetof(ZarrArraySettings, storage_dimension_order) == 48,
               "storage_dimension_order");
_Static_assert(sizeof(ZarrDimensionProperties) == 40, "ZarrDimensionProperties size");
_Static_assert(offsetof(ZarrDimensionProperties, array_size_px) == 12, "array_size_px");
_Static_assert(offsetof(ZarrDimensionProperties, chunk_size_px) == 16, "chunk_size_px");
_Static_assert(offsetof(ZarrDimensionProperties, shard_size_chunks) == 20,
               "shard_size_chunks");
_Static_assert(offsetof(ZarrDimensionProperties, scale) == 32, "scale");

/* aqz_dimension is the pixel-geometry subset of ZarrDimensionProperties:
 * the same field types, so a copy is a field-by-field assignment. */
_Static_assert(sizeof(((aqz_dimension*)0)->type) == sizeof(ZarrDimensionType), "type width");
_Static_assert(sizeof(((aqz_dimension*)0)->array_size_px) ==
                 sizeof(((ZarrDimensionProperties*)0)->array_size_px), "array_size_px width");
_Static_assert(sizeof(((aqz_dimension*)0)->chunk_size_px) ==
                 sizeof(((ZarrDimensionProperties*)0)->chunk_size_px), "chunk_size_px width");
_Static_assert(sizeof(((aqz_dimension*)0)->shard_size_chunks) ==
                 sizeof(((ZarrDimensionProperties*)0)->shard_size_chunks), "shard width");

/* Building an aqz_array_desc from a ZarrArraySettings, as the integration
 * does, type-checks without casts beyond enum ->
 * int32_t. */
int
aqz_pin_fill_desc(const ZarrArraySettings* s, aqz_dimension* dims, aqz_array_desc* d)
{
    for (size_t i = 0; i < s->dimension_count; ++i) {
        dims[i].type = s->dimensions[i].type;
        dims[i].array_size_px = s->dimensions[i].array_size_px;
        dims[i].chunk_size_px = s->dimensions[i].chunk_size_px;
        dims[i].shard_size_chunks = s->dimensions[i].shard_size_chunks;
    }
    d->dimensions = dims;
    d->dimension_count = s->dimension_count;
    d->data_type = s->data_type;
    d->multiscale = s->multiscale;
    d->downsampling_method = s->downsampling_method;
    d->max_levels = s->max_levels;
    d->storage_dimension_order = s->storage_dimension_order;
    d->device = 0;
    return 0;
}
