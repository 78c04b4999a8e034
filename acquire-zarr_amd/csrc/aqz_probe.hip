// aqz_probe.hip -- practical HBM rates of this device for the stage's access
// shapes (include/aqz_gpu_bench.h aqz_probe_hbm).  Measurement only: the
// bench reports the stage's rates next to these ceilings, measured in the
// same process on the same device.
#include "aqz_engine.hh"
#include "aqz_gpu_bench.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// U 16-B vectors per lane, loaded before any is used (the stage's kernels
// keep 128 B per lane in flight); U divisible by 3 for the 1/3 shapes.
// AQZ_PROBE_DEEP: 12 (192 B per lane, 48 KiB per workgroup).
constexpr int kU = 6;
constexpr int kUDeep = 12;

template<int MODE, bool NTS>
__device__ __forceinline__ void
put(u32x4* p, u32x4 v)
{
    if constexpr (NTS)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

template<int MODE, bool NTS, int kU = kU>
__global__ __launch_bounds__(256) void
probe_stream(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
             u32x4* __restrict__ dst3, uint32_t* __restrict__ sink)
{
    const uint64_t base = uint64_t(blockIdx.x) * (kU * 256) + threadIdx.x;
    u32x4 v[kU];
#pragma unroll
    for (int i = 0; i < kU; ++i)
        v[i] = __builtin_nontemporal_load(src + base + i * 256);
    if constexpr (MODE == AQZ_PROBE_READ) {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < kU; ++i)
            acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        if (acc == 0x9e3779b9u) // never: keeps the loads alive
            sink[0] = acc;
        return;
    }
    if constexpr (MODE == AQZ_PROBE_COPY || MODE == AQZ_PROBE_COPY_THIRD) {
#pragma unroll
        for (int i = 0; i < kU; ++i)
            put<MODE, NTS>(dst + base + i * 256, v[i]);
    }
    if constexpr (MODE == AQZ_PROBE_COPY_THIRD || MODE == AQZ_PROBE_READ_THIRD) {
        const uint64_t b3 = uint64_t(blockIdx.x) * (kU * 256 / 3) + threadIdx.x;
#pragma unroll
        for (int i = 0; i < kU / 3; ++i)
            put<MODE, NTS>(dst3 + b3 + i * 256, v[3 * i] ^ v[3 * i + 1] ^ v[3 * i + 2]);
    }
}

struct DevMem
{
    void* p = nullptr;
    aqz::DevBuf pieces; // AQZ_PROBE_PIECES
    ~DevMem()
    {
        if (p && !pieces.p)
            (void)hipFree(p);
    }
};

// hipMalloc, or (pieces) 2 MiB virtual-memory pieces as the stage's rings
hipError_t
probe_alloc(DevMem& m, size_t bytes, bool pieces)
{
    if (!pieces)
        return hipMalloc(&m.p, bytes);
    try {
        m.pieces.alloc(bytes, aqz::DevBuf::kVmm | (5u << 9));
    } catch (...) {
        return hipErrorOutOfMemory;
    }
    m.p = m.pieces.p;
    return hipSuccess;
}

} // namespace

namespace aqz {

uint64_t
probe_copy_third_read_bytes(uint64_t src_bytes, uint64_t dst_bytes)
{
    constexpr uint64_t wg = uint64_t(kUDeep) * 256 * 16; // a multiple of both
    if (dst_bytes < 2 * wg)
        return 0;
    const uint64_t r = std::min<uint64_t>(src_bytes, (dst_bytes - wg) / 4 * 3);
    return std::min<uint64_t>(r / wg, 0x7fffffffull) * wg;
}

// The stage's own bus shape (1 read : 4/3 write) from src into dst: dst
// receives the copy and behind it the third.  variant 0: nontemporal
// stores, 96 B per lane in flight; 1: the same with 192 B; 2: plain stores.
// third_only: the pyramid-only shape (1 read : 1/3 write, a stage without
// the level-0 split), the third at dst.  The placement search
// (Stage::calibrate_placement) takes the best of them over its random frames
// and the candidate's rings: the practical ceiling of the stage's shape in
// that memory, at the stage's launch size.
hipError_t
launch_probe_copy_third(const uint8_t* src, uint8_t* dst, uint64_t read_bytes,
                        hipStream_t stream, int variant, bool third_only)
{
    const uint64_t per_wg = uint64_t(variant == 1 ? kUDeep : kU) * 256 * 16;
    const uint64_t grid = read_bytes / per_wg;
    if (grid == 0 || grid > 0x7fffffffull || read_bytes % per_wg)
        return hipErrorInvalidValue;
    const auto* in = reinterpret_cast<const u32x4*>(src);
    auto* o = reinterpret_cast<u32x4*>(dst);
    auto* o3 = reinterpret_cast<u32x4*>(third_only ? dst : dst + read_bytes);
    const dim3 g{ uint32_t(grid), 1, 1 };
    if (third_only) {
        if (variant == 1)
            hipLaunchKernelGGL((probe_stream<AQZ_PROBE_READ_THIRD, true, kUDeep>), g, dim3(256),
                               0, stream, in, o, o3, nullptr);
        else if (variant == 2)
            hipLaunchKernelGGL((probe_stream<AQZ_PROBE_READ_THIRD, false>), g, dim3(256), 0,
                               stream, in, o, o3, nullptr);
        else
            hipLaunchKernelGGL((probe_stream<AQZ_PROBE_READ_THIRD, true>), g, dim3(256), 0,
                               stream, in, o, o3, nullptr);
    } else if (variant == 1)
        hipLaunchKernelGGL((probe_stream<AQZ_PROBE_COPY_THIRD, true, kUDeep>), g, dim3(256), 0,
                           stream, in, o, o3, nullptr);
    else if (variant == 2)
        hipLaunchKernelGGL((probe_stream<AQZ_PROBE_COPY_THIRD, false>), g, dim3(256), 0,
                           stream, in, o, o3, nullptr);
    else
        hipLaunchKernelGGL((probe_stream<AQZ_PROBE_COPY_THIRD, true>), g, dim3(256), 0,
                           stream, in, o, o3, nullptr);
    return hipGetLastError();
}

} // namespace aqz

extern "C" aqz_status
aqz_probe_hbm(int32_t device, int32_t shape, uint64_t bytes, uint32_t reps, double* ms,
              uint64_t* read_bytes)
{
    const int32_t kind = shape & 0xff;
    const bool plain = (shape & AQZ_PROBE_PLAIN_STORES) != 0;
    const bool pieces = (shape & AQZ_PROBE_PIECES) != 0;
    const bool deep = (shape & AQZ_PROBE_DEEP) != 0;
    if (!ms || kind < AQZ_PROBE_READ || kind > AQZ_PROBE_READ_THIRD || reps == 0 ||
        (shape & ~(0xff | AQZ_PROBE_PLAIN_STORES | AQZ_PROBE_PIECES | AQZ_PROBE_DEEP)) != 0)
        return AQZ_STATUS_INVALID_ARGUMENT;
    const uint64_t per_wg = uint64_t(deep ? kUDeep : kU) * 256 * 16;
    const uint64_t grid = bytes / per_wg;
    if (grid == 0 || grid > 0x7fffffffull)
        return AQZ_STATUS_INVALID_ARGUMENT;
    const uint64_t rd = grid * per_wg;
    constexpr int kRing = 4; // the source ring, well past the 256 MiB MALL
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
        return AQZ_STATUS_INVALID_ARGUMENT;
    aqz_status st = AQZ_STATUS_SUCCESS;
    {
        DevMem src, dst, dst3, sink;
        hipStream_t s = nullptr;
        hipEvent_t a = nullptr, b = nullptr;
        auto ok = [&](hipError_t e) {
            if (e != hipSuccess && st == AQZ_STATUS_SUCCESS)
                st = e == hipErrorOutOfMemory ? AQZ_STATUS_OUT_OF_MEMORY
                                              : AQZ_STATUS_INTERNAL_ERROR;
            return e == hipSuccess;
        };
        if (ok(probe_alloc(src, rd * kRing, pieces)) && ok(probe_alloc(dst, rd, pieces)) &&
            ok(probe_alloc(dst3, rd / 3 + per_wg, pieces)) && ok(hipMalloc(&sink.p, 64)) &&
            ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) &&
            ok(hipEventCreate(&a)) && ok(hipEventCreate(&b)) &&
            ok(hipMemsetAsync(src.p, 1, rd * kRing, s))) {
            auto launch = [&](uint32_t r) {
                const auto* in = static_cast<const u32x4*>(src.p) + (r % kRing) * (rd / 16);
                auto* o = static_cast<u32x4*>(dst.p);
                auto* o3 = static_cast<u32x4*>(dst3.p);
                auto* k = static_cast<uint32_t*>(sink.p);
                const dim3 g{ uint32_t(grid), 1, 1 };
#define PROBE_LAUNCH(MODE)                                                     \
    if (plain && deep)                                                         \
        hipLaunchKernelGGL((probe_stream<MODE, false, kUDeep>), g, dim3(256), 0, s, in, o, \
                           o3, k);                                             \
    else if (deep)                                                             \
        hipLaunchKernelGGL((probe_stream<MODE, true, kUDeep>), g, dim3(256), 0, s, in, o, \
                           o3, k);                                             \
    else if (plain)                                                            \
        hipLaunchKernelGGL((probe_stream<MODE, false>), g, dim3(256), 0, s, in, o, o3, k); \
    else                                                                       \
        hipLaunchKernelGGL((probe_stream<MODE, true>), g, dim3(256), 0, s, in, o, o3, k)
                switch (kind) {
                    case AQZ_PROBE_READ: PROBE_LAUNCH(AQZ_PROBE_READ); break;
                    case AQZ_PROBE_COPY: PROBE_LAUNCH(AQZ_PROBE_COPY); break;
                    case AQZ_PROBE_COPY_THIRD: PROBE_LAUNCH(AQZ_PROBE_COPY_THIRD); break;
                    default: PROBE_LAUNCH(AQZ_PROBE_READ_THIRD);
                }
#undef PROBE_LAUNCH
            };
            for (uint32_t r = 0; r < 3; ++r)
                launch(r);
            float t = 0;
            if (ok(hipGetLastError()) && ok(hipEventRecord(a, s))) {
                for (uint32_t r = 0; r < reps; ++r)
                    launch(r);
                if (ok(hipEventRecord(b, s)) && ok(hipEventSynchronize(b)) &&
                    ok(hipEventElapsedTime(&t, a, b))) {
                    *ms = double(t) / reps;
                    if (read_bytes)
                        *read_bytes = rd;
                }
            }
        }
        if (s)
            (void)hipStreamSynchronize(s);
        if (a)
            (void)hipEventDestroy(a);
        if (b)
            (void)hipEventDestroy(b);
        if (s)
            (void)hipStreamDestroy(s);
    }
    (void)hipSetDevice(prev);
    return st;
}
