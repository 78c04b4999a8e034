// aqz_kernels.hip -- CDNA4 (gfx950) kernels of the multiscale stage.
//
// fused_pyramid<T,M>: one workgroup (256 threads = 4 waves) per level-0
//   region of RH x RW pixels (RW = 512 bytes of row, RH = 16..64 rows).
//   Each thread streams two 16-byte row vectors per pass (coalesced: 32
//   lanes cover one 512-B row segment), stores them straight into the
//   level-0 chunk tiles (Array::write_frame_to_chunks_, array.cpp:507-622),
//   reduces them 2x2 in registers to level 1 (scale_image, downsampler.cpp:
//   139-206), stores level 1 into its tiles and into LDS; levels 2..F are then
//   cascaded inside LDS with the per-level rounding and edge replication of
//   the chained CPU path.  has_data (chunk.cpp:41-56) is a per-chunk flag set
//   from a wave ballot.  HBM traffic = read input once + write every level once.
//
// level_kernel<T,M>: the generic one-level step used for 2x2x2 pyramids
//   (z pairs, average_two_frames, downsampler.cpp:208-246, 358-389), for
//   levels beyond the fused depth, and for levels whose XY does not shrink.
#include <hip/hip_runtime.h>

#include "aqz_params.hh"
#include "aqz_reduce.hh"

#include <cstring>

namespace aqz {
namespace {

__device__ __forceinline__ uint32_t
fdiv(uint32_t n, const FastDiv& f)
{
    return (__umulhi(n, f.m) + n) >> f.s;
}

template<typename T>
__device__ __forceinline__ bool
nonzero_bits(T v)
{
    // the reference scans bytes (chunk.cpp:50-51): -0.0 counts as data
    if constexpr (sizeof(T) == 1) {
        uint8_t u;
        __builtin_memcpy(&u, &v, 1);
        return u != 0;
    } else if constexpr (sizeof(T) == 2) {
        uint16_t u;
        __builtin_memcpy(&u, &v, 2);
        return u != 0;
    } else if constexpr (sizeof(T) == 4) {
        uint32_t u;
        __builtin_memcpy(&u, &v, 4);
        return u != 0;
    } else {
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        return u != 0;
    }
}

template<int BYTES>
struct VecT;
template<>
struct VecT<16>
{
    using type = uint4;
};
template<>
struct VecT<8>
{
    using type = uint2;
};
template<>
struct VecT<4>
{
    using type = uint32_t;
};
template<>
struct VecT<2>
{
    using type = uint16_t;
};
template<>
struct VecT<1>
{
    using type = uint8_t;
};

template<typename T, int N>
__device__ __forceinline__ void
store_vec(uint8_t* p, const T* v)
{
    using V = typename VecT<N * sizeof(T)>::type;
    V raw;
    __builtin_memcpy(&raw, v, N * sizeof(T));
    *reinterpret_cast<V*>(p) = raw;
}

// Collects has_data per chunk for one thread; flushes with a wave-level
// de-duplication (most lanes of a wave hit the same chunk).
struct FlagAcc
{
    uint32_t* ptr = nullptr;
    bool nz = false;

    __device__ __forceinline__ void note(uint32_t* p, bool z)
    {
        if (p != ptr) {
            if (nz)
                *ptr = 1u;
            ptr = p;
            nz = z;
        } else {
            nz |= z;
        }
    }

    // call in converged control flow
    __device__ __forceinline__ void flush_wave()
    {
        const bool want = nz && ptr != nullptr;
        const unsigned long long m = __ballot(want);
        if (m != 0) {
            const int leader = __ffsll(static_cast<long long>(m)) - 1;
            const unsigned long long lp = __shfl(
              static_cast<unsigned long long>(reinterpret_cast<uintptr_t>(ptr)),
              leader);
            const bool same =
              !want || reinterpret_cast<uintptr_t>(ptr) == uintptr_t(lp);
            if (__all(same)) {
                if (want && int(threadIdx.x & 63) == leader)
                    *ptr = 1u;
            } else if (want) {
                *ptr = 1u;
            }
        }
        ptr = nullptr;
        nz = false;
    }
};

// Base of frame `f` (batch-relative) of a level inside the layer ring.
__device__ __forceinline__ void
frame_base(const LevelGeom& g, uint32_t f, uint8_t*& fb, uint32_t*& fl)
{
    const uint32_t q = g.fid0_mod + f;
    const uint32_t ld = q / g.frames_per_layer;
    const uint32_t fm = q - ld * g.frames_per_layer;
    const uint32_t slot = (g.slot0 + ld) % g.n_slots;
    fb = g.base + uint64_t(slot) * g.slot_bytes + g.tab_off[fm];
    fl = g.flags + uint64_t(slot) * g.n_chunks + g.tab_grp[fm];
}

// Store a run of N pixels of row Y starting at column X into the chunk tiles
// (nvalid <= N pixels are inside the level).
template<typename T, int N>
__device__ __forceinline__ void
put_tile(const LevelGeom& g,
         uint8_t* fb,
         uint32_t* fl,
         uint32_t Y,
         uint32_t X,
         const T* v,
         int nvalid,
         FlagAcc& acc)
{
    const uint32_t ty = fdiv(Y, g.dth);
    const uint32_t ry = Y - ty * g.th;
    const uint32_t tx = fdiv(X, g.dtw);
    const uint32_t rx = X - tx * g.tw;
    if (nvalid == N && rx + N <= g.tw && (g.tw % N) == 0) {
        bool nz = false;
#pragma unroll
        for (int i = 0; i < N; ++i)
            nz |= nonzero_bits(v[i]);
        const uint32_t chunk = ty * g.ntx + tx;
        store_vec<T, N>(fb + uint64_t(chunk) * g.bpc +
                          uint64_t(ry * g.tw + rx) * sizeof(T),
                        v);
        acc.note(fl + chunk, nz);
    } else {
        for (int i = 0; i < nvalid; ++i) {
            const uint32_t xi = X + i;
            const uint32_t txi = fdiv(xi, g.dtw);
            const uint32_t rxi = xi - txi * g.tw;
            const uint32_t chunk = ty * g.ntx + txi;
            *reinterpret_cast<T*>(fb + uint64_t(chunk) * g.bpc +
                                  uint64_t(ry * g.tw + rxi) * sizeof(T)) =
              v[i];
            acc.note(fl + chunk, nonzero_bits(v[i]));
        }
    }
}

// One cascaded level K (2..6) inside LDS: prev (pitch RW >> (K-1)) -> cur.
template<typename T, int M, int K, uint32_t RW>
__device__ __forceinline__ void
deep_level(const FusedParams& p,
           uint32_t f,
           uint32_t y0,
           uint32_t x0,
           const T* prev,
           T* cur)
{
    const LevelGeom& g = p.lv[K];
    const LevelGeom& gp = p.lv[K - 1];
    constexpr uint32_t lw = RW >> K;
    constexpr uint32_t pw = RW >> (K - 1);
    const uint32_t lh = (1u << p.rh_log2) >> K;
    const uint32_t yk0 = y0 >> K, xk0 = x0 >> K;
    const uint32_t yp0 = y0 >> (K - 1), xp0 = x0 >> (K - 1);
    // last valid local row/col of the previous level inside this region
    const uint32_t pxmax = gp.W - 1 - xp0;
    const uint32_t pymax = gp.H - 1 - yp0;
    uint8_t* fb = nullptr;
    uint32_t* fl = nullptr;
    if (g.base)
        frame_base(g, f, fb, fl);
    T* scr = g.scratch ? reinterpret_cast<T*>(g.scratch) + uint64_t(f) * g.W * g.H
                       : nullptr;
    FlagAcc acc;
    for (uint32_t idx = threadIdx.x; idx < lh * lw; idx += 256) {
        const uint32_t ly = idx / lw, lx = idx % lw;
        const uint32_t Y = yk0 + ly, X = xk0 + lx;
        if (Y < g.H && X < g.W) {
            const uint32_t py = 2 * ly, px = 2 * lx;
            const uint32_t px1 = min(px + 1, pxmax);
            const uint32_t py1 = min(py + 1, pymax);
            const T v = reduce4<M, T>(prev[py * pw + px],
                                      prev[py * pw + px1],
                                      prev[py1 * pw + px],
                                      prev[py1 * pw + px1]);
            cur[ly * lw + lx] = v;
            if (fb)
                put_tile<T, 1>(g, fb, fl, Y, X, &v, 1, acc);
            if (scr)
                scr[uint64_t(Y) * g.W + X] = v;
        }
    }
    acc.flush_wave();
}

template<typename T, int M>
__global__ __launch_bounds__(256) void
fused_pyramid(const FusedParams p)
{
    constexpr int VEC = 16 / sizeof(T); // pixels per 16-B row vector
    constexpr int HV = VEC / 2;         // level-1 pixels per vector pair
    constexpr uint32_t RW = 32 * VEC;   // region width (512 B of row)
    // level-1 region (<= 32 rows) and level-2 region (<= 16 rows)
    __shared__ __attribute__((aligned(16))) T lds_a[32 * (RW / 2)];
    __shared__ __attribute__((aligned(16))) T lds_b[16 * (RW / 4)];

    const uint32_t tid = threadIdx.x;
    const uint32_t rp = tid >> 5; // row pair within a 16-row pass
    const uint32_t cv = tid & 31; // 16-B column vector
    const uint32_t nreg = p.nbx * p.nby;
    const uint32_t f = blockIdx.x / nreg;
    const uint32_t r = blockIdx.x - f * nreg;
    const uint32_t by = r / p.nbx;
    const uint32_t bx = r - by * p.nbx;
    const uint32_t y0 = by << p.rh_log2;
    const uint32_t x0 = bx * RW;
    const uint32_t npass = 1u << (p.rh_log2 - 4);

    const LevelGeom& g0 = p.lv[0];
    const LevelGeom& g1 = p.lv[1];
    const uint32_t W0 = g0.W, H0 = g0.H;
    const T* src = reinterpret_cast<const T*>(p.src + uint64_t(f) * p.src_stride);

    uint8_t *fb0 = nullptr, *fb1 = nullptr;
    uint32_t *fl0 = nullptr, *fl1 = nullptr;
    if (g0.base)
        frame_base(g0, f, fb0, fl0);
    const bool l1 = p.n_fused >= 1;
    if (l1 && g1.base)
        frame_base(g1, f, fb1, fl1);
    T* scr1 = (l1 && g1.scratch)
                ? reinterpret_cast<T*>(g1.scratch) + uint64_t(f) * g1.W * g1.H
                : nullptr;
    const bool keep_l1 = p.n_fused >= 2;

    FlagAcc acc0, acc1;
    for (uint32_t pass = 0; pass < npass; ++pass) {
        const uint32_t y = y0 + pass * 16 + 2 * rp;
        const uint32_t x = x0 + cv * VEC;
        if (y < H0 && x < W0) {
            const uint32_t ya = min(y + 1, H0 - 1); // bottom edge replicate
            T r0[VEC], r1[VEC];
            const int nv0 = int(min(uint32_t(VEC), W0 - x));
            if (p.vec_rows && nv0 == VEC) {
                const uint4 a = *reinterpret_cast<const uint4*>(
                  src + uint64_t(y) * W0 + x);
                const uint4 b = *reinterpret_cast<const uint4*>(
                  src + uint64_t(ya) * W0 + x);
                __builtin_memcpy(r0, &a, 16);
                __builtin_memcpy(r1, &b, 16);
            } else {
#pragma unroll
                for (int i = 0; i < VEC; ++i) {
                    // right edge replicate: clamp the column
                    const uint32_t xi = min(x + uint32_t(i), W0 - 1);
                    r0[i] = src[uint64_t(y) * W0 + xi];
                    r1[i] = src[uint64_t(ya) * W0 + xi];
                }
            }
            if (fb0) {
                put_tile<T, VEC>(g0, fb0, fl0, y, x, r0, nv0, acc0);
                if (y + 1 < H0)
                    put_tile<T, VEC>(g0, fb0, fl0, y + 1, x, r1, nv0, acc0);
            }
            if (l1) {
                T o[HV];
#pragma unroll
                for (int i = 0; i < HV; ++i)
                    o[i] = reduce4<M, T>(
                      r0[2 * i], r0[2 * i + 1], r1[2 * i], r1[2 * i + 1]);
                const uint32_t Y = y >> 1, X = x >> 1;
                const int nv1 = int(min(uint32_t(HV), g1.W - X));
                if (fb1)
                    put_tile<T, HV>(g1, fb1, fl1, Y, X, o, nv1, acc1);
                if (scr1)
                    for (int i = 0; i < nv1; ++i)
                        scr1[uint64_t(Y) * g1.W + X + i] = o[i];
                if (keep_l1) {
#pragma unroll
                    for (int i = 0; i < HV; ++i)
                        lds_a[(pass * 8 + rp) * (RW / 2) + cv * HV + i] = o[i];
                }
            }
        }
    }
    acc0.flush_wave();
    acc1.flush_wave();

    // cascaded levels 2..n_fused inside LDS (ping-pong A -> B -> A ...)
    if (p.n_fused >= 2) {
        __syncthreads();
        deep_level<T, M, 2, RW>(p, f, y0, x0, lds_a, lds_b);
    }
    if (p.n_fused >= 3) {
        __syncthreads();
        deep_level<T, M, 3, RW>(p, f, y0, x0, lds_b, lds_a);
    }
    if (p.n_fused >= 4) {
        __syncthreads();
        deep_level<T, M, 4, RW>(p, f, y0, x0, lds_a, lds_b);
    }
    if (p.n_fused >= 5) {
        __syncthreads();
        deep_level<T, M, 5, RW>(p, f, y0, x0, lds_b, lds_a);
    }
    if (p.n_fused >= 6) {
        __syncthreads();
        deep_level<T, M, 6, RW>(p, f, y0, x0, lds_a, lds_b);
    }
}

// ---------------------------------------------------------------------------
// Generic one-level step.  grid = (ceil(W*H/256), n_ops); one output pixel
// per thread.
// ---------------------------------------------------------------------------
template<int M, typename T>
__device__ __forceinline__ T
fetch(const T* s, bool scale, uint32_t Y, uint32_t X, uint32_t W, uint32_t Wp,
      uint32_t Hp)
{
    if (!scale)
        return s[uint64_t(Y) * W + X];
    const uint32_t py = 2 * Y, px = 2 * X;
    const uint32_t px1 = min(px + 1, Wp - 1), py1 = min(py + 1, Hp - 1);
    return reduce4<M, T>(s[uint64_t(py) * Wp + px],
                         s[uint64_t(py) * Wp + px1],
                         s[uint64_t(py1) * Wp + px],
                         s[uint64_t(py1) * Wp + px1]);
}

template<typename T, int M>
__global__ __launch_bounds__(256) void
level_kernel(const LevelParams p)
{
    const LevelOp op = p.ops[blockIdx.y];
    const LevelGeom& g = p.g;
    const uint64_t npx = uint64_t(g.W) * g.H;
    const uint64_t idx = uint64_t(blockIdx.x) * 256 + threadIdx.x;
    FlagAcc acc;
    if (idx < npx) {
        const uint32_t Y = uint32_t(idx / g.W);
        const uint32_t X = uint32_t(idx - uint64_t(Y) * g.W);
        T v = fetch<M, T>(reinterpret_cast<const T*>(op.a), op.a_scale != 0, Y,
                          X, g.W, p.Wp, p.Hp);
        if (op.b) {
            const T vb = fetch<M, T>(reinterpret_cast<const T*>(op.b),
                                     op.b_scale != 0, Y, X, g.W, p.Wp, p.Hp);
            v = reduce2<M, T>(v, vb);
        }
        if (op.scratch_out)
            reinterpret_cast<T*>(op.scratch_out)[idx] = v;
        if (op.has_tile)
            put_tile<T, 1>(g, g.base + op.tile_off, g.flags + op.flag_off, Y,
                           X, &v, 1, acc);
    }
    acc.flush_wave();
}

// Zero-fill whole frames of a chunk layer (final partial layer flush).
__global__ void
zero_frame_tiles(uint8_t* fb, uint64_t bpc, uint32_t n_tiles,
                 uint32_t tile_bytes)
{
    const uint32_t t = blockIdx.y;
    if (t >= n_tiles)
        return;
    uint8_t* p = fb + uint64_t(t) * bpc;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < tile_bytes;
         i += gridDim.x * 256)
        p[i] = 0;
}

} // namespace

// ---------------------------------------------------------------------------
// Host launchers: dtype x method dispatch.
// ---------------------------------------------------------------------------

#define AQZ_DISPATCH(DT, M, CALL)                                              \
    switch (DT) {                                                              \
        case 0: AQZ_DISPATCH_M(uint8_t, M, CALL); break;                       \
        case 1: AQZ_DISPATCH_M(uint16_t, M, CALL); break;                      \
        case 2: AQZ_DISPATCH_M(uint32_t, M, CALL); break;                      \
        case 3: AQZ_DISPATCH_M(uint64_t, M, CALL); break;                      \
        case 4: AQZ_DISPATCH_M(int8_t, M, CALL); break;                        \
        case 5: AQZ_DISPATCH_M(int16_t, M, CALL); break;                       \
        case 6: AQZ_DISPATCH_M(int32_t, M, CALL); break;                       \
        case 7: AQZ_DISPATCH_M(int64_t, M, CALL); break;                       \
        case 8: AQZ_DISPATCH_M(float, M, CALL); break;                         \
        case 9: AQZ_DISPATCH_M(double, M, CALL); break;                        \
        default: return hipErrorInvalidValue;                                  \
    }

#define AQZ_DISPATCH_M(T, M, CALL)                                             \
    switch (M) {                                                               \
        case 0: CALL(T, 0); break;                                             \
        case 1: CALL(T, 1); break;                                             \
        case 2: CALL(T, 2); break;                                             \
        case 3: CALL(T, 3); break;                                             \
        default: return hipErrorInvalidValue;                                  \
    }

hipError_t
launch_fused_pyramid(int dtype, int method, const FusedParams& p,
                     hipStream_t stream)
{
    const uint64_t blocks = uint64_t(p.n_frames) * p.nbx * p.nby;
    if (blocks == 0)
        return hipSuccess;
    if (blocks > 0x7fffffffull || p.n_fused > uint32_t(kMaxFused) ||
        p.rh_log2 < 4 || p.rh_log2 > 6)
        return hipErrorInvalidValue;
#define CALL(T, MM)                                                            \
    hipLaunchKernelGGL((fused_pyramid<T, MM>), dim3(uint32_t(blocks)),         \
                       dim3(256), 0, stream, p)
    AQZ_DISPATCH(dtype, method, CALL)
#undef CALL
    return hipGetLastError();
}

hipError_t
launch_level(int dtype, int method, const LevelParams& p, hipStream_t stream)
{
    const uint64_t npx = uint64_t(p.g.W) * p.g.H;
    if (p.n_ops == 0 || npx == 0)
        return hipSuccess;
    const uint64_t bx = (npx + 255) / 256;
    if (bx > 0x7fffffffull || p.n_ops > 65535)
        return hipErrorInvalidValue;
#define CALL(T, MM)                                                            \
    hipLaunchKernelGGL((level_kernel<T, MM>), dim3(uint32_t(bx), p.n_ops),    \
                       dim3(256), 0, stream, p)
    AQZ_DISPATCH(dtype, method, CALL)
#undef CALL
    return hipGetLastError();
}

hipError_t
launch_zero_frame_tiles(uint8_t* fb, uint64_t bpc, uint32_t n_tiles,
                        uint32_t tile_bytes, hipStream_t stream)
{
    if (n_tiles == 0 || tile_bytes == 0)
        return hipSuccess;
    const uint32_t gx = min((tile_bytes + 255) / 256, 64u);
    hipLaunchKernelGGL(zero_frame_tiles, dim3(gx, n_tiles), dim3(256), 0,
                       stream, fb, bpc, n_tiles, tile_bytes);
    return hipGetLastError();
}

const char*
fused_kernel_symbol_hint()
{
    return "fused_pyramid";
}

} // namespace aqz
