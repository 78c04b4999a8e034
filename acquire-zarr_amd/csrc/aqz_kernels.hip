// aqz_kernels.hip -- CDNA4 (gfx950) kernels of the multiscale stage.
//
// fused_pyramid<T,M> (interior regions) / fused_pyramid_edge<T,M> (edges):
//   a region is RH rows x 512 bytes of row of one level-0 frame.  256 threads
//   (4 waves); every thread streams two 16-byte row vectors per 16-row pass
//   (32 lanes cover one 512-B row segment: fully coalesced), stores them
//   straight into the level-0 chunk tiles (Array::write_frame_to_chunks_,
//   array.cpp:507-622), reduces them 2x2 in registers to level 1
//   (scale_image, downsampler.cpp:139-206), meets the row below through a
//   cross-lane swap for level 2, and cascades levels 3..F inside LDS with the
//   per-level rounding and edge replication of the chained CPU path.
//   has_data (chunk.cpp:41-56) is one word per chunk, set after a wave
//   ballot.  HBM traffic = read the input once + write every level once.
//   The interior kernel is persistent (grid = resident workgroups) and
//   prefetches the next pass's rows while it stores the current one.
//
// level_kernel<T,M>: the generic one-level step used for 2x2x2 pyramids
//   (z pairs, average_two_frames, downsampler.cpp:208-246, 358-389), for
//   levels deeper than the fused cascade, and for levels whose XY does not
//   shrink.
#include <hip/hip_runtime.h>

#include <type_traits>

#include "aqz_params.hh"
#include "aqz_reduce.hh"

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

// Stores / loads through global (address space 1) pointers: the tile
// pointers come out of the FrameRef tables, so without the cast the
// compiler can only prove a generic pointer and emits flat_* instructions.
// NT selects the nontemporal form at compile time (a runtime branch between
// a plain and a nontemporal access of the same address folds into one plain
// access and loses the hint).
template<typename V>
using gptr = __attribute__((address_space(1))) V*;

template<bool NT, typename V>
__device__ __forceinline__ void
gstore(uint8_t* p, V v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, (gptr<V>)(p));
    else
        *(gptr<V>)(p) = v;
}

template<bool NT, typename V>
__device__ __forceinline__ V
gload(const uint8_t* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load((const gptr<V>)(p));
    else
        return *(const gptr<V>)(p);
}

// N pixels as one store of N * sizeof(T) bytes
template<typename T, int N, bool NT>
__device__ __forceinline__ void
gstore_px(uint8_t* p, const T* v)
{
    typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    constexpr int B = N * int(sizeof(T));
    if constexpr (B == 16) {
        u32x4v w;
        __builtin_memcpy(&w, v, 16);
        gstore<NT>(p, w);
    } else if constexpr (B == 8) {
        u32x2v w;
        __builtin_memcpy(&w, v, 8);
        gstore<NT>(p, w);
    } else {
        using V = typename VecT<B>::type;
        V w;
        __builtin_memcpy(&w, v, B);
        gstore<NT>(p, w);
    }
}

template<typename T, int N, bool NT = false>
__device__ __forceinline__ void
store_vec(uint8_t* p, const T* v)
{
    gstore_px<T, N, NT>(p, v);
}

template<typename T, int N>
__device__ __forceinline__ bool
any_nonzero(const T* v)
{
    bool nz = false;
#pragma unroll
    for (int i = 0; i < N; ++i)
        nz |= nonzero_bits(v[i]);
    return nz;
}

// Collects has_data per chunk for one thread; flushes with a wave-level
// de-duplication (most lanes of a wave hit the same chunk).
struct FlagAcc
{
    uint32_t* ptr = nullptr;
    bool nz = false;
    uint32_t tag = 1;

    __device__ __forceinline__ void note(uint32_t* p, bool z)
    {
        if (p != ptr) {
            if (nz)
                *ptr = tag;
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
                    *ptr = tag;
            } else if (want) {
                *ptr = tag;
            }
        }
        ptr = nullptr;
        nz = false;
    }
};

// chunk tiling of one level
struct Tiles
{
    uint32_t tw, th, ntx;
    FastDiv dtw, dth;
    uint64_t bpc;
};

__device__ __forceinline__ Tiles
tiles_of(const FusedParams& p, int k)
{
    return Tiles{ p.tw, p.th, p.ntx[k], p.dtw, p.dth, p.bpc };
}

__device__ __forceinline__ Tiles
tiles_of(const LevelGeom& g)
{
    return Tiles{ g.tw, g.th, g.ntx, g.dtw, g.dth, g.bpc };
}

// Where frame f (batch-relative) of level k lands, and its has_data tag.
struct Ref
{
    uint8_t* tiles;
    uint32_t* flags;
    uint32_t tag;
};

__device__ __forceinline__ Ref
frame_ref(const FusedParams& p, int k, uint32_t f)
{
    const LevelRefs& l = p.lr[k];
    if (!l.table)
        return Ref{ nullptr, nullptr, 0 };
    uint32_t q = l.r0 + f; // < 2 * period: a launch spans at most one wrap
    uint32_t tag = l.tag0;
    if (q >= l.period) {
        q -= l.period;
        ++tag;
    }
    const FrameRef r = l.table[q];
    return Ref{ r.tiles, r.flags, tag };
}

// Store a run of N pixels of row Y starting at column X into the chunk tiles
// of one frame (nvalid <= N pixels are inside the level).
template<typename T, int N>
__device__ __forceinline__ void
put_tile(const Tiles& g, uint8_t* fb, uint32_t* fl, uint32_t Y, uint32_t X,
         const T* v, int nvalid, FlagAcc& acc)
{
    const uint32_t ty = fdiv(Y, g.dth);
    const uint32_t ry = Y - ty * g.th;
    const uint32_t tx = fdiv(X, g.dtw);
    const uint32_t rx = X - tx * g.tw;
    if (nvalid == N && rx + N <= g.tw && (g.tw % N) == 0) {
        const uint32_t chunk = ty * g.ntx + tx;
        store_vec<T, N>(fb + uint64_t(chunk) * g.bpc +
                          uint64_t(ry * g.tw + rx) * sizeof(T),
                        v);
        acc.note(fl + chunk, any_nonzero<T, N>(v));
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
deep_level(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0,
           const T* prev, T* cur)
{
    constexpr uint32_t lw = RW >> K;
    constexpr uint32_t pw = RW >> (K - 1);
    const uint32_t Wk = p.W[K], Hk = p.H[K];
    const uint32_t lh = (1u << p.rh_log2) >> K;
    const uint32_t yk0 = y0 >> K, xk0 = x0 >> K;
    // last valid local row/col of the previous level inside this region
    const uint32_t pxmax = p.W[K - 1] - 1 - (x0 >> (K - 1));
    const uint32_t pymax = p.H[K - 1] - 1 - (y0 >> (K - 1));
    const Ref ref = frame_ref(p, K, f);
    const Tiles tg = tiles_of(p, K);
    T* scr = (p.scratch_level == uint32_t(K))
               ? reinterpret_cast<T*>(p.scratch) + uint64_t(f) * Wk * Hk
               : nullptr;
    FlagAcc acc;
    acc.tag = ref.tag;
    for (uint32_t idx = threadIdx.x; idx < lh * lw; idx += 256) {
        const uint32_t ly = idx / lw, lx = idx % lw;
        const uint32_t Y = yk0 + ly, X = xk0 + lx;
        if (Y < Hk && X < Wk) {
            const uint32_t py = 2 * ly, px = 2 * lx;
            const uint32_t px1 = min(px + 1, pxmax);
            const uint32_t py1 = min(py + 1, pymax);
            const T v = reduce4<M, T>(prev[py * pw + px],
                                      prev[py * pw + px1],
                                      prev[py1 * pw + px],
                                      prev[py1 * pw + px1]);
            cur[ly * lw + lx] = v;
            if (ref.tiles)
                put_tile<T, 1>(tg, ref.tiles, ref.flags, Y, X, &v, 1, acc);
            if (scr)
                scr[uint64_t(Y) * Wk + X] = v;
        }
    }
    acc.flush_wave();
}

// The last two cascaded levels K and K+1 in one step, no barrier between
// them: each thread owns one level-(K+1) pixel, computes the 2x2 level-K
// pixels under it from level K-1 in LDS (pitch RW >> (K-1)), stores them,
// and reduces them (with the edge replication of scale_image when a level-K
// row/column falls outside the level) to its level-(K+1) pixel.
template<typename T, int M, int K, uint32_t RW>
__device__ __forceinline__ void
deep_pair(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0,
          const T* prev)
{
    constexpr uint32_t lw1 = RW >> (K + 1);
    constexpr uint32_t pw = RW >> (K - 1);
    const uint32_t lh1 = (1u << p.rh_log2) >> (K + 1);
    const uint32_t Wk = p.W[K], Hk = p.H[K], W1 = p.W[K + 1], H1 = p.H[K + 1];
    const uint32_t yk0 = y0 >> K, xk0 = x0 >> K;
    const uint32_t y10 = y0 >> (K + 1), x10 = x0 >> (K + 1);
    const uint32_t pxmax = p.W[K - 1] - 1 - (x0 >> (K - 1));
    const uint32_t pymax = p.H[K - 1] - 1 - (y0 >> (K - 1));
    const Ref rk = frame_ref(p, K, f);
    const Ref r1 = frame_ref(p, K + 1, f);
    const Tiles tk = tiles_of(p, K), t1 = tiles_of(p, K + 1);
    T* scrk = (p.scratch_level == uint32_t(K))
                ? reinterpret_cast<T*>(p.scratch) + uint64_t(f) * Wk * Hk
                : nullptr;
    T* scr1 = (p.scratch_level == uint32_t(K + 1))
                ? reinterpret_cast<T*>(p.scratch) + uint64_t(f) * W1 * H1
                : nullptr;
    FlagAcc acck, acc1;
    acck.tag = rk.tag;
    acc1.tag = r1.tag;
    for (uint32_t idx = threadIdx.x; idx < lh1 * lw1; idx += 256) {
        const uint32_t ly = idx / lw1, lx = idx % lw1;
        const uint32_t Y1 = y10 + ly, X1 = x10 + lx;
        if (Y1 < H1 && X1 < W1) {
            T v[2][2];
#pragma unroll
            for (int a = 0; a < 2; ++a) {
#pragma unroll
                for (int b = 0; b < 2; ++b) {
                    const uint32_t ky = 2 * ly + a, kx = 2 * lx + b; // level-K local
                    // (rows/cols past the level are clamped here and never
                    // stored; the level-(K+1) reduce replicates instead)
                    const uint32_t py = min(2 * ky, pymax), px = min(2 * kx, pxmax);
                    const uint32_t px1 = min(px + 1, pxmax), py1 = min(py + 1, pymax);
                    v[a][b] = reduce4<M, T>(prev[py * pw + px], prev[py * pw + px1],
                                            prev[py1 * pw + px], prev[py1 * pw + px1]);
                    const uint32_t Yk = yk0 + ky, Xk = xk0 + kx;
                    if (Yk < Hk && Xk < Wk) {
                        if (rk.tiles)
                            put_tile<T, 1>(tk, rk.tiles, rk.flags, Yk, Xk, &v[a][b], 1,
                                           acck);
                        if (scrk)
                            scrk[uint64_t(Yk) * Wk + Xk] = v[a][b];
                    }
                }
            }
            // edge replication of level K inside the level-(K+1) reduce
            const bool right = xk0 + 2 * lx + 1 < Wk;
            const bool down = yk0 + 2 * ly + 1 < Hk;
            const T here = v[0][0];
            const T rt = right ? v[0][1] : here;
            const T dn = down ? v[1][0] : here;
            const T dg = down ? (right ? v[1][1] : v[1][0]) : rt;
            const T q = reduce4<M, T>(here, rt, dn, dg);
            if (r1.tiles)
                put_tile<T, 1>(t1, r1.tiles, r1.flags, Y1, X1, &q, 1, acc1);
            if (scr1)
                scr1[uint64_t(Y1) * W1 + X1] = q;
        }
    }
    acck.flush_wave();
    acc1.flush_wave();
}

// Levels 3..n_fused of one region; level 2 is in lds_b.  Every level but
// the last two goes through LDS behind a barrier; the last two are one step.
template<typename T, int M, uint32_t RW>
__device__ __forceinline__ void
deep_levels(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0,
            T* lds_a, T* lds_b)
{
    const uint32_t n = p.n_fused;
    if (n < 3)
        return;
    __syncthreads();
    if (n == 3) {
        deep_level<T, M, 3, RW>(p, f, y0, x0, lds_b, lds_a);
        return;
    }
    const bool pair = (p.knobs & 1u) == 0;
    if (n == 4 && pair) {
        deep_pair<T, M, 3, RW>(p, f, y0, x0, lds_b);
        return;
    }
    deep_level<T, M, 3, RW>(p, f, y0, x0, lds_b, lds_a);
    __syncthreads();
    if (n == 4) {
        deep_level<T, M, 4, RW>(p, f, y0, x0, lds_a, lds_b);
        return;
    }
    if (n == 5) {
        deep_pair<T, M, 4, RW>(p, f, y0, x0, lds_a);
        return;
    }
    deep_level<T, M, 4, RW>(p, f, y0, x0, lds_a, lds_b);
    __syncthreads();
    deep_pair<T, M, 5, RW>(p, f, y0, x0, lds_b);
}

// ---- interior cascade (levels >= 3) ----------------------------------------
// An interior region lies wholly inside level 0, so every level-k pixel of it
// exists and so do its four parents: no clamping.  Stores address the tiles
// with 32-bit offsets from the frame's FrameRef (the host keeps the fast path
// to layers < 4 GiB) and raise has_data with a plain per-pixel store, which
// keeps these rarely-run loops from pinning registers the row passes need.
template<typename T>
__device__ __forceinline__ void
put_px(const FusedParams& p, int k, const Ref& r, uint32_t Y, uint32_t X, T v)
{
    const uint32_t ty = fdiv(Y, p.dth), tx = fdiv(X, p.dtw);
    const uint32_t chunk = ty * p.ntx[k] + tx;
    const uint32_t off = chunk * uint32_t(p.bpc) +
                         ((Y - ty * p.th) * p.tw + (X - tx * p.tw)) * uint32_t(sizeof(T));
    *reinterpret_cast<T*>(r.tiles + off) = v;
    if (nonzero_bits(v))
        r.flags[chunk] = r.tag;
}

template<typename T>
__device__ __forceinline__ T*
scratch_of(const FusedParams& p, int k, uint32_t f)
{
    return p.scratch_level == uint32_t(k)
             ? reinterpret_cast<T*>(p.scratch) + uint64_t(f) * p.W[k] * p.H[k]
             : nullptr;
}

template<typename T, int M, int K, uint32_t RW>
__device__ __forceinline__ void
lean_level(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0, const T* prev,
           T* cur)
{
    constexpr uint32_t lw = RW >> K, pw = RW >> (K - 1);
    const uint32_t n = ((1u << p.rh_log2) >> K) * lw;
    const Ref ref = frame_ref(p, K, f);
    T* scr = scratch_of<T>(p, K, f);
#pragma unroll 1
    for (uint32_t idx = threadIdx.x; idx < n; idx += 256) {
        const uint32_t ly = idx / lw, lx = idx % lw;
        const T* q = prev + 2 * ly * pw + 2 * lx;
        const T v = reduce4<M, T>(q[0], q[1], q[pw], q[pw + 1]);
        cur[idx] = v;
        const uint32_t Y = (y0 >> K) + ly, X = (x0 >> K) + lx;
        if (ref.tiles)
            put_px<T>(p, K, ref, Y, X, v);
        if (scr)
            scr[uint64_t(Y) * p.W[K] + X] = v;
    }
}

// levels K and K+1 in one step: each thread owns one level-(K+1) pixel
template<typename T, int M, int K, uint32_t RW>
__device__ __forceinline__ void
lean_pair(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0, const T* prev)
{
    constexpr uint32_t lw1 = RW >> (K + 1), pw = RW >> (K - 1);
    const uint32_t n = ((1u << p.rh_log2) >> (K + 1)) * lw1;
    const Ref rk = frame_ref(p, K, f), r1 = frame_ref(p, K + 1, f);
    T* scrk = scratch_of<T>(p, K, f);
    T* scr1 = scratch_of<T>(p, K + 1, f);
#pragma unroll 1
    for (uint32_t idx = threadIdx.x; idx < n; idx += 256) {
        const uint32_t ly = idx / lw1, lx = idx % lw1;
        T v[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
            for (int b = 0; b < 2; ++b) {
                const T* q = prev + (4 * ly + 2 * a) * pw + 4 * lx + 2 * b;
                v[a][b] = reduce4<M, T>(q[0], q[1], q[pw], q[pw + 1]);
                const uint32_t Y = (y0 >> K) + 2 * ly + a, X = (x0 >> K) + 2 * lx + b;
                if (rk.tiles)
                    put_px<T>(p, K, rk, Y, X, v[a][b]);
                if (scrk)
                    scrk[uint64_t(Y) * p.W[K] + X] = v[a][b];
            }
        }
        const T w = reduce4<M, T>(v[0][0], v[0][1], v[1][0], v[1][1]);
        const uint32_t Y1 = (y0 >> (K + 1)) + ly, X1 = (x0 >> (K + 1)) + lx;
        if (r1.tiles)
            put_px<T>(p, K + 1, r1, Y1, X1, w);
        if (scr1)
            scr1[uint64_t(Y1) * p.W[K + 1] + X1] = w;
    }
}

// Levels 3..n_fused of an interior region; level 2 is in lds_b.
template<typename T, int M, uint32_t RW>
__device__ __forceinline__ void
lean_levels(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0, T* lds_a,
            T* lds_b)
{
    const uint32_t n = p.n_fused;
    if (n < 3)
        return;
    __syncthreads();
    if (n == 3) {
        lean_level<T, M, 3, RW>(p, f, y0, x0, lds_b, lds_a);
    } else if (n == 4) {
        lean_pair<T, M, 3, RW>(p, f, y0, x0, lds_b);
    } else if (n == 5) {
        lean_level<T, M, 3, RW>(p, f, y0, x0, lds_b, lds_a);
        __syncthreads();
        lean_pair<T, M, 4, RW>(p, f, y0, x0, lds_a);
    } else {
        lean_level<T, M, 3, RW>(p, f, y0, x0, lds_b, lds_a);
        __syncthreads();
        lean_level<T, M, 4, RW>(p, f, y0, x0, lds_a, lds_b);
        __syncthreads();
        lean_pair<T, M, 5, RW>(p, f, y0, x0, lds_b);
    }
}

// Edge regions (or layouts the fast path does not cover): every access
// bounds-checked, columns and rows clamped for the edge replication of
// scale_image (downsampler.cpp:187-196); level 1 -> lds_a, level 2 -> lds_b.
template<typename T, int M, uint32_t RW>
__device__ void
generic_region(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0,
               T* lds_a, T* lds_b)
{
    constexpr int VEC = 16 / sizeof(T);
    constexpr int HV = VEC / 2;
    const uint32_t tid = threadIdx.x;
    const uint32_t rp = tid >> 5;
    const uint32_t cv = tid & 31;
    const uint32_t npass = 1u << (p.rh_log2 - 4);
    const uint32_t W0 = p.W[0], H0 = p.H[0];
    const T* src = reinterpret_cast<const T*>(p.src + uint64_t(f) * p.src_stride);

    const Ref r0ref = frame_ref(p, 0, f);
    const bool l1 = p.n_fused >= 1;
    const Ref r1ref = l1 ? frame_ref(p, 1, f) : Ref{ nullptr, nullptr, 0 };
    const Tiles tg0 = tiles_of(p, 0);
    const Tiles tg1 = tiles_of(p, 1);
    T* scr1 = (l1 && p.scratch_level == 1)
                ? reinterpret_cast<T*>(p.scratch) + uint64_t(f) * p.W[1] * p.H[1]
                : nullptr;
    const bool keep_l1 = p.n_fused >= 2;

    FlagAcc acc0, acc1;
    acc0.tag = r0ref.tag;
    acc1.tag = r1ref.tag;
    for (uint32_t pass = 0; pass < npass; ++pass) {
        const uint32_t y = y0 + pass * 16 + 2 * rp;
        const uint32_t x = x0 + cv * VEC;
        if (y < H0 && x < W0) {
            const uint32_t ya = min(y + 1, H0 - 1); // bottom edge replicate
            T r0[VEC], r1[VEC];
            const int nv0 = int(min(uint32_t(VEC), W0 - x));
            if (p.xy) {
                // acquisition-order source: storage (y, x) is src[x * H0 + y]
#pragma unroll
                for (int i = 0; i < VEC; ++i) {
                    const uint32_t xi = min(x + uint32_t(i), W0 - 1);
                    r0[i] = src[uint64_t(xi) * H0 + y];
                    r1[i] = src[uint64_t(xi) * H0 + ya];
                }
            } else if (p.vec_rows && nv0 == VEC) {
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
            if (r0ref.tiles) {
                put_tile<T, VEC>(tg0, r0ref.tiles, r0ref.flags, y, x, r0, nv0, acc0);
                if (y + 1 < H0)
                    put_tile<T, VEC>(tg0, r0ref.tiles, r0ref.flags, y + 1, x, r1,
                                     nv0, acc0);
            }
            if (l1) {
                T o[HV];
#pragma unroll
                for (int i = 0; i < HV; ++i)
                    o[i] = reduce4<M, T>(
                      r0[2 * i], r0[2 * i + 1], r1[2 * i], r1[2 * i + 1]);
                const uint32_t Y = y >> 1, X = x >> 1;
                const int nv1 = int(min(uint32_t(HV), p.W[1] - X));
                if (r1ref.tiles)
                    put_tile<T, HV>(tg1, r1ref.tiles, r1ref.flags, Y, X, o, nv1, acc1);
                if (scr1)
                    for (int i = 0; i < nv1; ++i)
                        scr1[uint64_t(Y) * p.W[1] + X + i] = o[i];
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
    if (p.n_fused >= 2) {
        __syncthreads();
        deep_level<T, M, 2, RW>(p, f, y0, x0, lds_a, lds_b);
    }
}

// ---------------------------------------------------------------------------
// Fast path for interior regions whose rows lie in one chunk-tile row at
// every fused level and whose 16-B vectors never straddle a tile: every
// thread's tile addresses are set up once per region.
// ---------------------------------------------------------------------------
struct FastTile
{
    uint8_t* p;      // (region row 0 at this level, this thread's column)
    uint32_t* flag;  // has_data word of that chunk
    uint32_t tag;
    bool nz;
};

template<typename T>
__device__ __forceinline__ FastTile
fast_tile(const FusedParams& p, int k, uint32_t f, uint32_t Y0, uint32_t X)
{
    FastTile t{ nullptr, nullptr, 0, false };
    const Ref ref = frame_ref(p, k, f);
    if (!ref.tiles)
        return t;
    t.tag = ref.tag;
    const uint32_t ty = fdiv(Y0, p.dth);
    const uint32_t tx = fdiv(X, p.dtw);
    const uint32_t ry = Y0 - ty * p.th;
    const uint32_t rx = X - tx * p.tw;
    const uint32_t chunk = ty * p.ntx[k] + tx;
    t.p = ref.tiles + uint64_t(chunk) * p.bpc + uint64_t(ry * p.tw + rx) * sizeof(T);
    t.flag = ref.flags + chunk;
    return t;
}

__device__ __forceinline__ void
flush_tile_flag(FastTile& t)
{
    FlagAcc a;
    a.ptr = t.flag;
    a.nz = t.nz;
    a.tag = t.tag;
    a.flush_wave();
    t.nz = false;
}

template<typename T>
__device__ __forceinline__ T
shfl_xor_t(T v, int mask)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        const uint32_t lo = __shfl_xor(uint32_t(u), mask);
        const uint32_t hi = __shfl_xor(uint32_t(u >> 32), mask);
        u = (uint64_t(hi) << 32) | lo;
        T r;
        __builtin_memcpy(&r, &u, 8);
        return r;
    } else {
        uint32_t u = 0;
        __builtin_memcpy(&u, &v, sizeof(T));
        u = __shfl_xor(u, mask);
        T r;
        __builtin_memcpy(&r, &u, sizeof(T));
        return r;
    }
}

template<typename T>
__device__ __forceinline__ T
shfl_down_t(T v, int d)
{
    if constexpr (sizeof(T) == 8) {
        uint64_t u;
        __builtin_memcpy(&u, &v, 8);
        const uint32_t lo = __shfl_down(uint32_t(u), d);
        const uint32_t hi = __shfl_down(uint32_t(u >> 32), d);
        u = (uint64_t(hi) << 32) | lo;
        T r;
        __builtin_memcpy(&r, &u, 8);
        return r;
    } else {
        uint32_t u = 0;
        __builtin_memcpy(&u, &v, sizeof(T));
        u = __shfl_down(u, d);
        T r;
        __builtin_memcpy(&r, &u, sizeof(T));
        return r;
    }
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template<bool NT>
__device__ __forceinline__ uint4
ld16(const uint8_t* s)
{
    const u32x4 v = gload<NT, u32x4>(s);
    return uint4{ v.x, v.y, v.z, v.w };
}

template<bool NT>
__device__ __forceinline__ void
st16(uint8_t* d, const uint4& a)
{
    gstore<NT>(d, u32x4{ a.x, a.y, a.z, a.w });
}

// The two 16-B row vectors of this thread for one pass of an interior region.
template<int NTM>
__device__ __forceinline__ void
load_pass(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0,
          uint32_t pass, uint32_t bpp, uint4& a, uint4& b)
{
    const uint32_t y = y0 + pass * 16 + 2 * (threadIdx.x >> 5);
    const uint64_t row = uint64_t(p.W[0]) * bpp;
    const uint8_t* s = p.src + uint64_t(f) * p.src_stride + uint64_t(y) * row +
                       uint64_t(x0 + (threadIdx.x & 31) * (16 / bpp)) * bpp;
    a = ld16<(NTM & 1) != 0>(s);
    b = ld16<(NTM & 1) != 0>(s + row);
}

// One 16-row pass of an interior region: level-0 tile rows, level 1 (2x2 in
// registers), level 2 (rows of lanes l and l^32 meet by a cross-lane swap).
template<typename T, int M, uint32_t RW, int NTM>
__device__ __forceinline__ void
fast_pass(const FusedParams& p, uint32_t pass, const uint4& ra, const uint4& rb,
          FastTile& t0, FastTile& t1, FastTile& t2, T* lds_l2)
{
    constexpr int VEC = 16 / sizeof(T);
    constexpr int HV = VEC / 2;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rp = threadIdx.x >> 5;
    const uint32_t cv = threadIdx.x & 31;
    const uint32_t trow = p.tw * uint32_t(sizeof(T)); // bytes per tile row
    if (t0.p) {
        const uint32_t dy = pass * 16 + 2 * rp;
        st16<(NTM & 2) != 0>(t0.p + uint64_t(dy) * trow, ra);
        st16<(NTM & 2) != 0>(t0.p + uint64_t(dy + 1) * trow, rb);
        t0.nz |= ((ra.x | ra.y | ra.z | ra.w) | (rb.x | rb.y | rb.z | rb.w)) != 0u;
    }
    if (p.n_fused < 1)
        return;
    T r0[VEC], r1[VEC];
    __builtin_memcpy(r0, &ra, 16);
    __builtin_memcpy(r1, &rb, 16);
    T o[HV];
#pragma unroll
    for (int i = 0; i < HV; ++i)
        o[i] = reduce4<M, T>(r0[2 * i], r0[2 * i + 1], r1[2 * i], r1[2 * i + 1]);
    if (t1.p && !(p.knobs & 4u)) {
        store_vec<T, HV, (NTM & 4) != 0>(t1.p + uint64_t(pass * 8 + rp) * trow, o);
        t1.nz |= any_nonzero<T, HV>(o);
    }
    if (p.n_fused < 2)
        return;
    const uint32_t row2 = pass * 4 + (rp >> 1);
    if constexpr (HV >= 2) {
        constexpr int QV = HV / 2;
        // level-1 row below lives in lane ^ 32: move HV*sizeof(T) = 8 bytes
        uint2 mine, below;
        __builtin_memcpy(&mine, o, 8);
        below.x = __shfl_xor(mine.x, 32);
        below.y = __shfl_xor(mine.y, 32);
        T b[HV];
        __builtin_memcpy(b, &below, 8);
        if (lane < 32) {
            T q[QV];
#pragma unroll
            for (int j = 0; j < QV; ++j)
                q[j] = reduce4<M, T>(o[2 * j], o[2 * j + 1], b[2 * j], b[2 * j + 1]);
            if (t2.p && !(p.knobs & 8u)) {
                store_vec<T, QV, (NTM & 4) != 0>(t2.p + uint64_t(row2) * trow, q);
                t2.nz |= any_nonzero<T, QV>(q);
            }
            if (lds_l2) {
#pragma unroll
                for (int j = 0; j < QV; ++j)
                    lds_l2[row2 * (RW / 4) + cv * QV + j] = q[j];
            }
        }
    } else {
        // one level-1 pixel per lane: the 2x2 block spans lanes l, l+1,
        // l^32, (l^32)+1
        const T b = shfl_xor_t(o[0], 32);
        const T rt = shfl_down_t(o[0], 1);
        const T brt = shfl_down_t(b, 1);
        if (lane < 32 && (cv & 1) == 0) {
            const T q = reduce4<M, T>(o[0], rt, b, brt);
            if (t2.p) {
                store_vec<T, 1>(t2.p + uint64_t(row2) * trow, &q);
                t2.nz |= nonzero_bits(q);
            }
            if (lds_l2)
                lds_l2[row2 * (RW / 4) + (cv >> 1)] = q;
        }
    }
}

// Workgroups are dealt round-robin over the 8 XCDs (block b -> XCD b mod 8).
// With xcd_order, the blocks of one XCD walk one contiguous eighth of the
// launch's regions, so horizontally adjacent regions -- whose level >= 3
// rows share cache lines -- meet in the same L2 and leave it as whole lines.
__device__ __forceinline__ uint32_t
region_of_block(const FusedParams& p)
{
    const uint32_t b = blockIdx.x;
    if (!p.xcd_order)
        return b;
    const uint32_t per = gridDim.x >> 3;
    if (b >= (per << 3))
        return b;
    const uint32_t x = b & 7u;
    uint32_t i = (b >> 3) + p.xrot[x];
    if (i >= per)
        i -= per;
    if (p.xskew) {
        // step s of the range visits region u of frame (s + u) mod R: the
        // regions in flight on one XCD write their tiles at different
        // frame offsets inside the chunks instead of all at the same one
        const uint32_t nreg = p.nbx_in * p.nby_in;
        const uint32_t s = fdiv(i, p.d_nreg_in);
        const uint32_t u = i - s * nreg;
        i = ((s + u) & p.xskew) * nreg + u;
    }
    return x * per + i;
}

// x * xcd_rot mod (blocks / 8) for the 8 XCDs (region_of_block)
static FusedParams
with_xcd_rotation(const FusedParams& p, uint64_t blocks)
{
    FusedParams q = p;
    const uint64_t per = blocks >> 3;
    for (uint32_t x = 0; x < 8; ++x)
        q.xrot[x] = per ? uint32_t((uint64_t(x) * p.xcd_rot) % per) : 0u;
    const uint64_t nreg = uint64_t(p.nbx_in) * p.nby_in;
    const uint64_t R = nreg ? per / nreg : 0;
    q.xskew = (p.xskew && p.xcd_order && R >= 2 && per % nreg == 0 && (R & (R - 1)) == 0)
                ? uint32_t(R - 1)
                : 0u;
    return q;
}

// Region q of a frame -> (row, column) of regions: row-major, or
// column-major, so that consecutive workgroups walk down one column of
// chunk tiles and write each tile's rows as one contiguous run.  Tuning knob
// 1024 flips the kernel's default (same-stage A/B, tools/knob_ab.py: the
// 2-D strip kernel is 2-3% faster row-major, the 2x2x2 strip kernel 2%
// faster column-major).
__device__ __forceinline__ void
region_xy(const FusedParams& p, uint32_t q, uint32_t& by, uint32_t& bx, bool colmajor)
{
    // values, then selects: assigning by / bx inside the branches made the
    // compiler pick the store address per branch and keep both in scratch
    const bool cm = colmajor != ((p.knobs & 1024u) != 0);
    uint32_t a, b;
    if (cm) {
        a = q / p.nby_in; // column
        b = q - a * p.nby_in;
    } else {
        a = fdiv(q, p.d_nbx_in); // row
        b = q - a * p.nbx_in;
    }
    by = cm ? b : a;
    bx = cm ? a : b;
}

// Interior regions, one per workgroup (region r of n_frames * nby_in * nbx_in).
// The rows of up to kPassBatch passes are loaded before any is reduced, so a
// wave keeps its whole region in flight; then level 0 goes to its tiles,
// levels 1-2 are formed in registers, and levels >= 3 in LDS.  Not a
// persistent loop: a grid-stride loop lets the compiler keep every
// cascade invariant live across the row passes, which costs occupancy.
constexpr uint32_t kPassBatch = 4;

template<typename T, int M, int NTM>
__global__ __launch_bounds__(256) void
fused_pyramid(const FusedParams p)
{
    constexpr int VEC = 16 / sizeof(T); // pixels per 16-B row vector
    constexpr uint32_t RW = 32 * VEC;   // region width (512 B of row)
    __shared__ __attribute__((aligned(16))) T lds_a[(kMaxRegionRows / 2) * (RW / 2)];
    __shared__ __attribute__((aligned(16))) T lds_b[(kMaxRegionRows / 4) * (RW / 4)];

    const uint32_t r = region_of_block(p);
    const uint32_t f = fdiv(r, p.d_nreg_in);
    const uint32_t q = r - f * (p.nbx_in * p.nby_in);
    const uint32_t by = fdiv(q, p.d_nbx_in);
    const uint32_t y0 = by << p.rh_log2;
    const uint32_t x0 = (q - by * p.nbx_in) * RW;
    const uint32_t npass = 1u << (p.rh_log2 - 4);
    const uint32_t cv = threadIdx.x & 31;

    FastTile t0 = fast_tile<T>(p, 0, f, y0, x0 + cv * VEC);
    FastTile t1{}, t2{};
    if (p.n_fused >= 1)
        t1 = fast_tile<T>(p, 1, f, y0 >> 1, (x0 >> 1) + cv * (VEC / 2));
    if (p.n_fused >= 2)
        t2 = fast_tile<T>(p, 2, f, y0 >> 2,
                          (x0 >> 2) + (VEC >= 4 ? cv * (VEC / 4) : (cv >> 1)));
    T* lds_l2 = p.n_fused >= 3 ? lds_b : nullptr;

    for (uint32_t p0 = 0; p0 < npass; p0 += kPassBatch) {
        uint4 ra[kPassBatch], rb[kPassBatch];
#pragma unroll
        for (uint32_t i = 0; i < kPassBatch; ++i) // passes past npass re-read the last
            load_pass<NTM>(p, f, y0, x0, min(p0 + i, npass - 1), sizeof(T), ra[i], rb[i]);
#pragma unroll
        for (uint32_t i = 0; i < kPassBatch; ++i)
            if (p0 + i < npass)
                fast_pass<T, M, RW, NTM>(p, p0 + i, ra[i], rb[i], t0, t1, t2, lds_l2);
    }
    if (!(p.knobs & 32u)) {
        flush_tile_flag(t0);
        flush_tile_flag(t1);
        flush_tile_flag(t2);
    }
    if (!(p.knobs & 16u))
        lean_levels<T, M, RW>(p, f, y0, x0, lds_a, lds_b);
}

// XY-transposed storage order fused into the strip kernel's region load
// (transpose_frame, array.cpp:488-534, applied before the split and the
// downsampler, :525-533).  The region's storage rows [y0, y0+64) x columns
// [x0, x0+RW) are acquisition columns [y0, y0+64) of acquisition rows
// [x0, x0+RW): the workgroup reads those rows as coalesced 64-pixel segments
// (8 x 16 B per lane), stores them in LDS as column pairs (c, c+1), and each
// thread gathers its storage row vectors: ra[i] = storage row ry + 4i, rb[i]
// = the row below, both from one LDS read per pixel pair.  Pair index pc of
// row r sits at (pc + r + r / VEC) mod 32, so the 32 lanes of a gather
// (rows cv * VEC + k) hit distinct banks.
// SLOTS tiles of LDS, one per group of 256 threads loading its own region
// (slot = the group; fused_pyramid_strip3d_pair loads two planes at once).
template<typename T, int NTM, int SLOTS = 1>
__device__ __forceinline__ void
load_region_xy(const FusedParams& p, uint32_t f, uint32_t y0, uint32_t x0, uint32_t ry,
               uint32_t cv, uint4 (&ra)[4], uint4 (&rb)[4], uint32_t tid = threadIdx.x,
               uint32_t slot = 0)
{
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    typedef typename std::conditional<
      sizeof(T) == 1, uint16_t,
      typename std::conditional<sizeof(T) == 2, uint32_t, uint64_t>::type>::type PT;
    constexpr uint32_t VEC = 16 / sizeof(T);
    constexpr uint32_t RW = 32 * VEC;      // acquisition rows of the region
    constexpr uint32_t VR = 4 * sizeof(T); // 16-B vectors per 64-pixel row segment
    constexpr uint32_t PV = 8 / sizeof(T); // column pairs per 16-B vector
    __shared__ PT xt_slots[SLOTS * RW * 32]; // 32 KiB per slot
    static_assert(sizeof(PT) * RW * 32 == 32768, "one transpose slot is 32 KiB");
    // with the pair kernel's 16 KiB level-1 exchange: 2 x 32 + 16 = 80 KiB
    // per workgroup, two workgroups per CU in gfx950's 160 KiB
    static_assert(SLOTS * 32768 + (SLOTS > 1 ? 16384 : 0) <= 163840 / 2,
                  "the XY kernels' LDS must leave room for two workgroups per CU");
    PT* const xt = xt_slots + slot * (RW * 32);
    const uint64_t pitch = uint64_t(p.H[0]) * sizeof(T); // acquisition row bytes
    const uint8_t* s =
      p.src + uint64_t(f) * p.src_stride + uint64_t(x0) * pitch + uint64_t(y0) * sizeof(T);
    u32x4v v[8];
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t idx = tid + 256u * j;
        const uint32_t r = idx / VR, c16 = idx % VR;
        v[j] = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(r) * pitch + c16 * 16u);
    }
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        const uint32_t idx = tid + 256u * j;
        const uint32_t r = idx / VR, c16 = idx % VR;
        PT e[PV];
        __builtin_memcpy(e, &v[j], 16);
#pragma unroll
        for (uint32_t q = 0; q < PV; ++q)
            xt[r * 32u + ((c16 * PV + q + r + r / VEC) & 31u)] = e[q];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t pc = (ry + 4u * i) >> 1; // ry is even
        T a[VEC], b[VEC];
#pragma unroll
        for (uint32_t k = 0; k < VEC; ++k) {
            const uint32_t r = cv * VEC + k;
            const PT e = xt[r * 32u + ((pc + r + cv) & 31u)];
            T two[2];
            __builtin_memcpy(two, &e, sizeof(PT));
            a[k] = two[0];
            b[k] = two[1];
        }
        __builtin_memcpy(&ra[i], a, 16);
        __builtin_memcpy(&rb[i], b, 16);
    }
}

// ---------------------------------------------------------------------------
// Interior regions of 64 rows with pixels of <= 4 bytes ("strip" kernel).
// Wave w owns the region's rows [16w, 16w+16): level 1 is a 2x2 in
// registers, level 2 meets the row below through a lane^32 swap, and levels
// 3 and 4 combine level-2 rows that the same lane already holds (rows of
// different passes) and columns of the same or a neighbouring lane -- so the
// cascade down to level 4 needs no LDS and no barrier.  Only pyramids deeper
// than 4 levels hand their one level-4 row per wave to LDS for levels 5-6.
// ---------------------------------------------------------------------------
// NTM: compile-time nontemporal policy -- bit 1 input loads, bit 2 level-0
// tile stores, bit 4 level-1/2 stores (the launcher maps p.nt onto one of the
// instantiated policies).
// XY: the source is in acquisition order (load_region_xy).
template<typename T, int M, int NTM, bool XY = false>
__global__ __launch_bounds__(256) void
fused_pyramid_strip(const FusedParams p)
{
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    constexpr int VEC = 16 / sizeof(T); // pixels per 16-B row vector
    constexpr int HV = VEC / 2;         // level-1 pixels per lane
    constexpr int QV = VEC / 4;         // level-2 pixels per lane
    constexpr uint32_t RW = 32 * VEC;   // region width
    static_assert(QV >= 1, "strip kernel needs <= 4-byte pixels");
    // level 3: N3 pixels per lane, one lane in S3 holds pixels
    constexpr int N3 = QV >= 2 ? QV / 2 : 1;
    constexpr int S3 = QV >= 2 ? 1 : 2;
    constexpr int N4 = N3 >= 2 ? N3 / 2 : 1;
    constexpr int S4 = N3 >= 2 ? S3 : 2 * S3;
    __shared__ __attribute__((aligned(16))) T lds4[4 * (RW / 16)];
    __shared__ __attribute__((aligned(16))) T lds5[2 * (RW / 32)];

    const uint32_t r = region_of_block(p);
    const uint32_t f = fdiv(r, p.d_nreg_in);
    const uint32_t q = r - f * (p.nbx_in * p.nby_in);
    uint32_t by, bx;
    region_xy(p, q, by, bx, false);
    const uint32_t y0 = by << 6;
    const uint32_t x0 = bx * RW;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t hw = (threadIdx.x >> 5) & 1u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cv = threadIdx.x & 31u;
    const uint32_t trow = p.tw * uint32_t(sizeof(T)); // bytes per tile row
    const uint32_t nf = p.n_fused;

    // this half-wave's rows: y0 + ry + 4i + {0, 1}, i = 0..3
    const uint32_t ry = 16 * w + 2 * hw;
    uint4 ra[4], rb[4];
    if constexpr (XY) {
        load_region_xy<T, NTM>(p, f, y0, x0, ry, cv, ra, rb);
    } else {
        const uint64_t row = uint64_t(p.W[0]) * sizeof(T);
        const uint8_t* s = p.src + uint64_t(f) * p.src_stride + uint64_t(y0 + ry) * row +
                           uint64_t(x0 + cv * VEC) * sizeof(T);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4v a = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(4 * i) * row);
            const u32x4v b = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(4 * i + 1) * row);
            ra[i] = uint4{ a.x, a.y, a.z, a.w };
            rb[i] = uint4{ b.x, b.y, b.z, b.w };
        }
    }
    FastTile t0 = fast_tile<T>(p, 0, f, y0 + ry, x0 + cv * VEC);
    FastTile t1{}, t2{};
    if (nf >= 1)
        t1 = fast_tile<T>(p, 1, f, (y0 >> 1) + 8 * w + hw, (x0 >> 1) + cv * HV);
    if (nf >= 2)
        t2 = fast_tile<T>(p, 2, f, (y0 >> 2) + 4 * w, (x0 >> 2) + cv * QV);
    T q2[4][QV]; // level-2 rows 4w + i (meaningful in lanes < 32)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        if (t0.p) {
            gstore<(NTM & 2) != 0>(t0.p + uint64_t(4 * i) * trow,
                                   u32x4v{ ra[i].x, ra[i].y, ra[i].z, ra[i].w });
            gstore<(NTM & 2) != 0>(t0.p + uint64_t(4 * i + 1) * trow,
                                   u32x4v{ rb[i].x, rb[i].y, rb[i].z, rb[i].w });
            t0.nz |= ((ra[i].x | ra[i].y | ra[i].z | ra[i].w) |
                      (rb[i].x | rb[i].y | rb[i].z | rb[i].w)) != 0u;
        }
        if (nf < 1)
            continue;
        T r0[VEC], r1[VEC], o[HV];
        __builtin_memcpy(r0, &ra[i], 16);
        __builtin_memcpy(r1, &rb[i], 16);
#pragma unroll
        for (int j = 0; j < HV; ++j)
            o[j] = reduce4<M, T>(r0[2 * j], r0[2 * j + 1], r1[2 * j], r1[2 * j + 1]);
        if (t1.p) {
            gstore_px<T, HV, (NTM & 4) != 0>(t1.p + uint64_t(2 * i) * trow, o);
            t1.nz |= any_nonzero<T, HV>(o);
        }
        if (nf < 2)
            continue;
        // the level-1 row below lives in lane ^ 32 (HV * sizeof(T) = 8 bytes)
        uint2 mine, below;
        __builtin_memcpy(&mine, o, 8);
        below.x = __shfl_xor(mine.x, 32);
        below.y = __shfl_xor(mine.y, 32);
        T b[HV];
        __builtin_memcpy(b, &below, 8);
#pragma unroll
        for (int j = 0; j < QV; ++j)
            q2[i][j] = reduce4<M, T>(o[2 * j], o[2 * j + 1], b[2 * j], b[2 * j + 1]);
        if (lane < 32 && t2.p) {
            gstore_px<T, QV, (NTM & 4) != 0>(t2.p + uint64_t(i) * trow, q2[i]);
            t2.nz |= any_nonzero<T, QV>(q2[i]);
        }
    }
    if (!(p.knobs & 32u)) { // tuning knob 32: no has_data stores (A/B only)
        flush_tile_flag(t0);
        flush_tile_flag(t1);
        flush_tile_flag(t2);
    }
    if (nf < 3 || (p.knobs & 8u))
        return;

    // level 3: rows 2w + r from level-2 rows 2r, 2r+1 of this lane
    T v3[2][N3];
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
        const T* a = q2[2 * rr];
        const T* c = q2[2 * rr + 1];
        if constexpr (QV >= 2) {
#pragma unroll
            for (int j = 0; j < N3; ++j)
                v3[rr][j] = reduce4<M, T>(a[2 * j], a[2 * j + 1], c[2 * j], c[2 * j + 1]);
        } else {
            const T ar = shfl_down_t(a[0], 1), cr = shfl_down_t(c[0], 1);
            v3[rr][0] = reduce4<M, T>(a[0], ar, c[0], cr);
        }
    }
    {
        const bool valid = lane < 32 && (cv % S3) == 0;
        FastTile t3{};
        if (valid)
            t3 = fast_tile<T>(p, 3, f, (y0 >> 3) + 2 * w, (x0 >> 3) + (cv / S3) * N3);
        if (t3.p) {
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                gstore_px<T, N3, false>(t3.p + uint64_t(rr) * trow, v3[rr]);
                t3.nz |= any_nonzero<T, N3>(v3[rr]);
            }
        }
        flush_tile_flag(t3);
    }
    if (nf < 4)
        return;

    // level 4: row w
    T v4[N4];
    if constexpr (N3 >= 2) {
#pragma unroll
        for (int j = 0; j < N4; ++j)
            v4[j] = reduce4<M, T>(v3[0][2 * j], v3[0][2 * j + 1], v3[1][2 * j],
                                  v3[1][2 * j + 1]);
    } else {
        const T ar = shfl_down_t(v3[0][0], S3), cr = shfl_down_t(v3[1][0], S3);
        v4[0] = reduce4<M, T>(v3[0][0], ar, v3[1][0], cr);
    }
    const bool valid4 = lane < 32 && (cv % S4) == 0;
    {
        FastTile t4{};
        if (valid4)
            t4 = fast_tile<T>(p, 4, f, (y0 >> 4) + w, (x0 >> 4) + (cv / S4) * N4);
        if (t4.p) {
            gstore_px<T, N4, false>(t4.p, v4);
            t4.nz |= any_nonzero<T, N4>(v4);
        }
        flush_tile_flag(t4);
    }
    if (nf < 5)
        return;
    // levels 5-6 across the waves, from the level-4 rows in LDS
    if (valid4) {
#pragma unroll
        for (int j = 0; j < N4; ++j)
            lds4[w * (RW / 16) + (cv / S4) * N4 + j] = v4[j];
    }
    __syncthreads();
    if (nf == 5)
        lean_level<T, M, 5, RW>(p, f, y0, x0, lds4, lds5);
    else
        lean_pair<T, M, 5, RW>(p, f, y0, x0, lds4);
}

// Edge regions (right column strip, bottom row strip; or every region when
// the fast path does not apply): one workgroup per region, fully checked.
template<typename T, int M>
__global__ __launch_bounds__(256) void
fused_pyramid_edge(const FusedParams p)
{
    constexpr int VEC = 16 / sizeof(T);
    constexpr uint32_t RW = 32 * VEC;
    __shared__ __attribute__((aligned(16))) T lds_a[(kMaxRegionRows / 2) * (RW / 2)];
    __shared__ __attribute__((aligned(16))) T lds_b[(kMaxRegionRows / 4) * (RW / 4)];
    const uint32_t right = p.nby_in * (p.nbx - p.nbx_in);
    const uint32_t per_frame = p.nbx * p.nby - p.nbx_in * p.nby_in;
    const uint32_t f = blockIdx.x / per_frame;
    const uint32_t e = blockIdx.x - f * per_frame;
    uint32_t by, bx;
    if (e < right) {
        const uint32_t w = p.nbx - p.nbx_in;
        by = e / w;
        bx = p.nbx_in + (e - by * w);
    } else {
        const uint32_t e2 = e - right;
        by = p.nby_in + e2 / p.nbx;
        bx = e2 - (by - p.nby_in) * p.nbx;
    }
    const uint32_t y0 = by << p.rh_log2, x0 = bx * RW;
    generic_region<T, M, RW>(p, f, y0, x0, lds_a, lds_b);
    deep_levels<T, M, RW>(p, f, y0, x0, lds_a, lds_b);
}

// ---------------------------------------------------------------------------
// 2x2x2 pyramid (z-halving levels), interior regions, regular z schedule.
// A workgroup owns one region of G consecutive level-0 planes (G = 2^number
// of z-halving levels), so every z pair of every level is formed inside it:
// level k plane = reduce2(xy(earlier plane), xy(later plane)) exactly as
// Downsampler::add_frame orders it (XY first, then average_two_frames with
// the earlier plane first, downsampler.cpp:341-389).  Levels 1-2 in
// registers (the earlier plane of a pair is held), levels >= 3 per plane in
// LDS.  Host guarantees: sizeof(T) <= 4, interior region, every fused level
// halves XY, every z-halving level has an even input plane count, the
// launch starts at a group boundary with no pending partial plane.
// ---------------------------------------------------------------------------
template<typename T, int M, int K, uint32_t RW>
__device__ __forceinline__ void
deep3d_level(const FusedParams& p, uint32_t grp, uint32_t y0, uint32_t x0,
             const T* prev, T* cur, uint32_t g_prev)
{
    constexpr uint32_t lw = RW >> K;
    constexpr uint32_t pw = RW >> (K - 1);
    const uint32_t lh = (1u << p.rh_log2) >> K;
    const uint32_t ph = (1u << p.rh_log2) >> (K - 1);
    const uint32_t zk = (p.zmask >> K) & 1u;
    const uint32_t g = g_prev >> zk;
    const uint32_t yk0 = y0 >> K, xk0 = x0 >> K;
    const Tiles tg = tiles_of(p, K);
    for (uint32_t q = 0; q < g; ++q) {
        const Ref ref = frame_ref(p, K, grp * g + q);
        FlagAcc acc;
        acc.tag = ref.tag;
        const T* a = prev + (zk ? 2 * q : q) * ph * pw;
        const T* b = a + ph * pw; // the later plane of the pair
        for (uint32_t idx = threadIdx.x; idx < lh * lw; idx += 256) {
            const uint32_t ly = idx / lw, lx = idx % lw;
            const uint32_t o0 = (2 * ly) * pw + 2 * lx;
            T v = reduce4<M, T>(a[o0], a[o0 + 1], a[o0 + pw], a[o0 + pw + 1]);
            if (zk)
                v = reduce2<M, T>(
                  v, reduce4<M, T>(b[o0], b[o0 + 1], b[o0 + pw], b[o0 + pw + 1]));
            cur[q * lh * lw + ly * lw + lx] = v;
            if (ref.tiles)
                put_tile<T, 1>(tg, ref.tiles, ref.flags, yk0 + ly, xk0 + lx, &v, 1, acc);
        }
        acc.flush_wave();
    }
}

// per-thread column part of a level's tile address inside a frame
struct ColTile
{
    uint64_t off;   // chunk*bpc + (ry0*tw + rx)*bpp
    uint32_t chunk;
};

__device__ __forceinline__ ColTile
col_tile(const FusedParams& p, int k, uint32_t Y0, uint32_t X, uint32_t bpp)
{
    const uint32_t ty = fdiv(Y0, p.dth), tx = fdiv(X, p.dtw);
    const uint32_t ry = Y0 - ty * p.th, rx = X - tx * p.tw;
    const uint32_t chunk = ty * p.ntx[k] + tx;
    return ColTile{ uint64_t(chunk) * p.bpc + uint64_t(ry * p.tw + rx) * bpp, chunk };
}

__device__ __forceinline__ void
flush_planes(const FusedParams& p, int k, uint32_t first, uint32_t g,
             uint32_t chunk, uint32_t nzmask)
{
    for (uint32_t q = 0; q < g; ++q) {
        const Ref ref = frame_ref(p, k, first + q);
        FlagAcc a;
        a.ptr = ref.flags ? ref.flags + chunk : nullptr;
        a.nz = (nzmask >> q) & 1u;
        a.tag = ref.tag;
        a.flush_wave();
    }
}

template<typename T, int M, int NTM>
__global__ __launch_bounds__(256) void
fused_pyramid_3d(const FusedParams p)
{
    // NTM: compile-time nontemporal policy, as fused_pyramid_strip
    constexpr int VEC = 16 / sizeof(T);
    constexpr int HV = VEC / 2;
    constexpr int QV = HV / 2;
    constexpr uint32_t RW = 32 * VEC;
    static_assert(QV >= 1, "2x2x2 fused kernel needs <= 4-byte pixels");
    __shared__ __attribute__((aligned(16)))
    T lds_a[kMaxPlanes3d / 2 * (kMaxRegionRows / 8) * (RW / 8)];
    __shared__ __attribute__((aligned(16)))
    T lds_b[kMaxPlanes3d / 2 * (kMaxRegionRows / 4) * (RW / 4)];

    const uint32_t nreg = p.nbx_in * p.nby_in;
    const uint32_t blk = region_of_block(p);
    const uint32_t grp = fdiv(blk, p.d_nreg_in);
    const uint32_t r = blk - grp * nreg;
    const uint32_t by = fdiv(r, p.d_nbx_in);
    const uint32_t y0 = by << p.rh_log2;
    const uint32_t x0 = (r - by * p.nbx_in) * RW;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t rp = threadIdx.x >> 5;
    const uint32_t cv = threadIdx.x & 31;
    const uint32_t npass = 1u << (p.rh_log2 - 4);
    const uint32_t G = p.G;
    const uint32_t z1 = (p.zmask >> 1) & 1u, z2 = (p.zmask >> 2) & 1u;
    const uint32_t g1 = G >> z1, g2 = g1 >> z2;
    const uint32_t trow = p.tw * uint32_t(sizeof(T));
    const bool l2 = p.n_fused >= 2;
    T* lds_l2 = p.n_fused >= 3 ? lds_b : nullptr;
    const uint32_t l2_rows = (1u << p.rh_log2) >> 2;

    const ColTile c0 = col_tile(p, 0, y0, x0 + cv * VEC, sizeof(T));
    const ColTile c1 = col_tile(p, 1, y0 >> 1, (x0 >> 1) + cv * HV, sizeof(T));
    const ColTile c2 = col_tile(p, 2, y0 >> 2, (x0 >> 2) + cv * QV, sizeof(T));
    uint32_t nz0 = 0, nz1 = 0, nz2 = 0;

    T h1[HV], h2[QV]; // earlier planes of the current z pairs
    // units = (pass, plane) pairs in pass-major order, processed in order
    // (z pairs); the rows of the next two units are in flight while one is
    // reduced
    const uint32_t units = npass * G;
    uint4 ca, cb, na{}, nb{};
    load_pass<NTM>(p, grp * G, y0, x0, 0, sizeof(T), ca, cb);
    if (units > 1)
        load_pass<NTM>(p, grp * G + (1 % G), y0, x0, 1 / G, sizeof(T), na, nb);
    for (uint32_t u = 0; u < units; ++u) {
        const uint32_t pass = u / G, pl = u - pass * G;
        uint4 fa{}, fb{};
        if (u + 2 < units) {
            const uint32_t pn = (u + 2) / G;
            load_pass<NTM>(p, grp * G + (u + 2 - pn * G), y0, x0, pn, sizeof(T), fa, fb);
        }
        // level 0: this plane's tile rows
        const Ref f0 = frame_ref(p, 0, grp * G + pl);
        if (f0.tiles) {
            const uint32_t dy = pass * 16 + 2 * rp;
            st16<(NTM & 2) != 0>(f0.tiles + c0.off + uint64_t(dy) * trow, ca);
            st16<(NTM & 2) != 0>(f0.tiles + c0.off + uint64_t(dy + 1) * trow, cb);
            if (((ca.x | ca.y | ca.z | ca.w) | (cb.x | cb.y | cb.z | cb.w)) != 0u)
                nz0 |= 1u << pl;
        }
        if (p.n_fused >= 1) {
            T r0[VEC], r1[VEC], o[HV];
            __builtin_memcpy(r0, &ca, 16);
            __builtin_memcpy(r1, &cb, 16);
#pragma unroll
            for (int i = 0; i < HV; ++i)
                o[i] = reduce4<M, T>(r0[2 * i], r0[2 * i + 1], r1[2 * i], r1[2 * i + 1]);
            bool emit1 = true;
            uint32_t q1 = pl;
            if (z1) {
                if ((pl & 1u) == 0) {
#pragma unroll
                    for (int i = 0; i < HV; ++i)
                        h1[i] = o[i];
                    emit1 = false;
                } else {
#pragma unroll
                    for (int i = 0; i < HV; ++i)
                        o[i] = reduce2<M, T>(h1[i], o[i]);
                    q1 = pl >> 1;
                }
            }
            if (emit1) {
                const Ref f1 = frame_ref(p, 1, grp * g1 + q1);
                if (f1.tiles) {
                    store_vec<T, HV, (NTM & 4) != 0>(
                      f1.tiles + c1.off + uint64_t(pass * 8 + rp) * trow, o);
                    if (any_nonzero<T, HV>(o))
                        nz1 |= 1u << q1;
                }
                if (l2) {
                    uint2 mine, below;
                    __builtin_memcpy(&mine, o, 8);
                    below.x = __shfl_xor(mine.x, 32);
                    below.y = __shfl_xor(mine.y, 32);
                    T b[HV], q[QV];
                    __builtin_memcpy(b, &below, 8);
#pragma unroll
                    for (int j = 0; j < QV; ++j)
                        q[j] = reduce4<M, T>(o[2 * j], o[2 * j + 1], b[2 * j], b[2 * j + 1]);
                    bool emit2 = true;
                    uint32_t q2 = q1;
                    if (z2) {
                        if ((q1 & 1u) == 0) {
#pragma unroll
                            for (int j = 0; j < QV; ++j)
                                h2[j] = q[j];
                            emit2 = false;
                        } else {
#pragma unroll
                            for (int j = 0; j < QV; ++j)
                                q[j] = reduce2<M, T>(h2[j], q[j]);
                            q2 = q1 >> 1;
                        }
                    }
                    if (emit2 && lane < 32) {
                        const uint32_t row2 = pass * 4 + (rp >> 1);
                        const Ref f2 = frame_ref(p, 2, grp * g2 + q2);
                        if (f2.tiles) {
                            store_vec<T, QV, (NTM & 4) != 0>(
                              f2.tiles + c2.off + uint64_t(row2) * trow, q);
                            if (any_nonzero<T, QV>(q))
                                nz2 |= 1u << q2;
                        }
                        if (lds_l2) {
#pragma unroll
                            for (int j = 0; j < QV; ++j)
                                lds_l2[q2 * l2_rows * (RW / 4) + row2 * (RW / 4) + cv * QV + j] = q[j];
                        }
                    }
                }
            }
        }
        ca = na;
        cb = nb;
        na = fa;
        nb = fb;
    }
    flush_planes(p, 0, grp * G, G, c0.chunk, nz0);
    if (p.n_fused >= 1)
        flush_planes(p, 1, grp * g1, g1, c1.chunk, nz1);
    if (l2)
        flush_planes(p, 2, grp * g2, g2, c2.chunk, nz2);

    // levels >= 3 per plane through LDS (level-2 planes are in lds_b, plane
    // stride (RH/4) x (RW/4))
    if (p.n_fused >= 3) {
        __syncthreads();
        deep3d_level<T, M, 3, RW>(p, grp, y0, x0, lds_b, lds_a, g2);
        uint32_t g = g2 >> ((p.zmask >> 3) & 1u);
        if (p.n_fused >= 4) {
            __syncthreads();
            deep3d_level<T, M, 4, RW>(p, grp, y0, x0, lds_a, lds_b, g);
            g >>= (p.zmask >> 4) & 1u;
        }
        if (p.n_fused >= 5) {
            __syncthreads();
            deep3d_level<T, M, 5, RW>(p, grp, y0, x0, lds_b, lds_a, g);
            g >>= (p.zmask >> 5) & 1u;
        }
        if (p.n_fused >= 6) {
            __syncthreads();
            deep3d_level<T, M, 6, RW>(p, grp, y0, x0, lds_a, lds_b, g);
        }
    }
}

// ---------------------------------------------------------------------------
// 2x2x2 pyramid with the strip kernel's register cascade (64-row interior
// regions, pixels <= 4 B, at most 4 fused levels).  One workgroup owns one
// region of G consecutive planes and walks them in order.  Per plane, wave w
// holds the region's rows [16w, 16w+16) as the strip kernel does: level 0 is
// stored from registers, level 1 is a 2x2 in registers, level 2 meets the
// row below through a lane^32 swap, levels 3-4 combine rows the lane already
// holds.  A z-halving level k keeps its earlier plane's XY result in
// registers (h1..h4) and emits mean2(earlier, later) on the odd plane
// (downsampler.cpp:366-385, average_two_frames :208-246), so the cascade
// needs no LDS and no barrier.  NTM as fused_pyramid_strip.  Host
// guarantees as fused_pyramid_3d, plus rh_log2 == 6 and n_fused <= 4.
// XY: the planes are in acquisition order (XY-transposed storage order,
// array.cpp:488-534): each plane's region comes through load_region_xy, the
// strip kernel's LDS transpose (a barrier per plane; no prefetch).
// ---------------------------------------------------------------------------
template<typename T, int M, int NTM, int PF, bool XY = false>
__global__ __launch_bounds__(256) void
fused_pyramid_strip3d(const FusedParams p)
{
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    constexpr int VEC = 16 / sizeof(T);
    constexpr int HV = VEC / 2;
    constexpr int QV = VEC / 4;
    constexpr uint32_t RW = 32 * VEC;
    static_assert(QV >= 1, "strip 3-D kernel needs <= 4-byte pixels");
    constexpr int N3 = QV >= 2 ? QV / 2 : 1;
    constexpr int S3 = QV >= 2 ? 1 : 2;
    constexpr int N4 = N3 >= 2 ? N3 / 2 : 1;
    constexpr int S4 = N3 >= 2 ? S3 : 2 * S3;

    const uint32_t nreg = p.nbx_in * p.nby_in;
    const uint32_t blk = region_of_block(p);
    const uint32_t grp = fdiv(blk, p.d_nreg_in);
    const uint32_t r = blk - grp * nreg;
    uint32_t by, bx;
    region_xy(p, r, by, bx, true);
    const uint32_t y0 = by << 6;
    const uint32_t x0 = bx * RW;
    const uint32_t w = threadIdx.x >> 6;
    const uint32_t hw = (threadIdx.x >> 5) & 1u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t cv = threadIdx.x & 31u;
    const uint32_t trow = p.tw * uint32_t(sizeof(T));
    const uint32_t nf = p.n_fused;
    const uint32_t G = p.G;
    const uint32_t zm = p.zmask;
    const uint32_t ry = 16 * w + 2 * hw;
    const uint64_t row = uint64_t(p.W[0]) * sizeof(T);
    const uint8_t* src0 = XY ? p.src
                             : p.src + uint64_t(grp * G) * p.src_stride +
                                 uint64_t(y0 + ry) * row + uint64_t(x0 + cv * VEC) * sizeof(T);
    const bool v3ok = lane < 32 && (cv % S3) == 0;
    const bool v4ok = lane < 32 && (cv % S4) == 0;

    // earlier planes of the z pairs, packed (a lane's level-1 row is 8 B, its
    // level-2 row 4 B): 16 VGPRs instead of 48 for u8
    uint2 h1[4];
    uint32_t h2[4];
    T h3[2][N3], h4[N4];
    const uint32_t g1 = G >> ((zm >> 1) & 1u);
    const uint32_t g2 = g1 >> ((zm >> 2) & 1u);
    const uint32_t g3 = g2 >> ((zm >> 3) & 1u);
    const uint32_t g4 = g3 >> ((zm >> 4) & 1u);
    // plane pl's rows are in ra/rb; the next plane's loads are issued as soon
    // as this plane's level-0 stores and level-1 sums no longer need them, so
    // they are in flight while levels 1-4 are formed and stored
    uint4 ra[4], rb[4];
    auto load_plane = [&](uint32_t pl) {
        if constexpr (XY) {
            if (pl > 0)
                __syncthreads(); // every wave has gathered the previous plane
            // opaque per plane: the loop-invariant LDS / global addresses of
            // the transpose are recomputed, not hoisted (and held) across
            // the plane loop
            uint32_t tid = threadIdx.x, ryo = ry, cvo = cv;
            asm volatile("" : "+v"(tid), "+v"(ryo), "+v"(cvo));
            load_region_xy<T, NTM>(p, grp * G + pl, y0, x0, ryo, cvo, ra, rb, tid);
            return;
        }
        const uint8_t* s = src0 + uint64_t(pl) * p.src_stride;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4v a = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(4 * i) * row);
            const u32x4v b = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(4 * i + 1) * row);
            ra[i] = uint4{ a.x, a.y, a.z, a.w };
            rb[i] = uint4{ b.x, b.y, b.z, b.w };
        }
    };
    if (PF)
        load_plane(0);
    for (uint32_t pl = 0; pl < G; ++pl) {
        if (!PF)
            load_plane(pl);
        // which levels emit a frame at this plane, and its index there (a
        // z-halving level emits on the later plane of each pair); uniform
        uint32_t i1 = pl, i2, i3, i4;
        bool e1 = nf >= 1, e2, e3, e4;
        if (zm & 2u) {
            e1 = e1 && (i1 & 1u);
            i1 >>= 1;
        }
        i2 = i1;
        e2 = e1 && nf >= 2;
        if (zm & 4u) {
            e2 = e2 && (i2 & 1u);
            i2 >>= 1;
        }
        i3 = i2;
        e3 = e2 && nf >= 3;
        if (zm & 8u) {
            e3 = e3 && (i3 & 1u);
            i3 >>= 1;
        }
        i4 = i3;
        e4 = e3 && nf >= 4;
        if (zm & 16u) {
            e4 = e4 && (i4 & 1u);
            i4 >>= 1;
        }
        // level 0
        {
            FastTile t0 = fast_tile<T>(p, 0, grp * G + pl, y0 + ry, x0 + cv * VEC);
            if (t0.p) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    gstore<(NTM & 2) != 0>(t0.p + uint64_t(4 * i) * trow,
                                           u32x4v{ ra[i].x, ra[i].y, ra[i].z, ra[i].w });
                    gstore<(NTM & 2) != 0>(t0.p + uint64_t(4 * i + 1) * trow,
                                           u32x4v{ rb[i].x, rb[i].y, rb[i].z, rb[i].w });
                    t0.nz |= ((ra[i].x | ra[i].y | ra[i].z | ra[i].w) |
                              (rb[i].x | rb[i].y | rb[i].z | rb[i].w)) != 0u;
                }
            }
            flush_tile_flag(t0);
        }
        // level-1 2x2 sums of this plane (8 B per row pair)
        uint2 o1[4];
        if (nf >= 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                T r0[VEC], r1[VEC], o[HV];
                __builtin_memcpy(r0, &ra[i], 16);
                __builtin_memcpy(r1, &rb[i], 16);
#pragma unroll
                for (int j = 0; j < HV; ++j)
                    o[j] = reduce4<M, T>(r0[2 * j], r0[2 * j + 1], r1[2 * j], r1[2 * j + 1]);
                __builtin_memcpy(&o1[i], o, 8);
            }
        }
        if (PF && pl + 1 < G)
            load_plane(pl + 1);
        if (nf < 1)
            continue;
        // levels 1-2, one level-1 row (8w + hw + 2i) at a time
        FastTile t1{}, t2{};
        if (e1)
            t1 = fast_tile<T>(p, 1, grp * g1 + i1, (y0 >> 1) + 8 * w + hw, (x0 >> 1) + cv * HV);
        if (e2 && lane < 32)
            t2 = fast_tile<T>(p, 2, grp * g2 + i2, (y0 >> 2) + 4 * w, (x0 >> 2) + cv * QV);
        uint32_t q2w[4]; // level-2 rows 4w + i of this lane, packed
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            T o[HV];
            __builtin_memcpy(o, &o1[i], 8);
            if (zm & 2u) {
                if (!e1) {
                    __builtin_memcpy(&h1[i], o, 8);
                    continue;
                }
                T a[HV];
                __builtin_memcpy(a, &h1[i], 8);
#pragma unroll
                for (int j = 0; j < HV; ++j)
                    o[j] = reduce2<M, T>(a[j], o[j]);
            }
            if (t1.p) {
                gstore_px<T, HV, (NTM & 4) != 0>(t1.p + uint64_t(2 * i) * trow, o);
                t1.nz |= any_nonzero<T, HV>(o);
            }
            if (nf < 2)
                continue;
            uint2 mine, below;
            __builtin_memcpy(&mine, o, 8);
            below.x = __shfl_xor(mine.x, 32);
            below.y = __shfl_xor(mine.y, 32);
            T b[HV], q[QV];
            __builtin_memcpy(b, &below, 8);
#pragma unroll
            for (int j = 0; j < QV; ++j)
                q[j] = reduce4<M, T>(o[2 * j], o[2 * j + 1], b[2 * j], b[2 * j + 1]);
            if (zm & 4u) {
                if (!e2) {
                    __builtin_memcpy(&h2[i], q, 4);
                    continue;
                }
                T a[QV];
                __builtin_memcpy(a, &h2[i], 4);
#pragma unroll
                for (int j = 0; j < QV; ++j)
                    q[j] = reduce2<M, T>(a[j], q[j]);
            }
            if (t2.p) {
                gstore_px<T, QV, (NTM & 4) != 0>(t2.p + uint64_t(i) * trow, q);
                t2.nz |= any_nonzero<T, QV>(q);
            }
            __builtin_memcpy(&q2w[i], q, 4);
        }
        flush_tile_flag(t1);
        flush_tile_flag(t2);
        if (!e2 || nf < 3)
            continue;
        // level 3: rows 2w + rr from level-2 rows 2rr, 2rr+1 of this lane
        T v3[2][N3];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            T a[QV], c[QV];
            __builtin_memcpy(a, &q2w[2 * rr], 4);
            __builtin_memcpy(c, &q2w[2 * rr + 1], 4);
            if constexpr (QV >= 2) {
#pragma unroll
                for (int j = 0; j < N3; ++j)
                    v3[rr][j] = reduce4<M, T>(a[2 * j], a[2 * j + 1], c[2 * j], c[2 * j + 1]);
            } else {
                const T ar = shfl_down_t(a[0], 1), cr = shfl_down_t(c[0], 1);
                v3[rr][0] = reduce4<M, T>(a[0], ar, c[0], cr);
            }
        }
        if (zm & 8u) {
            if (!e3) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr)
#pragma unroll
                    for (int j = 0; j < N3; ++j)
                        h3[rr][j] = v3[rr][j];
                continue;
            }
#pragma unroll
            for (int rr = 0; rr < 2; ++rr)
#pragma unroll
                for (int j = 0; j < N3; ++j)
                    v3[rr][j] = reduce2<M, T>(h3[rr][j], v3[rr][j]);
        }
        {
            FastTile t3{};
            if (v3ok)
                t3 = fast_tile<T>(p, 3, grp * g3 + i3, (y0 >> 3) + 2 * w,
                                  (x0 >> 3) + (cv / S3) * N3);
            if (t3.p) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    gstore_px<T, N3, false>(t3.p + uint64_t(rr) * trow, v3[rr]);
                    t3.nz |= any_nonzero<T, N3>(v3[rr]);
                }
            }
            flush_tile_flag(t3);
        }
        if (nf < 4)
            continue;
        // level 4: row w
        T v4[N4];
        if constexpr (N3 >= 2) {
#pragma unroll
            for (int j = 0; j < N4; ++j)
                v4[j] = reduce4<M, T>(v3[0][2 * j], v3[0][2 * j + 1], v3[1][2 * j],
                                      v3[1][2 * j + 1]);
        } else {
            const T ar = shfl_down_t(v3[0][0], S3), cr = shfl_down_t(v3[1][0], S3);
            v4[0] = reduce4<M, T>(v3[0][0], ar, v3[1][0], cr);
        }
        if (zm & 16u) {
            if (!e4) {
#pragma unroll
                for (int j = 0; j < N4; ++j)
                    h4[j] = v4[j];
                continue;
            }
#pragma unroll
            for (int j = 0; j < N4; ++j)
                v4[j] = reduce2<M, T>(h4[j], v4[j]);
        }
        {
            FastTile t4{};
            if (v4ok)
                t4 = fast_tile<T>(p, 4, grp * g4 + i4, (y0 >> 4) + w,
                                  (x0 >> 4) + (cv / S4) * N4);
            if (t4.p) {
                gstore_px<T, N4, false>(t4.p, v4);
                t4.nz |= any_nonzero<T, N4>(v4);
            }
            flush_tile_flag(t4);
        }
    }
}


// ---------------------------------------------------------------------------
// 2x2x2 pyramids whose level 1 halves z, two planes at a time: 512 threads,
// the first 256 on plane 2j, the second 256 on plane 2j+1 of the same
// region (twice the loads in flight per workgroup, at the 2-D strip
// kernel's register count).  Both halves store their level-0 tile rows and
// form level 1 in registers; the first half hands its level-1 rows to the
// second through LDS (double-buffered by j, one barrier per pair), and the
// second half emits mean2(earlier, later) (average_two_frames,
// downsampler.cpp:208-246) and carries levels 2-4 exactly as
// fused_pyramid_strip3d does (later z pairs in registers across j).
// The default where it applies (not for XY); tuning knob 2 selects
// fused_pyramid_strip3d.  PF: pair j+1's loads are issued while pair j's
// levels 1-4 are formed (1.1-1.3% faster on C4, same stage,
// profiles/r05_c4_prefetch_ab.txt; knob 131072 turns it off, 107 VGPRs with
// it, 87 without).  WPE = 4 waves per SIMD (two 8-wave workgroups per
// CU): the register budget (128) holds the whole cascade with no scratch.
// The round-4 build ran 6 (80 VGPRs) and spilled 32 B per lane of u16 MEAN
// to scratch every pair -- 4.7% more HBM writes than the algorithmic bytes
// (profiles/r05_c4_pmc.json against r05_c4-single); knob 65536 keeps it for
// A/B.  XY: acquisition-order planes, each half through load_region_xy with
// its own 32 KiB LDS tile (2 x 32 KiB + the 16 KiB exchange = 80 KiB per
// workgroup); it spills even at 4 waves, so XY stages run the single-plane
// kernel unless knob 65536 asks for this one.
// ---------------------------------------------------------------------------
template<typename T, int M, int NTM, bool XY = false, int WPE = 4, int PF = 1>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE))) void
fused_pyramid_strip3d_pair(const FusedParams p)
{
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    constexpr int VEC = 16 / sizeof(T);
    constexpr int HV = VEC / 2;
    constexpr int QV = VEC / 4;
    constexpr uint32_t RW = 32 * VEC;
    static_assert(QV >= 1, "strip 3-D kernel needs <= 4-byte pixels");
    constexpr int N3 = QV >= 2 ? QV / 2 : 1;
    constexpr int S3 = QV >= 2 ? 1 : 2;
    constexpr int N4 = N3 >= 2 ? N3 / 2 : 1;
    constexpr int S4 = N3 >= 2 ? S3 : 2 * S3;
    __shared__ uint2 xch[2][4][256]; // level-1 rows of plane 2j, by j parity

    const uint32_t nreg = p.nbx_in * p.nby_in;
    const uint32_t blk = region_of_block(p);
    const uint32_t grp = fdiv(blk, p.d_nreg_in);
    const uint32_t r = blk - grp * nreg;
    uint32_t by, bx;
    region_xy(p, r, by, bx, true);
    const uint32_t y0 = by << 6;
    const uint32_t x0 = bx * RW;
    const uint32_t half = threadIdx.x >> 8;
    const uint32_t t = threadIdx.x & 255u;
    const uint32_t w = t >> 6;
    const uint32_t hw = (t >> 5) & 1u;
    const uint32_t lane = t & 63u;
    const uint32_t cv = t & 31u;
    const uint32_t trow = p.tw * uint32_t(sizeof(T));
    const uint32_t nf = p.n_fused;
    const uint32_t G = p.G;
    const uint32_t zm = p.zmask; // bit 1 set (host)
    const uint32_t ry = 16 * w + 2 * hw;
    const uint64_t row = uint64_t(p.W[0]) * sizeof(T);
    const uint8_t* src0 = XY ? p.src
                             : p.src + uint64_t(grp * G + half) * p.src_stride +
                                 uint64_t(y0 + ry) * row + uint64_t(x0 + cv * VEC) * sizeof(T);
    const bool v3ok = lane < 32 && (cv % S3) == 0;
    const bool v4ok = lane < 32 && (cv % S4) == 0;
    uint32_t h2[4];
    T h3[2][N3], h4[N4];
    const uint32_t g1 = G >> 1;
    const uint32_t g2 = g1 >> ((zm >> 2) & 1u);
    const uint32_t g3 = g2 >> ((zm >> 3) & 1u);
    const uint32_t g4 = g3 >> ((zm >> 4) & 1u);

    // this half's plane of pair jj into ra/rb; PF: pair j+1's loads are
    // issued as soon as pair j's level-0 stores and level-1 sums no longer
    // need them, so they are in flight across the exchange barrier and
    // levels 1-4 (not for XY, whose loads go through LDS behind barriers)
    uint4 ra[4], rb[4];
    auto load_pair = [&](uint32_t jj) {
        const uint8_t* s = src0 + uint64_t(2 * jj) * p.src_stride;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const u32x4v a = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(4 * i) * row);
            const u32x4v b = gload<(NTM & 1) != 0, u32x4v>(s + uint64_t(4 * i + 1) * row);
            ra[i] = uint4{ a.x, a.y, a.z, a.w };
            rb[i] = uint4{ b.x, b.y, b.z, b.w };
        }
    };
    if constexpr (!XY && PF)
        load_pair(0);
    for (uint32_t j = 0; 2 * j < G; ++j) {
        const uint32_t pl = 2 * j + half;
        if constexpr (XY) {
            // the previous pair's gathers are behind the level-1 exchange's
            // barrier; the transpose addresses are recomputed per pair
            uint32_t tid = t, ryo = ry, cvo = cv;
            asm volatile("" : "+v"(tid), "+v"(ryo), "+v"(cvo));
            load_region_xy<T, NTM, 2>(p, grp * G + pl, y0, x0, ryo, cvo, ra, rb, tid, half);
        } else if constexpr (!PF) {
            load_pair(j);
        }
        // level 0: both halves
        {
            FastTile t0 = fast_tile<T>(p, 0, grp * G + pl, y0 + ry, x0 + cv * VEC);
            if (t0.p) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    gstore<(NTM & 2) != 0>(t0.p + uint64_t(4 * i) * trow,
                                           u32x4v{ ra[i].x, ra[i].y, ra[i].z, ra[i].w });
                    gstore<(NTM & 2) != 0>(t0.p + uint64_t(4 * i + 1) * trow,
                                           u32x4v{ rb[i].x, rb[i].y, rb[i].z, rb[i].w });
                    t0.nz |= ((ra[i].x | ra[i].y | ra[i].z | ra[i].w) |
                              (rb[i].x | rb[i].y | rb[i].z | rb[i].w)) != 0u;
                }
            }
            flush_tile_flag(t0);
        }
        // level-1 2x2 sums of this half's plane
        uint2 o1[4];
        if (nf >= 1) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                T r0[VEC], r1[VEC], o[HV];
                __builtin_memcpy(r0, &ra[i], 16);
                __builtin_memcpy(r1, &rb[i], 16);
#pragma unroll
                for (int q = 0; q < HV; ++q)
                    o[q] = reduce4<M, T>(r0[2 * q], r0[2 * q + 1], r1[2 * q], r1[2 * q + 1]);
                __builtin_memcpy(&o1[i], o, 8);
            }
        }
        if constexpr (!XY && PF) {
            if (2 * (j + 1) < G)
                load_pair(j + 1);
        }
        if (nf < 1)
            continue;
        if (half == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                xch[j & 1][i][t] = o1[i];
        }
        __syncthreads();
        if (half == 0)
            continue;
        // second half: the pair's level 1, then levels 2-4 as strip3d with
        // the level-1 frame index j (the odd plane of the pair emits)
        uint32_t i2 = j, i3, i4;
        bool e2 = nf >= 2, e3, e4;
        if (zm & 4u) {
            e2 = e2 && (i2 & 1u);
            i2 >>= 1;
        }
        i3 = i2;
        e3 = e2 && nf >= 3;
        if (zm & 8u) {
            e3 = e3 && (i3 & 1u);
            i3 >>= 1;
        }
        i4 = i3;
        e4 = e3 && nf >= 4;
        if (zm & 16u) {
            e4 = e4 && (i4 & 1u);
            i4 >>= 1;
        }
        FastTile t1 = fast_tile<T>(p, 1, grp * g1 + j, (y0 >> 1) + 8 * w + hw,
                                   (x0 >> 1) + cv * HV);
        FastTile t2{};
        if (e2 && lane < 32)
            t2 = fast_tile<T>(p, 2, grp * g2 + i2, (y0 >> 2) + 4 * w, (x0 >> 2) + cv * QV);
        uint32_t q2w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            T o[HV], a[HV];
            __builtin_memcpy(o, &o1[i], 8);
            const uint2 e = xch[j & 1][i][t];
            __builtin_memcpy(a, &e, 8);
#pragma unroll
            for (int q = 0; q < HV; ++q)
                o[q] = reduce2<M, T>(a[q], o[q]);
            if (t1.p) {
                gstore_px<T, HV, (NTM & 4) != 0>(t1.p + uint64_t(2 * i) * trow, o);
                t1.nz |= any_nonzero<T, HV>(o);
            }
            if (nf < 2)
                continue;
            uint2 mine, below;
            __builtin_memcpy(&mine, o, 8);
            below.x = __shfl_xor(mine.x, 32);
            below.y = __shfl_xor(mine.y, 32);
            T b[HV], q[QV];
            __builtin_memcpy(b, &below, 8);
#pragma unroll
            for (int k = 0; k < QV; ++k)
                q[k] = reduce4<M, T>(o[2 * k], o[2 * k + 1], b[2 * k], b[2 * k + 1]);
            if (zm & 4u) {
                if (!e2) {
                    __builtin_memcpy(&h2[i], q, 4);
                    continue;
                }
                T hq[QV];
                __builtin_memcpy(hq, &h2[i], 4);
#pragma unroll
                for (int k = 0; k < QV; ++k)
                    q[k] = reduce2<M, T>(hq[k], q[k]);
            }
            if (t2.p) {
                gstore_px<T, QV, (NTM & 4) != 0>(t2.p + uint64_t(i) * trow, q);
                t2.nz |= any_nonzero<T, QV>(q);
            }
            __builtin_memcpy(&q2w[i], q, 4);
        }
        flush_tile_flag(t1);
        flush_tile_flag(t2);
        if (!e2 || nf < 3)
            continue;
        T v3[2][N3];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            T a[QV], c[QV];
            __builtin_memcpy(a, &q2w[2 * rr], 4);
            __builtin_memcpy(c, &q2w[2 * rr + 1], 4);
            if constexpr (QV >= 2) {
#pragma unroll
                for (int k = 0; k < N3; ++k)
                    v3[rr][k] = reduce4<M, T>(a[2 * k], a[2 * k + 1], c[2 * k], c[2 * k + 1]);
            } else {
                const T ar = shfl_down_t(a[0], 1), cr = shfl_down_t(c[0], 1);
                v3[rr][0] = reduce4<M, T>(a[0], ar, c[0], cr);
            }
        }
        if (zm & 8u) {
            if (!e3) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr)
#pragma unroll
                    for (int k = 0; k < N3; ++k)
                        h3[rr][k] = v3[rr][k];
                continue;
            }
#pragma unroll
            for (int rr = 0; rr < 2; ++rr)
#pragma unroll
                for (int k = 0; k < N3; ++k)
                    v3[rr][k] = reduce2<M, T>(h3[rr][k], v3[rr][k]);
        }
        {
            FastTile t3{};
            if (v3ok)
                t3 = fast_tile<T>(p, 3, grp * g3 + i3, (y0 >> 3) + 2 * w,
                                  (x0 >> 3) + (cv / S3) * N3);
            if (t3.p) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    gstore_px<T, N3, false>(t3.p + uint64_t(rr) * trow, v3[rr]);
                    t3.nz |= any_nonzero<T, N3>(v3[rr]);
                }
            }
            flush_tile_flag(t3);
        }
        if (nf < 4)
            continue;
        T v4[N4];
        if constexpr (N3 >= 2) {
#pragma unroll
            for (int k = 0; k < N4; ++k)
                v4[k] = reduce4<M, T>(v3[0][2 * k], v3[0][2 * k + 1], v3[1][2 * k],
                                      v3[1][2 * k + 1]);
        } else {
            const T ar = shfl_down_t(v3[0][0], S3), cr = shfl_down_t(v3[1][0], S3);
            v4[0] = reduce4<M, T>(v3[0][0], ar, v3[1][0], cr);
        }
        if (zm & 16u) {
            if (!e4) {
#pragma unroll
                for (int k = 0; k < N4; ++k)
                    h4[k] = v4[k];
                continue;
            }
#pragma unroll
            for (int k = 0; k < N4; ++k)
                v4[k] = reduce2<M, T>(h4[k], v4[k]);
        }
        {
            FastTile t4{};
            if (v4ok)
                t4 = fast_tile<T>(p, 4, grp * g4 + i4, (y0 >> 4) + w,
                                  (x0 >> 4) + (cv / S4) * N4);
            if (t4.p) {
                gstore_px<T, N4, false>(t4.p, v4);
                t4.nz |= any_nonzero<T, N4>(v4);
            }
            flush_tile_flag(t4);
        }
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
    acc.tag = op.tag;
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
            put_tile<T, 1>(tiles_of(g), g.base + op.tile_off,
                           g.flags + op.flag_off, Y, X, &v, 1, acc);
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

// z-slab assembly (Stage::import_frames): the tiles of frames [f0, f0 +
// gridDim.y) of one chunk layer copied from another stage's resident layer
// (a peer device's HBM over xGMI, or the same device) -- or zeroed when src
// is null -- at the same offsets (same geometry).  Block (x, f): tile
// blockIdx.x of frame f0 + blockIdx.y; the first lane also carries the
// chunk's has_data tag over.
__global__ __launch_bounds__(256) void
import_frame_tiles(uint8_t* dst, const uint8_t* src, const uint64_t* tab_off,
                   const uint32_t* tab_grp, uint32_t f0, uint64_t pitch, uint32_t tile_bytes,
                   uint32_t* dst_flags, const uint32_t* src_flags, uint32_t tag)
{
    const uint32_t f = f0 + blockIdx.y, t = blockIdx.x;
    const uint64_t off = tab_off[f] + uint64_t(t) * pitch;
    if ((tile_bytes & 15u) == 0 && (off & 15u) == 0) {
        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
        u32x4v* d = reinterpret_cast<u32x4v*>(dst + off);
        const u32x4v* s = reinterpret_cast<const u32x4v*>(src + off);
        for (uint32_t i = threadIdx.x; i < tile_bytes / 16u; i += 256)
            d[i] = src ? __builtin_nontemporal_load(s + i) : u32x4v{ 0, 0, 0, 0 };
    } else {
        for (uint32_t i = threadIdx.x; i < tile_bytes; i += 256)
            dst[off + i] = src ? src[off + i] : uint8_t(0);
    }
    if (src && threadIdx.x == 0) {
        const uint32_t c = tab_grp[f] + t;
        if (src_flags[c] == tag)
            dst_flags[c] = tag;
    }
}

// splitmix64 words (the tests' synthetic_frames stream, seed-offset): the
// placement calibration times its candidates on random frames, as the
// stage sees them, not on a constant fill.
__global__ void
fill_splitmix(uint64_t* p, uint64_t n, uint64_t seed)
{
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * 256) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = z ^ (z >> 31);
    }
}

} // namespace

hipError_t
launch_fill_random(void* p, uint64_t bytes, uint64_t seed, hipStream_t stream)
{
    const uint64_t n = bytes / 8;
    if (n == 0)
        return hipSuccess;
    const uint32_t grid = uint32_t(std::min<uint64_t>((n + 255) / 256, 8192));
    hipLaunchKernelGGL(fill_splitmix, dim3(grid), dim3(256), 0, stream,
                       static_cast<uint64_t*>(p), n, seed);
    return hipGetLastError();
}

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

// workgroups of the 2-D strip kernel per CU (launch_interior)
constexpr uint32_t kStripWgPerCu = 6;

// The strip kernel takes 64-row interior regions of <= 4-byte pixels when
// no level 3-4 output goes to scratch; fused_pyramid takes the rest.
template<typename T, int M>
void
launch_interior(uint32_t blocks, const FusedParams& p, hipStream_t stream)
{
    if constexpr (sizeof(T) <= 4) {
        if (p.xy) { // launch_fused_pyramid checked the strip kernel applies
            if (p.nt)
                hipLaunchKernelGGL((fused_pyramid_strip<T, M, 7, true>), dim3(blocks),
                                   dim3(256), 0, stream, p);
            else
                hipLaunchKernelGGL((fused_pyramid_strip<T, M, 0, true>), dim3(blocks),
                                   dim3(256), 0, stream, p);
            return;
        }
        if (p.rh_log2 == 6 && !(p.knobs & 128u) &&
            (p.scratch_level == 0 || p.scratch_level >= 5)) {
            // Occupancy: at most kStripWgPerCu workgroups per CU, held by
            // unused dynamic LDS (the kernel's registers would allow 8).
            // Same stage A/Bs, round 5 (profiles/r05_occupancy_cap.txt):
            // 6 per CU is 0.5-1.8% faster on C1, C2, C2-ref4 and C3 and
            // within 0.1% on C5 -- fewer streams of row reads in flight per
            // CU contend less for the memory channels.  Tuning knob bits
            // 13-15 = v: 0 the shipped cap, 1 uncapped, else v per CU.
            const uint32_t v = (p.knobs >> 13) & 7u;
            const uint32_t per_cu = v == 0 ? kStripWgPerCu : v;
            const uint32_t lds = per_cu > 1 ? (163840u / per_cu - 512u) & ~255u : 0u;
            switch (p.nt) {
                case 1:
                    hipLaunchKernelGGL((fused_pyramid_strip<T, M, 1>), dim3(blocks),
                                       dim3(256), lds, stream, p);
                    break;
                case 3:
                    hipLaunchKernelGGL((fused_pyramid_strip<T, M, 3>), dim3(blocks),
                                       dim3(256), lds, stream, p);
                    break;
                case 7:
                    hipLaunchKernelGGL((fused_pyramid_strip<T, M, 7>), dim3(blocks),
                                       dim3(256), lds, stream, p);
                    break;
                default:
                    hipLaunchKernelGGL((fused_pyramid_strip<T, M, 0>), dim3(blocks),
                                       dim3(256), lds, stream, p);
            }
            return;
        }
    }
    if (p.nt)
        hipLaunchKernelGGL((fused_pyramid<T, M, 7>), dim3(blocks), dim3(256), 0, stream, p);
    else
        hipLaunchKernelGGL((fused_pyramid<T, M, 0>), dim3(blocks), dim3(256), 0, stream, p);
}

hipError_t
launch_fused_pyramid(int dtype, int method, const FusedParams& p,
                     hipStream_t stream)
{
    if (p.n_fused > uint32_t(kMaxFused) || p.rh_log2 < 4 ||
        (1u << p.rh_log2) > uint32_t(kMaxRegionRows) || p.nbx_in > p.nbx ||
        p.nby_in > p.nby || (1u << p.rh_log2) < (1u << p.n_fused))
        return hipErrorInvalidValue;
    const uint64_t interior = uint64_t(p.n_frames) * p.nbx_in * p.nby_in;
    const uint64_t edge =
      uint64_t(p.n_frames) * (uint64_t(p.nbx) * p.nby - uint64_t(p.nbx_in) * p.nby_in);
    if (interior > 0x7fffffffull || edge > 0x7fffffffull)
        return hipErrorInvalidValue;
    // acquisition-order source: interior regions only through the strip kernel
    if (p.xy && interior &&
        !((dtype == 0 || dtype == 1 || dtype == 2 || dtype == 4 || dtype == 5 ||
           dtype == 6 || dtype == 8) &&
          p.rh_log2 == 6 &&
          !(p.knobs & 128u) && (p.scratch_level == 0 || p.scratch_level >= 5)))
        return hipErrorInvalidValue;
    const FusedParams pr = with_xcd_rotation(p, interior);
#define CALL(T, MM)                                                            \
    do {                                                                       \
        if (interior)                                                          \
            launch_interior<T, MM>(uint32_t(interior), pr, stream);            \
        if (edge)                                                              \
            hipLaunchKernelGGL((fused_pyramid_edge<T, MM>),                    \
                               dim3(uint32_t(edge)), dim3(256), 0, stream, p); \
    } while (0)
    AQZ_DISPATCH(dtype, method, CALL)
#undef CALL
    return hipGetLastError();
}

hipError_t
launch_fused_pyramid_3d(int dtype, int method, const FusedParams& p,
                        hipStream_t stream)
{
    const uint64_t blocks = uint64_t(p.n_frames / p.G) * p.nbx_in * p.nby_in;
    if (p.G == 0 || p.G > uint32_t(kMaxPlanes3d) || p.n_frames % p.G ||
        p.n_fused > uint32_t(kMaxFused) || (1u << p.rh_log2) < (1u << p.n_fused) ||
        (1u << p.rh_log2) > uint32_t(kMaxRegionRows) || blocks > 0x7fffffffull)
        return hipErrorInvalidValue;
    if (blocks == 0)
        return hipSuccess;
    // the register-cascade kernel takes 64-row regions down to 4 fused levels
    const bool strip = p.rh_log2 == 6 && p.n_fused <= 4 && !(p.knobs & 256u);
    // two planes at a time (fused_pyramid_strip3d_pair) when level 1 halves
    // z and the group holds whole pairs: 0.8-1.3% faster than one plane at a
    // time on C4, same stage (profiles/archive/r04_c4_pair_ab.txt); knob 2 keeps
    // fused_pyramid_strip3d
    // knob 65536: the round-4 pair kernels (6 waves per SIMD, spilling; the
    // pair for XY stages too)
    const bool r4 = (p.knobs & 65536u) != 0;
    const bool pair =
      strip && !(p.knobs & 2u) && (p.zmask & 2u) && p.G % 2 == 0 && (!p.xy || r4);
    // acquisition-order planes: only through the strip kernel's XY load
    if (p.xy && !(strip && dtype != 3 && dtype != 7 && dtype != 9))
        return hipErrorInvalidValue;
    const FusedParams pr = with_xcd_rotation(p, blocks);
#define CALL(T, MM)                                                            \
    do {                                                                       \
        const dim3 gd{ uint32_t(blocks), 1, 1 };                              \
        if (p.xy && pair && p.nt)                                             \
            hipLaunchKernelGGL((fused_pyramid_strip3d_pair<T, MM, 7, true>), gd, dim3(512), \
                               0, stream, pr);                                 \
        else if (p.xy && p.nt)                                                \
            hipLaunchKernelGGL((fused_pyramid_strip3d<T, MM, 7, 0, true>), gd, dim3(256), \
                               0, stream, pr);                                 \
        else if (pair && p.nt && r4)                                          \
            hipLaunchKernelGGL((fused_pyramid_strip3d_pair<T, MM, 7, false, 6, 0>), gd, \
                               dim3(512), 0, stream, pr);                      \
        else if (pair && p.nt && (p.knobs & 131072u))                         \
            hipLaunchKernelGGL((fused_pyramid_strip3d_pair<T, MM, 7, false, 4, 0>), gd, \
                               dim3(512), 0, stream, pr);                      \
        else if (pair && p.nt)                                                \
            hipLaunchKernelGGL((fused_pyramid_strip3d_pair<T, MM, 7>), gd, dim3(512), 0, \
                               stream, pr);                                    \
        else if (p.xy)                                                        \
            hipLaunchKernelGGL((fused_pyramid_strip3d<T, MM, 0, 0, true>), gd, dim3(256), \
                               0, stream, pr);                                 \
        else if (strip && p.nt && (p.knobs & 512u))                           \
            hipLaunchKernelGGL((fused_pyramid_strip3d<T, MM, 7, 0>), gd, dim3(256), 0, \
                               stream, pr);                                    \
        else if (strip && p.nt)                                               \
            hipLaunchKernelGGL((fused_pyramid_strip3d<T, MM, 7, 1>), gd, dim3(256), 0, \
                               stream, pr);                                    \
        else if (strip)                                                       \
            hipLaunchKernelGGL((fused_pyramid_strip3d<T, MM, 0, 1>), gd, dim3(256), 0, \
                               stream, pr);                                    \
        else if (p.nt)                                                        \
            hipLaunchKernelGGL((fused_pyramid_3d<T, MM, 7>), gd, dim3(256), 0,  \
                               stream, pr);                                    \
        else                                                                  \
            hipLaunchKernelGGL((fused_pyramid_3d<T, MM, 0>), gd, dim3(256), 0,  \
                               stream, pr);                                    \
    } while (0)
    switch (dtype) {
        case 0: AQZ_DISPATCH_M(uint8_t, method, CALL); break;
        case 1: AQZ_DISPATCH_M(uint16_t, method, CALL); break;
        case 2: AQZ_DISPATCH_M(uint32_t, method, CALL); break;
        case 4: AQZ_DISPATCH_M(int8_t, method, CALL); break;
        case 5: AQZ_DISPATCH_M(int16_t, method, CALL); break;
        case 6: AQZ_DISPATCH_M(int32_t, method, CALL); break;
        case 8: AQZ_DISPATCH_M(float, method, CALL); break;
        default: return hipErrorInvalidValue;
    }
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

// Y x X -> X x Y transpose of a batch of level-0 frames (Array::
// transpose_frame, array.cpp:488-504; applied before the split when the
// storage order swaps the two spatial dims, array.cpp:525-533, and the
// downsampler then sees the transposed frame).  64x64 tiles through LDS:
// both the row reads and the row writes are coalesced.  Pixels are moved as
// opaque words of their size.
template<typename W>
__global__ __launch_bounds__(256) void
transpose_frames(const W* __restrict__ src, W* __restrict__ dst, uint32_t rows,
                 uint32_t cols)
{
    __shared__ W tile[64][65];
    const uint64_t fe = uint64_t(rows) * cols;
    const W* s = src + blockIdx.z * fe;
    W* d = dst + blockIdx.z * fe;
    const uint32_t x0 = blockIdx.x * 64, y0 = blockIdx.y * 64;
    const uint32_t tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t r = ty + 4 * i;
        const uint32_t y = y0 + r, x = x0 + tx;
        if (y < rows && x < cols)
            tile[r][tx] = s[uint64_t(y) * cols + x];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t r = ty + 4 * i;
        const uint32_t oy = x0 + r, ox = y0 + tx; // output row = input column
        if (oy < cols && ox < rows)
            d[uint64_t(oy) * rows + ox] = tile[tx][r];
    }
}

hipError_t
launch_transpose_frames(const void* src, void* dst, uint32_t rows, uint32_t cols,
                        uint32_t n_frames, uint32_t bpp, hipStream_t stream)
{
    if (n_frames == 0 || rows == 0 || cols == 0)
        return hipSuccess;
    const dim3 grid((cols + 63) / 64, (rows + 63) / 64, n_frames);
    switch (bpp) {
        case 1:
            hipLaunchKernelGGL(transpose_frames<uint8_t>, grid, dim3(256), 0, stream,
                               static_cast<const uint8_t*>(src), static_cast<uint8_t*>(dst),
                               rows, cols);
            break;
        case 2:
            hipLaunchKernelGGL(transpose_frames<uint16_t>, grid, dim3(256), 0, stream,
                               static_cast<const uint16_t*>(src),
                               static_cast<uint16_t*>(dst), rows, cols);
            break;
        case 4:
            hipLaunchKernelGGL(transpose_frames<uint32_t>, grid, dim3(256), 0, stream,
                               static_cast<const uint32_t*>(src),
                               static_cast<uint32_t*>(dst), rows, cols);
            break;
        case 8:
            hipLaunchKernelGGL(transpose_frames<uint64_t>, grid, dim3(256), 0, stream,
                               static_cast<const uint64_t*>(src),
                               static_cast<uint64_t*>(dst), rows, cols);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// has_data of one chunk layer as 0/1 bytes: a chunk holds data of this layer
// when its word carries the layer's generation tag (Chunk::has_data,
// chunk.cpp:17-67)
__global__ void
flags_to_bytes(const uint32_t* flags, uint8_t* out, uint32_t n, uint32_t tag)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n)
        out[i] = flags[i] == tag ? 1 : 0;
}

hipError_t
launch_flags_to_bytes(const uint32_t* flags, uint8_t* out, uint32_t n, uint32_t tag,
                      hipStream_t stream)
{
    if (n == 0)
        return hipSuccess;
    hipLaunchKernelGGL(flags_to_bytes, dim3((n + 255) / 256), dim3(256), 0, stream,
                       flags, out, n, tag);
    return hipGetLastError();
}

hipError_t
launch_import_frames(uint8_t* dst, const uint8_t* src, const uint64_t* tab_off,
                     const uint32_t* tab_grp, uint32_t f0, uint32_t n_frames, uint32_t n_tiles,
                     uint64_t pitch, uint32_t tile_bytes, uint32_t* dst_flags,
                     const uint32_t* src_flags, uint32_t tag, hipStream_t stream)
{
    if (n_frames == 0 || n_tiles == 0)
        return hipSuccess;
    hipLaunchKernelGGL(import_frame_tiles, dim3(n_tiles, n_frames), dim3(256), 0, stream, dst,
                       src, tab_off, tab_grp, f0, pitch, tile_bytes, dst_flags, src_flags, tag);
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

} // namespace aqz
