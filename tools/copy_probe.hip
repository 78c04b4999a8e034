// Dev probe (not product): achievable HBM rates on this chip for the access
// shapes of the stage -- read-only, 1:1 copy, and 1 read : 1.33 write --
// under load/store flavours (plain, nontemporal), bytes in flight per lane
// and grid shapes.  Prints one line per variant.
//   hipcc -O3 --offload-arch=gfx950 tools/copy_probe.hip -o tools/copy_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,                  \
                    hipGetErrorString(e_));                                    \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template<bool NT>
__device__ __forceinline__ u32x4
ld(const u32x4* p)
{
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template<bool NT>
__device__ __forceinline__ void
st(u32x4* p, u32x4 v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// each workgroup: one contiguous block of U*256*16 bytes
template<int U, bool NTL, bool NTS, int MODE>
__global__ __launch_bounds__(256) void
k_stream(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
         u32x4* __restrict__ dst2, size_t nvec, unsigned* sink)
{
    const size_t base = size_t(blockIdx.x) * (U * 256) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i)
        v[i] = ld<NTL>(src + base + i * 256);
    if constexpr (MODE == 3) { // read 1 : write 1/3 (the pyramid-only shape)
        const size_t b2 = size_t(blockIdx.x) * (U * 256 / 3) + threadIdx.x;
#pragma unroll
        for (int i = 0; i < U / 3; ++i)
            st<NTS>(dst2 + b2 + i * 256, v[3 * i] ^ v[3 * i + 1] ^ v[3 * i + 2]);
    } else if constexpr (MODE == 0) { // read only
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < U; ++i)
            acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        if (acc == 0x12345678u)
            sink[0] = acc;
    } else {
#pragma unroll
        for (int i = 0; i < U; ++i)
            st<NTS>(dst + base + i * 256, v[i]);
        if constexpr (MODE == 2) { // + one third more written
            const size_t b2 = size_t(blockIdx.x) * (U * 256 / 3) + threadIdx.x;
#pragma unroll
            for (int i = 0; i < U / 3; ++i) {
                u32x4 w = v[3 * i] ^ v[3 * i + 1];
                st<NTS>(dst2 + b2 + i * 256, w);
            }
        }
    }
}

template<int U, bool NTL, bool NTS, int MODE>
void
run(const char* name, const u32x4* src, u32x4* dst, u32x4* dst2, size_t bytes,
    unsigned* sink, int ring)
{
    const size_t nvec = bytes / 16;
    const unsigned grid = unsigned(nvec / (U * 256));
    const size_t per = size_t(grid) * U * 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w)
        k_stream<U, NTL, NTS, MODE><<<grid, 256>>>(src, dst, dst2, nvec, sink);
    const int reps = 20;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) {
        const int i = r % ring;
        k_stream<U, NTL, NTS, MODE><<<grid, 256>>>(src + i * per, dst, dst2, nvec, sink);
    }
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double rd = double(per) * 16;
    const double wr = MODE == 0 ? 0 : rd * (MODE == 2 ? 4.0 / 3.0 : MODE == 3 ? 1.0 / 3.0 : 1.0);
    printf("%-28s U=%d grid=%7u  %.4f ms  read %.0f GB/s  bus %.0f GB/s\n", name, U,
           grid, ms, rd / ms / 1e6, (rd + wr) / ms / 1e6);
}

int
main()
{
    const size_t bytes = size_t(512) << 20; // per launch (64 C2 frames)
    const int ring = 4;
    void *src, *dst, *dst2;
    unsigned* sink;
    CK(hipMalloc(&src, bytes * ring));
    CK(hipMalloc(&dst, bytes));
    CK(hipMalloc(&dst2, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, bytes * ring));
    CK(hipMemset(dst, 0, bytes));
    CK(hipMemset(dst2, 0, bytes));
    auto s = (const u32x4*)src;
    auto d = (u32x4*)dst;
    auto d2 = (u32x4*)dst2;
    if (getenv("PROBE_ALLOCS")) {
        // bimodality check: the same copy into several separately
        // allocated destinations
        const int na = atoi(getenv("PROBE_ALLOCS"));
        std::vector<void*> ds(na), ds2(na);
        for (int i = 0; i < na; ++i) {
            CK(hipMalloc(&ds[i], bytes));
            CK(hipMalloc(&ds2[i], bytes));
            CK(hipMemset(ds[i], 0, bytes));
            CK(hipMemset(ds2[i], 0, bytes));
        }
        for (int rep = 0; rep < 2; ++rep)
            for (int i = 0; i < na; ++i) {
                char nm[64];
                snprintf(nm, sizeof nm, "copy+1/3 dst%d", i);
                run<6, false, false, 2>(nm, s, (u32x4*)ds[i], (u32x4*)ds2[i], bytes, sink, ring);
                snprintf(nm, sizeof nm, "copy dst%d", i);
                run<4, false, false, 1>(nm, s, (u32x4*)ds[i], (u32x4*)ds2[i], bytes, sink, ring);
            }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        run<4, false, false, 0>("read", s, d, d2, bytes, sink, ring);
        run<8, false, false, 0>("read", s, d, d2, bytes, sink, ring);
        run<4, true, false, 0>("read nt", s, d, d2, bytes, sink, ring);
        run<8, true, false, 0>("read nt", s, d, d2, bytes, sink, ring);
        run<2, false, false, 1>("copy", s, d, d2, bytes, sink, ring);
        run<4, false, false, 1>("copy", s, d, d2, bytes, sink, ring);
        run<8, false, false, 1>("copy", s, d, d2, bytes, sink, ring);
        run<4, true, false, 1>("copy ntl", s, d, d2, bytes, sink, ring);
        run<4, false, true, 1>("copy nts", s, d, d2, bytes, sink, ring);
        run<4, true, true, 1>("copy ntl nts", s, d, d2, bytes, sink, ring);
        run<8, true, true, 1>("copy ntl nts", s, d, d2, bytes, sink, ring);
        run<6, false, false, 2>("copy+1/3", s, d, d2, bytes, sink, ring);
        run<6, false, true, 2>("copy+1/3 nts", s, d, d2, bytes, sink, ring);
        run<6, true, true, 2>("copy+1/3 ntl nts", s, d, d2, bytes, sink, ring);
        run<12, false, false, 2>("copy+1/3", s, d, d2, bytes, sink, ring);
        run<6, false, false, 3>("read+1/3w", s, d, d2, bytes, sink, ring);
        run<6, true, false, 3>("read+1/3w ntl", s, d, d2, bytes, sink, ring);
        run<6, false, true, 3>("read+1/3w nts", s, d, d2, bytes, sink, ring);
        run<6, true, true, 3>("read+1/3w ntl nts", s, d, d2, bytes, sink, ring);
        run<12, true, true, 3>("read+1/3w ntl nts", s, d, d2, bytes, sink, ring);
        printf("\n");
    }
    return 0;
}
