// Dev probe (not product): where does the allocation-dependent bimodality
// of the 1 read : 1.33 write shape come from?  
//   E1  one pool; the 1/3 destination's offset swept in 2 MiB steps
//   E2  the same at 64 KiB steps over the first 2 MiB
//   E3  the main destination's offset swept (1/3 destination fixed)
//   E4  fresh hipMalloc pairs, repeated
//   E5  nontemporal stores on each stream
// Every line: ms per 512 MiB-of-input launch, bus TB/s.
//   hipcc -O3 --offload-arch=gfx950 tools/alloc_probe.hip -o tools/alloc_probe
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
__device__ __forceinline__ void
st(u32x4* p, u32x4 v)
{
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// each workgroup: 6*256*16 B read, the same written to dst, 1/3 to dst2
template<bool NT1, bool NT2>
__global__ __launch_bounds__(256) void
k_copy13(const u32x4* __restrict__ src, u32x4* __restrict__ dst, u32x4* __restrict__ dst2)
{
    constexpr int U = 6;
    const size_t base = size_t(blockIdx.x) * (U * 256) + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i)
        v[i] = src[base + i * 256];
#pragma unroll
    for (int i = 0; i < U; ++i)
        st<NT1>(dst + base + i * 256, v[i]);
    const size_t b2 = size_t(blockIdx.x) * (U * 256 / 3) + threadIdx.x;
#pragma unroll
    for (int i = 0; i < U / 3; ++i)
        st<NT2>(dst2 + b2 + i * 256, v[3 * i] ^ v[3 * i + 1]);
}

static const size_t kBytes = size_t(512) << 20;
static const int kRing = 4;

template<bool NT1 = false, bool NT2 = false>
static float
time_copy13(const uint8_t* src, uint8_t* dst, uint8_t* dst2)
{
    const size_t nvec = kBytes / 16;
    const unsigned grid = unsigned(nvec / (6 * 256));
    const size_t per = size_t(grid) * 6 * 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto s = (const u32x4*)src;
    for (int w = 0; w < 2; ++w)
        k_copy13<NT1, NT2><<<grid, 256>>>(s, (u32x4*)dst, (u32x4*)dst2);
    const int reps = 12;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r)
        k_copy13<NT1, NT2><<<grid, 256>>>(s + (r % kRing) * per, (u32x4*)dst, (u32x4*)dst2);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

static void
line(const char* tag, long off, float ms)
{
    const double bus = double(kBytes) * (1 + 4.0 / 3.0);
    printf("%-10s %10ld  %.4f ms  bus %.2f TB/s\n", tag, off, ms, bus / ms / 1e9);
    fflush(stdout);
}

int
main()
{
    uint8_t *src, *pool;
    const size_t pool_bytes = size_t(3) << 30;
    CK(hipMalloc(&src, kBytes * kRing));
    CK(hipMalloc(&pool, pool_bytes));
    CK(hipMemset(src, 1, kBytes * kRing));
    CK(hipMemset(pool, 0, pool_bytes));
    uint8_t* dst = pool;
    uint8_t* d2base = pool + kBytes;
    const size_t MiB = size_t(1) << 20;
    // E1: 1/3 destination offset, 2 MiB steps
    for (int k = 0; k < 48; ++k)
        line("E1", long(k * 2), time_copy13(src, dst, d2base + k * 2 * MiB));
    // E2: 64 KiB steps inside the first 2 MiB
    for (int k = 0; k < 32; ++k)
        line("E2", long(k * 64), time_copy13(src, dst, d2base + k * 64 * 1024));
    // E3: main destination offset (dst2 fixed behind the sweep range)
    uint8_t* d2fixed = pool + kBytes + 200 * MiB + 128 * MiB;
    for (int k = 0; k < 32; ++k)
        line("E3", long(k * 2), time_copy13(src, pool + k * 2 * MiB, d2fixed));
    // E4: fresh allocations
    for (int i = 0; i < 10; ++i) {
        uint8_t *a, *b;
        CK(hipMalloc(&a, kBytes));
        CK(hipMalloc(&b, kBytes / 2));
        CK(hipMemset(a, 0, kBytes));
        CK(hipMemset(b, 0, kBytes / 2));
        line("E4", i, time_copy13(src, a, b));
        line("E4nts2", i, time_copy13<false, true>(src, a, b));
        line("E4nts12", i, time_copy13<true, true>(src, a, b));
        // keep them: the next pair lands elsewhere
    }
    // E5: nontemporal variants at the pool's first placement
    line("E5plain", 0, time_copy13<false, false>(src, dst, d2base));
    line("E5nts1", 0, time_copy13<true, false>(src, dst, d2base));
    line("E5nts2", 0, time_copy13<false, true>(src, dst, d2base));
    line("E5nts12", 0, time_copy13<true, true>(src, dst, d2base));
    return 0;
}
