// Dev probe (not product): do plain streaming kernels run at different
// rates in different device allocations of one process?  Allocates N
// buffers of S MiB one after another (all held), then times a read-only,
// a write-only and a copy (read buffer i, write buffer i+1) nontemporal
// streaming kernel on each, R rounds, printing GB/s per buffer.
//   hipcc --offload-arch=gfx950 -O3 tools/region_probe.hip -o tools/region_probe
//   tools/region_probe [N=12] [S=2048] [R=3]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                       \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) rd(const u32x4* __restrict__ p, size_t n, u32x4* sink)
{
    u32x4 acc = { 0, 0, 0, 0 };
    const size_t stride = size_t(gridDim.x) * 256 * 8;
    for (size_t i = size_t(blockIdx.x) * 256 * 8 + threadIdx.x; i < n; i += stride) {
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = __builtin_nontemporal_load(p + i + k * 256);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            acc ^= v[k];
    }
    if (acc.x == 0x12345678u && acc.y == 7u)
        sink[threadIdx.x] = acc;
}

__global__ void __launch_bounds__(256) wr(u32x4* __restrict__ p, size_t n)
{
    const size_t stride = size_t(gridDim.x) * 256 * 8;
    for (size_t i = size_t(blockIdx.x) * 256 * 8 + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u32x4 v = { u32x4(i).x, 1u, 2u, 3u };
            __builtin_nontemporal_store(v, p + i + k * 256);
        }
    }
}

__global__ void __launch_bounds__(256) cp(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                          size_t n)
{
    const size_t stride = size_t(gridDim.x) * 256 * 8;
    for (size_t i = size_t(blockIdx.x) * 256 * 8 + threadIdx.x; i < n; i += stride) {
        u32x4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            v[k] = __builtin_nontemporal_load(s + i + k * 256);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            __builtin_nontemporal_store(v[k], d + i + k * 256);
    }
}

int main(int argc, char** argv)
{
    const int N = argc > 1 ? atoi(argv[1]) : 12;
    const size_t S = size_t(argc > 2 ? atoi(argv[2]) : 2048) << 20;
    const int R = argc > 3 ? atoi(argv[3]) : 3;
    std::vector<u32x4*> b(N);
    for (int i = 0; i < N; ++i) {
        CK(hipMalloc(&b[i], S));
        CK(hipMemset(b[i], 0, S));
    }
    u32x4* sink;
    CK(hipMalloc(&sink, 4096));
    const size_t n = S / 16;
    const int grid = 256 * 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("buffer  ptr  read_GBs  write_GBs  copy_bus_GBs (S=%zu MiB)\n", S >> 20);
    for (int r = 0; r < R; ++r) {
        for (int i = 0; i < N; ++i) {
            float t[3];
            for (int k = 0; k < 3; ++k) {
                for (int w = 0; w < 2; ++w) { // warm + timed
                    CK(hipEventRecord(e0));
                    const int reps = w ? 5 : 1;
                    for (int q = 0; q < reps; ++q) {
                        if (k == 0)
                            rd<<<grid, 256>>>(b[i], n, sink);
                        else if (k == 1)
                            wr<<<grid, 256>>>(b[i], n);
                        else
                            cp<<<grid, 256>>>(b[i], b[(i + 1) % N], n / 2);
                    }
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    t[k] = ms / reps;
                }
            }
            printf("r%d b%02d %p %8.1f %8.1f %8.1f\n", r, i, (void*)b[i], S / t[0] / 1e6,
                   S / t[1] / 1e6, S / t[2] / 1e6);
            fflush(stdout);
        }
    }
    return 0;
}
