// Block shuffle kernel (aqz::launch_shuffle_blocks) on a C2 level-0 layer
// (64 chunks x 8 MiB u16, 256 KiB blocks) against a device memcpy of the
// same bytes.
//   hipcc --offload-arch=gfx950 -O2 -std=c++20 -Iacquire-zarr_amd/csrc -Iinclude \
//     tools/shuffle_probe.cpp -Lacquire-zarr_amd -laqz_gpu \
//     -Wl,-rpath,'$ORIGIN/../acquire-zarr_amd' -o tools/shuffle_probe
#include "aqz_codec.hh"

#include <cstdio>
#include <cstdlib>

#define HIPC(x)                                                                 \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

int
main()
{
    const uint32_t n_chunks = 64, nbytes = 256 * 256 * 64 * 2, bs = 256 * 1024;
    const size_t N = size_t(n_chunks) * nbytes;
    uint8_t *src, *dst;
    HIPC(hipMalloc(&src, N));
    HIPC(hipMalloc(&dst, N));
    HIPC(hipMemset(src, 7, N));
    hipEvent_t a, b;
    HIPC(hipEventCreate(&a));
    HIPC(hipEventCreate(&b));
    for (uint32_t sh : { 1u, 2u, 0u }) {
        aqz::ShuffleParams p{ src, nbytes, n_chunks, nullptr, 0, nbytes, 2, sh, bs,
                              nbytes / bs, dst };
        HIPC(aqz::launch_shuffle_blocks(p, nullptr));
        HIPC(hipDeviceSynchronize());
        HIPC(hipEventRecord(a));
        for (int r = 0; r < 10; ++r)
            HIPC(aqz::launch_shuffle_blocks(p, nullptr));
        HIPC(hipEventRecord(b));
        HIPC(hipEventSynchronize(b));
        float ms;
        HIPC(hipEventElapsedTime(&ms, a, b));
        std::printf("shuffle %u: %.3f ms per 512 MiB layer, %.0f GB/s read+write\n", sh, ms / 10,
                    2.0 * N / (ms / 10) / 1e6);
    }
    HIPC(hipEventRecord(a));
    for (int r = 0; r < 10; ++r)
        HIPC(hipMemcpyAsync(dst, src, N, hipMemcpyDeviceToDevice));
    HIPC(hipEventRecord(b));
    HIPC(hipEventSynchronize(b));
    float ms;
    HIPC(hipEventElapsedTime(&ms, a, b));
    std::printf("memcpy D2D: %.3f ms per layer, %.0f GB/s read+write\n", ms / 10,
                2.0 * N / (ms / 10) / 1e6);
    return 0;
}
