// Dev probe (not product): does the strip kernel's READ SHAPE cost HBM rate?
// The stage kernel reads a region of R rows x S bytes at the frame's row
// pitch (C2 / C3: 64 rows x 512 B at 4 KiB) per workgroup; the live probe
// (aqz_probe_hbm) reads 24 KiB contiguous per workgroup.  This times, on
// the same 2 GiB ring, read-only and read + 1/3 write with:
//   contiguous 32 KiB per workgroup,
//   R x S regions at a 4 KiB pitch (S = 512, 1024, 2048, 4096),
//   with and without the XCD-contiguous block order of the stage.
//   hipcc -O3 --offload-arch=gfx950 tools/shape_probe.hip -o tools/shape_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

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

// each workgroup: 32 KiB = 8 x 16 B per lane.  Region of R = 32768 / S rows
// of S bytes at pitch P; lanes of one load instruction cover S/16 lanes per
// row.  WRITE: also store 1/3 of it (xor of three vectors), contiguous.
template<bool WRITE, bool NTS>
__global__ __launch_bounds__(256) void
k_region(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t S,
         uint32_t P, uint32_t regions_per_band, uint32_t bands_per_frame,
         uint64_t frame_bytes, int xcd, unsigned* sink)
{
    uint32_t b = blockIdx.x;
    if (xcd) {
        const uint32_t per = gridDim.x >> 3;
        if (b < (per << 3))
            b = (b & 7u) * per + (b >> 3);
    }
    const uint32_t per_frame = regions_per_band * bands_per_frame;
    const uint32_t f = b / per_frame;
    const uint32_t q = b - f * per_frame;
    const uint32_t by = q / regions_per_band;
    const uint32_t bx = q - by * regions_per_band;
    const uint32_t R = 32768u / S;
    const uint32_t lpr = S / 16;            // lanes per row
    const uint32_t rpi = 256u / lpr;        // rows per load instruction (block-wide)
    const uint32_t t = threadIdx.x;
    const uint32_t row0 = t / lpr, col = (t - row0 * lpr) * 16;
    const uint8_t* base = src + f * frame_bytes + uint64_t(by) * R * P + uint64_t(bx) * S + col;
    u32x4 v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
        v[i] = __builtin_nontemporal_load(
            (const u32x4*)(base + uint64_t(row0 + i * rpi) * P));
    if constexpr (WRITE) {
        // 1/3 of 32 KiB, contiguous per block: lanes store 16 B, 8/3 vectors
        // per lane -> 3 stores of the first 2/3 lanes' ... keep it simple:
        // every lane stores 2 vectors, lanes < 171 a third (10.7 KiB)
        u32x4* o = (u32x4*)(dst + uint64_t(blockIdx.x) * 10944);
        const u32x4 a = v[0] ^ v[1] ^ v[2], c = v[3] ^ v[4] ^ v[5], e = v[6] ^ v[7];
        if constexpr (NTS) {
            __builtin_nontemporal_store(a, o + t);
            __builtin_nontemporal_store(c, o + 256 + t);
            if (t < 172)
                __builtin_nontemporal_store(e, o + 512 + t);
        } else {
            o[t] = a;
            o[256 + t] = c;
            if (t < 172)
                o[512 + t] = e;
        }
    } else {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i)
            acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
        if (acc == 0x12345678u)
            sink[0] = acc;
    }
}

int
main()
{
    const uint64_t frame = 4096ull * 2048; // C2: 2048 rows x 4 KiB (C3: 4096 x 4 KiB / 2)
    const uint32_t P = 4096;
    const uint64_t per_launch = 512ull << 20;
    const int ring = 4;
    uint8_t *src, *dst;
    unsigned* sink;
    CK(hipMalloc(&src, per_launch * ring));
    CK(hipMalloc(&dst, per_launch));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, per_launch * ring));
    CK(hipMemset(dst, 0, per_launch));
    hipEvent_t ea, eb;
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    const uint32_t frames = uint32_t(per_launch / frame);
    for (int rep = 0; rep < 2; ++rep)
        for (int mode = 0; mode < 3; ++mode)
            for (uint32_t S : { 4096u, 2048u, 1024u, 512u })
                for (int xcd = 0; xcd < 2; ++xcd) {
                    const uint32_t R = 32768u / S;
                    const uint32_t rpb = P / S, bpf = uint32_t(frame / P) / R;
                    const uint32_t grid = frames * rpb * bpf;
                    auto launch = [&](int i) {
                        const uint8_t* s = src + uint64_t(i % ring) * per_launch;
                        if (mode == 0)
                            k_region<false, false><<<grid, 256>>>(s, dst, S, P, rpb, bpf, frame,
                                                                  xcd, sink);
                        else if (mode == 1)
                            k_region<true, false><<<grid, 256>>>(s, dst, S, P, rpb, bpf, frame,
                                                                 xcd, sink);
                        else
                            k_region<true, true><<<grid, 256>>>(s, dst, S, P, rpb, bpf, frame,
                                                                xcd, sink);
                    };
                    for (int w = 0; w < 3; ++w)
                        launch(w);
                    const int reps = 40;
                    CK(hipEventRecord(ea));
                    for (int r = 0; r < reps; ++r)
                        launch(r);
                    CK(hipEventRecord(eb));
                    CK(hipEventSynchronize(eb));
                    float ms;
                    CK(hipEventElapsedTime(&ms, ea, eb));
                    ms /= reps;
                    const double rd = double(per_launch);
                    const double wr = mode ? double(grid) * 10944 : 0.0;
                    printf("%-14s S=%4u R=%2u xcd=%d  %.4f ms  read %.0f GB/s  bus %.0f GB/s\n",
                           mode == 0 ? "read" : mode == 1 ? "read+1/3" : "read+1/3 nts", S, R,
                           xcd, ms, rd / ms / 1e6, (rd + wr) / ms / 1e6);
                    fflush(stdout);
                }
    return 0;
}
