// PCIe copy engines on one MI355X: hipMemcpyAsync (which lands D2H as blit
// kernels) against hsa_amd_memory_async_copy (SDMA), alone and in duplex
// with a hipMemcpyAsync H2D, and what each D2H does to a latency-bound
// kernel running beside it.
//   hipcc --offload-arch=gfx950 -O2 tools/sdma_probe.cpp -lhsa-runtime64 \
//     -Lacquire-zarr_amd -laqz_gpu -Wl,-rpath,'$ORIGIN/../acquire-zarr_amd' -o tools/sdma_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include "../include/aqz_gpu.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define HIPC(x)                                                                 \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)
#define HSAC(x)                                                                 \
    do {                                                                        \
        hsa_status_t s_ = (x);                                                  \
        if (s_ != HSA_STATUS_SUCCESS) {                                         \
            std::fprintf(stderr, "%s:%d hsa status 0x%x\n", __FILE__, __LINE__, s_); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

static hsa_agent_t g_gpu{}, g_cpu{};

static hsa_status_t
agent_cb(hsa_agent_t a, void*)
{
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle)
        g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle)
        g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

// a latency-bound stand-in for the LZ4 walk: dependent LDS + global loads
__global__ __launch_bounds__(64) void
chase(const uint32_t* __restrict__ src, uint32_t* __restrict__ out, uint32_t n, int iters)
{
    __shared__ uint32_t t[1024];
    uint32_t x = blockIdx.x * 64 + threadIdx.x;
    for (int k = threadIdx.x; k < 1024; k += 64)
        t[k] = src[(blockIdx.x * 1024 + k) % n];
    __syncthreads();
    for (int i = 0; i < iters; ++i) {
        x = t[(x ^ (x >> 7)) & 1023] + src[(x * 2654435761u) % n];
        t[x & 1023] = x;
    }
    out[blockIdx.x * 64 + threadIdx.x] = x;
}

static double
now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int
main(int argc, char** argv)
{
    const size_t N = size_t(argc > 1 ? std::atoi(argv[1]) : 512) << 20;
    const size_t piece = size_t(32) << 20;
    HIPC(hipSetDevice(0));
    HIPC(hipFree(nullptr));
    HSAC(hsa_init());
    HSAC(hsa_iterate_agents(agent_cb, nullptr));
    uint32_t mask = 0, rec = 0;
    hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &mask);
    std::printf("sdma engines D2H available mask 0x%x\n", mask);
    if (hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &rec) == HSA_STATUS_SUCCESS)
        std::printf("preferred D2H mask 0x%x\n", rec);
    mask = 0;
    hsa_amd_memory_copy_engine_status(g_gpu, g_cpu, &mask);
    std::printf("sdma engines H2D available mask 0x%x\n", mask);

    uint8_t *dsrc, *ddst, *hsrc, *hdst;
    HIPC(hipMalloc(&dsrc, N));
    HIPC(hipMalloc(&ddst, N));
    HIPC(hipHostMalloc(&hsrc, N, hipHostMallocDefault));
    HIPC(hipHostMalloc(&hdst, N, hipHostMallocDefault));
    HIPC(hipMemset(dsrc, 1, N));
    std::memset(hsrc, 2, N);
    std::memset(hdst, 0, N);
    hipStream_t s1, s2, s3;
    HIPC(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
    hsa_signal_t sig;
    HSAC(hsa_signal_create(1, 0, nullptr, &sig));

    const int reps = 5;
    auto hip_d2h = [&](hipStream_t s) {
        for (size_t o = 0; o < N; o += piece)
            HIPC(hipMemcpyAsync(hdst + o, dsrc + o, std::min(piece, N - o), hipMemcpyDeviceToHost, s));
    };
    auto hip_h2d = [&](hipStream_t s) {
        for (size_t o = 0; o < N; o += piece)
            HIPC(hipMemcpyAsync(ddst + o, hsrc + o, std::min(piece, N - o), hipMemcpyHostToDevice, s));
    };
    // one SDMA copy of the whole buffer, or pieces chained by the signal
    auto hsa_d2h = [&](int engine, size_t pc) {
        const size_t np = (N + pc - 1) / pc;
        hsa_signal_store_screlease(sig, hsa_signal_value_t(np));
        for (size_t o = 0; o < N; o += pc) {
            const size_t n = std::min(pc, N - o);
            if (engine < 0)
                HSAC(hsa_amd_memory_async_copy(hdst + o, g_cpu, dsrc + o, g_gpu, n, 0, nullptr, sig));
            else
                HSAC(hsa_amd_memory_async_copy_on_engine(hdst + o, g_cpu, dsrc + o, g_gpu, n, 0,
                                                         nullptr, sig,
                                                         hsa_amd_sdma_engine_id_t(1u << engine),
                                                         true));
        }
    };
    auto hsa_wait = [&] {
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                         HSA_WAIT_STATE_BLOCKED) > 0) {
        }
    };
    auto rate = [&](double bytes, double t) { return bytes / t / 1e9; };

    // warm
    hip_d2h(s1);
    hip_h2d(s2);
    HIPC(hipDeviceSynchronize());
    hsa_d2h(-1, N);
    hsa_wait();

    double t;
    t = now();
    for (int r = 0; r < reps; ++r)
        hip_d2h(s1);
    HIPC(hipStreamSynchronize(s1));
    std::printf("hip D2H alone            %6.1f GB/s\n", rate(double(N) * reps, now() - t));
    t = now();
    for (int r = 0; r < reps; ++r)
        hip_h2d(s2);
    HIPC(hipStreamSynchronize(s2));
    std::printf("hip H2D alone            %6.1f GB/s\n", rate(double(N) * reps, now() - t));
    for (size_t pc : { N, piece }) {
        t = now();
        for (int r = 0; r < reps; ++r) {
            hsa_d2h(-1, pc);
            hsa_wait();
        }
        std::printf("hsa D2H alone (piece %4zu MiB) %6.1f GB/s\n", pc >> 20,
                    rate(double(N) * reps, now() - t));
    }
    for (int e = 0; e < 16; ++e) {
        uint32_t m = 0;
        hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &m);
        if (!(m & (1u << e)))
            continue;
        t = now();
        for (int r = 0; r < reps; ++r) {
            hsa_d2h(e, N);
            hsa_wait();
        }
        std::printf("hsa D2H engine %2d        %6.1f GB/s\n", e, rate(double(N) * reps, now() - t));
    }
    // duplex: hip H2D pieces + D2H (hip pieces / hsa)
    t = now();
    for (int r = 0; r < reps; ++r) {
        hip_h2d(s2);
        hip_d2h(s1);
    }
    HIPC(hipDeviceSynchronize());
    std::printf("duplex hip H2D + hip D2H  %6.1f GB/s total\n", rate(2.0 * N * reps, now() - t));
    t = now();
    for (int r = 0; r < reps; ++r) {
        hip_h2d(s2);
        hsa_d2h(-1, N);
        hsa_wait();
        HIPC(hipStreamSynchronize(s2));
    }
    std::printf("duplex hip H2D + hsa D2H  %6.1f GB/s total\n", rate(2.0 * N * reps, now() - t));

    // latency-bound kernel alone / with hip D2H / with hsa D2H
    const uint32_t nw = uint32_t(N / 4);
    uint32_t* out;
    HIPC(hipMalloc(&out, size_t(131072) * 64 * 4));
    auto kern = [&] {
        chase<<<131072, 64, 0, s3>>>(reinterpret_cast<const uint32_t*>(ddst), out, nw, 64);
    };
    kern();
    HIPC(hipStreamSynchronize(s3));
    hipEvent_t a, b;
    HIPC(hipEventCreate(&a));
    HIPC(hipEventCreate(&b));
    auto timed = [&](const char* what, int mode) {
        if (mode == 1)
            hip_d2h(s1);
        if (mode == 2)
            hsa_d2h(-1, N);
        HIPC(hipEventRecord(a, s3));
        kern();
        HIPC(hipEventRecord(b, s3));
        HIPC(hipEventSynchronize(b));
        float ms = 0;
        HIPC(hipEventElapsedTime(&ms, a, b));
        std::printf("chase kernel %-18s %7.3f ms\n", what, ms);
        HIPC(hipDeviceSynchronize());
        if (mode == 2)
            hsa_wait();
    };
    for (int r = 0; r < 2; ++r) {
        timed("alone", 0);
        timed("beside hip D2H", 1);
        timed("beside hsa D2H", 2);
    }
    // the device blosc-lz4 compressor (byte shuffle) on 64 camera-like
    // 256x256x64 u16 chunks, alone / beside each D2H
    {
        const uint64_t bpc = uint64_t(256) * 256 * 64 * 2;
        const uint32_t nch = uint32_t(N / bpc);
        std::vector<uint16_t> h(N / 2);
        uint32_t rs = 12345;
        for (size_t i = 0; i < h.size(); ++i) {
            rs = rs * 1664525u + 1013904223u;
            const int noise = int((rs >> 16) % 61) - 30;
            h[i] = uint16_t(1000 + int(200 * __builtin_sin(double(i % 1000000) / 977.0)) + noise);
        }
        HIPC(hipMemcpy(ddst, h.data(), N, hipMemcpyHostToDevice));
        for (int shuffle : { 1, 2 }) {
            aqz_compression cc{ 1, 5, shuffle };
            aqz_compressor* comp = nullptr;
            if (aqz_compressor_create(bpc, 2, &cc, &comp) != AQZ_STATUS_SUCCESS)
                return 2;
            const uint64_t cap = aqz_compressor_max_bytes(bpc, nch);
            uint8_t* frames;
            uint64_t* offs;
            HIPC(hipMalloc(&frames, cap));
            HIPC(hipMalloc(&offs, (nch + 1) * 8));
            auto ctimed = [&](const char* what, int mode) {
                if (mode == 1)
                    hip_d2h(s1);
                if (mode == 2)
                    hsa_d2h(-1, N);
                if (mode == 3)
                    hsa_d2h(0, N);
                HIPC(hipEventRecord(a, s3));
                for (int r = 0; r < 3; ++r)
                    aqz_compressor_run(comp, ddst, bpc, nch, frames, cap, offs, s3);
                HIPC(hipEventRecord(b, s3));
                HIPC(hipEventSynchronize(b));
                float ms = 0;
                HIPC(hipEventElapsedTime(&ms, a, b));
                std::printf("lz4 shuffle %d, 512 MiB  %-22s %7.3f ms per run\n", shuffle, what,
                            ms / 3);
                HIPC(hipDeviceSynchronize());
                if (mode >= 2)
                    hsa_wait();
            };
            for (int r = 0; r < 2; ++r) {
                ctimed("alone", 0);
                ctimed("beside hip D2H", 1);
                ctimed("beside hsa D2H", 2);
                ctimed("beside hsa D2H eng 0", 3);
            }
            aqz_compressor_destroy(comp);
            HIPC(hipFree(frames));
            HIPC(hipFree(offs));
        }
    }
    // correctness of the hsa path
    HIPC(hipMemset(dsrc, 0x5a, N));
    HIPC(hipDeviceSynchronize());
    hsa_d2h(-1, piece);
    hsa_wait();
    size_t bad = 0;
    for (size_t i = 0; i < N; i += 4093)
        bad += hdst[i] != 0x5a;
    std::printf("hsa D2H check: %s\n", bad ? "MISMATCH" : "ok");
    hsa_signal_destroy(sig);
    return bad ? 1 : 0;
}
