// split_probe -- host throughput of the level-0 tile split on this machine
// (dev probe, not product): a 2048x2048 u16 frame stream, 256x256 tiles,
// 64-frame chunk layers; T threads each own a row range of every frame.
// Variants:
//   copy      memcpy of the frame into a batch buffer (the hand-off's copy)
//   split     the tile split alone (memcpy per tile row)
//   both      copy + split of each 16-row block (the hand-off's pass)
//   both-nt   the same with nontemporal (streaming) stores for both writes
//   split-nt  the split alone, nontemporal stores
// Prints GB/s of input per variant and thread count.
// Argument 2 "pinned": the source frames (and the batch) in hipHostMalloc'd
// memory, as a camera's DMA ring (-DWITH_HIP, linked with libamdhip64).
//   g++ -O3 -std=c++20 -pthread tools/split_probe.cpp -o tools/split_probe
//   g++ -O3 -std=c++20 -pthread -DWITH_HIP -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
//     tools/split_probe.cpp -o split_probe -L/opt/rocm/lib -lamdhip64
#include <immintrin.h>
#ifdef WITH_HIP
#include <hip/hip_runtime_api.h>
#include <sys/mman.h>
#endif

#include <atomic>
#include <barrier>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr uint32_t W = 2048, H = 2048, BPP = 2, TW = 256, TH = 256, F = 64;
constexpr size_t ROW = size_t(W) * BPP, FRAME = ROW * H;
constexpr size_t BPC = size_t(TW) * TH * BPP * F;
constexpr uint32_t NTX = W / TW;

__attribute__((target("avx2"))) void
stream_copy(uint8_t* d, const uint8_t* s, size_t n)
{
    size_t i = 0;
    if ((reinterpret_cast<uintptr_t>(d) & 31) == 0) {
        for (; i + 128 <= n; i += 128) {
            __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
            __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
            __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
            __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
            _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
        }
    }
    std::memcpy(d + i, s + i, n - i);
}

template<bool NT>
void
split_rows(const uint8_t* frame, uint32_t fid, uint32_t r0, uint32_t r1, uint8_t* layer)
{
    const uint64_t internal = uint64_t(fid % F) * TW * TH * BPP;
    for (uint32_t r = r0; r < r1; ++r) {
        const uint8_t* src = frame + size_t(r) * ROW;
        const uint32_t ty = r / TH;
        const uint64_t drow = internal + uint64_t(r % TH) * TW * BPP;
        for (uint32_t tx = 0; tx < NTX; ++tx) {
            uint8_t* d = layer + uint64_t(ty * NTX + tx) * BPC + drow;
            if constexpr (NT)
                stream_copy(d, src + size_t(tx) * TW * BPP, size_t(TW) * BPP);
            else
                std::memcpy(d, src + size_t(tx) * TW * BPP, size_t(TW) * BPP);
        }
    }
}

} // namespace

int
main(int argc, char** argv)
{
    const uint32_t frames = argc > 1 ? uint32_t(std::atoi(argv[1])) : 256;
    const std::string kind = argc > 2 ? argv[2] : "pageable";
    const bool pinned = kind == "pinned" || kind == "pinned-thp" || kind == "pinned-numauser";
    std::vector<uint32_t> tcounts = { 4, 8, 12, 16 };
    const uint32_t R = 64; // distinct source frames (512 MiB, past the L3)
    std::vector<uint8_t> src_v;
    uint8_t* srcp = nullptr;
    uint8_t* batch = nullptr;
#ifdef WITH_HIP
    if (kind == "pinned" || kind == "pinned-numauser") {
        // pinned-numauser: pages placed by this thread's NUMA policy (run
        // under taskset on the GPU's node: local) instead of the runtime's
        const unsigned fl = kind == "pinned" ? hipHostMallocDefault : hipHostMallocNumaUser;
        void* p = nullptr;
        if (hipHostMalloc(&p, R * FRAME, fl) != hipSuccess)
            return 1;
        srcp = static_cast<uint8_t*>(p);
        if (hipHostMalloc(&p, 64 * FRAME, fl) != hipSuccess)
            return 1;
        batch = static_cast<uint8_t*>(p);
    } else if (kind == "pinned-thp") {
        // 2 MiB-aligned anonymous memory with transparent huge pages,
        // touched, then page-locked for DMA (hipHostRegister)
        auto thp = [](size_t n) -> uint8_t* {
            const size_t a = size_t(2) << 20;
            void* p = mmap(nullptr, n + a, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS,
                           -1, 0);
            if (p == MAP_FAILED)
                return nullptr;
            uint8_t* q = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(p) + a - 1) & ~(a - 1));
            madvise(q, n, MADV_HUGEPAGE);
            std::memset(q, 0, n);
            if (hipHostRegister(q, n, hipHostRegisterDefault) != hipSuccess)
                return nullptr;
            return q;
        };
        srcp = thp(R * FRAME);
        batch = thp(64 * FRAME);
        if (!srcp || !batch)
            return 1;
    }
#endif
    if (!srcp) {
        src_v.resize(R * FRAME);
        srcp = src_v.data();
        batch = static_cast<uint8_t*>(std::aligned_alloc(4096, 64 * FRAME));
    }
    for (size_t i = 0; i < size_t(R) * FRAME; i += 8) {
        const uint64_t x = i * 0x9e3779b97f4a7c15ull;
        std::memcpy(&srcp[i], &x, 8);
    }
    uint8_t* layer = static_cast<uint8_t*>(std::aligned_alloc(4096, NTX * NTX * BPC));
    std::memset(batch, 0, 64 * FRAME);
    std::memset(layer, 0, NTX * NTX * BPC);
    const char* names[] = { "copy", "split", "both", "both-nt", "split-nt" };
    const std::string only = argc > 3 ? argv[3] : "";
    for (int v = 0; v < 5; ++v)
        for (uint32_t T : tcounts) {
            if (!only.empty() && ("," + only + ",").find("," + std::string(names[v]) + ",") ==
                                   std::string::npos)
                continue;
            std::barrier sync(T);
            std::atomic<double> secs{ 0 };
            auto work = [&](uint32_t t) {
                const uint32_t per = (H + T - 1) / T;
                const uint32_t a = std::min(H, per * t), b = std::min(H, a + per);
                sync.arrive_and_wait();
                const auto t0 = std::chrono::steady_clock::now();
                for (uint32_t f = 0; f < frames; ++f) {
                    const uint8_t* fr = srcp + size_t(f % R) * FRAME;
                    uint8_t* bt = batch + size_t(f % 64) * FRAME;
                    for (uint32_t r = a; r < b; r += 16) {
                        const uint32_t e = std::min(b, r + 16);
                        const size_t o = size_t(r) * ROW, n = size_t(e - r) * ROW;
                        if (v == 0 || v == 2)
                            std::memcpy(bt + o, fr + o, n);
                        if (v == 3)
                            stream_copy(bt + o, fr + o, n);
                        if (v == 1 || v == 2)
                            split_rows<false>(fr, f, r, e, layer);
                        if (v == 3 || v == 4)
                            split_rows<true>(fr, f, r, e, layer);
                    }
                    _mm_sfence();
                    sync.arrive_and_wait(); // frame by frame, as the hand-off
                }
                const double s =
                  std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (t == 0)
                    secs = s;
            };
            std::vector<std::thread> th;
            for (uint32_t t = 0; t < T; ++t)
                th.emplace_back(work, t);
            for (auto& x : th)
                x.join();
            std::printf("{\"variant\": \"%s\", \"source\": \"%s\", \"threads\": %u, "
                        "\"input_gbs\": %.2f}\n",
                        names[v], kind.c_str(), T,
                        double(frames) * FRAME / secs / 1e9);
            std::fflush(stdout);
        }
    if (src_v.empty()) {
#ifdef WITH_HIP
        if (kind == "pinned" || kind == "pinned-numauser") {
            (void)hipHostFree(srcp);
            (void)hipHostFree(batch);
        }
#endif
    } else {
        std::free(batch);
    }
    std::free(layer);
    return 0;
}
