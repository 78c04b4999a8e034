// Host-only entry points of the C ABI under AddressSanitizer +
// UndefinedBehaviorSanitizer (VERDICT r01 "host hygiene": aqz_capi.cpp's
// host-only entry points).  tests/test_sanitize_cpu.py compiles
// csrc/aqz_capi.cpp and csrc/aqz_geometry.cpp host-side with the
// sanitizers and links them ahead of libaqz_gpu.so, so these instrumented
// definitions are the ones that run; nothing here touches a GPU.  Every
// call is made with valid, boundary and invalid arguments (null pointers,
// short buffers, bad enum values) and its result checked.
#include "aqz_gpu.h"

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#define CHECK(c)                                                               \
    do {                                                                       \
        if (!(c)) {                                                            \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

static uint32_t
crc32c_bitwise(const uint8_t* p, size_t n)
{
    uint32_t c = ~0u;
    for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k)
            c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    }
    return ~c;
}

static std::vector<aqz_dimension>
random_dims(std::mt19937& rng)
{
    auto r = [&](int lo, int hi) { return uint32_t(int(rng() % uint32_t(hi - lo + 1)) + lo); };
    const int nd = int(r(3, 5));
    std::vector<aqz_dimension> d;
    d.push_back({ AQZ_DIM_TIME, r(0, 2) * 4, r(1, 5), r(1, 2) });
    for (int i = 0; i < nd - 3; ++i)
        d.push_back({ int32_t(r(0, 2)), r(1, 6), r(1, 3), r(1, 2) });
    d.push_back({ AQZ_DIM_SPACE, r(1, 300), r(1, 40), r(1, 3) });
    d.push_back({ AQZ_DIM_SPACE, r(1, 300), r(1, 40), r(1, 3) });
    return d;
}

static void
strings()
{
    CHECK(aqz_version() && std::strlen(aqz_version()) > 0);
    for (int s = -3; s < 40; ++s)
        CHECK(aqz_status_message(aqz_status(s)) != nullptr);
    for (int m = -2; m < 8; ++m) {
        const char* n = aqz_downsampling_method_name(m);
        size_t len = 0;
        const aqz_status s = aqz_downsampling_metadata_json(m, nullptr, 0, &len);
        if (m < 0 || m > 3) {
            CHECK(s != AQZ_STATUS_SUCCESS);
            continue;
        }
        CHECK(n && s == AQZ_STATUS_SUCCESS && len > 0);
        std::vector<char> buf(len + 1, 'x');
        // too small: reports the length, writes nothing past cap
        size_t l2 = 0;
        CHECK(aqz_downsampling_metadata_json(m, buf.data(), len / 2, &l2) ==
              AQZ_STATUS_OVERFLOW);
        CHECK(l2 == len);
        CHECK(aqz_downsampling_metadata_json(m, buf.data(), len + 1, &l2) ==
              AQZ_STATUS_SUCCESS);
        CHECK(std::strlen(buf.data()) == len && buf[0] == '{');
    }
}

static void
dims(std::mt19937& rng)
{
    aqz_dims* d = nullptr;
    CHECK(aqz_dims_create(nullptr, 3, AQZ_DTYPE_UINT16, nullptr, &d) != AQZ_STATUS_SUCCESS);
    CHECK(aqz_dims_create(nullptr, 0, AQZ_DTYPE_UINT16, nullptr, nullptr) !=
          AQZ_STATUS_SUCCESS);
    for (int it = 0; it < 300; ++it) {
        const auto v = random_dims(rng);
        const int dtype = int(rng() % 12) - 1; // includes invalid types
        const aqz_status s = aqz_dims_create(v.data(), v.size(), dtype, nullptr, &d);
        if (dtype < 0 || dtype >= AQZ_DTYPE_COUNT) {
            CHECK(s != AQZ_STATUS_SUCCESS);
            continue;
        }
        if (s != AQZ_STATUS_SUCCESS)
            continue;
        CHECK(aqz_dims_ndims(d) == v.size());
        aqz_dimension out;
        for (size_t i = 0; i < v.size(); ++i) {
            CHECK(aqz_dims_get(d, i, &out) == AQZ_STATUS_SUCCESS);
            CHECK(out.array_size_px == v[i].array_size_px);
        }
        CHECK(aqz_dims_get(d, v.size(), &out) != AQZ_STATUS_SUCCESS);
        CHECK(aqz_dims_get(d, 0, nullptr) != AQZ_STATUS_SUCCESS);
        const uint64_t nch = aqz_dims_number_of_chunks_in_memory(d);
        (void)aqz_dims_bytes_per_chunk(d);
        for (uint64_t f = 0; f < 40; ++f) {
            (void)aqz_dims_tile_group_offset(d, f);
            (void)aqz_dims_chunk_internal_offset(d, f);
            (void)aqz_dims_transpose_frame_id(d, f);
            for (uint32_t k = 0; k < v.size() + 1; ++k)
                (void)aqz_dims_chunk_lattice_index(d, f, k);
        }
        for (uint32_t c = 0; c < std::min<uint64_t>(nch * 2, 300); ++c) {
            (void)aqz_dims_shard_index_for_chunk(d, c);
            (void)aqz_dims_shard_internal_index(d, c);
        }
        int32_t sup = -1;
        uint32_t nb = 0, cpb = 0;
        uint64_t fpb = 0;
        CHECK(aqz_dims_dim1_banding(d, &sup, &nb, &fpb, &cpb) == AQZ_STATUS_SUCCESS);
        CHECK(sup == 0 || sup == 1);
        // null outputs are skipped or rejected, never written through
        (void)aqz_dims_dim1_banding(d, nullptr, nullptr, nullptr, nullptr);
        aqz_dims_destroy(d);
        d = nullptr;
    }
    aqz_dims_destroy(nullptr);
}

static void
levels(std::mt19937& rng)
{
    for (int it = 0; it < 300; ++it) {
        const auto v = random_dims(rng);
        const uint32_t ml = rng() % 6;
        uint32_t n = 0;
        CHECK(aqz_pyramid_levels(v.data(), v.size(), ml, &n, nullptr, 0) == AQZ_STATUS_SUCCESS);
        CHECK(n >= 1);
        std::vector<aqz_dimension> out(size_t(n) * v.size());
        if (n > 1) // one level short of room
            CHECK(aqz_pyramid_levels(v.data(), v.size(), ml, &n, out.data(),
                                     out.size() - v.size()) != AQZ_STATUS_SUCCESS);
        CHECK(aqz_pyramid_levels(v.data(), v.size(), ml, &n, out.data(), out.size()) ==
              AQZ_STATUS_SUCCESS);
        for (uint32_t l = 1; l < n; ++l)
            for (size_t i = 0; i < v.size(); ++i)
                CHECK(out[l * v.size() + i].array_size_px <=
                      out[(l - 1) * v.size() + i].array_size_px);
    }
    CHECK(aqz_pyramid_levels(nullptr, 3, 2, nullptr, nullptr, 0) != AQZ_STATUS_SUCCESS);
}

static void
memory(std::mt19937& rng)
{
    for (int it = 0; it < 200; ++it) {
        auto v = random_dims(rng);
        aqz_array_desc desc{ v.data(), v.size(), int32_t(rng() % 10), int32_t(rng() % 2),
                             int32_t(rng() % 4), uint32_t(rng() % 4), nullptr, 0 };
        aqz_stage_options o{ uint32_t(1 + rng() % 3), uint32_t(1 + rng() % 64), 0 };
        aqz_memory_usage m{};
        const aqz_status s = aqz_stage_estimate_memory(&desc, (it & 1) ? &o : nullptr, &m);
        if (s == AQZ_STATUS_SUCCESS)
            CHECK(m.device_bytes > 0);
    }
    CHECK(aqz_stage_estimate_memory(nullptr, nullptr, nullptr) != AQZ_STATUS_SUCCESS);
    aqz_memory_usage m{};
    CHECK(aqz_stage_estimate_memory(nullptr, nullptr, &m) != AQZ_STATUS_SUCCESS);
    CHECK(aqz_stage_memory_usage(nullptr, &m) == AQZ_STATUS_INVALID_ARGUMENT);
}

static void
shards(std::mt19937& rng)
{
    for (size_t n : { size_t(0), size_t(1), size_t(3), size_t(4), size_t(7), size_t(1000),
                      size_t(4097) }) {
        std::vector<uint8_t> b(n + 3);
        for (auto& x : b)
            x = uint8_t(rng());
        // unaligned starts
        for (size_t o = 0; o < 3; ++o)
            CHECK(aqz_crc32c(b.data() + o, n) == crc32c_bitwise(b.data() + o, n));
    }
    CHECK(aqz_crc32c(nullptr, 10) == 0);
    for (uint32_t cps : { 1u, 2u, 5u, 64u, 1000u }) {
        std::vector<uint64_t> off(cps), ext(cps);
        for (uint32_t i = 0; i < cps; ++i) {
            const bool skip = rng() % 4 == 0;
            off[i] = skip ? UINT64_MAX : rng();
            ext[i] = skip ? UINT64_MAX : rng() % 100000;
        }
        const size_t nb = aqz_shard_table_bytes(cps);
        CHECK(nb == size_t(cps) * 16 + 4);
        std::vector<uint8_t> t(nb);
        CHECK(aqz_shard_table(off.data(), ext.data(), cps, t.data(), nb - 1) ==
              AQZ_STATUS_OVERFLOW);
        CHECK(aqz_shard_table(off.data(), ext.data(), cps, t.data(), nb) == AQZ_STATUS_SUCCESS);
        for (uint32_t i = 0; i < cps; ++i) {
            uint64_t a, e;
            std::memcpy(&a, t.data() + 16 * i, 8);
            std::memcpy(&e, t.data() + 16 * i + 8, 8);
            CHECK(a == off[i] && e == ext[i]);
        }
        uint32_t crc;
        std::memcpy(&crc, t.data() + nb - 4, 4);
        CHECK(crc == crc32c_bitwise(t.data(), nb - 4));
        CHECK(aqz_shard_table(nullptr, ext.data(), cps, t.data(), nb) != AQZ_STATUS_SUCCESS);
    }
}

// Stage entry points reject null handles and bad descriptors before any
// device work.
static void
null_handles()
{
    CHECK(aqz_stage_create(nullptr, nullptr, nullptr) == AQZ_STATUS_INVALID_ARGUMENT);
    aqz_stage* st = reinterpret_cast<aqz_stage*>(0x1);
    CHECK(aqz_stage_create(nullptr, nullptr, &st) != AQZ_STATUS_SUCCESS && st == nullptr);
    aqz_dimension bad[3] = { { AQZ_DIM_TIME, 0, 1, 1 }, { AQZ_DIM_SPACE, 8, 4, 1 },
                             { AQZ_DIM_SPACE, 8, 4, 1 } };
    aqz_array_desc d{ bad, 3, 99, 1, 0, 0, nullptr, 0 }; // invalid dtype
    CHECK(aqz_stage_create(&d, nullptr, &st) != AQZ_STATUS_SUCCESS);
    uint8_t frame[64] = {};
    CHECK(aqz_stage_append(nullptr, frame, 1, AQZ_MEM_HOST) == AQZ_STATUS_INVALID_ARGUMENT);
    CHECK(aqz_stage_finalize(nullptr) == AQZ_STATUS_INVALID_ARGUMENT);
    CHECK(aqz_stage_wait_copies(nullptr) == AQZ_STATUS_INVALID_ARGUMENT);
    CHECK(aqz_stage_n_levels(nullptr) == 0);
    CHECK(aqz_stage_frames_written(nullptr, 0) == 0);
    aqz_stage_destroy(nullptr);
}

int
main()
{
    std::mt19937 rng(99);
    strings();
    dims(rng);
    levels(rng);
    memory(rng);
    shards(rng);
    null_handles();
    std::printf("capi sanitizer driver: clean\n");
    return 0;
}
