// CPU checks of the binding's host-side helpers (integration/aqz_handoff.hh):
// AQZ_DEVICE parsing (select_device) and the z-slab plan (plan_z_slabs).
// Built and run by tests/test_binding_cpu.py; needs no GPU and no library.
#include "aqz_handoff.hh"

#include <cstdio>
#include <cstdlib>

namespace {
int fails = 0;
void
expect(bool ok, const char* what)
{
    if (!ok) {
        std::printf("FAIL %s\n", what);
        ++fails;
    }
}
} // namespace

int
main()
{
    using aqz_binding::plan_z_slabs;
    using aqz_binding::select_device;
    // AQZ_DEVICE: round robin over the visible devices by default
    unsetenv("AQZ_DEVICE");
    const int a = select_device(4), b = select_device(4), c = select_device(4);
    expect(a >= 0 && a < 4 && b == (a + 1) % 4 && c == (a + 2) % 4, "auto round robin");
    expect(select_device(0) == -1, "no device visible");
    setenv("AQZ_DEVICE", "2", 1);
    expect(select_device(4) == 2 && select_device(4) == 2, "fixed device");
    expect(select_device(2) == -1, "device out of range");
    setenv("AQZ_DEVICE", "off", 1);
    expect(select_device(4) == -1, "off");
    setenv("AQZ_DEVICE", "3,1", 1);
    const int d0 = select_device(8), d1 = select_device(8);
    expect((d0 == 3 && d1 == 1) || (d0 == 1 && d1 == 3), "list round robin");
    setenv("AQZ_DEVICE", "1,9", 1);
    expect(select_device(4) == -1, "list entry out of range");
    unsetenv("AQZ_DEVICE");

    // z slabs: bounds are multiples of the alignment and cover the planes
    const auto p = plan_z_slabs(256, 4, 4);
    expect(p.planes == 256 && p.begin.size() == 4, "4 slabs of 256");
    for (size_t r = 0; r < p.begin.size(); ++r) {
        expect(p.begin[r] == 64 * r && p.end[r] == 64 * (r + 1), "even slabs");
        expect(p.begin[r] % 4 == 0 && p.end[r] % 4 == 0, "aligned");
    }
    const auto q = plan_z_slabs(64, 3, 4);
    expect(q.begin.size() == 3 && q.begin[0] == 0 && q.end[2] == 64, "3 slabs cover 64");
    for (size_t r = 0; r + 1 < q.begin.size(); ++r)
        expect(q.end[r] == q.begin[r + 1] && q.end[r] % 4 == 0, "3 slabs contiguous, aligned");
    expect(plan_z_slabs(64, 1, 4).begin.empty(), "one slab: no plan");
    expect(plan_z_slabs(8, 4, 4).begin.empty(), "fewer aligned units than slabs");
    expect(plan_z_slabs(66, 2, 4).begin.empty(), "planes not a multiple of the alignment");
    setenv("AQZ_Z_SLABS", "4", 1);
    expect(aqz_binding::slabs_from_env() == 4, "AQZ_Z_SLABS");
    setenv("AQZ_Z_SLABS", "junk", 1);
    expect(aqz_binding::slabs_from_env() == 1, "AQZ_Z_SLABS invalid");
    std::printf("%s\n", fails ? "FAILED" : "OK");
    // the level-0 side: on the host for a raw hand-off of an array stored in
    // acquisition row order; on the device with a codec or an XY order
    {
        using aqz_binding::level0_on_host_for;
        aqz_dimension d[3] = { { AQZ_DIM_TIME, 0, 8, 1 }, { AQZ_DIM_SPACE, 64, 16, 1 },
                               { AQZ_DIM_SPACE, 64, 16, 1 } };
        const size_t same[3] = { 0, 1, 2 }, xy[3] = { 0, 2, 1 };
        aqz_array_desc a{ d, 3, AQZ_DTYPE_UINT16, 1, AQZ_METHOD_MEAN, 0, nullptr, 0 };
        const aqz_compression raw{ AQZ_CODEC_NONE, 0, 0 }, lz4{ AQZ_CODEC_BLOSC_LZ4, 1, 1 };
        expect(level0_on_host_for(a, raw), "raw, acquisition order: host");
        expect(!level0_on_host_for(a, lz4), "blosc-lz4: device");
        a.storage_dimension_order = same;
        expect(level0_on_host_for(a, raw), "identity storage order: host");
        a.storage_dimension_order = xy;
        expect(!level0_on_host_for(a, raw), "XY storage order: device");
    }
    return fails ? 1 : 0;
}
