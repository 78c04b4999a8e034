// synth_frames.hh -- TEST INFRASTRUCTURE ONLY: the synthetic frames the
// native harnesses (handoff_replay, binding_exec) make for timing runs.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace aqz_test {

inline uint64_t
splitmix(uint64_t& s)
{
    uint64_t z = (s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// camera-like frames (smooth background + noise; bench.py run_e2e) or
// random bytes, R distinct frames reused round robin
inline std::vector<uint8_t>
synth_frames(uint32_t kind, int32_t dtype, uint64_t fbytes, uint32_t R)
{
    std::vector<uint8_t> v(size_t(R) * fbytes);
    uint64_t s = 0x5eed;
    if (kind == 2 || (dtype != 0 && dtype != 1)) {
        for (size_t i = 0; i + 8 <= v.size(); i += 8) {
            const uint64_t x = splitmix(s);
            std::memcpy(&v[i], &x, 8);
        }
        return v;
    }
    const size_t bpp = dtype == 1 ? 2 : 1;
    const size_t n = v.size() / bpp;
    for (size_t i = 0; i < n; ++i) {
        const uint64_t r = splitmix(s);
        // sum of 4 uniforms: roughly normal noise, sigma ~ 30
        const double g = (double(r & 0xffff) + double((r >> 16) & 0xffff) +
                          double((r >> 32) & 0xffff) + double(r >> 48)) / 65536.0 - 2.0;
        double x = 1000.0 + 200.0 * std::sin(double(i % (n / R)) / 977.0) + 52.0 * g;
        if (bpp == 1)
            x /= 8.0;
        x = std::max(0.0, std::min(bpp == 1 ? 255.0 : 65535.0, x));
        if (bpp == 2) {
            const uint16_t w = uint16_t(x);
            std::memcpy(&v[i * 2], &w, 2);
        } else {
            v[i] = uint8_t(x);
        }
    }
    return v;
}

} // namespace aqz_test
