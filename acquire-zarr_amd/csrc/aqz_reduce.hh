// aqz_reduce.hh -- the 2x2 and z-pair reducers, bit-exact with the reference
// (src/streaming/downsampler.cpp:39-137).
//
// MEAN: the reference's "overflow-safe" integral overloads (:53-62, :114-123)
// are removed by SFINAE, so `(a+b+c+d)/4` and `(a+b)/2` run for every type:
//   8/16-bit -> promoted to int, exact sum, truncating division;
//   32/64-bit -> the sum wraps modulo 2^N (computed here in the unsigned
//   type, which is the wrap the reference exhibits), truncating division;
//   float/double -> ((a+b)+c)+d then /4 (x*0.25 is the same correctly
//   rounded value as x/4), no reassociation, no contraction, denormals kept.
// MIN/MAX: compare-select in the reference's order (strict <, >); never the
// hardware v_min/v_max, whose NaN and signed-zero rules differ.
// DECIMATE: the top-left pixel; z-decimate keeps the earlier plane.
#pragma once

#include <cstdint>
#include <type_traits>

#ifndef AQZ_HD
#if defined(__HIPCC__)
#define AQZ_HD __host__ __device__ __forceinline__
#else
#define AQZ_HD inline
#endif
#endif

namespace aqz {

enum Method : int
{
    kDecimate = 0,
    kMean = 1,
    kMin = 2,
    kMax = 3
};

template<typename T>
AQZ_HD T
mean4(T a, T b, T c, T d)
{
    if constexpr (std::is_floating_point_v<T>) {
        T s = a + b;
        s = s + c;
        s = s + d;
        return s * T(0.25);
    } else if constexpr (sizeof(T) < 4) {
        return static_cast<T>((int(a) + int(b) + int(c) + int(d)) / 4);
    } else {
        using U = std::make_unsigned_t<T>;
        const U s = U(a) + U(b) + U(c) + U(d);
        return static_cast<T>(static_cast<T>(s) / T(4));
    }
}

template<typename T>
AQZ_HD T
mean2(T a, T b)
{
    if constexpr (std::is_floating_point_v<T>) {
        return (a + b) * T(0.5);
    } else if constexpr (sizeof(T) < 4) {
        return static_cast<T>((int(a) + int(b)) / 2);
    } else {
        using U = std::make_unsigned_t<T>;
        const U s = U(a) + U(b);
        return static_cast<T>(static_cast<T>(s) / T(2));
    }
}

// (a, b, c, d) = (here, right, down, diag), downsampler.cpp:193-198
template<int M, typename T>
AQZ_HD T
reduce4(T a, T b, T c, T d)
{
    if constexpr (M == kDecimate) {
        return a;
    } else if constexpr (M == kMean) {
        return mean4<T>(a, b, c, d);
    } else if constexpr (M == kMin) {
        T v = a;
        v = (b < v) ? b : v;
        v = (c < v) ? c : v;
        v = (d < v) ? d : v;
        return v;
    } else {
        T v = a;
        v = (b > v) ? b : v;
        v = (c > v) ? c : v;
        v = (d > v) ? d : v;
        return v;
    }
}

// a = earlier plane, b = later plane (downsampler.cpp:374-375, 243-245)
template<int M, typename T>
AQZ_HD T
reduce2(T a, T b)
{
    if constexpr (M == kDecimate) {
        return a;
    } else if constexpr (M == kMean) {
        return mean2<T>(a, b);
    } else if constexpr (M == kMin) {
        return a < b ? a : b;
    } else {
        return a > b ? a : b;
    }
}

} // namespace aqz
