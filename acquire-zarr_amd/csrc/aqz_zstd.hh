// aqz_zstd.hh -- building blocks of the device zstd encoder (RFC 8878), as
// __host__ __device__ functions so the same code runs in the kernels
// (aqz_codec.hip, zstd_*) and in the CPU test encoder (tests/zstd/zstd_host.cpp) that
// libzstd decodes.
//
// What the encoder emits (every piece a decoder must accept, nothing more):
//   frame    magic, Single_Segment descriptor + Frame_Content_Size, no
//            checksum, no dictionary (ZSTD_compress's defaults)
//   blocks   Raw, RLE or Compressed; at most kBlock bytes of content
//   literals Raw, RLE, or Huffman in 4 streams; the first Huffman block of
//            a frame carries the tree description (weights FSE-compressed,
//            or direct when <= 128 weights), later blocks reuse it
//            (Treeless literals)
//   sequences none, or LZ matches coded with the predefined FSE
//            distributions of literal length, match length and offset codes
//            (Symbol_Compression_Modes = 0); offsets are always new offsets
//            (Offset_Value = offset + 3, no repeat codes)
//
// The FSE table construction and state transitions follow the normative
// decoding tables of RFC 8878 4.1.1 (spread step (size>>1)+(size>>3)+3,
// "less than 1" symbols at the top); encoding runs the streams backwards so
// the decoder reads them forwards.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace aqz {
namespace zstd {

// content bytes of one zstd block, the parallel unit of the device encoder:
// one workgroup, whose sequences are FSE-coded by one lane -- 8 KiB keeps
// that serial chain short and four times as many of them in flight as
// 32 KiB blocks did (encode 4.6 -> see DESIGN.md), for ~15 bytes of block
// and literal headers per block
constexpr uint32_t kBlock = 8 * 1024;
constexpr uint32_t kHufMaxBits = 11;
constexpr uint32_t kWeightsLog = 6; // FSE accuracy of the Huffman weights

__host__ __device__ inline uint32_t
highbit(uint32_t v) // v > 0
{
    return 31u - uint32_t(__builtin_clz(v));
}

// LSB-first bit writer over a byte buffer (the zstd bitstream order).
struct BitW
{
    uint8_t* p;
    uint32_t cap;
    uint32_t pos;
    uint64_t acc;
    uint32_t n;
    bool ovf;
    __host__ __device__ void init(uint8_t* dst, uint32_t c)
    {
        p = dst;
        cap = c;
        pos = 0;
        acc = 0;
        n = 0;
        ovf = false;
    }
    __host__ __device__ void add(uint64_t v, uint32_t nb) // nb <= 32
    {
        acc |= (v & ((1ull << nb) - 1ull)) << n;
        n += nb;
        while (n >= 8) {
            if (pos < cap)
                p[pos] = uint8_t(acc);
            else
                ovf = true;
            ++pos;
            acc >>= 8;
            n -= 8;
        }
    }
    // pad the last byte with zeros (no end mark); bytes, 0 on overflow
    __host__ __device__ uint32_t pad()
    {
        if (n) {
            if (pos < cap)
                p[pos] = uint8_t(acc);
            else
                ovf = true;
            ++pos;
            acc = 0;
            n = 0;
        }
        return ovf ? 0 : pos;
    }
    // end mark (one 1 bit) then pad: a backward-read bitstream
    __host__ __device__ uint32_t close()
    {
        add(1, 1);
        return pad();
    }
};

// ---- FSE -------------------------------------------------------------------
constexpr uint32_t kFseMaxLog = 6;  // predefined sequence tables, Huffman weights
constexpr uint32_t kSeqMaxLog = 9;  // custom sequence tables (LL/ML 9, OF 8)
constexpr uint32_t kFseMaxSym = 53;

template<uint32_t LOG>
struct FseTable
{
    uint16_t st[1u << LOG];   // next state values, by symbol
    uint32_t dnb[kFseMaxSym]; // deltaNbBits
    int32_t dfs[kFseMaxSym];  // deltaFindState
    uint32_t al;
};
using FseCT = FseTable<kFseMaxLog>;

// norm: normalized counts of symbols 0..maxsym (-1 = "less than 1"),
// summing to 1 << al.  false when the distribution is not valid.
template<uint32_t LOG>
struct FseBuildWorkT
{
    uint8_t sym[1u << LOG];
    uint32_t cumul[kFseMaxSym + 1];
};
using FseBuildWork = FseBuildWorkT<kFseMaxLog>;

template<uint32_t LOG>
__host__ __device__ inline bool
fse_build(FseTable<LOG>& ct, const int16_t* norm, uint32_t maxsym, uint32_t al,
          FseBuildWorkT<LOG>& bw)
{
    if (al > LOG || maxsym >= kFseMaxSym)
        return false;
    const uint32_t ts = 1u << al, mask = ts - 1, step = (ts >> 1) + (ts >> 3) + 3;
    uint8_t* sym = bw.sym;
    uint32_t* cumul = bw.cumul;
    uint32_t high = ts - 1;
    cumul[0] = 0;
    for (uint32_t s = 0; s <= maxsym; ++s) {
        if (norm[s] == -1) {
            cumul[s + 1] = cumul[s] + 1;
            sym[high--] = uint8_t(s);
        } else {
            if (norm[s] < 0)
                return false;
            cumul[s + 1] = cumul[s] + uint32_t(norm[s]);
        }
    }
    if (cumul[maxsym + 1] != ts)
        return false;
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxsym; ++s)
        for (int i = 0; i < norm[s]; ++i) {
            sym[pos] = uint8_t(s);
            pos = (pos + step) & mask;
            while (pos > high)
                pos = (pos + step) & mask;
        }
    if (pos != 0)
        return false;
    for (uint32_t u = 0; u < ts; ++u)
        ct.st[cumul[sym[u]]++] = uint16_t(ts + u);
    uint32_t total = 0;
    for (uint32_t s = 0; s <= maxsym; ++s) {
        const int n = norm[s];
        if (n == 0) {
            ct.dnb[s] = ((al + 1) << 16) - ts;
            ct.dfs[s] = 0;
        } else if (n == -1 || n == 1) {
            ct.dnb[s] = (al << 16) - ts;
            ct.dfs[s] = int32_t(total) - 1;
            total += 1;
        } else {
            const uint32_t mbo = al - highbit(uint32_t(n) - 1);
            const uint32_t msp = uint32_t(n) << mbo;
            ct.dnb[s] = (mbo << 16) - msp;
            ct.dfs[s] = int32_t(total) - n;
            total += uint32_t(n);
        }
    }
    ct.al = al;
    return true;
}

template<uint32_t LOG>
__host__ __device__ inline bool
fse_build(FseTable<LOG>& ct, const int16_t* norm, uint32_t maxsym, uint32_t al)
{
    FseBuildWorkT<LOG> bw;
    return fse_build(ct, norm, maxsym, al, bw);
}

// first (= last encoded) symbol: the smallest state, no bits out
template<uint32_t LOG>
__host__ __device__ inline uint32_t
fse_init(const FseTable<LOG>& ct, uint32_t s)
{
    const uint32_t nbo = (ct.dnb[s] + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - ct.dnb[s];
    return ct.st[int32_t(v >> nbo) + ct.dfs[s]];
}

template<uint32_t LOG, class W>
__host__ __device__ inline void
fse_enc(W& w, uint32_t& state, const FseTable<LOG>& ct, uint32_t s)
{
    const uint32_t nbo = (state + ct.dnb[s]) >> 16;
    w.add(state, nbo);
    state = ct.st[int32_t(state >> nbo) + ct.dfs[s]];
}

template<uint32_t LOG, class W>
__host__ __device__ inline void
fse_flush(W& w, uint32_t state, const FseTable<LOG>& ct)
{
    w.add(state, ct.al);
}

// The table description (RFC 8878 4.1.1): accuracy log, then each
// probability + 1 in a variable number of bits, zero runs as 2-bit repeat
// flags.  Bytes written, 0 on error.
__host__ __device__ inline uint32_t
fse_write_ncount(uint8_t* out, uint32_t cap, const int16_t* norm, uint32_t maxsym,
                 uint32_t al)
{
    BitW w;
    w.init(out, cap);
    w.add(al - 5, 4);
    const int ts = 1 << al;
    int remaining = ts + 1, threshold = ts;
    uint32_t nb = al + 1, s = 0;
    bool prev0 = false;
    while (s <= maxsym && remaining > 1) {
        if (prev0) {
            uint32_t start = s;
            while (s <= maxsym && norm[s] == 0)
                ++s;
            if (s > maxsym)
                return 0;
            while (s >= start + 24) {
                start += 24;
                w.add(0xFFFFu, 16);
            }
            while (s >= start + 3) {
                start += 3;
                w.add(3, 2);
            }
            w.add(s - start, 2);
        }
        int count = norm[s++];
        const int mx = (2 * threshold - 1) - remaining;
        remaining -= count < 0 ? -count : count;
        ++count;
        if (count >= threshold)
            count += mx;
        w.add(uint32_t(count), nb - (count < mx ? 1u : 0u));
        prev0 = count == 1;
        if (remaining < 1)
            return 0;
        while (remaining < threshold) {
            --nb;
            threshold >>= 1;
        }
    }
    if (remaining != 1)
        return 0;
    return w.pad();
}

// ---- Huffman ---------------------------------------------------------------
// Workspace of the Huffman construction (LDS in the kernel).
struct HufWork
{
    uint32_t cnt[256];
    uint16_t sorted[256]; // symbols present, by (count, symbol)
    uint32_t wt[511];
    uint16_t par[511];
    uint8_t dep[511];
};

// Code lengths (<= maxbits) of an optimal prefix code for the n symbols
// w.sorted[0..n) (n >= 2) with counts w.cnt; two-queue construction.  A code
// longer than maxbits halves the counts (order-preserving) and rebuilds;
// either way the code is complete, as zstd's weights require.
__host__ __device__ inline void
huf_lengths_sorted(HufWork& w, uint32_t n, uint8_t* len, uint32_t maxbits)
{
    for (;;) {
        for (uint32_t i = 0; i < n; ++i)
            w.wt[i] = w.cnt[w.sorted[i]];
        uint32_t li = 0, ii = n, ni = n;
        while (ni < 2 * n - 1) {
            uint32_t a, b;
            if (li < n && (ii >= ni || w.wt[li] <= w.wt[ii]))
                a = li++;
            else
                a = ii++;
            if (li < n && (ii >= ni || w.wt[li] <= w.wt[ii]))
                b = li++;
            else
                b = ii++;
            w.wt[ni] = w.wt[a] + w.wt[b];
            w.par[a] = w.par[b] = uint16_t(ni);
            ++ni;
        }
        w.dep[2 * n - 2] = 0;
        uint32_t mx = 0;
        for (int k = int(2 * n) - 3; k >= 0; --k) {
            w.dep[k] = uint8_t(w.dep[w.par[k]] + 1);
            if (uint32_t(k) < n && w.dep[k] > mx)
                mx = w.dep[k];
        }
        if (mx <= maxbits) {
            for (uint32_t i = 0; i < n; ++i)
                len[w.sorted[i]] = w.dep[i];
            return;
        }
        for (uint32_t i = 0; i < n; ++i)
            w.cnt[w.sorted[i]] = (w.cnt[w.sorted[i]] + 1) >> 1;
    }
}

// The same from a histogram (serial sort); returns the symbols present.
// len[] is zero for absent symbols; one symbol present gets length 1.
__host__ __device__ inline uint32_t
huf_lengths(const uint32_t* cnt_in, uint8_t* len, uint32_t maxbits)
{
    HufWork w;
    uint32_t n = 0;
    for (uint32_t s = 0; s < 256; ++s) {
        w.cnt[s] = cnt_in[s];
        len[s] = 0;
        if (w.cnt[s])
            w.sorted[n++] = uint16_t(s);
    }
    for (uint32_t i = 1; i < n; ++i) { // insertion sort by count, stable
        const uint16_t x = w.sorted[i];
        uint32_t j = i;
        while (j > 0 && w.cnt[w.sorted[j - 1]] > w.cnt[x]) {
            w.sorted[j] = w.sorted[j - 1];
            --j;
        }
        w.sorted[j] = x;
    }
    if (n == 1)
        len[w.sorted[0]] = 1;
    if (n >= 2)
        huf_lengths_sorted(w, n, len, maxbits);
    return n;
}

// A literal histogram too flat for Huffman to pay: every byte value present
// and none above 5/4 of the mean (entropy >= 7.68 bits; random bytes, the low
// bit planes of noisy data).  Literals stay raw; the encoders skip the table.
__host__ __device__ inline bool
huf_flat(uint32_t present, uint32_t maxcnt, uint64_t total)
{
    return present == 256 && uint64_t(maxcnt) * 1024u < total * 5u;
}

// Workspace of the tree description (LDS in the kernel).
struct TreeWork
{
    uint8_t w[256];
    uint8_t tmp[160];
    FseCT ct;
    FseBuildWork bw;
    int16_t norm[kHufMaxBits + 1];
    uint32_t wc[kHufMaxBits + 1];
    uint32_t nper[kHufMaxBits + 2];
    uint32_t start[kHufMaxBits + 2];
};

// Canonical codes (RFC 8878 4.2.2: longest codes first, symbol order within
// a length).  Returns the largest length.
__host__ __device__ inline uint32_t
huf_codes(const uint8_t* len, uint16_t* code, TreeWork& tw)
{
    for (uint32_t L = 0; L < kHufMaxBits + 2; ++L) {
        tw.nper[L] = 0;
        tw.start[L] = 0;
    }
    uint32_t mx = 0;
    for (uint32_t s = 0; s < 256; ++s) {
        tw.nper[len[s]]++;
        if (len[s] > mx)
            mx = len[s];
    }
    uint32_t v = 0;
    for (uint32_t L = mx; L >= 1; --L) {
        tw.start[L] = v;
        v = (v + tw.nper[L]) >> 1;
    }
    for (uint32_t s = 0; s < 256; ++s)
        code[s] = len[s] ? uint16_t(tw.start[len[s]]++) : 0;
    return mx;
}

// Huffman tree description (RFC 8878 4.2.1): the weights of symbols
// 0..last-1 (last = the largest symbol present, its weight implied),
// FSE-compressed or, when that does not pay and last <= 128, 4 bits each.
// Returns bytes written (<= 129), 0 when it cannot be described (> 128
// weights that FSE does not compress): the caller stores raw literals.
__host__ __device__ inline uint32_t
huf_write_tree(const uint8_t* len, uint32_t maxbits, uint8_t* out, TreeWork& tw)
{
    uint32_t last = 0;
    for (uint32_t s = 0; s < 256; ++s)
        if (len[s])
            last = s;
    const uint32_t nw = last; // weights transmitted
    uint8_t* w = tw.w;
    uint32_t* wc = tw.wc;
    for (uint32_t v = 0; v <= kHufMaxBits; ++v)
        wc[v] = 0;
    uint32_t wmax = 0;
    for (uint32_t s = 0; s < nw; ++s) {
        w[s] = len[s] ? uint8_t(maxbits + 1 - len[s]) : 0;
        wc[w[s]]++;
        if (w[s] > wmax)
            wmax = w[s];
    }
    // FSE-compressed weights (2 interleaved states, as FSE_compress)
    if (nw > 2) {
        bool single = false;
        for (uint32_t v = 0; v <= wmax; ++v)
            single |= wc[v] == nw;
        if (!single) {
            const uint32_t al = kWeightsLog, ts = 1u << al;
            int16_t* norm = tw.norm;
            uint32_t sum = 0, big = 0;
            for (uint32_t v = 0; v <= wmax; ++v) {
                uint32_t q = uint32_t((uint64_t(wc[v]) * ts) / nw);
                if (wc[v] && q == 0)
                    q = 1;
                norm[v] = int16_t(q);
                sum += q;
                if (wc[v] > wc[big])
                    big = v;
            }
            const int fix = int(norm[big]) + int(ts) - int(sum);
            if (fix >= 1) {
                norm[big] = int16_t(fix);
                FseCT& ct = tw.ct;
                uint8_t* tmp = tw.tmp;
                const uint32_t hn = fse_build(ct, norm, wmax, al, tw.bw)
                                      ? fse_write_ncount(tmp, sizeof(tw.tmp), norm, wmax, al)
                                      : 0;
                if (hn) {
                    BitW bw;
                    bw.init(tmp + hn, sizeof(tw.tmp) - hn);
                    uint32_t s1, s2;
                    int i = int(nw);
                    if (nw & 1) {
                        s1 = fse_init(ct, w[--i]);
                        s2 = fse_init(ct, w[--i]);
                        fse_enc(bw, s1, ct, w[--i]);
                    } else {
                        s2 = fse_init(ct, w[--i]);
                        s1 = fse_init(ct, w[--i]);
                    }
                    while (i > 0) {
                        fse_enc(bw, s2, ct, w[--i]);
                        fse_enc(bw, s1, ct, w[--i]);
                    }
                    fse_flush(bw, s2, ct);
                    fse_flush(bw, s1, ct);
                    const uint32_t sn = bw.close();
                    if (sn && hn + sn < 128 && (nw > 128 || hn + sn < (nw + 1) / 2)) {
                        const uint32_t fsz = hn + sn;
                        out[0] = uint8_t(fsz);
                        for (uint32_t k = 0; k < fsz; ++k)
                            out[1 + k] = tmp[k];
                        return 1 + fsz;
                    }
                }
            }
        }
    }
    if (nw == 0 || nw > 128)
        return 0;
    out[0] = uint8_t(127 + nw);
    for (uint32_t i = 0; i < nw; i += 2)
        out[1 + i / 2] = uint8_t(w[i] << 4 | (i + 1 < nw ? w[i + 1] : 0));
    return 1 + (nw + 1) / 2;
}

// host-side conveniences (their own workspace)
inline uint32_t
huf_codes(const uint8_t* len, uint16_t* code)
{
    TreeWork tw;
    return huf_codes(len, code, tw);
}
inline uint32_t
huf_write_tree(const uint8_t* len, uint32_t maxbits, uint8_t* out)
{
    TreeWork tw;
    return huf_write_tree(len, maxbits, out, tw);
}

// ---- headers ---------------------------------------------------------------
__host__ __device__ inline void
put_le(uint8_t* o, uint64_t v, uint32_t n)
{
    for (uint32_t k = 0; k < n; ++k)
        o[k] = uint8_t(v >> (8 * k));
}

__host__ __device__ inline uint32_t
frame_header_bytes(uint64_t content)
{
    return 5 + (content < 256 ? 1 : content < 65536 + 256 ? 2 : content <= 0xFFFFFFFFull ? 4 : 8);
}

__host__ __device__ inline uint32_t
write_frame_header(uint8_t* o, uint64_t content)
{
    put_le(o, 0xFD2FB528u, 4);
    if (content < 256) {
        o[4] = 0x20;
        o[5] = uint8_t(content);
        return 6;
    }
    if (content < 65536 + 256) {
        o[4] = 0x60;
        put_le(o + 5, content - 256, 2);
        return 7;
    }
    if (content <= 0xFFFFFFFFull) {
        o[4] = 0xA0;
        put_le(o + 5, content, 4);
        return 9;
    }
    o[4] = 0xE0;
    put_le(o + 5, content, 8);
    return 13;
}

// block header: last flag, type (0 raw, 1 RLE, 2 compressed), size
__host__ __device__ inline void
write_block_header(uint8_t* o, bool last, uint32_t type, uint32_t size)
{
    put_le(o, uint32_t(last) | type << 1 | size << 3, 3);
}

// Raw (type 0) or RLE (type 1) literals section header
__host__ __device__ inline uint32_t
lit_header_raw_bytes(uint32_t n)
{
    return n < 32 ? 1 : n < 4096 ? 2 : 3;
}
__host__ __device__ inline uint32_t
write_lit_header_raw(uint8_t* o, uint32_t type, uint32_t n)
{
    if (n < 32) {
        o[0] = uint8_t(type | n << 3);
        return 1;
    }
    if (n < 4096) {
        put_le(o, type | 1u << 2 | n << 4, 2);
        return 2;
    }
    put_le(o, type | 3u << 2 | n << 4, 3);
    return 3;
}

// Compressed (type 2) or Treeless (type 3) literals header, 4 streams
__host__ __device__ inline uint32_t
lit_header_huf_bytes(uint32_t regen, uint32_t csize)
{
    const uint32_t m = regen > csize ? regen : csize;
    return m < 1024 ? 3 : m < 16384 ? 4 : 5;
}
__host__ __device__ inline uint32_t
write_lit_header_huf(uint8_t* o, uint32_t type, uint32_t regen, uint32_t csize)
{
    const uint32_t nb = lit_header_huf_bytes(regen, csize);
    if (nb == 3)
        put_le(o, type | 1u << 2 | uint64_t(regen) << 4 | uint64_t(csize) << 14, 3);
    else if (nb == 4)
        put_le(o, type | 2u << 2 | uint64_t(regen) << 4 | uint64_t(csize) << 18, 4);
    else
        put_le(o, type | 3u << 2 | uint64_t(regen) << 4 | uint64_t(csize) << 22, 5);
    return nb;
}

// The 4 literal streams of n literals: stream k holds literals
// [k * seg, min(n, (k + 1) * seg)), seg = (n + 3) / 4.
__host__ __device__ inline uint32_t
lit_segment(uint32_t n)
{
    return (n + 3) / 4;
}

// ---- sequences (predefined distributions, RFC 8878 3.1.1.3.2.2) -----------
__host__ __device__ inline const int16_t*
ll_default_norm()
{
    static constexpr int16_t v[36] = { 4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                       2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1 };
    return v;
}
__host__ __device__ inline const int16_t*
ml_default_norm()
{
    static constexpr int16_t v[53] = { 1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1 };
    return v;
}
__host__ __device__ inline const int16_t*
of_default_norm()
{
    static constexpr int16_t v[29] = { 1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1 };
    return v;
}

// literal length -> code; extra bits = ll - base
__host__ __device__ inline uint32_t
ll_code(uint32_t ll)
{
    if (ll < 16)
        return ll;
    if (ll < 64) {
        // 16,18,20,22 (1 bit) 24,28 (2) 32,40 (3) 48 (4)
        if (ll < 24)
            return 16 + (ll - 16) / 2;
        if (ll < 32)
            return 20 + (ll - 24) / 4;
        if (ll < 48)
            return 22 + (ll - 32) / 8;
        return 24;
    }
    return highbit(ll) + 19;
}
__host__ __device__ inline uint32_t
ll_base(uint32_t code)
{
    if (code < 16)
        return code;
    if (code < 20)
        return 16 + 2 * (code - 16);
    if (code < 22)
        return 24 + 4 * (code - 20);
    if (code < 24)
        return 32 + 8 * (code - 22);
    if (code == 24)
        return 48;
    return 1u << (code - 19);
}
__host__ __device__ inline uint32_t
ll_bits(uint32_t code)
{
    if (code < 16)
        return 0;
    if (code < 20)
        return 1;
    if (code < 22)
        return 2;
    if (code < 24)
        return 3;
    if (code == 24)
        return 4;
    return code - 19;
}

// match length (>= 3) -> code over mlBase = ml - 3
__host__ __device__ inline uint32_t
ml_code(uint32_t ml)
{
    const uint32_t b = ml - 3;
    if (b < 32)
        return b;
    if (b < 128) {
        // 32..38 step 2 (1 bit), 40,44 (2), 48,56 (3), 64,80 (4), 96 (5)
        if (b < 40)
            return 32 + (b - 32) / 2;
        if (b < 48)
            return 36 + (b - 40) / 4;
        if (b < 64)
            return 38 + (b - 48) / 8;
        if (b < 96)
            return 40 + (b - 64) / 16;
        return 42;
    }
    return highbit(b) + 36;
}
__host__ __device__ inline uint32_t
ml_base(uint32_t code) // in match length (mlBase + 3)
{
    uint32_t b;
    if (code < 32)
        b = code;
    else if (code < 36)
        b = 32 + 2 * (code - 32);
    else if (code < 38)
        b = 40 + 4 * (code - 36);
    else if (code < 40)
        b = 48 + 8 * (code - 38);
    else if (code < 42)
        b = 64 + 16 * (code - 40);
    else if (code == 42)
        b = 96;
    else
        b = 1u << (code - 36);
    return b + 3;
}
__host__ __device__ inline uint32_t
ml_bits(uint32_t code)
{
    if (code < 32)
        return 0;
    if (code < 36)
        return 1;
    if (code < 38)
        return 2;
    if (code < 40)
        return 3;
    if (code < 42)
        return 4;
    if (code == 42)
        return 5;
    return code - 36;
}

// Sequences section header (count + modes byte, predefined tables); bytes
__host__ __device__ inline uint32_t
write_seq_header(uint8_t* o, uint32_t nseq)
{
    if (nseq == 0) {
        o[0] = 0;
        return 1;
    }
    uint32_t k;
    if (nseq < 128) {
        o[0] = uint8_t(nseq);
        k = 1;
    } else if (nseq < 0x7F00) {
        o[0] = uint8_t((nseq >> 8) + 0x80);
        o[1] = uint8_t(nseq);
        k = 2;
    } else {
        o[0] = 0xFF;
        put_le(o + 1, nseq - 0x7F00, 2);
        k = 3;
    }
    o[k] = 0; // LL, OF, ML: predefined
    return k + 1;
}

struct SeqTables
{
    FseCT ll, ml, of;
};

__host__ __device__ inline bool
build_seq_tables(SeqTables& t)
{
    return fse_build(t.ll, ll_default_norm(), 35, 6) && fse_build(t.ml, ml_default_norm(), 52, 6) &&
           fse_build(t.of, of_default_norm(), 28, 5);
}

// One sequence: lit literals, then a match of len >= 3 at distance off.
struct Seq
{
    uint32_t lit, len, off;
};

// The sequences bitstream of n >= 1 sequences (get(i) -> Seq), written
// backwards as ZSTD_encodeSequences does; bytes, 0 on overflow.
template<class Get>
__host__ __device__ inline uint32_t
encode_sequences(const SeqTables& t, Get get, uint32_t n, uint8_t* out, uint32_t cap)
{
    BitW w;
    w.init(out, cap);
    Seq z = get(n - 1);
    uint32_t llc = ll_code(z.lit), mlc = ml_code(z.len), ofv = z.off + 3, ofc = highbit(ofv);
    uint32_t sml = fse_init(t.ml, mlc), sof = fse_init(t.of, ofc), sll = fse_init(t.ll, llc);
    w.add(z.lit - ll_base(llc), ll_bits(llc));
    w.add(z.len - ml_base(mlc), ml_bits(mlc));
    w.add(ofv - (1u << ofc), ofc);
    for (int i = int(n) - 2; i >= 0; --i) {
        z = get(uint32_t(i));
        llc = ll_code(z.lit);
        mlc = ml_code(z.len);
        ofv = z.off + 3;
        ofc = highbit(ofv);
        fse_enc(w, sof, t.of, ofc);
        fse_enc(w, sml, t.ml, mlc);
        fse_enc(w, sll, t.ll, llc);
        w.add(z.lit - ll_base(llc), ll_bits(llc));
        w.add(z.len - ml_base(mlc), ml_bits(mlc));
        w.add(ofv - (1u << ofc), ofc);
    }
    fse_flush(w, sml, t.ml);
    fse_flush(w, sof, t.of);
    fse_flush(w, sll, t.ll);
    return w.close();
}

// sequence packing of the device parse: lit (16 bits), len (16), off (16)
__host__ __device__ inline uint64_t
pack_seq(uint32_t lit, uint32_t len, uint32_t off)
{
    return uint64_t(lit) | uint64_t(len) << 16 | uint64_t(off) << 32;
}
__host__ __device__ inline Seq
unpack_seq(uint64_t v)
{
    return Seq{ uint32_t(v & 0xFFFFu), uint32_t((v >> 16) & 0xFFFFu), uint32_t(v >> 32) };
}

// Minimum match length for a block whose bytes have entropy H bits: a match
// pays when its literal cost beats a sequence's cost.  With the predefined
// sequence tables a sequence is ~16 bits (CPU model sweep,
// tests/zstd/zstd_host.cpp MATCH_BITS); with tables fitted to the segment
// ~12 (tools/zstd_lab.cpp sweep: dim sCMOS plain zstd 2.86 -> 3.11).
constexpr float kMatchBits = 16.0f;
constexpr float kMatchBitsFitted = 12.0f;
__host__ __device__ inline uint32_t
min_match(float H, uint32_t cap, float bits = kMatchBits)
{
    const float h = H > 0.25f ? H : 0.25f;
    uint32_t m = uint32_t(bits / h + 0.999f);
    return m < 4 ? 4 : (m > cap ? cap : m);
}

} // namespace zstd
} // namespace aqz
