// aqz_codec.hip -- blosc1 + LZ4 compression of a resident chunk layer on
// gfx950 (see aqz_codec.hh for the parity contract).
//
//   lz4_streams         one 64-lane wave per split stream: gathers the
//                       stream out of its block through the byte shuffle
//                       or bitshuffle into LDS, then LZ4-encodes it:
//                       every lane hashes one position of a 64-position
//                       window against an LDS hash table (4-byte probe),
//                       a wave ballot marks the positions with a match,
//                       and the wave walks those greedily, extending each
//                       match 64 bytes per step (ballot of mismatches).
//   chunk_layout        per chunk: record offsets of its streams (block
//                       scan) and the frame size; memcpyed when the frame
//                       would not be smaller than the chunk (blosc's rule)
//   scan_offsets        frame offsets of the layer (exclusive scan)
//   write_frames        header, block starts and stream records, back to
//                       back in chunk order
#include "aqz_codec.hh"
#include "aqz_zstd.hh"

namespace aqz {

BloscGeom
make_blosc_geom(uint32_t nbytes, uint32_t typesize, uint32_t shuffle)
{
    BloscGeom g{};
    g.nbytes = nbytes;
    g.typesize = typesize;
    g.shuffle = shuffle;
    uint64_t bs = uint64_t(kLz4StreamMax) * typesize;
    if (bs > nbytes)
        bs = nbytes;
    bs -= bs % typesize;
    if (bs == 0)
        bs = nbytes; // fewer bytes than one pixel
    g.blocksize = uint32_t(bs);
    g.nfull = bs ? nbytes / g.blocksize : 0;
    g.left = bs ? nbytes % g.blocksize : 0;
    // the blosc1 decoder's split rule (never for the leftover block)
    g.ns_full = (typesize <= 16 && g.blocksize / typesize >= 128) ? typesize : 1;
    g.spc = g.nfull * g.ns_full + (g.left ? 1u : 0u);
    g.nblocks = g.nfull + (g.left ? 1u : 0u);
    g.slot = g.blocksize / g.ns_full;
    if (g.left > g.slot)
        g.slot = g.left;
    return g;
}

namespace {

constexpr uint32_t kHashSize = 1u << kLz4HashLog;

__device__ __forceinline__ uint32_t
lds_rd32(const uint32_t* w, uint32_t pos)
{
    const uint32_t lo = w[pos >> 2], hi = w[(pos >> 2) + 1];
    return __builtin_amdgcn_alignbyte(hi, lo, pos & 3u);
}

// Which stream of which block a (chunk, stream index) is.
struct StreamRef
{
    uint32_t j;     // block
    uint32_t s;     // stream inside the block
    uint32_t ns;    // streams of that block
    uint32_t bsize; // block bytes
    uint32_t len;   // stream bytes
};

__device__ __forceinline__ StreamRef
stream_ref(const BloscGeom& g, uint32_t q)
{
    StreamRef r;
    if (q < g.nfull * g.ns_full) {
        r.j = q / g.ns_full;
        r.s = q - r.j * g.ns_full;
        r.ns = g.ns_full;
        r.bsize = g.blocksize;
    } else {
        r.j = g.nfull;
        r.s = 0;
        r.ns = 1;
        r.bsize = g.left;
    }
    r.len = r.bsize / r.ns;
    return r;
}

// Byte x (0 <= x < bsize) of the shuffled block (c-blosc 1.x shuffle /
// bitshuffle; a block whose element count is not a multiple of 8 is not
// bit-shuffled).
__device__ __forceinline__ uint8_t
shuffled_byte(const uint8_t* blk, uint32_t bsize, uint32_t ts, uint32_t sh, uint32_t x)
{
    const uint32_t ne = bsize / ts;
    if (sh == 1 && ts > 1) {
        if (x >= ne * ts)
            return blk[x];
        const uint32_t jj = x / ne, i = x - jj * ne;
        return blk[i * ts + jj];
    }
    if (sh == 2 && ne % 8 == 0 && ne * ts == bsize) {
        const uint32_t row = ne / 8;
        const uint32_t r = x / row, m = x - r * row;
        const uint32_t jj = r >> 3, b = r & 7u;
        uint32_t v = 0;
        for (uint32_t k = 0; k < 8; ++k)
            v |= ((blk[(8 * m + k) * ts + jj] >> b) & 1u) << k;
        return uint8_t(v);
    }
    return blk[x];
}

// 8x8 bit transpose: byte b of the result holds bit b of every input byte
// (input byte k -> result bit k).
__device__ __forceinline__ uint64_t
transpose8(uint64_t x)
{
    uint64_t t;
    t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
    x = x ^ t ^ (t << 7);
    t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
    x = x ^ t ^ (t << 14);
    t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
    x = x ^ t ^ (t << 28);
    return x;
}

// Stream bytes -> LDS.  Fast paths for the split byte-shuffle / bitshuffle
// streams of 16-B aligned blocks; everything else byte by byte.
__device__ void
gather_stream(const BloscGeom& g, const StreamRef& r, const uint8_t* blk, uint8_t* sb)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t ts = g.typesize;
    const uint32_t ne = r.bsize / ts;
    const bool aligned = (reinterpret_cast<uintptr_t>(blk) & 15u) == 0;
    if (g.shuffle == 1 && ts > 1 && r.ns == ts && aligned && (ts == 2 || ts == 4 || ts == 8)) {
        // byte r.s of elements 4w .. 4w+3 -> word w
        uint32_t* sw = reinterpret_cast<uint32_t*>(sb);
#pragma unroll 8
        for (uint32_t w = lane; w < ne / 4; w += 64) {
            uint8_t e[32];
            if (ts == 2) {
                const uint2 v = *reinterpret_cast<const uint2*>(blk + 8 * w);
                __builtin_memcpy(e, &v, 8);
            } else if (ts == 4) {
                const uint4 v = *reinterpret_cast<const uint4*>(blk + 16 * w);
                __builtin_memcpy(e, &v, 16);
            } else {
                const uint4 v0 = *reinterpret_cast<const uint4*>(blk + 32 * w);
                const uint4 v1 = *reinterpret_cast<const uint4*>(blk + 32 * w + 16);
                __builtin_memcpy(e, &v0, 16);
                __builtin_memcpy(e + 16, &v1, 16);
            }
            sw[w] = uint32_t(e[r.s]) | uint32_t(e[ts + r.s]) << 8 |
                    uint32_t(e[2 * ts + r.s]) << 16 | uint32_t(e[3 * ts + r.s]) << 24;
        }
        for (uint32_t i = (ne / 4) * 4 + lane; i < ne; i += 64)
            sb[i] = blk[i * ts + r.s];
        return;
    }
    if (g.shuffle == 2 && r.ns == ts && ne % 8 == 0 && ne * ts == r.bsize) {
        // stream r.s = the 8 bit-planes of byte r.s of every element
        const uint32_t row = ne / 8;
#pragma unroll 4
        for (uint32_t m = lane; m < row; m += 64) {
            uint64_t x = 0;
            for (uint32_t k = 0; k < 8; ++k)
                x |= uint64_t(blk[(8 * m + k) * ts + r.s]) << (8 * k);
            x = transpose8(x);
            for (uint32_t b = 0; b < 8; ++b)
                sb[b * row + m] = uint8_t(x >> (8 * b));
        }
        return;
    }
    const uint32_t x0 = r.s * r.len;
    for (uint32_t k = lane; k < r.len; k += 64)
        sb[k] = shuffled_byte(blk, r.bsize, ts, g.shuffle, x0 + k);
}

// ---- LZ4 encoder: one wave per stream -----------------------------------
// Wave-wide inclusive prefix sum.
__device__ __forceinline__ uint32_t
wave_incl_scan(uint32_t x)
{
    const uint32_t lane = threadIdx.x & 63u;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (int(lane) >= d)
            x += y;
    }
    return x;
}

// value of lane i (wave-uniform i): v_readlane, no LDS round trip
__device__ __forceinline__ uint32_t
rdlane(uint32_t v, uint32_t i)
{
    return uint32_t(__builtin_amdgcn_readlane(int(v), int(i)));
}

// Length-extension bytes: n_ext bytes 255 ... 255, then the remainder.
__device__ __forceinline__ void
put_len_ext_lane(uint8_t* d, uint32_t n_ext, uint32_t rest)
{
    for (uint32_t k = 0; k + 1 < n_ext; ++k)
        d[k] = 255;
    if (n_ext)
        d[n_ext - 1] = uint8_t(rest - 255 * (n_ext - 1));
}

// Copies n stream bytes sb[s0..) to d with the whole wave.
__device__ __forceinline__ void
copy_lits(uint8_t* d, const uint8_t* sb, uint32_t s0, uint32_t n)
{
    for (uint32_t k = threadIdx.x; k < n; k += 64)
        d[k] = sb[s0 + k];
}

constexpr uint32_t kLenCap = 32; // match bytes measured per position up front
constexpr uint32_t kWin = 4;     // 64-position windows probed per batch
constexpr uint32_t kShortLits = 16; // literal runs copied by one lane

// LZ4 block of sb[0, L) -> dst; returns the compressed size, or 0 when it
// would not be smaller than L - 1 bytes (the caller then stores the stream
// raw, which blosc signals by csize == L).
//
// Per 64-position window: (A) every lane hashes its position, probes the
// table (any earlier position with the same hash is a valid candidate, so
// concurrent table stores may land in any order), verifies 4 bytes and
// measures the match up to kLenCap bytes with word compares; (B) the wave
// walks the ballot of match starts greedily with scalar steps, extending
// only matches that reached kLenCap (64 bytes per ballot), and records the
// window's sequences one per lane; (C) the sequences are encoded in
// parallel: a wave scan places them, each lane writes its token, lengths
// and offset, and the wave copies the literal runs.
__device__ uint32_t
lz4_wave(const uint8_t* sb, const uint32_t* sw, uint32_t L, uint16_t* table, uint8_t* dst)
{
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < kHashSize / 2; i += 64)
        reinterpret_cast<uint32_t*>(table)[i] = 0;
    __syncthreads();
    if (L < 13)
        return 0;
    const uint32_t mflimit = L - 12;   // last position a match may start
    const uint32_t matchlimit = L - 5; // a match ends at or before here
    const uint32_t cap = L - 1;
    uint32_t anchor = 0, p = 0, op = 0;
    uint32_t misses = 0; // consecutive batches without a match
    for (uint32_t base = 0; base <= mflimit;) {
        // (A) four 64-position windows at once: four independent probe
        // chains per lane (a batch does not see its own table stores)
        uint32_t cand[kWin], mlen[kWin];
        uint64_t M[kWin];
#pragma unroll
        for (uint32_t k = 0; k < kWin; ++k) {
            const uint32_t q = base + 64 * k + lane;
            cand[k] = 0;
            mlen[k] = 0;
            if (q <= mflimit) {
                const uint32_t v = lds_rd32(sw, q);
                const uint32_t h = (v * 2654435761u) >> (32 - kLz4HashLog);
                const uint32_t e = table[h];
                table[h] = uint16_t(q + 1);
                // the hash candidate, else the byte before (a run: offset 1)
                uint32_t c = ~0u;
                if (e != 0 && lds_rd32(sw, e - 1) == v)
                    c = e - 1;
                else if (q > 0 && lds_rd32(sw, q - 1) == v)
                    c = q - 1;
                if (c != ~0u) {
                    const uint32_t lim = min(matchlimit - q, kLenCap);
                    uint32_t len = 4;
                    bool done = false;
                    while (len + 4 <= lim) {
                        const uint32_t x = lds_rd32(sw, q + len) ^ lds_rd32(sw, c + len);
                        if (x) {
                            len += uint32_t(__builtin_ctz(x)) >> 3;
                            done = true;
                            break;
                        }
                        len += 4;
                    }
                    if (!done) // the last < 4 bytes up to the limit
                        while (len < lim && sb[q + len] == sb[c + len])
                            ++len;
                    cand[k] = c;
                    mlen[k] = len;
                }
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < kWin; ++k)
            M[k] = __ballot(mlen[k] != 0);
        // (B)
        uint32_t s_lit0 = 0, s_lit = 0, s_off = 0, s_len = 4; // lane k: sequence k
        uint32_t nseq = 0;
#pragma unroll
        for (uint32_t k = 0; k < kWin; ++k) {
            const uint32_t wb = base + 64 * k;
            while (p < wb + 64) {
                const uint32_t sh = p > wb ? p - wb : 0;
                const uint64_t mm = M[k] & (~0ull << sh);
                if (mm == 0)
                    break;
                const uint32_t i = uint32_t(__ffsll(static_cast<long long>(mm))) - 1;
                const uint32_t qq = wb + i;
                const uint32_t cc = rdlane(cand[k], i);
                uint32_t len = rdlane(mlen[k], i);
                if (len == kLenCap) {
                    for (;;) {
                        const uint32_t a = qq + len + lane;
                        const bool eq = a < matchlimit && sb[a] == sb[cc + len + lane];
                        const uint64_t miss = __ballot(!eq);
                        if (miss == 0) {
                            len += 64;
                            continue;
                        }
                        len += uint32_t(__ffsll(static_cast<long long>(miss))) - 1;
                        break;
                    }
                }
                if (lane == nseq) {
                    s_lit0 = anchor;
                    s_lit = qq - anchor;
                    s_off = qq - cc;
                    s_len = len;
                }
                ++nseq;
                p = qq + len;
                anchor = p;
            }
        }
        // (C)
        if (nseq) {
            const bool mine = lane < nseq;
            const uint32_t ml = s_len - 4;
            const uint32_t le = s_lit >= 15 ? (s_lit - 15) / 255 + 1 : 0;
            const uint32_t me = ml >= 15 ? (ml - 15) / 255 + 1 : 0;
            const uint32_t sz = mine ? 1 + le + s_lit + 2 + me : 0;
            const uint32_t incl = wave_incl_scan(sz);
            const uint32_t total = rdlane(incl, nseq - 1);
            if (op + total > cap)
                return 0;
            if (mine) {
                uint8_t* d = dst + op + incl - sz;
                d[0] = uint8_t((s_lit < 15 ? s_lit : 15) << 4 | (ml < 15 ? ml : 15));
                put_len_ext_lane(d + 1, le, s_lit - 15);
                uint8_t* o = d + 1 + le + s_lit;
                o[0] = uint8_t(s_off & 255u);
                o[1] = uint8_t(s_off >> 8);
                put_len_ext_lane(o + 2, me, ml - 15);
            }
            // literal runs: short ones by their own lane, long ones by the wave
            if (mine && s_lit <= kShortLits) {
                uint8_t* d = dst + op + incl - sz + 1 + le;
                for (uint32_t k = 0; k < s_lit; ++k)
                    d[k] = sb[s_lit0 + k];
            }
            uint64_t longs = __ballot(mine && s_lit > kShortLits);
            while (longs) {
                const uint32_t k = uint32_t(__ffsll(static_cast<long long>(longs))) - 1;
                longs &= longs - 1;
                const uint32_t n = rdlane(s_lit, k);
                const uint32_t start = rdlane(incl - sz, k);
                const uint32_t lel = (n - 15) / 255 + 1;
                copy_lits(dst + op + start + 1 + lel, sb, rdlane(s_lit0, k), n);
            }
            op += total;
            misses = 0;
        } else {
            ++misses;
        }
        // incompressible runs are probed ever more sparsely (LZ4's
        // acceleration): after m batches without a match, m-1 are skipped
        const uint32_t skip = misses > 1 ? (misses - 1) * 64 * kWin : 0;
        base = max(base + 64 * kWin + skip, p & ~63u);
    }
    // the last literals
    const uint32_t n = L - anchor;
    const uint32_t le = n >= 15 ? (n - 15) / 255 + 1 : 0;
    if (op + 1 + le + n > cap)
        return 0;
    if (lane == 0) {
        dst[op] = uint8_t((n < 15 ? n : 15) << 4);
        put_len_ext_lane(dst + op + 1, le, n - 15);
    }
    copy_lits(dst + op + 1 + le, sb, anchor, n);
    return op + 1 + le + n;
}

__global__ __launch_bounds__(64) void
lz4_streams(const BloscParams p)
{
    __shared__ __attribute__((aligned(16))) uint32_t sw[kLz4StreamMax / 4 + 4];
    __shared__ __attribute__((aligned(16))) uint16_t table[kHashSize];
    const uint32_t gid = blockIdx.x;
    const uint32_t c = gid / p.g.spc, q = gid - c * p.g.spc;
    if (p.flags && p.flags[c] != p.tag) {
        if (threadIdx.x == 0)
            p.ssize[gid] = 0;
        return;
    }
    const StreamRef r = stream_ref(p.g, q);
    if (p.store_only) { // raw streams add up past nbytes + 16: memcpyed
        if (threadIdx.x == 0)
            p.ssize[gid] = r.len;
        return;
    }
    const uint8_t* blk = p.chunks + c * p.pitch + uint64_t(r.j) * p.g.blocksize;
    uint8_t* dst = p.scratch + uint64_t(gid) * p.g.slot;
    if (r.len > kLz4StreamMax) {
        // an oversized leftover block: stored raw, straight from HBM
        for (uint32_t k = threadIdx.x; k < r.len; k += 64)
            dst[k] = shuffled_byte(blk, r.bsize, p.g.typesize, p.g.shuffle, k);
        if (threadIdx.x == 0)
            p.ssize[gid] = r.len;
        return;
    }
    uint8_t* sb = reinterpret_cast<uint8_t*>(sw);
    gather_stream(p.g, r, blk, sb);
    for (uint32_t k = r.len + threadIdx.x; k < r.len + 8; k += 64)
        sb[k] = 0;
    __syncthreads();
    uint32_t n = lz4_wave(sb, sw, r.len, table, dst);
    if (n == 0) {
        // raw: words when the slot is 4-B aligned (slots are), bytes for the tail
        const uint32_t nw = (reinterpret_cast<uintptr_t>(dst) & 3u) ? 0 : r.len / 4;
        for (uint32_t k = threadIdx.x; k < nw; k += 64)
            reinterpret_cast<uint32_t*>(dst)[k] = sw[k];
        for (uint32_t k = nw * 4 + threadIdx.x; k < r.len; k += 64)
            dst[k] = sb[k];
        n = r.len;
    }
    if (threadIdx.x == 0)
        p.ssize[gid] = n;
}


// Exclusive block-wide scan of one value per thread (256 threads); returns
// the prefix, *total = the sum over the block.
__device__ uint32_t
block_scan256(uint32_t v, uint32_t* total)
{
    __shared__ uint32_t wsum[4];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (int(lane) >= d)
            x += y;
    }
    if (lane == 63)
        wsum[w] = x;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t k = 0; k < 4; ++k) {
        if (k < w)
            before += wsum[k];
        all += wsum[k];
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

__global__ __launch_bounds__(256) void
chunk_layout(const BloscParams p)
{
    const uint32_t c = blockIdx.x;
    const bool skip = p.flags && p.flags[c] != p.tag;
    const uint32_t hdr = 16 + 4 * p.g.nblocks;
    uint32_t carry = hdr;
    for (uint32_t q0 = 0; q0 < p.g.spc; q0 += 256) {
        const uint32_t q = q0 + threadIdx.x;
        const uint32_t rec = q < p.g.spc ? 4 + p.ssize[uint64_t(c) * p.g.spc + q] : 0;
        uint32_t tot;
        const uint32_t pre = block_scan256(rec, &tot);
        if (q < p.g.spc)
            p.spos[uint64_t(c) * p.g.spc + q] = carry + pre;
        carry += tot;
    }
    if (threadIdx.x == 0) {
        const bool memcpyed = uint64_t(carry) > uint64_t(p.g.nbytes) + 16;
        p.fsize[c] = skip ? 0 : (memcpyed ? p.g.nbytes + 16 : carry);
        p.mode[c] = memcpyed ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void
scan_offsets(const uint32_t* fsize, const uint32_t* order, uint64_t* offsets,
             uint64_t* cstart, uint32_t n)
{
    __shared__ uint64_t carry_s;
    if (threadIdx.x == 0)
        carry_s = 0;
    __syncthreads();
    for (uint32_t i0 = 0; i0 < n; i0 += 256) {
        const uint32_t i = i0 + threadIdx.x;
        const uint32_t c = i < n ? (order ? order[i] : i) : 0;
        const uint32_t v = i < n ? fsize[c] : 0;
        uint32_t tot;
        const uint32_t pre = block_scan256(v, &tot);
        const uint64_t carry = carry_s;
        if (i < n) {
            offsets[i] = carry + pre;
            cstart[c] = carry + pre;
        }
        __syncthreads();
        if (threadIdx.x == 0)
            carry_s = carry + tot;
        __syncthreads();
    }
    if (threadIdx.x == 0)
        offsets[n] = carry_s;
}

__device__ __forceinline__ void
put32(uint8_t* d, uint32_t v)
{
    d[0] = uint8_t(v);
    d[1] = uint8_t(v >> 8);
    d[2] = uint8_t(v >> 16);
    d[3] = uint8_t(v >> 24);
}

// n bytes s -> d for any alignment of either, by the whole workgroup:
// dword stores at dword-aligned destinations, each assembled from two
// aligned source dwords (v_alignbyte); only the head and tail go by byte.
// Never reads past s + n.
__device__ __forceinline__ void
copy_bytes(uint8_t* d, const uint8_t* s, uint32_t n)
{
    const uint32_t t = threadIdx.x, nt = blockDim.x;
    uint32_t head = (4u - uint32_t(reinterpret_cast<uintptr_t>(d) & 3u)) & 3u;
    if (head > n)
        head = n;
    for (uint32_t k = t; k < head; k += nt)
        d[k] = s[k];
    d += head;
    s += head;
    n -= head;
    const uint32_t nw = n / 4;
    uint32_t* dw = reinterpret_cast<uint32_t*>(d);
    const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(s) & 3u);
    if (sh == 0) {
        const uint32_t* sw = reinterpret_cast<const uint32_t*>(s);
        for (uint32_t i = t; i < nw; i += nt)
            dw[i] = sw[i];
    } else {
        // source dwords i and i+1 cover destination dword i; the last one
        // would read up to 3 bytes past the end, so it goes by byte
        const uint32_t* sw = reinterpret_cast<const uint32_t*>(s - sh);
        for (uint32_t i = t; i + 1 < nw; i += nt)
            dw[i] = __builtin_amdgcn_alignbyte(sw[i + 1], sw[i], sh);
        if (nw > 0 && t == 0)
            for (uint32_t k = 4 * (nw - 1); k < 4 * nw; ++k)
                d[k] = s[k];
    }
    for (uint32_t k = 4 * nw + t; k < n; k += nt)
        d[k] = s[k];
}

__global__ __launch_bounds__(256) void
write_frames(const BloscParams p)
{
    const uint32_t gid = blockIdx.x;
    const uint32_t c = gid / p.g.spc, q = gid - c * p.g.spc;
    const uint32_t fs = p.fsize[c];
    if (fs == 0)
        return;
    uint8_t* o = p.out + p.cstart[c];
    const bool memcpyed = p.mode[c] != 0;
    if (q == 0 && threadIdx.x == 0) {
        o[0] = 2; // BLOSC_VERSION_FORMAT
        o[1] = 1; // BLOSC_LZ4_VERSION_FORMAT
        o[2] = uint8_t(1u << 5 | (p.g.shuffle == 1 ? 0x1u : 0u) |
                       (p.g.shuffle == 2 ? 0x4u : 0u) | (memcpyed ? 0x2u : 0u));
        o[3] = uint8_t(p.g.typesize);
        put32(o + 4, p.g.nbytes);
        put32(o + 8, p.g.blocksize);
        put32(o + 12, fs);
    }
    const uint8_t* chunk = p.chunks + c * p.pitch;
    if (memcpyed) {
        const uint32_t per = (p.g.nbytes + p.g.spc - 1) / p.g.spc;
        const uint32_t x0 = min(p.g.nbytes, q * per), x1 = min(p.g.nbytes, x0 + per);
        copy_bytes(o + 16 + x0, chunk + x0, x1 - x0);
        return;
    }
    const uint64_t sidx = uint64_t(c) * p.g.spc;
    if (q == 0) {
        for (uint32_t j = threadIdx.x; j < p.g.nblocks; j += 256)
            put32(o + 16 + 4 * j, p.spos[sidx + j * p.g.ns_full]);
    }
    const uint32_t n = p.ssize[gid];
    uint8_t* rec = o + p.spos[gid];
    if (threadIdx.x == 0)
        put32(rec, n);
    copy_bytes(rec + 4, p.scratch + uint64_t(gid) * p.g.slot, n);
}

// One workgroup per (block, chunk, part): the c-blosc 1.x byte shuffle (byte
// jj of element i -> jj * ne + i) or bitshuffle (bit b of byte jj of element
// 8m + k -> bit k of byte m of plane 8 jj + b) of one block, the block's
// elements split over gridDim.z parts (small layers: enough workgroups to
// keep the loads in flight).  The scalar fallbacks run in part 0.
__global__ __launch_bounds__(256) void
shuffle_blocks(const ShuffleParams p)
{
    const uint32_t j = blockIdx.x, c = blockIdx.y, part = blockIdx.z, np = gridDim.z;
    if (p.flags && p.flags[c] != p.tag)
        return;
    const uint32_t t = threadIdx.x;
    const uint32_t b0 = j * p.blocksize;
    const uint32_t bsize = min(p.blocksize, p.nbytes - b0);
    const uint32_t ts = p.typesize;
    const uint32_t ne = bsize / ts;
    // restrict: the stores may not alias the next loads, so several loads
    // stay in flight (without it every load waited for the previous
    // iteration's stores: 1.1 TB/s)
    const uint8_t* __restrict__ src = p.chunks + c * p.pitch + b0;
    uint8_t* __restrict__ dst = p.out + uint64_t(c) * p.nbytes + b0;
    const bool src16 = (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
    if (p.shuffle == 1 && ts > 1) {
        uint32_t done = 0; // elements handled by the vector path
        if ((ts == 2 || ts == 4 || ts == 8) && src16) {
            const uint32_t vec = 16 / ts; // elements per 16-B load
            const bool dst_ok = (reinterpret_cast<uintptr_t>(dst) % vec) == 0 && ne % vec == 0;
            if (dst_ok) {
                // this part's 16-B words, in batches of 4 rounds: 4
                // independent loads per lane in flight, then their stores
                const uint32_t nw = ne / vec;
                const uint32_t lo = uint32_t(uint64_t(nw) * part / np);
                const uint32_t hi = uint32_t(uint64_t(nw) * (part + 1) / np);
                // 8 nontemporal 16-B loads in flight per lane, then their
                // stores (4 plain loads: 0.70 ms per 512 MiB layer, 8 nt:
                // 0.42 ms; nt stores: no gain)
                constexpr uint32_t kB = 8;
                for (uint32_t w0 = lo; w0 < hi; w0 += kB * 256) {
                    uint4 v[kB];
#pragma unroll
                    for (uint32_t u = 0; u < kB; ++u) {
                        const uint32_t w = w0 + u * 256 + t;
                        typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
                        if (w < hi) {
                            const u32x4v a = __builtin_nontemporal_load(
                              reinterpret_cast<const u32x4v*>(src + 16ull * w));
                            v[u] = uint4{ a.x, a.y, a.z, a.w };
                        }
                    }
#pragma unroll
                    for (uint32_t u = 0; u < kB; ++u) {
                        const uint32_t w = w0 + u * 256 + t;
                        if (w >= hi)
                            continue;
                        uint8_t e[16];
                        __builtin_memcpy(e, &v[u], 16);
                        for (uint32_t jj = 0; jj < ts; ++jj) {
                            uint8_t o[8];
                            for (uint32_t k = 0; k < vec; ++k)
                                o[k] = e[k * ts + jj];
                            uint8_t* d = dst + uint64_t(jj) * ne + uint64_t(w) * vec;
                            if (vec == 8) {
                                uint2 x;
                                __builtin_memcpy(&x, o, 8);
                                *reinterpret_cast<uint2*>(d) = x;
                            } else if (vec == 4) {
                                uint32_t x;
                                __builtin_memcpy(&x, o, 4);
                                *reinterpret_cast<uint32_t*>(d) = x;
                            } else {
                                uint16_t x;
                                __builtin_memcpy(&x, o, 2);
                                *reinterpret_cast<uint16_t*>(d) = x;
                            }
                        }
                    }
                }
                done = ne;
            }
        }
        if (part != 0)
            return;
        for (uint32_t x = t; x < (ne - done) * ts; x += 256) {
            const uint32_t i = done + x / ts, jj = x % ts;
            dst[uint64_t(jj) * ne + i] = src[uint64_t(i) * ts + jj];
        }
        for (uint32_t x = ne * ts + t; x < bsize; x += 256)
            dst[x] = src[x];
        return;
    }
    if (p.shuffle == 2 && ne % 8 == 0 && ne * ts == bsize) {
        const uint32_t row = ne / 8;
        const uint32_t lo = uint32_t(uint64_t(row) * part / np);
        const uint32_t hi = uint32_t(uint64_t(row) * (part + 1) / np);
#pragma unroll 4
        for (uint32_t m = lo + t; m < hi; m += 256) {
            const uint8_t* g = src + uint64_t(8) * m * ts; // 8 elements
            for (uint32_t jj = 0; jj < ts; ++jj) {
                uint64_t x = 0;
                for (uint32_t k = 0; k < 8; ++k)
                    x |= uint64_t(g[k * ts + jj]) << (8 * k);
                x = transpose8(x);
                for (uint32_t b = 0; b < 8; ++b)
                    dst[uint64_t(jj * 8 + b) * row + m] = uint8_t(x >> (8 * b));
            }
        }
        return;
    }
    if (part != 0)
        return;
    for (uint32_t x = t; x < bsize; x += 256)
        dst[x] = src[x];
}


// ---- device zstd (aqz_codec.hh ZstdParams; format pieces in aqz_zstd.hh) ----
//   zstd_parse   per 4 KiB unit, one wave (match mode): greedy LZ parse with
//                the LZ4 encoder's window probing (4 x 64 positions hashed
//                per batch against an LDS table, ballot, scalar walk), a
//                minimum match length from the unit's byte entropy; packed
//                sequences and the literal bytes go to the unit's slots, the
//                literal histogram to its block
//   zstd_hist    per zstd block (literals-only mode): byte histogram
//   zstd_table   per segment (one zstd frame): Huffman code of the frame's
//                literals and its tree description
//   zstd_encode  per zstd block: RLE when one byte value; the 4 Huffman
//                streams, one wave each (lane-parallel bit packing: each lane
//                owns a run of literals, a suffix scan of their bit counts
//                places it -- a stream is written last literal first); the
//                sequences pre-coded (codes + extra bits) and compacted
//   zstd_seqenc  one lane per block: the sequences' FSE bitstream
//                (backwards); compressed iff smaller than the block counted
//                with the tree
//   zstd_segment per segment: which block carries the tree, block offsets,
//                frame bytes; a blosc record larger than its block is raw
//   zstd_chunk   per chunk: blosc record offsets / memcpyed rule, frame bytes
//   zstd_write   per zstd block: headers, tree, payload or raw bytes
constexpr uint32_t kZMinHuf = 64; // fewer literals: raw (as the host model)
// a Huffman stream is kept only when it is not larger than its literals:
// room for 8 bits per literal (+ end mark and the word a code straddles)
constexpr uint32_t kZStreamWords = (zstd::kBlock / 4 * 8) / 32 + 4;
static_assert(4 * kZStreamWords <= 4096, "stream buffers fit the encode kernel's LDS");

struct ZBlock
{
    uint32_t c, j, b, seg, len, seglen, nb, grp;
};

__device__ __forceinline__ ZBlock
zblock(const ZstdParams& p, uint32_t g)
{
    ZBlock z;
    z.b = g % p.bps;
    z.seg = g / p.bps;
    z.c = z.seg / p.nseg;
    z.j = z.seg - z.c * p.nseg;
    const uint64_t s0 = uint64_t(z.j) * p.seg_bytes;
    z.seglen = uint32_t(min(uint64_t(p.seg_bytes), uint64_t(p.nbytes) - s0));
    z.nb = (z.seglen + zstd::kBlock - 1) / zstd::kBlock;
    const uint32_t o = z.b * zstd::kBlock;
    z.len = o < z.seglen ? min(zstd::kBlock, z.seglen - o) : 0;
    z.grp = z.seg * p.ngrp + (z.b >> p.hgrp_log2);
    return z;
}

__device__ __forceinline__ const uint8_t*
zblock_src(const ZstdParams& p, const ZBlock& z)
{
    return p.src + z.c * p.src_pitch + uint64_t(z.j) * p.seg_bytes + uint64_t(z.b) * zstd::kBlock;
}

__device__ __forceinline__ bool
zchunk_skip(const ZstdParams& p, uint32_t c)
{
    return p.flags && p.flags[c] != p.tag;
}

// Far candidates for the parse: libzstd's levels >= 3 find most of their
// matches on noisy camera data 8 KiB - 2 MiB back -- 5-byte coincidences no
// unit-local window sees (tools/zstd_lab.cpp).  A segment's positions are
// split by a 32-bit hash of their 5-byte key into p.far_slices slices; one
// workgroup per (segment, slice) walks the whole segment in order, one parse
// unit (kZSub bytes) per step, and keeps for its slice a table of 2^kFarLog
// entries in LDS: (position + 1) << far_tb | tag, the most recent position
// per bucket.  Each step first probes (a tag-equal entry is the candidate:
// far[i] = its position + 1, else 0), then inserts the step's positions (LDS
// atomic max: the latest wins), so a position sees every earlier unit; the
// parse's own table covers its unit.  The next step's bytes are loaded while
// the current one is probed.  The slices of one segment run on one XCD
// (their far[] stores interleave in the same lines).  The parse verifies
// every candidate.  A layer of few segments splits each into p.far_ranges
// ranges walked at once: a range first inserts the p.far_warm steps before
// it without probing, so it misses only candidates further back than that
// (e2e zstd level 3: 22.5 -> 28.4 GB/s, the same bytes to 4 digits).
constexpr uint32_t kFarThreads = 1024;
static_assert(kZSub == 4 * kFarThreads, "one parse unit per far step, 4 positions a thread");

__device__ __forceinline__ uint32_t
far_hash(uint32_t lo, uint32_t hi)
{
    // the two products kept apart: fused into v_mad_u64_u32, their sum took
    // a 64-bit addend whose undefined high half the allocator could place in
    // a register a prefetch is loading, and the step waited for that load
    uint32_t m0 = lo * 0x9E3779B1u, m1 = hi * 0x7FEB352Du;
    asm volatile("" : "+v"(m0));
    asm volatile("" : "+v"(m1));
    uint32_t h = m0 + m1;
    h ^= h >> 15;
    h *= 0x846CA68Bu;
    h ^= h >> 16;
    return h;
}

__global__ __launch_bounds__(kFarThreads) void
zstd_far(const ZstdParams p)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t T[]; // 2^far_log entries
    // a segment's workgroups: S hash slices x R ranges
    const uint32_t S = p.far_slices, R = p.far_ranges, SR = S * R;
    const uint32_t nb = gridDim.x, b = blockIdx.x;
    const uint32_t grp = 8u * SR, full = nb - nb % grp;
    uint32_t seg, sr;
    if (b < full) { // groups of 8 segments x S*R workgroups, a segment's on XCD b % 8
        seg = (b / grp) * 8 + (b & 7u);
        sr = (b % grp) >> 3;
    } else {
        seg = b / SR;
        sr = b % SR;
    }
    const uint32_t slice = sr % S, range = sr / S;
    const uint32_t c = seg / p.nseg, j = seg - c * p.nseg;
    if (zchunk_skip(p, c))
        return;
    const uint64_t s0 = uint64_t(j) * p.seg_bytes;
    const uint32_t len = uint32_t(min(uint64_t(p.seg_bytes), uint64_t(p.nbytes) - s0));
    const uint8_t* src = p.src + c * p.src_pitch + s0;
    uint32_t* far = p.far + uint64_t(seg) * p.seg_bytes;
    const uint32_t t = threadIdx.x, TB = p.far_tb, tmask = (1u << TB) - 1u, FL = p.far_log;
    const uint32_t sbits = 31u - uint32_t(__builtin_clz(S)); // log2 of the slices
    const uint32_t bshift = 32u - sbits - FL;
    for (uint32_t i = t; i < (1u << FL); i += kFarThreads)
        T[i] = 0;
    // positions with fewer than 5 bytes after them have no key
    const uint32_t nkey = len >= 5 ? len - 4 : 0;
    if (slice == 0 && range == 0)
        for (uint32_t i = nkey + t; i < len; i += kFarThreads)
            far[i] = 0;
    const uint32_t nsteps = (nkey + kZSub - 1) / kZSub;
    // one step: probe the slice's positions among [i0, i0 + 4) (bytes
    // [i0, i0 + 8) in a, d), store their candidates, then insert them
    auto hash4 = [&](uint32_t a, uint32_t d, uint32_t* h) {
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            h[k] = far_hash(__builtin_amdgcn_alignbyte(d, a, k), (d >> (8 * k)) & 255u);
    };
    // positions [ibeg, iend) are probed (and their candidates stored), the
    // ones from iwarm inserted; the single-range walk: 0, 0, nkey
    auto step = [&](uint32_t i0, const uint32_t* h, auto&& store, uint32_t iwarm, uint32_t ibeg,
                    uint32_t iend) {
        bool mine[4], probe[4];
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t i = i0 + k;
            mine[k] = i >= iwarm && i < iend &&
                      (sbits == 0 || (h[k] >> (32u - sbits)) == slice);
            probe[k] = mine[k] && i >= ibeg;
            uint32_t fv = 0;
            if (probe[k]) {
                const uint32_t e = T[(h[k] >> bshift) & ((1u << FL) - 1u)];
                fv = (e != 0 && (e & tmask) == (h[k] & tmask)) ? (e >> TB) : 0u;
            }
            store(i, probe[k], fv);
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < 4; ++k)
            if (mine[k])
                atomicMax(&T[(h[k] >> bshift) & ((1u << FL) - 1u)],
                          ((i0 + k + 1) << TB) | (h[k] & tmask));
        __syncthreads();
    };
    if ((len & 3u) == 0 && uint64_t(len) * 4 < (uint64_t(1) << 31)) {
        // Buffer loads and stores: a load past the segment reads 0 and a
        // store to another slice's position goes to an out-of-range offset
        // and is dropped, so no memory access sits under a branch and the
        // compiler's wait before a step's first use of its bytes leaves the
        // younger loads and the stores in flight.  The bytes are loaded
        // kFarAhead steps ahead.  (len % 4 == 0: a dword is in or out.)
        constexpr uint32_t kFarAhead = 4;
        const __amdgpu_buffer_rsrc_t sr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<uint8_t*>(src), 0, int32_t(len), 0x00020000);
        const __amdgpu_buffer_rsrc_t fr =
          __builtin_amdgcn_make_buffer_rsrc(far, 0, int32_t(nkey * 4), 0x00020000);
        auto ld = [&](uint32_t off) -> uint32_t {
            return __builtin_amdgcn_raw_buffer_load_b32(sr, int32_t(off), 0, 0);
        };
        auto st = [&](uint32_t i, bool m, uint32_t fv) {
            __builtin_amdgcn_raw_buffer_store_b32(fv, fr, int32_t(m ? 4 * i : 0x80000000u), 0,
                                                  0);
        };
        // this workgroup's range of steps [s1, s2), warmed up from s0
        const uint32_t per = (nsteps + R - 1) / R;
        const uint32_t s1 = min(range * per, nsteps), s2 = min(s1 + per, nsteps);
        const uint32_t s0 = s1 > p.far_warm ? s1 - p.far_warm : 0u;
        const uint32_t iwarm = s0 * kZSub, ibeg = s1 * kZSub, iend = min(s2 * kZSub, nkey);
        uint32_t ra[kFarAhead], rd[kFarAhead];
        // the prologue issues what a step issues (two loads, four stores;
        // the stores out of range, dropped): the compiler's wait at the loop
        // head merges this path with the back edge, and a shorter queue here
        // would make it wait for all but the last step's loads there
#pragma unroll
        for (uint32_t u = 0; u < kFarAhead; ++u) {
            ra[u] = ld((s0 + u) * kZSub + 4 * t);
            rd[u] = ld((s0 + u) * kZSub + 4 * t + 4);
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) // distinct, unmergeable offsets
                __builtin_amdgcn_raw_buffer_store_b32(0u, fr, int32_t(0x80000000u + 256 * (4 * u + k)),
                                                      0, 0);
        }
        __syncthreads();
        // whole groups of kFarAhead steps: a step past the segment loads
        // zeros and stores nothing (no break, so each ra/rd keeps its
        // register and a load is waited for only where it is used)
        for (uint32_t s = s0; s < s2; s += kFarAhead) {
#pragma unroll
            for (uint32_t u = 0; u < kFarAhead; ++u) {
                const uint32_t i0 = (s + u) * kZSub + 4 * t;
                // hash first: ra/rd are dead before their next load is
                // issued into them (no copy at the loop's back edge, which
                // would wait for the loads of the last steps)
                uint32_t h[4];
                hash4(ra[u], rd[u], h);
                ra[u] = ld(i0 + kFarAhead * kZSub);
                rd[u] = ld(i0 + kFarAhead * kZSub + 4);
                step(i0, h, st, iwarm, ibeg, iend);
            }
        }
        return;
    }
    // the generic walk (a segment of len % 4 != 0): one range, the whole segment
    if (range != 0)
        return;
    // bytes [i0, i0 + 8) of this thread's step (zero past the segment)
    auto load = [&](uint32_t i0, uint32_t& a, uint32_t& d) {
        if (i0 + 8 <= len) {
            a = *reinterpret_cast<const uint32_t*>(src + i0);
            d = *reinterpret_cast<const uint32_t*>(src + i0 + 4);
        } else {
            a = d = 0;
            for (uint32_t k = 0; k < 8 && i0 + k < len; ++k)
                (k < 4 ? a : d) |= uint32_t(src[i0 + k]) << (8 * (k & 3u));
        }
    };
    auto gst = [&](uint32_t i, bool m, uint32_t fv) {
        if (m)
            far[i] = fv;
    };
    uint32_t a = 0, d = 0;
    if (4 * t < nkey)
        load(4 * t, a, d);
    __syncthreads();
    for (uint32_t b0 = 0; b0 < nkey; b0 += kZSub) {
        const uint32_t i0 = b0 + 4 * t;
        uint32_t na = 0, nd = 0;
        if (i0 + kZSub < nkey)
            load(i0 + kZSub, na, nd);
        uint32_t h[4];
        hash4(a, d, h);
        step(i0, h, gst, 0u, 0u, nkey);
        a = na;
        d = nd;
    }
}

// FAR: p.far holds zstd_far's candidates; a lane keeps the longer of its
// local match and the verified far one (>= kFarMin bytes, measured up to 16).
template<uint32_t HIST, uint32_t HLOG, bool FAR = false>
__global__ __launch_bounds__(64) void
zstd_parse(const ZstdParams p)
{
    __shared__ __attribute__((aligned(16))) uint32_t sw[(HIST + kZSub) / 4 + 4];
    __shared__ uint16_t table[1u << HLOG];
    __shared__ uint32_t lh[256];
    // FAR: the units are dealt to the 8 XCDs in contiguous ranges (block b
    // runs on XCD b mod 8), so an XCD walks its chunks in order and the far
    // candidates its units verify -- mostly within the last MiB of the same
    // chunk -- were just read through the same L2
    uint32_t q = blockIdx.x;
    if constexpr (FAR) {
        const uint32_t per = gridDim.x >> 3;
        if (q < (per << 3))
            q = (q & 7u) * per + (q >> 3);
    }
    const uint32_t g = q / kZSubBlocks, k = q - g * kZSubBlocks;
    const uint32_t lane = threadIdx.x;
    const ZBlock z = zblock(p, g);
    const uint32_t so = k * kZSub;
    // the unit's sequences go straight to its global slots (lane 0 stores;
    // LDS is the occupancy limit, kZSubSeq of them would take 8 KiB)
    uint64_t* sseq = p.seqs + uint64_t(q) * kZSubSeq;
    const uint32_t L = so < z.len ? min(kZSub, z.len - so) : 0;
    if (L == 0 || zchunk_skip(p, z.c)) {
        if (lane == 0) {
            p.snseq[q] = 0;
            p.snlit[q] = 0;
            p.stail[q] = 0;
        }
        return;
    }
    const uint8_t* src = zblock_src(p, z) + so;
    // units tile their segment in kZSub steps, so H is a multiple of kZSub
    const uint32_t H = min(HIST, z.b * zstd::kBlock + so);
    uint8_t* sb = reinterpret_cast<uint8_t*>(sw);
    for (uint32_t b = lane; b < 256; b += 64)
        lh[b] = 0;
    for (uint32_t i = lane; i < (1u << HLOG) / 2; i += 64)
        reinterpret_cast<uint32_t*>(table)[i] = 0;
    if (HIST > 0 && H > 0) {
        const uint8_t* hs = src - H;
        if ((reinterpret_cast<uintptr_t>(hs) & 15u) == 0) {
            const uint4* h16 = reinterpret_cast<const uint4*>(hs);
            for (uint32_t w = lane; w < H / 16; w += 64)
                reinterpret_cast<uint4*>(sw)[w] = h16[w];
        } else {
            for (uint32_t i = lane; i < H; i += 64)
                sb[i] = hs[i];
        }
    }
    const bool whole = L == kZSub && (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
    if (whole) {
        // lane l holds bytes [64l, 64l + 64): staged to LDS and counted from
        // registers, one LDS atomic per run of equal bytes (the high byte
        // planes of shuffled camera data are long runs; per-byte atomics on
        // them serialised on one address)
        const uint4* s16 = reinterpret_cast<const uint4*>(src) + 4 * lane;
        uint4 r[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            r[j] = s16[j];
        __syncthreads(); // lh zeroed
#pragma unroll
        for (int j = 0; j < 4; ++j)
            reinterpret_cast<uint4*>(sw)[H / 16 + 4 * lane + j] = r[j];
        uint32_t cur = r[0].x & 255u, run = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t wd[4] = { r[j].x, r[j].y, r[j].z, r[j].w };
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const uint32_t v = (wd[k] >> (8 * b)) & 255u;
                    if (v != cur) {
                        atomicAdd(&lh[cur], run);
                        cur = v;
                        run = 0;
                    }
                    ++run;
                }
        }
        atomicAdd(&lh[cur], run);
        if (lane < 2)
            sw[(H + kZSub) / 4 + lane] = 0;
    } else {
        uint8_t* ub = sb + H;
        if ((reinterpret_cast<uintptr_t>(src) & 3u) == 0) {
            const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
            for (uint32_t w = lane; w < L / 4; w += 64)
                sw[H / 4 + w] = s4[w];
            for (uint32_t i = (L & ~3u) + lane; i < L; i += 64)
                ub[i] = src[i];
        } else {
            for (uint32_t i = lane; i < L; i += 64)
                ub[i] = src[i];
        }
        for (uint32_t i = L + lane; i < L + 8; i += 64)
            ub[i] = 0;
        __syncthreads();
        for (uint32_t i = lane; i < L; i += 64)
            atomicAdd(&lh[ub[i]], 1u);
    }
    __syncthreads();
    if (HIST > 0 && H > 0) {
        // the history's positions into the table (insert only; concurrent
        // stores to one slot land in any order: every entry is a valid
        // earlier position)
        for (uint32_t i = lane; i < H; i += 64) {
            const uint32_t v = lds_rd32(sw, i);
            table[(v * 2654435761u) >> (32 - HLOG)] = uint16_t(i + 1);
        }
        __syncthreads();
    }
    float e = 0.f;
    uint32_t one = 256; // the unit's only byte value, if it has one
    for (uint32_t b = lane; b < 256; b += 64)
        if (lh[b]) {
            const float pr = float(lh[b]) / float(L);
            e -= pr * __log2f(pr);
            if (lh[b] == L)
                one = b;
        }
    for (int d = 32; d > 0; d >>= 1) {
        e += __shfl_xor(e, d);
        one = min(one, uint32_t(__shfl_xor(int(one), d)));
    }
    // a block is RLE only when its bytes are one value -- its literals being
    // one value is not enough once matches copy from the history
    if (lane == 0)
        p.sval[q] = one;
    const uint32_t minlen = zstd::min_match(e, kLenCap, float(p.match_bits));
    // lh keeps the unit's byte histogram: it is the literal histogram
    // when the parse finds no sequence

    // greedy parse: probe four 64-position windows, walk the matches
    // (positions are LDS offsets: the unit starts at H)
    uint32_t nseq = 0, anchor = H, p0 = H, misses = 0;
    bool full = false;
    if (L >= 8) {
        const uint32_t mflimit = H + L - 4; // last position a match may start
        const uint32_t matchlimit = H + L;  // a match ends at or before here
        // FAR: the segment, its far candidates, the unit's segment offset
        const uint8_t* seg = p.src + z.c * p.src_pitch + uint64_t(z.j) * p.seg_bytes;
        const uint32_t* farp = FAR ? p.far + uint64_t(z.seg) * p.seg_bytes : nullptr;
        const uint32_t ubase = z.b * zstd::kBlock + so;
        for (uint32_t base = H; base <= mflimit && !full;) {
            uint32_t cand[kWin], mlen[kWin];
            uint64_t M[kWin];
#pragma unroll
            for (uint32_t w = 0; w < kWin; ++w) {
                const uint32_t qq = base + 64 * w + lane;
                cand[w] = 0;
                mlen[w] = 0;
                if (qq <= mflimit) {
                    const uint32_t v = lds_rd32(sw, qq);
                    const uint32_t h = (v * 2654435761u) >> (32 - HLOG);
                    const uint32_t en = table[h];
                    table[h] = uint16_t(qq + 1);
                    uint32_t c = ~0u;
                    if (en != 0 && en - 1 < qq && lds_rd32(sw, en - 1) == v)
                        c = en - 1;
                    else if (qq > 0 && lds_rd32(sw, qq - 1) == v)
                        c = qq - 1;
                    if (c != ~0u) {
                        const uint32_t lim = min(matchlimit - qq, kLenCap);
                        uint32_t len = 4;
                        bool done = false;
                        while (len + 4 <= lim) {
                            const uint32_t x = lds_rd32(sw, qq + len) ^ lds_rd32(sw, c + len);
                            if (x) {
                                len += uint32_t(__builtin_ctz(x)) >> 3;
                                done = true;
                                break;
                            }
                            len += 4;
                        }
                        if (!done)
                            while (len < lim && sb[qq + len] == sb[c + len])
                                ++len;
                        if (len >= minlen) {
                            cand[w] = qq - c; // distance
                            mlen[w] = len;
                        }
                    }
                    if constexpr (FAR) {
                        const uint32_t sp = ubase + (qq - H);
                        const uint32_t fv = (p.dbg & 2u) ? 0u : farp[sp];
                        if (fv != 0 && fv - 1 < sp && !(p.dbg & 1u)) {
                            // bytes of the candidate from global memory: one
                            // 8-B load holds its first 8 - (fp & 3) >= 5;
                            // the next 8 only when those all match
                            typedef uint32_t u32x2 __attribute__((ext_vector_type(2), aligned(4)));
                            const uint32_t fp = fv - 1, wi = fp >> 2, sh = 8u * (fp & 3u);
                            const uint32_t nw = (z.seglen + 3u) >> 2; // words of the segment
                            const uint32_t* a4 = reinterpret_cast<const uint32_t*>(seg) + wi;
                            const u32x2 v = wi + 2 <= nw ? *reinterpret_cast<const u32x2*>(a4)
                                                   : u32x2{ a4[0], 0u };
                            const uint64_t cw = (uint64_t(v.y) << 32 | v.x) >> sh;
                            const uint64_t mine =
                              uint64_t(lds_rd32(sw, qq + 4)) << 32 | lds_rd32(sw, qq);
                            const uint32_t avail = 8u - (fp & 3u);
                            const uint64_t x = (cw ^ mine) & (~0ull >> (64u - 8u * avail));
                            uint32_t flen = x ? uint32_t(__builtin_ctzll(x)) >> 3 : avail;
                            if (flen == avail) {
                                // candidate bytes [avail, avail + 8) are words
                                // wi + 2, wi + 3
                                const uint32_t w2 = wi + 2;
                                const u32x2 u = w2 + 2 <= nw
                                                  ? *reinterpret_cast<const u32x2*>(a4 + 2)
                                                  : u32x2{ w2 < nw ? a4[2] : 0u, 0u };
                                const uint64_t x2 =
                                  (uint64_t(u.y) << 32 | u.x) ^
                                  (uint64_t(lds_rd32(sw, qq + avail + 4)) << 32 |
                                   lds_rd32(sw, qq + avail));
                                flen += x2 ? uint32_t(__builtin_ctzll(x2)) >> 3 : 8u;
                            }
                            flen = min(flen, min(matchlimit - qq, 16u));
                            if (flen >= kFarMin && flen > mlen[w] && sp - fp <= kZOffMax &&
                                !(p.dbg & 4u)) {
                                cand[w] = sp - fp;
                                mlen[w] = flen;
                            }
                        }
                    }
                }
            }
#pragma unroll
            for (uint32_t w = 0; w < kWin; ++w)
                M[w] = __ballot(mlen[w] != 0);
            bool any = false;
#pragma unroll
            for (uint32_t w = 0; w < kWin; ++w) {
                const uint32_t wb = base + 64 * w;
                // FAR (matches at most positions): the greedy walk's next
                // step from each lane's match, the first match at or after
                // its end (64: none in this window; 65: the match reached
                // kLenCap and may run longer)
                const uint32_t ml = mlen[w];
                uint32_t jmp = 64u;
                if (ml == kLenCap) {
                    jmp = 65u;
                } else if (ml != 0 && lane + ml < 64u) {
                    const uint64_t nx = M[w] & (~0ull << (lane + ml));
                    jmp = nx ? uint32_t(__ffsll(static_cast<long long>(nx))) - 1 : 64u;
                }
                const uint32_t end = wb + lane + ml; // this lane's match end
                while (!FAR && p0 < wb + 64 && !full) {
                    // few matches (no far candidates): one step per match
                    const uint32_t sh = p0 > wb ? p0 - wb : 0;
                    const uint64_t mm = M[w] & (~0ull << sh);
                    if (mm == 0)
                        break;
                    const uint32_t i = uint32_t(__ffsll(static_cast<long long>(mm))) - 1;
                    const uint32_t qq = wb + i;
                    const uint32_t dist = rdlane(cand[w], i);
                    uint32_t len = rdlane(mlen[w], i);
                    if (len == kLenCap) {
                        const uint32_t cc = qq - dist;
                        for (;;) {
                            const uint32_t a = qq + len + lane;
                            const bool eq = a < matchlimit && sb[a] == sb[cc + len + lane];
                            const uint64_t miss = __ballot(!eq);
                            if (miss == 0) {
                                len += 64;
                                continue;
                            }
                            len += uint32_t(__ffsll(static_cast<long long>(miss))) - 1;
                            break;
                        }
                    }
                    if (lane == 0)
                        sseq[nseq] = zstd::pack_seq(qq - anchor, len, dist);
                    ++nseq;
                    full = nseq == kZSubSeq;
                    p0 = qq + len;
                    anchor = p0;
                    any = true;
                }
                while (FAR && p0 < wb + 64 && !full) {
                    const uint32_t sh = p0 > wb ? p0 - wb : 0;
                    const uint64_t mm = M[w] & (~0ull << sh);
                    if (mm == 0)
                        break;
                    // the chain of greedy matches from the first: one
                    // readlane per match; the sequences are then packed and
                    // stored by their own lanes at once
                    uint32_t s = uint32_t(__ffsll(static_cast<long long>(mm))) - 1;
                    const uint32_t room = kZSubSeq - nseq;
                    uint64_t sel = 0;
                    uint32_t cnt = 0;
                    bool cap = false;
                    for (;;) {
                        const uint32_t j = rdlane(jmp, s);
                        if (j == 65u) {
                            cap = true;
                            break;
                        }
                        sel |= 1ull << s;
                        if (++cnt == room || j >= 64u)
                            break;
                        s = j;
                    }
                    if (sel) {
                        const uint64_t below = sel & ((1ull << lane) - 1ull);
                        const int prev = below ? 63 - __clzll(static_cast<long long>(below)) : -1;
                        const uint32_t pend = __shfl(end, prev < 0 ? 0 : prev);
                        if ((sel >> lane) & 1ull)
                            sseq[nseq + uint32_t(__popcll(below))] = zstd::pack_seq(
                              wb + lane - (prev < 0 ? anchor : pend), ml, cand[w]);
                        nseq += cnt;
                        p0 = rdlane(end, 63u - uint32_t(__clzll(static_cast<long long>(sel))));
                        anchor = p0;
                        full = nseq == kZSubSeq;
                        any = true;
                    }
                    if (cap && !full) {
                        // a local match that reached kLenCap: measured on,
                        // 64 bytes per ballot
                        const uint32_t qq = wb + s;
                        const uint32_t dist = rdlane(cand[w], s);
                        const uint32_t cc = qq - dist;
                        uint32_t len = kLenCap;
                        for (;;) {
                            const uint32_t a = qq + len + lane;
                            const bool eq = a < matchlimit && sb[a] == sb[cc + len + lane];
                            const uint64_t miss = __ballot(!eq);
                            if (miss == 0) {
                                len += 64;
                                continue;
                            }
                            len += uint32_t(__ffsll(static_cast<long long>(miss))) - 1;
                            break;
                        }
                        if (lane == 0)
                            sseq[nseq] = zstd::pack_seq(qq - anchor, len, dist);
                        ++nseq;
                        full = nseq == kZSubSeq;
                        p0 = qq + len;
                        anchor = p0;
                        any = true;
                    }
                }
            }
            misses = any ? 0 : misses + 1;
            const uint32_t skip =
              misses > 1 && !(p.dbg & 8u) ? (misses - 1) * 64 * kWin : 0;
            base = max(base + 64 * kWin + skip, p0 & ~63u);
        }
    }
    __threadfence_block(); // lane 0's sequence stores, read back below
    __syncthreads();
    // literal runs -> the unit's literal slot, and their histogram
    uint8_t* lo = p.lits + uint64_t(q) * kZSub;
    if (nseq == 0) {
        // every byte is a literal: the unit's histogram is the literal one
        if (whole) {
            for (uint32_t w = lane; w < kZSub / 16; w += 64)
                reinterpret_cast<uint4*>(lo)[w] = reinterpret_cast<const uint4*>(sw)[H / 16 + w];
        } else {
            for (uint32_t i = lane; i < L; i += 64)
                lo[i] = sb[H + i];
        }
        __syncthreads();
        for (uint32_t b = lane; b < 256; b += 64)
            if (lh[b])
                atomicAdd(&p.hist[uint64_t(g) * 256 + b], lh[b]);
        if (lane == 0) {
            p.snseq[q] = 0;
            p.snlit[q] = L;
            p.stail[q] = L;
        }
        return;
    }
    for (uint32_t b = lane; b < 256; b += 64)
        lh[b] = 0;
    __syncthreads();
    uint32_t at = 0, pos = H;
    for (uint32_t s0 = 0; s0 < nseq; s0 += 64) {
        // 64 sequences per load, one per lane, walked through readlane
        const uint64_t mine = s0 + lane < nseq ? sseq[s0 + lane] : 0;
        const uint32_t mlo = uint32_t(mine), mhi = uint32_t(mine >> 32);
        const uint32_t m = min(64u, nseq - s0);
        for (uint32_t j = 0; j < m; ++j) {
            const zstd::Seq v =
              zstd::unpack_seq(uint64_t(rdlane(mlo, j)) | uint64_t(rdlane(mhi, j)) << 32);
            if (!(p.dbg & 16u)) // A/B: 16 = no literal gather (frames invalid)
                for (uint32_t i = lane; i < v.lit; i += 64) {
                    const uint8_t x = sb[pos + i];
                    lo[at + i] = x;
                    atomicAdd(&lh[x], 1u);
                }
            at += v.lit;
            pos += v.lit + v.len;
        }
    }
    const uint32_t tail = H + L - pos;
    for (uint32_t i = lane; i < tail; i += 64) {
        const uint8_t x = sb[pos + i];
        lo[at + i] = x;
        atomicAdd(&lh[x], 1u);
    }
    at += tail;
    __syncthreads();
    for (uint32_t b = lane; b < 256; b += 64)
        if (lh[b])
            atomicAdd(&p.hist[uint64_t(g) * 256 + b], lh[b]);
    if (lane == 0) {
        p.snseq[q] = nseq;
        p.snlit[q] = at;
        p.stail[q] = tail;
    }
}

__global__ __launch_bounds__(256) void
zstd_hist(const ZstdParams p)
{
    __shared__ uint32_t h[4][256];
    const uint32_t g = blockIdx.x, t = threadIdx.x, w = t >> 6;
    const ZBlock z = zblock(p, g);
    const bool skip = z.len == 0 || zchunk_skip(p, z.c);
    for (uint32_t k = 0; k < 4; ++k)
        h[k][t] = 0;
    __syncthreads();
    if (!skip) {
        const uint8_t* s = zblock_src(p, z);
        uint32_t done = 0;
        if ((reinterpret_cast<uintptr_t>(s) & 3u) == 0) {
            const uint32_t* sw = reinterpret_cast<const uint32_t*>(s);
            for (uint32_t i = t; i < z.len / 4; i += 256) {
                const uint32_t v = sw[i];
                atomicAdd(&h[w][v & 255u], 1u);
                atomicAdd(&h[w][(v >> 8) & 255u], 1u);
                atomicAdd(&h[w][(v >> 16) & 255u], 1u);
                atomicAdd(&h[w][v >> 24], 1u);
            }
            done = z.len & ~3u;
        }
        for (uint32_t i = done + t; i < z.len; i += 256)
            atomicAdd(&h[w][s[i]], 1u);
    }
    __syncthreads();
    p.hist[uint64_t(g) * 256 + t] = h[0][t] + h[1][t] + h[2][t] + h[3][t];
}

__global__ __launch_bounds__(64) void
zstd_table(const ZstdParams p)
{
    __shared__ zstd::HufWork w;
    __shared__ zstd::TreeWork tw;
    __shared__ uint64_t key[256];
    __shared__ uint8_t len[256];
    __shared__ uint16_t code[256];
    __shared__ uint8_t tree[160];
    __shared__ uint32_t npresent, tree_n, mode;
    // one Huffman group (2^hgrp_log2 blocks of a segment)
    const uint32_t gi = blockIdx.x, t = threadIdx.x;
    const uint32_t s = gi / p.ngrp, b0 = (gi - s * p.ngrp) << p.hgrp_log2;
    const uint32_t b1 = min(p.bps, b0 + (1u << p.hgrp_log2));
    if (zchunk_skip(p, s / p.nseg))
        return;
    if (t == 0)
        npresent = 0;
    __syncthreads();
    uint32_t mx = 0, tot = 0;
    for (uint32_t k = t; k < 256; k += 64) {
        uint32_t a = 0;
        for (uint32_t b = b0; b < b1; ++b)
            a += p.hist[(uint64_t(s) * p.bps + b) * 256 + k];
        w.cnt[k] = a;
        key[k] = uint64_t(a) << 8 | k;
        len[k] = 0;
        code[k] = 0;
        if (a)
            atomicAdd(&npresent, 1u);
        mx = max(mx, a);
        tot += a;
    }
    for (int d = 32; d > 0; d >>= 1) {
        mx = max(mx, uint32_t(__shfl_xor(int(mx), d)));
        tot += uint32_t(__shfl_xor(int(tot), d));
    }
    __syncthreads();
    if (zstd::huf_flat(npresent, mx, tot)) {
        // raw literals: no sort, no construction
        ZstdSegTable& T0 = p.tab[gi];
        for (uint32_t k = t; k < 256; k += 64) {
            T0.code[k] = 0;
            T0.len[k] = 0;
        }
        if (t == 0) {
            T0.mode = 0;
            T0.tree_n = 0;
        }
        return;
    }
    // bitonic sort of (count, symbol), 64 lanes x 2 pairs
    for (uint32_t size = 2; size <= 256; size <<= 1)
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t q = t; q < 128; q += 64) {
                const uint32_t i = 2 * q - (q & (stride - 1));
                const uint32_t j = i + stride;
                const bool up = (i & size) == 0;
                const uint64_t a = key[i], b = key[j];
                if ((a > b) == up) {
                    key[i] = b;
                    key[j] = a;
                }
            }
            __syncthreads();
        }
    const uint32_t n = npresent;
    for (uint32_t k = t; k < n; k += 64)
        w.sorted[k] = uint16_t(key[256 - n + k] & 255u);
    __syncthreads();
    // the serial construction on lane 0, every array in LDS
    if (t == 0) {
        mode = n == 1 ? 1 : 0;
        tree_n = 0;
        if (n >= 2) {
            zstd::huf_lengths_sorted(w, n, len, zstd::kHufMaxBits);
            const uint32_t mb = zstd::huf_codes(len, code, tw);
            tree_n = zstd::huf_write_tree(len, mb, tree, tw);
            mode = tree_n ? 2 : 0;
        }
    }
    __syncthreads();
    ZstdSegTable& T = p.tab[gi];
    for (uint32_t k = t; k < 256; k += 64) {
        T.code[k] = code[k];
        T.len[k] = len[k];
    }
    for (uint32_t k = t; k < tree_n; k += 64)
        T.tree[k] = tree[k];
    if (t == 0) {
        T.mode = mode;
        T.tree_n = tree_n;
    }
}

// A sequence's codes and extra bits in one word: llc (6) | mlc (6) | ofc (5)
// | ll extra (13) | ml extra (11) | offset extra (23).  A block's sequence
// has < 2 * kZSub literals (its unit's and the previous unit's tail: LL
// extra <= 13 bits) and a match ends inside its unit (length <= kZSub: ML
// extra <= 11 bits); far matches reach < 2^24 - 3 back (OF extra <= 23 bits).
static_assert(2 * kZSub <= 8192 && kZSub <= 4096, "sequence word field widths");
__device__ __forceinline__ uint64_t
zseq_codes(const zstd::Seq& v)
{
    const uint32_t llc = zstd::ll_code(v.lit), mlc = zstd::ml_code(v.len);
    const uint32_t ofv = v.off + 3, ofc = zstd::highbit(ofv);
    return uint64_t(llc) | uint64_t(mlc) << 6 | uint64_t(ofc) << 12 |
           uint64_t(v.lit - zstd::ll_base(llc)) << 17 |
           uint64_t(v.len - zstd::ml_base(mlc)) << 30 | uint64_t(ofv - (1u << ofc)) << 41;
}

// zstd::BitW's bitstream with 4-byte stores: whole bytes until the output
// is 4-byte aligned, then a dword per 32 bits (a lane per block writes its
// own stream, so every store instruction touches 64 lines: 4x fewer of them)
struct BitW32
{
    uint8_t* p;
    uint32_t cap, pos, n;
    uint64_t acc;
    bool ovf;
    __device__ void init(uint8_t* dst, uint32_t c)
    {
        p = dst;
        cap = c;
        pos = 0;
        n = 0;
        acc = 0;
        ovf = false;
    }
    __device__ void byte()
    {
        if (pos < cap)
            p[pos] = uint8_t(acc);
        else
            ovf = true;
        ++pos;
        acc >>= 8;
        n -= 8;
    }
    __device__ void add(uint64_t v, uint32_t nb) // nb <= 32
    {
        acc |= (v & ((1ull << nb) - 1ull)) << n;
        n += nb;
        if (n < 32)
            return;
        while (n >= 8 && ((reinterpret_cast<uintptr_t>(p) + pos) & 3u))
            byte();
        if (n >= 32) {
            if (pos + 4 <= cap)
                *reinterpret_cast<uint32_t*>(p + pos) = uint32_t(acc);
            else
                ovf = true;
            pos += 4;
            acc >>= 32;
            n -= 32;
        }
    }
    // end mark (one 1 bit), then the whole bytes and the padded last one
    __device__ uint32_t close()
    {
        add(1, 1);
        while (n >= 8)
            byte();
        if (n) {
            n = 8;
            byte();
            n = 0;
        }
        return ovf ? 0 : pos;
    }
};

// zstd::encode_sequences over pre-coded sequences (same bitstream), with
// the predefined tables (LDS) or a segment's fitted ones (global)
template<class TL, class TO, class TM>
__device__ uint32_t
zseq_encode(const TL& tll, const TO& tof, const TM& tml, const uint64_t* sv, uint32_t n,
            uint8_t* out, uint32_t cap)
{
    struct
    {
        const TL& ll;
        const TO& of;
        const TM& ml;
    } t{ tll, tof, tml };
    BitW32 w;
    w.init(out, cap);
    uint64_t v = sv[n - 1];
    uint32_t llc = uint32_t(v & 63u), mlc = uint32_t((v >> 6) & 63u), ofc = uint32_t((v >> 12) & 31u);
    uint32_t sml = zstd::fse_init(t.ml, mlc), sof = zstd::fse_init(t.of, ofc),
             sll = zstd::fse_init(t.ll, llc);
    w.add((v >> 17) & 0x1FFFu, zstd::ll_bits(llc));
    w.add((v >> 30) & 0x7FFu, zstd::ml_bits(mlc));
    w.add(v >> 41, ofc);
    // sequences n-2 .. 0, kSeqAhead at a time: the next group's words are
    // loaded while this group is coded.  (The bit writer's stores sit under
    // branches, so the compiler waits for every store before a loaded word is
    // used: one wait per group, not one per sequence.)  Indices below 0 load
    // word 0 and are not coded.
    constexpr int kSeqAhead = 8;
    uint64_t cur[kSeqAhead], nxt[kSeqAhead];
    int hi = int(n) - 2;
#pragma unroll
    for (int u = 0; u < kSeqAhead; ++u)
        cur[u] = sv[max(hi - u, 0)];
    for (; hi >= 0; hi -= kSeqAhead) {
#pragma unroll
        for (int u = 0; u < kSeqAhead; ++u)
            nxt[u] = sv[max(hi - kSeqAhead - u, 0)];
#pragma unroll
        for (int u = 0; u < kSeqAhead; ++u) {
            if (hi - u < 0)
                break;
            v = cur[u];
            llc = uint32_t(v & 63u);
            mlc = uint32_t((v >> 6) & 63u);
            ofc = uint32_t((v >> 12) & 31u);
            zstd::fse_enc(w, sof, t.of, ofc);
            zstd::fse_enc(w, sml, t.ml, mlc);
            zstd::fse_enc(w, sll, t.ll, llc);
            w.add((v >> 17) & 0x1FFFu, zstd::ll_bits(llc));
            w.add((v >> 30) & 0x7FFu, zstd::ml_bits(mlc));
            w.add(v >> 41, ofc);
        }
#pragma unroll
        for (int u = 0; u < kSeqAhead; ++u)
            cur[u] = nxt[u];
    }
    zstd::fse_flush(w, sml, t.ml);
    zstd::fse_flush(w, sof, t.of);
    zstd::fse_flush(w, sll, t.ll);
    return w.close();
}

// literal i of block g: the block's bytes (literals only) or the parse
// units' literal slots (pre = literal prefix of the units)
struct ZLits
{
    const uint8_t* base; // block bytes, or the block's first unit slot
    const uint32_t* pre; // [kZSubBlocks + 1] or nullptr
    __device__ __forceinline__ uint8_t operator()(uint32_t i) const
    {
        if (!pre)
            return base[i];
        uint32_t k = 0;
        while (k + 1 < kZSubBlocks && pre[k + 1] <= i)
            ++k;
        return base[uint64_t(k) * kZSub + (i - pre[k])];
    }
};

__global__ __launch_bounds__(256) void
zstd_encode(const ZstdParams p)
{
    // the 4 Huffman streams, later the staged sequences and their stream
    __shared__ uint32_t zbuf[4096];
    uint32_t(*buf)[kZStreamWords] = reinterpret_cast<uint32_t(*)[kZStreamWords]>(zbuf);
    __shared__ uint16_t code[256];
    __shared__ uint8_t clen[256];
    __shared__ int32_t rle;
    __shared__ uint32_t ssz[4];
    __shared__ uint32_t pre[kZSubBlocks + 1], spre[kZSubBlocks + 1], carry[kZSubBlocks];
    __shared__ uint32_t dec[4]; // literal section bytes, literal type, literal payload
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    const ZBlock z = zblock(p, g);
    if (z.len == 0 || zchunk_skip(p, z.c)) {
        if (t == 0)
            p.bkind[g] = 3;
        return;
    }
    if (t == 0) {
        rle = -1;
        pre[0] = 0;
        spre[0] = 0;
        if (p.match) {
            const uint64_t u0 = uint64_t(g) * kZSubBlocks;
            uint32_t cr = 0;
            for (uint32_t k = 0; k < kZSubBlocks; ++k) {
                pre[k + 1] = pre[k] + p.snlit[u0 + k];
                spre[k + 1] = spre[k] + p.snseq[u0 + k];
                carry[k] = cr;
                cr = p.snseq[u0 + k] ? p.stail[u0 + k] : cr + p.snlit[u0 + k];
            }
        } else {
            for (uint32_t k = 0; k < kZSubBlocks; ++k) {
                pre[k + 1] = z.len;
                spre[k + 1] = 0;
            }
        }
    }
    __syncthreads();
    const uint32_t nl = pre[kZSubBlocks], nseq = spre[kZSubBlocks];
    if (!p.match) {
        if (nl > 0 && p.hist[uint64_t(g) * 256 + t] == nl)
            rle = int32_t(t); // one byte value in the whole block
    } else if (t == 0) {
        // every unit of the block holds one and the same value
        uint32_t v = 512;
        for (uint32_t k = 0; k < kZSubBlocks; ++k)
            if (k * kZSub < z.len) {
                const uint32_t u = p.sval[uint64_t(g) * kZSubBlocks + k];
                v = (v == 512 || v == u) ? u : 256;
            }
        if (v < 256)
            rle = int32_t(v);
    }
    __syncthreads();
    if (rle >= 0) {
        if (t == 0) {
            p.bkind[g] = 1;
            p.bpay[g] = uint32_t(rle);
        }
        return;
    }
    const ZstdSegTable& T = p.tab[z.grp];
    const ZLits lit{ p.match ? p.lits + uint64_t(g) * kZSubBlocks * kZSub : zblock_src(p, z),
                     p.match ? pre : nullptr };
    const bool try_huf = T.mode == 2 && nl >= kZMinHuf;
    if (try_huf) {
        code[t] = T.code[t];
        clen[t] = T.len[t];
        for (uint32_t i = t; i < 4 * kZStreamWords; i += 256)
            zbuf[i] = 0;
    }
    __syncthreads();
    // stream w on wave w; literals are read coalesced (lane l takes literal
    // s + l of each run of 64).  First every stream's bit count, then --
    // only if Huffman wins for the block -- the bits are placed by a suffix
    // scan of their code lengths: a stream is written last literal first
    const uint32_t w = t >> 6, lane = t & 63u;
    const uint32_t seg4 = try_huf ? zstd::lit_segment(nl) : 0;
    const uint32_t a = min(nl, w * seg4), e = min(nl, (w + 1) * seg4);
    uint32_t k = 0; // parse unit of this lane's literal (match mode)
    auto sym_at = [&](uint32_t i) -> uint8_t {
        if (!lit.pre)
            return lit.base[i];
        while (k + 1 < kZSubBlocks && pre[k + 1] <= i)
            ++k;
        while (i < pre[k])
            --k;
        return lit.base[uint64_t(k) * kZSub + (i - pre[k])];
    };
    uint32_t bits = 0;
    bool fits = false;
    if (try_huf) {
        for (uint32_t i = a + lane; i < e; i += 64)
            bits += clen[sym_at(i)];
        for (int dd = 32; dd > 0; dd >>= 1)
            bits += __shfl_xor(bits, dd);
        fits = bits + 1 <= 8 * (e - a) + 32;
        if (lane == 0)
            ssz[w] = fits ? bits / 8 + 1 : 0x7fffffffu;
    }
    __syncthreads();
    uint8_t* d = p.scratch + uint64_t(g) * zstd::kBlock;
    if (t == 0) {
        // literals: Huffman when it beats raw counted with the tree
        uint32_t ltype = 0, lpay = nl, lsec = zstd::lit_header_raw_bytes(nl) + nl;
        if (try_huf) {
            const uint64_t pay64 = 6ull + ssz[0] + ssz[1] + ssz[2] + ssz[3];
            const uint32_t pay = uint32_t(min(pay64, uint64_t(0x7fffffffu)));
            const uint32_t wt = T.tree_n + pay;
            const uint32_t hs = zstd::lit_header_huf_bytes(nl, wt) + wt;
            if (hs < lsec) {
                ltype = 2;
                lpay = pay;
                lsec = hs;
            }
        }
        dec[1] = ltype;
        dec[2] = lpay;
        dec[0] = lsec;
    }
    __syncthreads();
    const uint32_t ltype = dec[1], lpay = dec[2], lsec = dec[0];
    if (lsec + 1 >= z.len) { // not smaller even without sequences
        if (t == 0)
            p.bkind[g] = 0;
        return;
    }
    if (ltype == 2) { // every stream fits (a stream that did not lost)
        uint32_t* sb = buf[w];
        uint32_t base = 0;
        for (uint32_t cs = e; cs > a;) {
            const uint32_t s0 = cs > a + 64 ? cs - 64 : a;
            const uint32_t i = s0 + lane;
            uint32_t n = 0, v = 0;
            if (i < cs) {
                const uint8_t sym = sym_at(i);
                n = clen[sym];
                v = code[sym];
            }
            uint32_t x = n; // inclusive suffix sum over the run
            for (int dd = 1; dd < 64; dd <<= 1) {
                const uint32_t y = __shfl_down(x, dd);
                if (lane + uint32_t(dd) < 64)
                    x += y;
            }
            const uint32_t pos = base + x - n;
            if (n) {
                const uint32_t o = pos & 31u;
                atomicOr(&sb[pos >> 5], v << o);
                if (o + n > 32)
                    atomicOr(&sb[(pos >> 5) + 1], v >> (32 - o));
            }
            base += __shfl(x, 0);
            cs = s0;
        }
        if (lane == 0)
            atomicOr(&sb[bits >> 5], 1u << (bits & 31u)); // end mark
        __syncthreads();
    }
    // the literal payload -> scratch[0, lpay)
    if (ltype == 2) {
        if (t == 0) {
            zstd::put_le(d, ssz[0], 2);
            zstd::put_le(d + 2, ssz[1], 2);
            zstd::put_le(d + 4, ssz[2], 2);
        }
        uint32_t at = 6;
        for (uint32_t k = 0; k < 4; ++k) {
            const uint8_t* sbk = reinterpret_cast<const uint8_t*>(buf[k]);
            for (uint32_t i = t; i < ssz[k]; i += 256)
                d[at + i] = sbk[i];
            at += ssz[k];
        }
    } else {
        for (uint32_t i = t; i < nl; i += 256)
            d[i] = lit(i);
    }
    // the sequences: pre-coded (codes + extra bits, one word each) and
    // compacted in place into the block's first sequence slots; the FSE
    // bitstream is built by zstd_seqenc, one lane per block
    if (nseq == 0) {
        if (t == 0) {
            d[lpay] = 0; // sequence section header: no sequences
            p.bnseq[g] = 0;
            p.bkind[g] = 2;
            p.bltype[g] = uint8_t(ltype);
            p.bpay[g] = lpay;
            p.bseqb[g] = 1;
            p.bnlit[g] = nl;
        }
        return;
    }
    // code counts of the block -> the segment's (zstd_seqtab fits its
    // sequence tables to them); the LDS stream buffers are free by now
    constexpr uint32_t kPer = kZSubBlocks * kZSubSeq / 256;
    static_assert(kZSubBlocks * kZSubSeq % 256 == 0, "whole sequences per thread");
    uint32_t* cnt = zbuf; // [3][64]: LL, OF, ML codes
    __syncthreads();
    for (uint32_t i = t; i < 3 * 64; i += 256)
        cnt[i] = 0;
    __syncthreads();
    uint64_t* gs = p.seqs + uint64_t(g) * kZSubBlocks * kZSubSeq;
    uint64_t cw[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j) {
        const uint32_t i = t + 256 * j;
        cw[j] = 0;
        if (i < nseq) {
            uint32_t k = 0;
            while (k + 1 < kZSubBlocks && spre[k + 1] <= i)
                ++k;
            zstd::Seq v = zstd::unpack_seq(gs[uint64_t(k) * kZSubSeq + (i - spre[k])]);
            if (i == spre[k])
                v.lit += carry[k];
            cw[j] = zseq_codes(v);
            atomicAdd(&cnt[cw[j] & 63u], 1u);                     // LL
            atomicAdd(&cnt[64 + ((cw[j] >> 12) & 31u)], 1u);      // OF
            atomicAdd(&cnt[128 + ((cw[j] >> 6) & 63u)], 1u);      // ML
        }
    }
    __syncthreads(); // every slot read before any is overwritten
#pragma unroll
    for (uint32_t j = 0; j < kPer; ++j)
        if (t + 256 * j < nseq)
            gs[t + 256 * j] = cw[j];
    for (uint32_t i = t; i < 3 * 64; i += 256)
        if (cnt[i])
            atomicAdd(&p.scount[uint64_t(z.seg) * 192 + i], cnt[i]);
    if (t == 0) {
        p.bkind[g] = 4; // sequences pending (zstd_seqenc)
        p.bltype[g] = uint8_t(ltype);
        p.bpay[g] = lpay;
        p.bseqb[g] = nseq;
        p.bnseq[g] = nseq;
        p.bnlit[g] = nl;
    }
}

// Sequence tables of a segment, one wave: LL / OF / ML FSE distributions
// fitted to the segment's code counts (accuracy log 5..9, the one with the
// fewest bits counted with its description), kept when the three together
// beat the predefined distributions.  The serial part runs on lane 0.
__device__ bool
zfit(const uint32_t* cnt, uint32_t maxlog, int16_t* norm, uint32_t& al_out,
     uint32_t& maxsym_out, float& bits_out, int16_t* nm, uint8_t* tmp)
{
    // nm [kFseMaxSym] and tmp [128]: LDS workspaces of the caller (private
    // arrays indexed at run time would live in scratch memory)
    uint32_t ms = 0, nz = 0;
    uint64_t total = 0;
    for (uint32_t s = 0; s < 64; ++s)
        if (cnt[s]) {
            ms = s;
            ++nz;
            total += cnt[s];
        }
    if (nz < 2 || ms >= zstd::kFseMaxSym)
        return false;
    float best = 3.0e38f;
    for (uint32_t al = 5; al <= maxlog; ++al) {
        const int ts = 1 << al;
        int used = 0, big = -1;
        for (uint32_t s = 0; s <= ms; ++s) {
            if (!cnt[s]) {
                nm[s] = 0;
                continue;
            }
            const float pr = float(cnt[s]) * float(ts) / float(total);
            if (pr < 1.0f) {
                nm[s] = -1;
                used += 1;
            } else {
                const int v = int(pr + 0.5f);
                nm[s] = int16_t(v);
                used += v;
            }
            if (big < 0 || cnt[s] > cnt[big])
                big = int(s);
        }
        const int fix = nm[big] + (ts - used);
        if (nm[big] < 0 || fix < 1)
            continue;
        nm[big] = int16_t(fix);
        const uint32_t d = zstd::fse_write_ncount(tmp, 128, nm, ms, al);
        if (!d)
            continue;
        float b = 8.0f * float(d);
        for (uint32_t s = 0; s <= ms; ++s)
            if (cnt[s])
                b += float(cnt[s]) * (float(al) - (nm[s] < 0 ? 0.0f : __log2f(float(nm[s]))));
        if (b < best) {
            best = b;
            al_out = al;
            for (uint32_t s = 0; s <= ms; ++s)
                norm[s] = nm[s];
        }
    }
    maxsym_out = ms;
    bits_out = best;
    return best < 3.0e38f;
}

__device__ float
zpredef_bits(const uint32_t* cnt, const int16_t* norm, uint32_t maxsym, uint32_t al)
{
    float b = 0.0f;
    for (uint32_t s = 0; s < 64; ++s)
        if (cnt[s]) {
            if (s > maxsym)
                return 3.0e38f;
            b += float(cnt[s]) * (float(al) - (norm[s] < 0 ? 0.0f : __log2f(float(norm[s]))));
        }
    return b;
}

__global__ __launch_bounds__(64) void
zstd_seqtab(const ZstdParams p)
{
    __shared__ uint32_t cnt[3][64];
    __shared__ int16_t norm[3][zstd::kFseMaxSym];
    __shared__ int16_t nmw[3][zstd::kFseMaxSym];
    __shared__ uint8_t tmpw[3][128];
    __shared__ zstd::FseBuildWorkT<zstd::kSeqMaxLog> bw[3];
    // the tables and their descriptions are built in LDS, one lane per table
    // (LL, OF, ML), then copied out by the wave
    __shared__ zstd::FseTable<zstd::kSeqMaxLog> tt[3];
    __shared__ uint8_t desc[sizeof(ZstdSeqSeg::desc)];
    __shared__ uint32_t al[3], ms[3], okf[3], okb[3];
    __shared__ float fb[3], pb[3];
    __shared__ uint32_t res_mode, res_n;
    const uint32_t s = blockIdx.x, t = threadIdx.x;
    ZstdSeqSeg& Q = p.sqt[s];
    if (zchunk_skip(p, s / p.nseg)) {
        if (t == 0)
            Q.mode = 0;
        return;
    }
    for (uint32_t f = 0; f < 3; ++f)
        cnt[f][t] = p.scount[uint64_t(s) * 192 + f * 64 + t];
    __syncthreads();
    if (t < 3) {
        const uint32_t maxlog[3] = { 9, 8, 9 };
        uint32_t a = 0, m = 0;
        float b = 0.f;
        okf[t] = zfit(cnt[t], maxlog[t], norm[t], a, m, b, nmw[t], tmpw[t]) ? 1u : 0u;
        al[t] = a;
        ms[t] = m;
        fb[t] = b;
        pb[t] = t == 0   ? zpredef_bits(cnt[0], zstd::ll_default_norm(), 35, 6)
                : t == 1 ? zpredef_bits(cnt[1], zstd::of_default_norm(), 28, 5)
                         : zpredef_bits(cnt[2], zstd::ml_default_norm(), 52, 6);
    }
    __syncthreads();
    const bool want = okf[0] && okf[1] && okf[2] && p.fit &&
                      fb[0] + fb[1] + fb[2] < pb[0] + pb[1] + pb[2];
    if (t == 0) {
        res_mode = 0;
        res_n = 0;
        if (want) {
            uint32_t n = 0;
            bool ok = true;
            for (uint32_t f = 0; f < 3 && ok; ++f) {
                const uint32_t d = zstd::fse_write_ncount(desc + n, sizeof(desc) - n,
                                                          norm[f], ms[f], al[f]);
                ok = d != 0;
                n += d;
            }
            if (ok) {
                res_n = n;
                res_mode = 2;
            }
        }
    }
    if (t < 3)
        okb[t] = want && zstd::fse_build(tt[t], norm[t], ms[t], al[t], bw[t]) ? 1u : 0u;
    __syncthreads();
    const bool fitted = res_mode == 2 && okb[0] && okb[1] && okb[2];
    if (fitted) {
        for (uint32_t i = t; i < sizeof(tt[0]) / 4; i += 64) {
            reinterpret_cast<uint32_t*>(&Q.ll)[i] = reinterpret_cast<const uint32_t*>(&tt[0])[i];
            reinterpret_cast<uint32_t*>(&Q.of)[i] = reinterpret_cast<const uint32_t*>(&tt[1])[i];
            reinterpret_cast<uint32_t*>(&Q.ml)[i] = reinterpret_cast<const uint32_t*>(&tt[2])[i];
        }
        for (uint32_t i = t; i < res_n; i += 64)
            Q.desc[i] = desc[i];
    }
    if (t == 0) {
        Q.desc_n = fitted ? res_n : 0;
        Q.mode = fitted ? 2u : 0u;
    }
}

// The FSE sequence bitstream of every block with pending sequences, one
// lane per block: the state chain is serial within a block, so 64 blocks
// advance together per wave instead of one lane per 256-thread workgroup.
// The predefined tables sit in LDS; each lane reads its block's pre-coded
// sequences (last first, one ahead) and writes the bitstream after the
// block's literal payload in scratch.  Then the block's kind: compressed
// iff the whole block (literal section + sequences) beats raw.
__global__ __launch_bounds__(64) void
zstd_seqenc(const ZstdParams p)
{
    // one wave per (segment, 64 of its blocks): the segment's tables -- the
    // predefined ones or its fitted ones -- in LDS, so the FSE state chains
    // look them up at LDS latency
    __shared__ zstd::SeqTables seqt;
    __shared__ zstd::FseTable<zstd::kSeqMaxLog> fll, fof, fml;
    const uint32_t gpseg = (p.bps + 63) / 64;
    const uint32_t s = blockIdx.x / gpseg, k0 = (blockIdx.x - s * gpseg) * 64;
    const ZstdSeqSeg& Q = p.sqt[s];
    const bool fitted = !zchunk_skip(p, s / p.nseg) && Q.mode == 2;
    if (fitted) {
        for (uint32_t i = threadIdx.x; i < sizeof(fll) / 4; i += 64) {
            reinterpret_cast<uint32_t*>(&fll)[i] = reinterpret_cast<const uint32_t*>(&Q.ll)[i];
            reinterpret_cast<uint32_t*>(&fof)[i] = reinterpret_cast<const uint32_t*>(&Q.of)[i];
            reinterpret_cast<uint32_t*>(&fml)[i] = reinterpret_cast<const uint32_t*>(&Q.ml)[i];
        }
    } else {
        for (uint32_t i = threadIdx.x; i < sizeof(zstd::SeqTables) / 4; i += 64)
            reinterpret_cast<uint32_t*>(&seqt)[i] = reinterpret_cast<const uint32_t*>(p.seqt)[i];
    }
    __syncthreads();
    const uint32_t b = k0 + threadIdx.x;
    const uint64_t g = uint64_t(s) * p.bps + b;
    if (b >= p.bps || p.bkind[g] != 4)
        return;
    const ZBlock z = zblock(p, uint32_t(g));
    const uint32_t nseq = p.bseqb[g], lpay = p.bpay[g], nl = p.bnlit[g];
    uint32_t lsec;
    if (p.bltype[g] == 2) {
        const uint32_t wt = p.tab[z.grp].tree_n + lpay;
        lsec = zstd::lit_header_huf_bytes(nl, wt) + wt;
    } else {
        lsec = zstd::lit_header_raw_bytes(nl) + nl;
    }
    // [count][modes, patched by zstd_write][bitstream]; the table
    // descriptions of a fitted segment are counted as if this block carried
    // them (as the tree), so the decision does not depend on which block does
    uint8_t* so = p.scratch + g * zstd::kBlock + lpay;
    const uint32_t cap = zstd::kBlock - lpay;
    uint32_t sq = zstd::write_seq_header(so, nseq);
    const uint64_t* sv = p.seqs + g * kZSubBlocks * kZSubSeq;
    const uint32_t bcap = cap > sq ? cap - sq : 0;
    const uint32_t bits = fitted ? zseq_encode(fll, fof, fml, sv, nseq, so + sq, bcap)
                                 : zseq_encode(seqt.ll, seqt.of, seqt.ml, sv, nseq, so + sq, bcap);
    sq = bits ? sq + bits : 0;
    if (sq != 0 && lsec + sq + (fitted ? Q.desc_n : 0) < z.len) {
        p.bkind[g] = 2;
        p.bseqb[g] = sq;
    } else {
        p.bkind[g] = 0;
    }
}


// One wave per segment: the block carrying each Huffman group's tree (the
// group's first Huffman block) and the sequence tables' descriptions (the
// segment's first block with sequences, when its tables are fitted), each
// block's bytes, their offsets (a wave scan, 64 blocks per step) and the
// frame size.
__global__ __launch_bounds__(64) void
zstd_segment(const ZstdParams p)
{
    static_assert(64 % kHufGroup == 0 && 64 % (1u << kHufGroupPlainLog2) == 0,
                  "a wave step holds whole groups");
    const uint32_t gl = p.hgrp_log2, gn = 1u << gl;
    const uint64_t gmask = gn >= 64 ? ~0ull : (1ull << gn) - 1ull;
    const uint32_t s = blockIdx.x, lane = threadIdx.x;
    if (zchunk_skip(p, s / p.nseg)) {
        if (lane == 0)
            p.ssize[s] = 0;
        return;
    }
    const ZBlock z0 = zblock(p, s * p.bps);
    const ZstdSeqSeg& Q = p.sqt[s];
    const uint32_t desc_n = Q.mode == 2 ? Q.desc_n : 0;
    uint32_t scar = ~0u;
    for (uint32_t b0 = 0; b0 < z0.nb; b0 += 64) {
        const uint32_t b = b0 + lane;
        const uint32_t g = s * p.bps + b;
        const bool cmp = b < z0.nb && p.bkind[g] == 2;
        const uint64_t huf = __ballot(cmp && p.bltype[g] == 2);
        const uint64_t sqb = __ballot(cmp && p.bnseq[g] > 0);
        if (lane < (64u >> gl) && b0 + (lane << gl) < z0.nb) {
            const uint64_t m = (huf >> (lane << gl)) & gmask;
            p.carrier[s * p.ngrp + (b0 >> gl) + lane] =
              m ? b0 + (lane << gl) + uint32_t(__builtin_ctzll(m)) : ~0u;
        }
        if (scar == ~0u && sqb)
            scar = b0 + uint32_t(__ffsll(static_cast<long long>(sqb))) - 1;
    }
    __syncthreads(); // the carriers above, read below
    uint32_t pos = 0;
    for (uint32_t b0 = 0; b0 < z0.nb; b0 += 64) {
        const uint32_t b = b0 + lane;
        uint32_t sz = 0;
        if (b < z0.nb) {
            const uint32_t g = s * p.bps + b;
            const uint32_t blen = min(zstd::kBlock, z0.seglen - b * zstd::kBlock);
            const uint32_t k = p.bkind[g];
            if (k == 0) {
                sz = 3 + blen;
            } else if (k == 1) {
                sz = 4;
            } else if (k == 2) {
                const uint32_t nl = p.bnlit[g];
                const uint32_t gi = s * p.ngrp + (b >> gl);
                const uint32_t sd = scar == b ? desc_n : 0;
                if (p.bltype[g] == 2) {
                    const uint32_t cs = p.bpay[g] + (p.carrier[gi] == b ? p.tab[gi].tree_n : 0);
                    sz = 3 + zstd::lit_header_huf_bytes(nl, cs) + cs + p.bseqb[g] + sd;
                } else {
                    sz = 3 + zstd::lit_header_raw_bytes(nl) + nl + p.bseqb[g] + sd;
                }
            }
        }
        uint32_t x = sz; // inclusive prefix sum over the wave
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d);
            if (lane >= uint32_t(d))
                x += y;
        }
        if (b < z0.nb)
            p.bpos[s * p.bps + b] = pos + x - sz;
        pos += __shfl(x, 63);
    }
    if (lane == 0) {
        p.scarrier[s] = scar;
        const uint32_t frame = zstd::frame_header_bytes(z0.seglen) + pos;
        const bool raw = p.blosc && frame >= z0.seglen;
        p.sraw[s] = raw ? 1 : 0;
        p.ssize[s] = raw ? z0.seglen : frame;
    }
}

__global__ __launch_bounds__(256) void
zstd_chunk(const ZstdParams p)
{
    const uint32_t c = blockIdx.x;
    const bool skip = zchunk_skip(p, c);
    if (!p.blosc) {
        if (threadIdx.x == 0) {
            p.fsize[c] = skip ? 0 : p.ssize[c];
            p.mode[c] = 0;
        }
        return;
    }
    const uint32_t hdr = 16 + 4 * p.nseg;
    uint32_t carry = hdr;
    if (!p.store_only)
        for (uint32_t j0 = 0; j0 < p.nseg; j0 += 256) {
            const uint32_t j = j0 + threadIdx.x;
            const uint32_t rec = j < p.nseg ? 4 + p.ssize[uint64_t(c) * p.nseg + j] : 0;
            uint32_t tot;
            const uint32_t pre = block_scan256(rec, &tot);
            if (j < p.nseg)
                p.spos[uint64_t(c) * p.nseg + j] = carry + pre;
            carry += tot;
        }
    if (threadIdx.x == 0) {
        const bool memcpyed = p.store_only || uint64_t(carry) > uint64_t(p.nbytes) + 16;
        p.fsize[c] = skip ? 0 : (memcpyed ? p.nbytes + 16 : carry);
        p.mode[c] = memcpyed ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void
zstd_write(const ZstdParams p)
{
    const uint32_t g = blockIdx.x, t = threadIdx.x;
    const ZBlock z = zblock(p, g);
    const uint32_t fs = p.fsize[z.c];
    if (fs == 0 || z.len == 0)
        return;
    uint8_t* o = p.out + p.cstart[z.c];
    uint8_t* fr = o;
    if (p.blosc) {
        const bool memcpyed = p.mode[z.c] != 0;
        if (z.j == 0 && z.b == 0 && t == 0) {
            o[0] = 2; // BLOSC_VERSION_FORMAT
            o[1] = 1; // BLOSC_ZSTD_VERSION_FORMAT
            o[2] = uint8_t(4u << 5 | 0x10u | (p.shuffle == 1 ? 0x1u : 0u) |
                           (p.shuffle == 2 ? 0x4u : 0u) | (memcpyed ? 0x2u : 0u));
            o[3] = uint8_t(p.typesize);
            put32(o + 4, p.nbytes);
            put32(o + 8, p.seg_bytes);
            put32(o + 12, fs);
        }
        const uint64_t off = uint64_t(z.j) * p.seg_bytes + uint64_t(z.b) * zstd::kBlock;
        if (memcpyed) {
            copy_bytes(o + 16 + off, p.chunks + z.c * p.pitch + off, z.len);
            return;
        }
        const uint32_t sp = p.spos[z.seg];
        if (z.b == 0 && t == 0) {
            put32(o + 16 + 4 * z.j, sp);
            put32(o + sp, p.ssize[z.seg]);
        }
        fr = o + sp + 4;
        if (p.sraw[z.seg]) {
            copy_bytes(fr + uint64_t(z.b) * zstd::kBlock, zblock_src(p, z), z.len);
            return;
        }
    }
    const uint32_t fh = zstd::frame_header_bytes(z.seglen);
    if (z.b == 0 && t == 0)
        zstd::write_frame_header(fr, z.seglen);
    uint8_t* d = fr + fh + p.bpos[g];
    const bool last = z.b + 1 == z.nb;
    const uint32_t k = p.bkind[g];
    if (k == 0) {
        if (t == 0)
            zstd::write_block_header(d, last, 0, z.len);
        copy_bytes(d + 3, zblock_src(p, z), z.len);
    } else if (k == 1) {
        if (t == 0) {
            zstd::write_block_header(d, last, 1, z.len);
            d[3] = uint8_t(p.bpay[g]);
        }
    } else if (k == 2) {
        const uint32_t nl = p.bnlit[g], pay = p.bpay[g], sq = p.bseqb[g];
        const uint8_t* scr = p.scratch + uint64_t(g) * zstd::kBlock;
        // the sequences section: [count][modes][descriptions, carrier only][bits]
        const uint32_t ns = p.bnseq[g];
        const ZstdSeqSeg& Q = p.sqt[z.seg];
        const bool fitted = ns > 0 && Q.mode == 2;
        const bool scar = fitted && p.scarrier[z.seg] == z.b;
        const uint32_t sd = scar ? Q.desc_n : 0;
        uint8_t* q = d + 3;
        uint32_t lit_bytes = pay; // literal payload in scratch
        if (p.bltype[g] == 2) {
            const ZstdSegTable& T = p.tab[z.grp];
            const bool carry = p.carrier[z.grp] == z.b;
            const uint32_t cs = pay + (carry ? T.tree_n : 0);
            const uint32_t lh = zstd::lit_header_huf_bytes(nl, cs);
            if (t == 0) {
                zstd::write_block_header(d, last, 2, lh + cs + sq + sd);
                zstd::write_lit_header_huf(d + 3, carry ? 2 : 3, nl, cs);
            }
            q += lh;
            if (carry) {
                for (uint32_t i = t; i < T.tree_n; i += 256)
                    q[i] = T.tree[i];
                q += T.tree_n;
            }
        } else {
            const uint32_t lh = zstd::lit_header_raw_bytes(nl);
            if (t == 0) {
                zstd::write_block_header(d, last, 2, lh + nl + sq + sd);
                zstd::write_lit_header_raw(d + 3, 0, nl);
            }
            q += lh;
            lit_bytes = nl;
        }
        if (!fitted) {
            copy_bytes(q, scr, lit_bytes + sq);
        } else {
            // count bytes, then the modes byte: LL / OF / ML all
            // FSE_Compressed (2) in the carrier, Repeat (3) elsewhere
            const uint32_t kc = ns < 128 ? 1u : ns < 0x7F00 ? 2u : 3u;
            copy_bytes(q, scr, lit_bytes + kc);
            if (t == 0)
                q[lit_bytes + kc] = scar ? uint8_t(2u << 6 | 2u << 4 | 2u << 2)
                                         : uint8_t(3u << 6 | 3u << 4 | 3u << 2);
            uint8_t* qd = q + lit_bytes + kc + 1;
            for (uint32_t i = t; i < sd; i += 256)
                qd[i] = Q.desc[i];
            copy_bytes(qd + sd, scr + lit_bytes + kc + 1, sq - kc - 1);
        }
    }
}

} // namespace

hipError_t
launch_shuffle_blocks(const ShuffleParams& p, hipStream_t stream)
{
    if (p.n_chunks == 0 || p.nblocks == 0)
        return hipSuccess;
    if (p.nblocks > 0x7fffffffu || p.n_chunks > 65535u)
        return hipErrorInvalidValue;
    // parts per block: at least ~2048 workgroups in all (a C2 level-1 layer
    // is 32 blocks x 16 chunks), at most 16
    const uint64_t wg = uint64_t(p.nblocks) * p.n_chunks;
    const uint32_t parts = uint32_t(std::min<uint64_t>(16, std::max<uint64_t>(1, (2048 + wg - 1) / wg)));
    hipLaunchKernelGGL(shuffle_blocks, dim3(p.nblocks, p.n_chunks, parts), dim3(256), 0, stream,
                       p);
    return hipGetLastError();
}

hipError_t
launch_blosc_lz4(const BloscParams& p, hipStream_t stream)
{
    if (p.n_chunks == 0)
        return hipSuccess;
    const uint64_t ns = uint64_t(p.n_chunks) * p.g.spc;
    if (ns > 0x7fffffffull || p.g.spc == 0)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(lz4_streams, dim3(uint32_t(ns)), dim3(64), 0, stream, p);
    hipLaunchKernelGGL(chunk_layout, dim3(p.n_chunks), dim3(256), 0, stream, p);
    hipLaunchKernelGGL(scan_offsets, dim3(1), dim3(256), 0, stream, p.fsize, p.order,
                       p.offsets, p.cstart, p.n_chunks);
    hipLaunchKernelGGL(write_frames, dim3(uint32_t(ns)), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t
launch_zstd(const ZstdParams& p, hipStream_t stream)
{
    if (p.n_chunks == 0)
        return hipSuccess;
    const uint64_t nseg = uint64_t(p.n_chunks) * p.nseg;
    const uint64_t nblk = nseg * p.bps;
    if (nblk * kZSubBlocks > 0x7fffffffull || p.nseg == 0 || p.bps == 0 ||
        uint64_t(p.bps) * zstd::kBlock < p.seg_bytes)
        return hipErrorInvalidValue;
    if (p.hgrp_log2 > 5 || p.ngrp != ((p.bps + (1u << p.hgrp_log2) - 1) >> p.hgrp_log2))
        return hipErrorInvalidValue;
    if (!p.store_only) {
        hipError_t e = hipMemsetAsync(p.scount, 0, nseg * 192 * 4, stream);
        if (e != hipSuccess)
            return e;
        if (p.match) {
            e = hipMemsetAsync(p.hist, 0, nblk * 256 * 4, stream);
            if (e != hipSuccess)
                return e;
            const dim3 gd(uint32_t(nblk * kZSubBlocks));
            if (p.far) {
                const uint32_t S = p.far_slices;
                if (!(S == 1 || S == 2 || S == 4 || S == 8) || p.far_tb < 6 ||
                    p.far_log < 10 || p.far_log > kFarLog ||
                    p.far_tb + p.far_log + (S == 8 ? 3 : S == 4 ? 2 : S == 2 ? 1 : 0) > 32 ||
                    (reinterpret_cast<uintptr_t>(p.src) & 3u) || (p.src_pitch & 3u) ||
                    (p.seg_bytes & 3u))
                    return hipErrorInvalidValue;
                static const hipError_t attr = hipFuncSetAttribute(
                  reinterpret_cast<const void*>(zstd_far),
                  hipFuncAttributeMaxDynamicSharedMemorySize, int(4u << kFarLog));
                if (attr != hipSuccess)
                    return attr;
                const uint32_t R = p.far_ranges;
                if (!(R == 1 || R == 2 || R == 4 || R == 8))
                    return hipErrorInvalidValue;
                hipLaunchKernelGGL(zstd_far, dim3(uint32_t(nseg * p.far_slices * R)),
                                   dim3(kFarThreads), size_t(4) << p.far_log, stream, p);
            }
            if (p.phist == 0 && !p.far)
                hipLaunchKernelGGL((zstd_parse<0, kLz4HashLog>), gd, dim3(64), 0, stream, p);
            else if (p.phist <= kZHist1 && !p.far)
                hipLaunchKernelGGL((zstd_parse<kZHist1, 13>), gd, dim3(64), 0, stream, p);
            else if (!p.far)
                hipLaunchKernelGGL((zstd_parse<kZHist2, 14>), gd, dim3(64), 0, stream, p);
            else if (p.phist == 0)
                hipLaunchKernelGGL((zstd_parse<0, kLz4HashLog, true>), gd, dim3(64), 0, stream, p);
            else if (p.phist <= kZHist1)
                hipLaunchKernelGGL((zstd_parse<kZHist1, 13, true>), gd, dim3(64), 0, stream, p);
            else
                hipLaunchKernelGGL((zstd_parse<kZHist2, 14, true>), gd, dim3(64), 0, stream, p);
        } else {
            hipLaunchKernelGGL(zstd_hist, dim3(uint32_t(nblk)), dim3(256), 0, stream, p);
        }
        hipLaunchKernelGGL(zstd_table, dim3(uint32_t(nseg * p.ngrp)), dim3(64), 0, stream, p);
        hipLaunchKernelGGL(zstd_encode, dim3(uint32_t(nblk)), dim3(256), 0, stream, p);
        hipLaunchKernelGGL(zstd_seqtab, dim3(uint32_t(nseg)), dim3(64), 0, stream, p);
        if (p.match)
            hipLaunchKernelGGL(zstd_seqenc, dim3(uint32_t(nseg * ((p.bps + 63) / 64))), dim3(64), 0,
                               stream, p);
        hipLaunchKernelGGL(zstd_segment, dim3(uint32_t(nseg)), dim3(64), 0, stream, p);
    }
    hipLaunchKernelGGL(zstd_chunk, dim3(p.n_chunks), dim3(256), 0, stream, p);
    hipLaunchKernelGGL(scan_offsets, dim3(1), dim3(256), 0, stream, p.fsize, p.order,
                       p.offsets, p.cstart, p.n_chunks);
    hipLaunchKernelGGL(zstd_write, dim3(uint32_t(nblk)), dim3(256), 0, stream, p);
    return hipGetLastError();
}

} // namespace aqz
