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

// One workgroup per (block, chunk): the c-blosc 1.x byte shuffle (byte jj
// of element i -> jj * ne + i) or bitshuffle (bit b of byte jj of element
// 8m + k -> bit k of byte m of plane 8 jj + b) of one block.
__global__ __launch_bounds__(256) void
shuffle_blocks(const ShuffleParams p)
{
    const uint32_t j = blockIdx.x, c = blockIdx.y;
    if (p.flags && p.flags[c] != p.tag)
        return;
    const uint32_t t = threadIdx.x;
    const uint32_t b0 = j * p.blocksize;
    const uint32_t bsize = min(p.blocksize, p.nbytes - b0);
    const uint32_t ts = p.typesize;
    const uint32_t ne = bsize / ts;
    const uint8_t* src = p.chunks + c * p.pitch + b0;
    uint8_t* dst = p.out + uint64_t(c) * p.nbytes + b0;
    const bool src16 = (reinterpret_cast<uintptr_t>(src) & 15u) == 0;
    if (p.shuffle == 1 && ts > 1) {
        uint32_t done = 0; // elements handled by the vector path
        if ((ts == 2 || ts == 4 || ts == 8) && src16) {
            const uint32_t vec = 16 / ts; // elements per 16-B load
            const bool dst_ok = (reinterpret_cast<uintptr_t>(dst) % vec) == 0 && ne % vec == 0;
            if (dst_ok) {
                for (uint32_t w = t; w < ne / vec; w += 256) {
                    const uint4 v = *reinterpret_cast<const uint4*>(src + 16ull * w);
                    uint8_t e[16];
                    __builtin_memcpy(e, &v, 16);
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
                done = ne;
            }
        }
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
        for (uint32_t m = t; m < row; m += 256) {
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
    for (uint32_t x = t; x < bsize; x += 256)
        dst[x] = src[x];
}

} // namespace

hipError_t
launch_shuffle_blocks(const ShuffleParams& p, hipStream_t stream)
{
    if (p.n_chunks == 0 || p.nblocks == 0)
        return hipSuccess;
    if (p.nblocks > 0x7fffffffu || p.n_chunks > 65535u)
        return hipErrorInvalidValue;
    hipLaunchKernelGGL(shuffle_blocks, dim3(p.nblocks, p.n_chunks), dim3(256), 0, stream, p);
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

} // namespace aqz
