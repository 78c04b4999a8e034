/*
 * aqz_codec_oracle.c -- CPU ORACLE for the chunk-compression row (SURVEY
 * §8f rank 2) and the shard index (§8f rank 3).  TEST INFRASTRUCTURE ONLY:
 * tests/ use it to decode what the HIP compressor produced.  Nothing under
 * acquire-zarr_amd/ links or calls it.
 *
 * The reference compresses a chunk with c-blosc's blosc_compress_ctx
 * (zarr.common.cpp:106-140, called from Chunk::compress_and_take_buffer,
 * chunk.cpp:78-106) -- a THIRD-PARTY dependency absent from /root/reference
 * (vcpkg.json pins blosc >= 1.21.5; the image ships c-blosc 1.21.0 and
 * lz4 1.9.3 under /opt/conda, used by the tests as a second, independent
 * decoder).  This file restates the PUBLISHED formats:
 *   - the blosc1 frame: 16-byte header (version, versionlz, flags,
 *     typesize, nbytes, blocksize, cbytes; flags bit0 byte shuffle, bit1
 *     memcpyed, bit2 bit shuffle, bit4 "don't split", bits 5-7 codec),
 *     then one int32 start offset per block, then per block one
 *     (int32 csize, bytes) record per split stream; a stream whose csize
 *     equals its length is stored raw;
 *   - the byte shuffle and the bitshuffle (bit-plane transpose of groups
 *     of 8 elements) of a block;
 *   - the LZ4 block format (token, literal run, 16-bit offset, match run;
 *     the last 5 bytes are literals and the last match starts at least 12
 *     bytes before the end -- enforced here so an encoder that breaks the
 *     rule fails the test even where a lenient decoder would not);
 *   - CRC-32C (Castagnoli, reflected 0x82F63B78), the checksum of the shard
 *     index table (shard.cpp:145-166).
 */
#include "aqz_oracle.h"

#include <string.h>

static uint32_t
rd32(const uint8_t* p)
{
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
           (uint32_t)p[3] << 24;
}

/* ---- byte shuffle of one block ------------------------------------------ */
void
or_shuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst)
{
    const size_t ne = n / ts;
    for (size_t j = 0; j < ts; ++j)
        for (size_t i = 0; i < ne; ++i)
            dst[j * ne + i] = src[i * ts + j];
    memcpy(dst + ne * ts, src + ne * ts, n - ne * ts);
}

void
or_unshuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst)
{
    const size_t ne = n / ts;
    for (size_t j = 0; j < ts; ++j)
        for (size_t i = 0; i < ne; ++i)
            dst[i * ts + j] = src[j * ne + i];
    memcpy(dst + ne * ts, src + ne * ts, n - ne * ts);
}

/* ---- bitshuffle of one block (c-blosc 1.x): when the block holds a
 * multiple of 8 elements it is transposed to ts*8 bit-planes (plane
 * r = 8*byte + bit, each ne/8 bytes; bit k of plane byte m = that bit of
 * element 8m+k); any other block is copied unchanged. */
void
or_bitshuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst)
{
    const size_t ne = n / ts;
    if (ne % 8 != 0 || ne * ts != n) {
        memcpy(dst, src, n);
        return;
    }
    const size_t row = ne / 8;
    memset(dst, 0, ne * ts);
    for (size_t i = 0; i < ne; ++i)
        for (size_t j = 0; j < ts; ++j)
            for (size_t b = 0; b < 8; ++b)
                if ((src[i * ts + j] >> b) & 1u)
                    dst[(j * 8 + b) * row + i / 8] |= (uint8_t)(1u << (i % 8));
    memcpy(dst + ne * ts, src + ne * ts, n - ne * ts);
}

void
or_bitunshuffle(size_t ts, size_t n, const uint8_t* src, uint8_t* dst)
{
    const size_t ne = n / ts;
    if (ne % 8 != 0 || ne * ts != n) {
        memcpy(dst, src, n);
        return;
    }
    const size_t row = ne / 8;
    memset(dst, 0, ne * ts);
    for (size_t i = 0; i < ne; ++i)
        for (size_t j = 0; j < ts; ++j)
            for (size_t b = 0; b < 8; ++b)
                if ((src[(j * 8 + b) * row + i / 8] >> (i % 8)) & 1u)
                    dst[i * ts + j] |= (uint8_t)(1u << b);
    memcpy(dst + ne * ts, src + ne * ts, n - ne * ts);
}

/* ---- LZ4 block decoder (strict) ----------------------------------------- */
long
or_lz4_decompress(const uint8_t* src, size_t csize, uint8_t* dst, size_t dsize)
{
    size_t ip = 0, op = 0;
    if (csize == 0)
        return -1;
    for (;;) {
        if (ip >= csize)
            return -1;
        const unsigned token = src[ip++];
        size_t lit = token >> 4;
        if (lit == 15) {
            unsigned b;
            do {
                if (ip >= csize)
                    return -1;
                b = src[ip++];
                lit += b;
            } while (b == 255);
        }
        if (ip + lit > csize || op + lit > dsize)
            return -1;
        memcpy(dst + op, src + ip, lit);
        ip += lit;
        op += lit;
        if (ip == csize) /* last sequence: literals only */
            break;
        if (ip + 2 > csize)
            return -1;
        const size_t off = (size_t)src[ip] | (size_t)src[ip + 1] << 8;
        ip += 2;
        if (off == 0 || off > op)
            return -1;
        size_t ml = token & 15u;
        if (ml == 15) {
            unsigned b;
            do {
                if (ip >= csize)
                    return -1;
                b = src[ip++];
                ml += b;
            } while (b == 255);
        }
        ml += 4;
        if (op + 12 > dsize)            /* MFLIMIT: match starts too late */
            return -1;
        if (op + ml + 5 > dsize)        /* LASTLITERALS */
            return -1;
        for (size_t k = 0; k < ml; ++k) /* overlapping copy, byte by byte */
            dst[op + k] = dst[op + k - off];
        op += ml;
    }
    return op == dsize ? (long)op : -1;
}

/* ---- blosc1 frame ------------------------------------------------------- */
int
or_blosc_frame_info(const uint8_t* src, size_t srcsize, or_blosc_info* info)
{
    if (srcsize < 16)
        return -1;
    info->version = src[0];
    info->versionlz = src[1];
    info->flags = src[2];
    info->typesize = src[3];
    info->nbytes = rd32(src + 4);
    info->blocksize = rd32(src + 8);
    info->cbytes = rd32(src + 12);
    return 0;
}

/* nsplits rule of the blosc1 decoder: a full block is split into typesize
 * streams unless the frame says "don't split", typesize > 16 or the block
 * holds fewer than 128 elements; a leftover block is never split. */
static size_t
n_streams(const or_blosc_info* h, size_t bsize, int leftover)
{
    if (!(h->flags & 0x10) && h->typesize <= 16 && h->typesize > 0 &&
        bsize / h->typesize >= 128 && !leftover)
        return h->typesize;
    return 1;
}

long
or_blosc_decompress(const uint8_t* src, size_t srcsize, uint8_t* dst, size_t dstcap,
                    uint8_t* tmp)
{
    or_blosc_info h;
    if (or_blosc_frame_info(src, srcsize, &h) != 0)
        return -1;
    if (h.version != 2 || h.cbytes > srcsize || h.nbytes > dstcap || h.typesize == 0)
        return -2;
    if (h.flags & 0x2) { /* memcpyed */
        if (h.cbytes != h.nbytes + 16)
            return -3;
        memcpy(dst, src + 16, h.nbytes);
        return (long)h.nbytes;
    }
    if ((h.flags >> 5) != 1 || h.versionlz != 1) /* LZ4 only */
        return -4;
    if (h.blocksize == 0 || h.nbytes == 0)
        return h.nbytes == 0 ? 0 : -5;
    const size_t nfull = h.nbytes / h.blocksize;
    const size_t left = h.nbytes % h.blocksize;
    const size_t nblocks = nfull + (left ? 1 : 0);
    if (16 + 4 * nblocks > h.cbytes)
        return -6;
    for (size_t j = 0; j < nblocks; ++j) {
        const int lo = (j == nfull);
        const size_t bsize = lo ? left : h.blocksize;
        const size_t ns = n_streams(&h, bsize, lo);
        const size_t ne = bsize / ns;
        size_t p = rd32(src + 16 + 4 * j);
        for (size_t s = 0; s < ns; ++s) {
            if (p + 4 > h.cbytes)
                return -7;
            const size_t cb = rd32(src + p);
            p += 4;
            if (p + cb > h.cbytes)
                return -8;
            if (cb == ne)
                memcpy(tmp + s * ne, src + p, ne);
            else if (or_lz4_decompress(src + p, cb, tmp + s * ne, ne) != (long)ne)
                return -9;
            p += cb;
        }
        uint8_t* out = dst + j * h.blocksize;
        if ((h.flags & 0x1) && h.typesize > 1)
            or_unshuffle(h.typesize, bsize, tmp, out);
        else if (h.flags & 0x4)
            or_bitunshuffle(h.typesize, bsize, tmp, out);
        else
            memcpy(out, tmp, bsize);
    }
    return (long)h.nbytes;
}

/* ---- CRC-32C (shard index checksum) ------------------------------------- */
uint32_t
or_crc32c(const uint8_t* p, size_t n)
{
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k)
            c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
    }
    return c ^ 0xFFFFFFFFu;
}
