// aqz_codec.hh -- device chunk compression: the blosc1
// frame of Chunk::compress_and_take_buffer (chunk.cpp:78-106) ->
// zarr::compress_in_place (zarr.common.cpp:106-140) ->
// blosc_compress_ctx(clevel, shuffle, typesize, ..., "lz4", blocksize 0, 1
// thread), produced on the GPU for a whole resident chunk layer at once.
//
// Output parity is at the decoded level: any blosc1 decoder returns the
// chunk bytes.  The frame differs from c-blosc's own in two documented
// choices -- the block size (kLz4StreamMax bytes per split stream, so a
// stream fits in LDS; the header records it, and zarr.json says blocksize
// 0 = "whatever the frame says") and the LZ4 match finder (parallel hash
// probing instead of LZ4_compress_fast's sequential scan) -- so the
// compressed bytes differ while every decoded byte is identical.
#pragma once

#include "aqz_zstd.hh"

#include <hip/hip_runtime.h>

#include <cstdint>

namespace aqz {

// bytes of one LZ4-compressed stream (resident in LDS while it is encoded)
// and the hash table size.  The encoder is latency-bound, so occupancy
// rules: 4 KiB streams + a 1024-entry table (6 KiB of LDS, 77 VGPRs: 24
// waves/CU) ran camera-like u16 chunks 1.4x (byte shuffle) and 1.3x
// (bitshuffle) faster than 8 KiB + 2048 entries (12 KiB, 103 VGPRs: 13
// waves/CU) for a ratio 0.3-1.2% lower; 2 KiB streams were no faster.
constexpr uint32_t kLz4StreamMax = 4096;
constexpr int kLz4HashLog = 10;

// The blosc1 frame geometry shared by every chunk of a layer.
struct BloscGeom
{
    uint32_t nbytes;    // chunk bytes (blosc nbytes)
    uint32_t typesize;  // bytes per pixel
    uint32_t shuffle;   // 0 none, 1 byte shuffle, 2 bit shuffle
    uint32_t blocksize;
    uint32_t nfull;     // full blocks
    uint32_t left;      // bytes of the trailing (leftover) block, 0 = none
    uint32_t ns_full;   // streams per full block: typesize (split) or 1
    uint32_t spc;       // streams per chunk
    uint32_t slot;      // scratch bytes per stream (>= its length)
    uint32_t nblocks;
};

// Block size and split rule; throws nothing (callers validate inputs).
BloscGeom make_blosc_geom(uint32_t nbytes, uint32_t typesize, uint32_t shuffle);

struct BloscParams
{
    BloscGeom g;
    const uint8_t* chunks;  // chunk c at chunks + c * pitch
    uint64_t pitch;
    uint32_t n_chunks;
    const uint32_t* flags;  // has_data words (nullptr: every chunk has data)
    uint32_t tag;           // a chunk has data iff flags[c] == tag
    uint8_t* scratch;       // [n_chunks * spc] stream slots of g.slot bytes
    uint32_t* ssize;        // [n_chunks * spc] bytes stored per stream
    uint32_t* spos;         // [n_chunks * spc] record offset inside the frame
    uint32_t* fsize;        // [n_chunks] frame bytes (0: chunk skipped)
    uint8_t* mode;          // [n_chunks] 1: memcpyed frame
    const uint32_t* order;  // [n_chunks] output position -> chunk (nullptr:
                            // chunk order); shard-major for shard packing
    uint64_t* offsets;      // [n_chunks + 1] frame offsets in out, in output
                            // order; [n] = total
    uint64_t* cstart;       // [n_chunks] frame offset of each chunk
    uint8_t* out;           // frames, back to back in output order
    uint32_t store_only;    // clevel 0: every frame memcpyed, no LZ4
};

// Enqueue the whole layer: streams -> per-chunk layout -> offsets -> frames.
hipError_t launch_blosc_lz4(const BloscParams& p, hipStream_t stream);

} // namespace aqz

namespace aqz {

// Block shuffle of a resident chunk layer for the host-side zstd codecs
// (aqz_hostzstd.hh): block j of chunk c (blocks of `blocksize` bytes) goes,
// byte- or bit-shuffled as c-blosc 1.x does it, to
// out + c * nbytes + j * blocksize.  Chunks whose flag is not `tag` are
// skipped (flags may be null).
struct ShuffleParams
{
    const uint8_t* chunks;
    uint64_t pitch;
    uint32_t n_chunks;
    const uint32_t* flags;
    uint32_t tag;
    uint32_t nbytes, typesize, shuffle, blocksize, nblocks;
    uint8_t* out;
};
hipError_t launch_shuffle_blocks(const ShuffleParams& p, hipStream_t stream);

} // namespace aqz

namespace aqz {

// Device zstd (aqz_zstd.hh for the format pieces): blosc1 frames with the
// zstd codec (one zstd frame per blosc block, "don't split") or plain zstd
// frames (one per chunk), for a whole resident chunk layer.  A segment is
// what one zstd frame holds (a blosc block, or a chunk); it is cut into
// zstd blocks of zstd::kBlock bytes, the parallel unit.
// The Huffman table of a group of zstd blocks (at most kHufGroup, 64 KiB):
// the literal statistics of a shuffled blosc block change at its byte or bit
// planes, so one table per segment fits no plane (tools/zstd_lab.cpp: c-blosc's
// ratio within 1% with group tables, 6% short with segment tables).  A group
// is one plane where planes are shorter than kHufGroup blocks at blosc
// clevel >= 7 (bitshuffle: a u16 plane of a 256 KiB block is 16 KiB, 2
// blocks; tools/zstd_lab.cpp with far candidates: dim sCMOS 3.20 -> 3.37,
// camera 1.972 -> 1.983, c-blosc clevel 5 3.14 / 1.974) -- four times the
// tables to build (zstd_table 0.5 -> 2.5 ms per 512 MiB layer).
// Unshuffled data (plain zstd, or blosc without a shuffle) keeps its
// statistics across a chunk: groups of kHufGroupPlain blocks (256 KiB),
// a quarter of the tables to build (tools/zstd_lab.cpp hufgroup=8/16/32:
// camera-like 1.596 / 1.596 / 1.596, dim 3.260 / 3.260 / 3.260).
// The first Huffman block of a group carries the tree, the rest are Treeless.
constexpr uint32_t kHufGroup = 8;
constexpr uint32_t kHufGroupPlainLog2 = 5;

// log2 of the blocks per Huffman group for a segment of seg_bytes
inline uint32_t
zstd_huf_group_log2(uint32_t shuffle, uint32_t typesize, uint32_t seg_bytes, int32_t clevel)
{
    if (shuffle == 0)
        return kHufGroupPlainLog2;
    uint32_t lg = 3; // kHufGroup
    if (shuffle == 2 && typesize > 0 && clevel >= 7) {
        const uint32_t plane = seg_bytes / (8u * typesize);
        while (lg > 0 && (zstd::kBlock << lg) > plane)
            --lg;
    }
    return lg;
}
struct ZstdSegTable
{
    uint32_t mode;   // 0 raw literals, 1 one symbol, 2 Huffman
    uint32_t tree_n; // bytes of the tree description
    uint32_t pad[2];
    uint16_t code[256];
    uint8_t len[256];
    uint8_t tree[160];
};

// The sequence tables of a segment (one zstd frame): FSE_Compressed tables
// built from the segment's literal-length / offset / match-length code
// counts, described by the first block with sequences (mode 2) and repeated
// by the others (mode 3); or the predefined distributions (mode 0) when
// they cost less.
struct ZstdSeqSeg
{
    uint32_t mode;      // 0 predefined, 2 custom
    uint32_t desc_n;    // bytes of the three table descriptions (LL, OF, ML)
    uint32_t pad[2];
    uint8_t desc[256];
    zstd::FseTable<zstd::kSeqMaxLog> ll, of, ml;
};

struct ZstdParams
{
    const uint8_t* src;     // segment data: chunk c at src + c * src_pitch
    uint64_t src_pitch;
    const uint8_t* chunks;  // the unshuffled chunks (memcpyed blosc frames)
    uint64_t pitch;
    uint32_t n_chunks, nbytes, typesize, shuffle;
    uint32_t blosc;         // 1 blosc-zstd frames, 0 plain zstd frames
    uint32_t seg_bytes;     // bytes per segment (blosc block size or nbytes)
    uint32_t nseg;          // segments per chunk
    uint32_t bps;           // zstd block slots per segment
    uint32_t store_only;    // blosc clevel 0: every frame memcpyed
    uint32_t match;         // 1: LZ sequences (zstd_parse); 0: literals only
    uint32_t match_bits;    // a match must save this many literal bits
    uint32_t phist;         // parse history: bytes before a unit its matches
                            // may reach (0, kZHist1, kZHist2: the level)
    uint32_t ngrp;          // Huffman groups per segment
    uint32_t hgrp_log2;     // log2 of the zstd blocks per Huffman group (<= 5)
    uint32_t fit;           // 1: fitted sequence tables allowed (AQZ_ZSTD_FIT=0: predefined)
    // far candidates (zstd_far; plain zstd at level >= 5): per segment
    // position the most recent earlier position with the same 5-byte key,
    // + 1 (0: none), [n_chunks * nseg * seg_bytes]; nullptr: no far pass
    uint32_t* far;
    uint32_t far_tb;        // tag bits of a far table entry (32 - position bits)
    uint32_t far_slices;    // hash slices (workgroups) per segment: 1, 2, 4 or 8
    uint32_t far_log;       // log2 of a slice's table entries (<= kFarLog)
    uint32_t far_ranges;    // ranges per segment walked in parallel (1, 2, 4, 8;
                            // each warmed up with the far_warm steps before it)
    uint32_t far_warm;      // steps a range after the first inserts first
    uint32_t dbg;           // parse A/B switches (bench option zstd_flags; 0 = shipped)
    const uint32_t* flags;  // has_data words (nullptr: every chunk has data)
    uint32_t tag;
    const zstd::SeqTables* seqt; // predefined sequence tables (device)
    // per parse unit (kZSubBlocks per zstd block, kZSub bytes each)
    uint8_t* lits;          // literal bytes, kZSub per unit
    uint64_t* seqs;         // kZSubSeq packed sequences per unit
    uint32_t* snseq, *snlit, *stail;
    uint32_t* sval;         // the unit's one byte value, 256 when it has several
    // per zstd block ([n_chunks * nseg * bps])
    uint32_t* hist;         // [.. * 256] literal histogram
    uint8_t* bkind;         // 0 raw, 1 RLE, 2 compressed, 3 none, 4 sequences pending
    uint8_t* bltype;        // compressed: literals 0 raw, 2 Huffman
    uint32_t* bpay;         // compressed: literal payload bytes; RLE: the byte
    uint32_t* bseqb;        // compressed: sequences section bytes
    uint32_t* bnlit;        // literals of the block
    uint32_t* bpos;         // block offset after the frame header
    uint8_t* scratch;       // [literal payload][sequences section], zstd::kBlock each
    uint32_t* bnseq;        // sequences of the block
    // per Huffman group ([n_chunks * nseg * ngrp])
    ZstdSegTable* tab;
    uint32_t* carrier;      // block of the group carrying its tree (~0: none)
    // per segment ([n_chunks * nseg])
    uint32_t* scount;       // [.. * 3 * 64] LL / OF / ML code counts
    ZstdSeqSeg* sqt;        // sequence tables
    uint32_t* scarrier;     // block carrying the sequence table descriptions
    uint32_t* ssize;        // record bytes (zstd frame, or the raw block)
    uint8_t* sraw;          // 1: record stored raw (blosc)
    uint32_t* spos;         // record offset inside the chunk frame (blosc)
    // per chunk
    uint32_t* fsize;
    uint8_t* mode;          // 1: memcpyed blosc frame
    const uint32_t* order;
    uint64_t* offsets;
    uint64_t* cstart;
    uint8_t* out;
};

// parse units of a zstd block: 4 KiB, one wave each (LDS-resident, as the
// LZ4 encoder's streams), at most kZSubSeq sequences each
constexpr uint32_t kZSub = 4096;
constexpr uint32_t kZSubBlocks = zstd::kBlock / kZSub;
constexpr uint32_t kZSubSeq = 1024; // a match is >= 4 bytes
// parse history of the levels (zstd level >= 3: 12 KiB, >= 7: 28 KiB; blosc
// clevel c is zstd level 2c - 1)
constexpr uint32_t kZHist1 = 12 * 1024;
constexpr uint32_t kZHist2 = 28 * 1024;
// far candidates (zstd_far): hash slices of 2^15 entries (128 KiB of LDS
// each, one workgroup per slice walking the whole segment); a far match is
// >= 5 bytes.  tools/zstd_lab.cpp, 8 MiB chunks, no LDS history: 4 slices
// (2^17 entries) camera-like 1.458 -> 1.596, dim sCMOS 3.070 -> 3.260; 8
// slices camera 1.624 (libzstd level 5: 1.699 / 3.377)
constexpr uint32_t kFarLog = 15;
constexpr uint32_t kFarMin = 5;
// a far range after the first inserts at least the 1 MiB before it first (no
// probes), and at least two of the chunk's planes (the previous planes are
// where camera data repeats)
constexpr uint32_t kFarWarm = 256; // steps of kZSub bytes
constexpr uint32_t kZOffMax = (1u << 24) - 4; // largest match distance (aqz_codec.hip zseq_codes)
// tag bits for a segment of seg_bytes split into `slices` hash slices of
// 2^far_log entries (0: segments too large for the pass)
inline uint32_t
zstd_far_tag_bits(uint32_t seg_bytes, uint32_t slices, uint32_t far_log = kFarLog)
{
    uint32_t pb = 0, sb = 0;
    while (pb < 32 && (uint64_t(1) << pb) <= seg_bytes) // positions + 1 <= seg_bytes
        ++pb;
    while ((1u << sb) < slices)
        ++sb;
    const uint32_t room = 32 - sb - far_log; // hash bits left for the tag
    const uint32_t tb = 32 - pb < room ? 32 - pb : room;
    return tb >= 6 ? tb : 0;
}

hipError_t launch_zstd(const ZstdParams& p, hipStream_t stream);

} // namespace aqz
