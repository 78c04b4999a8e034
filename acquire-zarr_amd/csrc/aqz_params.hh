// aqz_params.hh -- plain structs shared by the host engine and the HIP
// kernels (passed by value as kernel arguments).
#pragma once

#include <cstdint>

namespace aqz {

// n / d for n < 2^31 as (umulhi(n, m) + n) >> s; d >= 1.
struct FastDiv
{
    uint32_t d, m, s;
};

inline FastDiv
make_fastdiv(uint32_t d)
{
    uint32_t s = 0;
    while ((uint64_t(1) << s) < d)
        ++s;
    const uint64_t m =
      ((uint64_t(1) << 32) * ((uint64_t(1) << s) - d)) / d + 1;
    return FastDiv{ d, static_cast<uint32_t>(m), s };
}

// Geometry + output plumbing of one pyramid level for one launch.
struct LevelGeom
{
    uint32_t W, H;          // level pixel dims
    uint32_t tw, th, ntx;   // chunk tile dims, tiles along x
    FastDiv dtw, dth;
    uint64_t bpc;           // bytes per chunk
    uint64_t slot_bytes;    // bytes per resident chunk layer
    uint32_t n_chunks;      // chunks per layer
    uint32_t n_slots;       // resident layers (ring)
    uint32_t frames_per_layer;
    uint32_t fid0_mod;      // (level frame id of batch frame 0) % frames_per_layer
    uint32_t slot0;         // ring slot of the layer holding batch frame 0
    uint8_t* base;          // chunk-layer ring (nullptr: no tile output)
    uint32_t* flags;        // has_data, [n_slots * n_chunks]
    const uint64_t* tab_off; // [frames_per_layer]: group*bpc + internal offset
    const uint32_t* tab_grp; // [frames_per_layer]: tile_group_offset
    uint8_t* scratch;       // row-major frames (nullptr: none), stride W*H
};

constexpr int kMaxFused = 6;
constexpr int kMaxRegionRows = 128; // LDS is sized for this region height
constexpr int kMaxPlanes3d = 8;     // level-0 planes per 2x2x2 group

// Where a frame of a level lands: the base of its tiles inside its resident
// chunk layer (= slot base + tile_group_offset*bytes_per_chunk +
// chunk_internal_offset, array.dimensions.cpp:264-314) and its has_data
// words.  One table per level covers a full ring period (n_slots *
// frames_per_layer frames), built once at stage creation.
struct FrameRef
{
    uint8_t* tiles;
    uint32_t* flags;
};

// A level's frames of one launch: frame f has ring-period index (r0 + f)
// mod period; its has_data tag is the slot generation + 1 (so has_data words
// never need clearing: a chunk has data iff its word equals the tag of the
// layer resident in that slot).
struct LevelRefs
{
    const FrameRef* table; // nullptr: this level is not tile-split
    uint32_t r0, period, tag0;
};

// The fused pyramid launch.  Chunk sizes are the same at every level
// (downsample_dimension keeps chunk_size_px, downsampler.cpp:15-17), so only
// the level extents vary per level.
struct FusedParams
{
    const uint8_t* src;      // level-0 frames, row-major (xy: acquisition order)
    uint64_t src_stride;     // bytes between frames
    uint32_t xy;             // 1: src holds acquisition-order frames (XY-transposed storage
                             // order): storage pixel (y, x) is src[x * H[0] + y]
                             // (transpose_frame, array.cpp:488-534, fused into the loads)
    LevelRefs lr[kMaxFused + 1];
    uint8_t* scratch;        // row-major frames of level scratch_level
    uint32_t scratch_level;  // 0: no scratch output
    uint32_t n_frames;
    uint32_t n_fused;        // levels 1..n_fused computed here (<= kMaxFused)
    uint32_t rh_log2;        // region height = 1 << rh_log2 (>= 4)
    uint32_t nbx, nby;       // regions per frame along x / y
    uint32_t nbx_in, nby_in; // interior (fast-path) regions along x / y
    uint32_t vec_rows;       // 1: every row start is 16-B aligned
    uint32_t fast_ok;        // 1: tiles fit the interior fast path
    uint32_t nt;             // bit0: non-temporal input loads, bit1: nt level-0 stores
    uint32_t knobs;          // tuning A/B switches (0 = shipped defaults)
    uint32_t xcd_order;      // 1: interior regions walk XCD-contiguous ranges
    uint32_t xcd_rot;        // XCD x starts its range x * xcd_rot regions in
    uint32_t xrot[8];        // (launcher-filled: x * xcd_rot mod range)
    uint32_t xskew;          // frames per XCD range - 1 when skewed (power of 2), else 0
    uint32_t G;              // 2x2x2 kernel: level-0 planes per group
    uint32_t zmask;          // 2x2x2 kernel: bit k = level k halves z
    uint32_t tw, th;         // chunk tile (x, y) in pixels
    FastDiv dtw, dth;
    uint64_t bpc;            // bytes per chunk
    FastDiv d_nreg_in, d_nbx_in;
    uint32_t W[kMaxFused + 1], H[kMaxFused + 1], ntx[kMaxFused + 1];
};

// One output frame (or partial plane) of the generic level kernel.  Pixel
// value = R2(A, B) if b != nullptr else A, where A/B are the 2x2 reduction
// of a/b when *_scale, else a/b itself (Downsampler::add_frame's
// next_level_frame and average2_fun_, downsampler.cpp:341-389).
struct LevelOp
{
    const uint8_t* a;       // earlier plane (or the only one)
    const uint8_t* b;       // later plane, or nullptr
    uint8_t* scratch_out;   // row-major destination or nullptr
    uint64_t tile_off;      // byte offset of this frame in the layer ring
    uint32_t flag_off;      // flag index of this frame's chunk group
    uint32_t tag;           // has_data tag (slot generation + 1)
    uint32_t a_scale, b_scale, has_tile;
};

struct LevelParams
{
    uint32_t Wp, Hp;         // source (level k-1) dims
    LevelGeom g;             // level k
    const LevelOp* ops;
    uint32_t n_ops;
};

} // namespace aqz
