#include <cstdio>
// aqz_engine.cpp -- see aqz_engine.hh.  Citations are to
// /root/reference/src/streaming/.
#include "aqz_engine.hh"

#include <hsa/hsa_ext_amd.h>
#include "aqz_zstd.hh"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace aqz {


constexpr int kMemDevice = 1;
constexpr int kMemHostPinned = 2;

void
hip_check(hipError_t e, const char* what)
{
    if (e != hipSuccess) {
        (void)hipGetLastError(); // clear
        throw Error(e == hipErrorOutOfMemory ? 6 : 5,
                    std::string(what) + ": " + hipGetErrorString(e));
    }
}

// rings of at least this many bytes in all go to the 2 MiB-piece arena
constexpr uint64_t kArenaMinRings = uint64_t(256) << 20;
constexpr unsigned kArenaFlags = DevBuf::kVmm | (5u << 9); // 2 MiB pieces

// A large work buffer: from 2 MiB virtual-memory pieces when `vmm` and at
// least 64 MiB (CodecTuning::vmm), else hipMalloc.
static void
alloc_large(DevBuf& b, size_t bytes, bool vmm)
{
    if (b.p && !b.view && b.n >= bytes)
        return;
    b.alloc(bytes, vmm && bytes >= (size_t(64) << 20) ? kArenaFlags : 0u);
}

DevBuf::~DevBuf()
{
    release();
}

// A failed release leaks device memory silently unless it is said: the
// destructor path cannot throw, so it is logged once per kind.
static void
release_check(hipError_t e, const char* what)
{
    if (e == hipSuccess)
        return;
    (void)hipGetLastError();
    static std::atomic<unsigned> said{ 0 };
    if (said.fetch_add(1) < 8)
        std::fprintf(stderr, "aqz: %s failed while releasing device memory: %s\n", what,
                     hipGetErrorString(e));
}

void
DevBuf::release()
{
    if (p && !view) {
        if (vmm_span) {
            // every piece was its own hipMemMap: unmapped one by one, then
            // the handles and the reserved range
            for (size_t i = 0; i < vmm_mapped; ++i)
                release_check(hipMemUnmap(p + i * vmm_piece, vmm_piece), "hipMemUnmap");
            for (auto h : vmm)
                release_check(hipMemRelease(h), "hipMemRelease");
            release_check(hipMemAddressFree(p, vmm_span), "hipMemAddressFree");
        } else {
            release_check(hipFree(p), "hipFree");
        }
    }
    p = nullptr;
    n = 0;
    view = false;
    vmm.clear();
    vmm_span = 0;
    vmm_piece = 0;
    vmm_mapped = 0;
}

DevBuf::DevBuf(DevBuf&& o) noexcept
{
    *this = std::move(o);
}

DevBuf&
DevBuf::operator=(DevBuf&& o) noexcept
{
    if (this != &o) {
        release();
        p = o.p;
        n = o.n;
        view = o.view;
        vmm = std::move(o.vmm);
        vmm_span = o.vmm_span;
        vmm_piece = o.vmm_piece;
        vmm_mapped = o.vmm_mapped;
        o.p = nullptr;
        o.n = 0;
        o.view = false;
        o.vmm.clear();
        o.vmm_span = 0;
        o.vmm_piece = 0;
        o.vmm_mapped = 0;
    }
    return *this;
}

void
DevBuf::set_view(uint8_t* q, size_t bytes)
{
    release();
    p = q;
    n = bytes;
    view = true;
}

void
DevBuf::alloc(size_t bytes, unsigned flags)
{
    if (p && !view && n >= bytes)
        return;
    release();
    if (bytes == 0)
        return;
    void* q = nullptr;
    if (flags & kVmm) {
        int dev = 0;
        hip_check(hipGetDevice(&dev), "hipGetDevice");
        hipMemAllocationProp prop{};
        prop.type = hipMemAllocationTypePinned;
        prop.location.type = hipMemLocationTypeDevice;
        prop.location.id = dev;
        size_t gran = 0;
        hip_check(hipMemGetAllocationGranularity(&gran, &prop,
                                                 hipMemAllocationGranularityRecommended),
                  "hipMemGetAllocationGranularity");
        // bits 9-13 = v: pieces of 2^(16 + v) bytes (v <= 14: 64 KiB .. 1 GiB;
        // at least the granularity); 31: one piece of the whole size
        const unsigned v = (flags >> 9) & 31u;
        const size_t piece =
          v == 31u ? (bytes + gran - 1) / gran * gran
                   : std::max<size_t>(gran, size_t(1) << (16 + std::min(v, 14u)));
        const size_t span = (bytes + piece - 1) / piece * piece;
        size_t align = gran; // a power of two: the largest <= piece, <= 1 GiB
        while (align * 2 <= piece && align < (size_t(1) << 30))
            align *= 2;
        hip_check(hipMemAddressReserve(&q, span, align, nullptr, 0), "hipMemAddressReserve");
        // from here on release() undoes exactly what was done, also when a
        // create or map below throws
        p = static_cast<uint8_t*>(q);
        vmm_span = span;
        vmm_piece = piece;
        try {
            for (size_t off = 0; off < span; off += piece) {
                hipMemGenericAllocationHandle_t h{};
                hip_check(hipMemCreate(&h, piece, &prop, 0), "hipMemCreate");
                vmm.push_back(h);
                hip_check(hipMemMap(p + off, piece, 0, h, 0), "hipMemMap");
                ++vmm_mapped;
            }
            hipMemAccessDesc acc{};
            acc.location = prop.location;
            acc.flags = hipMemAccessFlagsProtReadWrite;
            hip_check(hipMemSetAccess(p, span, &acc, 1), "hipMemSetAccess");
        } catch (...) {
            release();
            throw;
        }
        n = bytes;
        return;
    }
    if (flags)
        hip_check(hipExtMallocWithFlags(&q, bytes, flags), "hipExtMallocWithFlags");
    else
        hip_check(hipMalloc(&q, bytes), "hipMalloc");
    p = static_cast<uint8_t*>(q);
    n = bytes;
}

PinnedBuf::~PinnedBuf()
{
    if (p)
        (void)hipHostFree(p);
}

void
PinnedBuf::alloc(size_t bytes)
{
    if (p && n >= bytes)
        return;
    if (p)
        (void)hipHostFree(p);
    p = nullptr;
    n = 0;
    if (bytes == 0)
        return;
    void* q = nullptr;
    hip_check(hipHostMalloc(&q, bytes, hipHostMallocDefault), "hipHostMalloc");
    p = static_cast<uint8_t*>(q);
    n = bytes;
}

// PCIe copies are issued in pieces: one large H2D and one large D2H on two
// streams do not overlap (measured 57 GB/s together, = either alone), while
// the same bytes in interleaved pieces run full duplex (86-96 GB/s).
static size_t
copy_piece_bytes()
{
    return size_t(32) << 20;
}

static void
memcpy_pieces(void* dst, const void* src, size_t n, hipMemcpyKind kind,
              hipStream_t stream)
{
    const size_t piece = copy_piece_bytes();
    for (size_t o = 0; o < n; o += piece)
        hip_check(hipMemcpyAsync(static_cast<uint8_t*>(dst) + o,
                                 static_cast<const uint8_t*>(src) + o,
                                 std::min(piece, n - o), kind, stream),
                  "hipMemcpyAsync");
}

// n chunks of bpc bytes, `pitch` apart in the source, packed into dst, in
// pieces of about copy_piece_bytes() (full-duplex PCIe, see memcpy_pieces)
static void
copy_chunks(void* dst, const uint8_t* src, uint64_t bpc, uint64_t pitch, uint32_t n,
            hipMemcpyKind kind, hipStream_t stream)
{
    if (pitch == bpc) {
        memcpy_pieces(dst, src, bpc * n, kind, stream);
        return;
    }
    const uint64_t per = std::max<uint64_t>(1, copy_piece_bytes() / bpc);
    for (uint64_t c = 0; c < n; c += per) {
        const uint64_t m = std::min<uint64_t>(per, n - c);
        if (m > 1)
            hip_check(hipMemcpy2DAsync(static_cast<uint8_t*>(dst) + c * bpc, bpc,
                                       src + c * pitch, pitch, bpc, m, kind, stream),
                      "hipMemcpy2DAsync");
        else // one chunk of at least a piece
            memcpy_pieces(static_cast<uint8_t*>(dst) + c * bpc, src + c * pitch, bpc,
                          kind, stream);
    }
}

// host threads for the pageable -> pinned staging copy (AQZ_COPY_THREADS, a
// deployment setting: it changes no output byte)
static unsigned
copy_workers()
{
    if (const char* s = std::getenv("AQZ_COPY_THREADS"))
        return unsigned(std::max(0, std::atoi(s)));
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return std::min(7u, hw / 2);
}

static hipMemcpyKind
kind_from(int src_mem, int dst_mem)
{
    if (src_mem == kMemDevice)
        return dst_mem == kMemDevice ? hipMemcpyDeviceToDevice
                                     : hipMemcpyDeviceToHost;
    return dst_mem == kMemDevice ? hipMemcpyHostToDevice : hipMemcpyHostToHost;
}

static bool
method_valid(int32_t m)
{
    return m >= 0 && m < 4;
}

// ===========================================================================
// Stage
// ===========================================================================
// page-locked host memory (hipHostMalloc / hipHostRegister)?
static bool
pinned_host(const void* p)
{
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// The HSA agents of HIP device `device` and of the host, for DMA-engine
// copies (hsa_amd_memory_async_copy).  false when either is not found.
static bool
find_hsa_agents(int device, hsa_agent_t* gpu, hsa_agent_t* cpu)
{
    hipDeviceProp_t prop{};
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || hsa_init() != HSA_STATUS_SUCCESS)
        return false;
    struct Find
    {
        uint32_t bdf, domain;
        hsa_agent_t gpu{ 0 }, cpu{ 0 };
    } f{ (uint32_t(prop.pciBusID) << 8) | (uint32_t(prop.pciDeviceID) << 3),
         uint32_t(prop.pciDomainID) };
    auto cb = [](hsa_agent_t a, void* data) -> hsa_status_t {
        auto* f = static_cast<Find*>(data);
        hsa_device_type_t t;
        if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS)
            return HSA_STATUS_SUCCESS;
        if (t == HSA_DEVICE_TYPE_CPU && !f->cpu.handle)
            f->cpu = a;
        if (t == HSA_DEVICE_TYPE_GPU) {
            uint32_t bdf = 0, dom = 0;
            hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_BDFID), &bdf);
            hsa_agent_get_info(a, hsa_agent_info_t(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
            if ((bdf & ~7u) == f->bdf && dom == f->domain)
                f->gpu = a;
        }
        return HSA_STATUS_SUCCESS;
    };
    if (hsa_iterate_agents(cb, &f) != HSA_STATUS_SUCCESS || !f.gpu.handle || !f.cpu.handle)
        return false;
    *gpu = f.gpu;
    *cpu = f.cpu;
    return true;
}

Stage::Stage(const ArrayDesc& desc, const StageOptions& opt)
  : desc_(desc)
  , opt_(opt)
{
    bpp_ = bytes_of_type(desc.dtype);
    if (desc.multiscale && !method_valid(desc.method))
        throw Error(1, "Invalid downsampling method");
    if (opt_.layer_slots == 0)
        opt_.layer_slots = 2;
    if (opt_.max_batch_frames == 0)
        opt_.max_batch_frames = 64;
    if (opt_.level0_on_host)
        opt_.skip_level0_split = true;

    auto base = std::make_unique<ArrayDimensions>(desc.dims, desc.dtype,
                                                  desc.storage_order);
    if (base->needs_xy_transposition()) {
        // Array::write_frame_to_chunks_ transposes the acquired frame
        // (array.cpp:525-533) and the downsampler sees the transposed frame
        // (multiscale.array.cpp:66-72): every level works in storage order
        if (opt_.level0_on_host)
            throw Error(9, "level0_split_on_host needs storage rows = acquisition rows "
                           "(no XY-transposed storage order)");
        xy_ = true;
        const size_t nd = desc.dims.size();
        acq_rows_ = desc.dims[nd - 2].array_size_px;
        acq_cols_ = desc.dims[nd - 1].array_size_px;
    }
    std::vector<std::vector<Dim>> levels;
    if (desc.multiscale)
        levels = make_pyramid_levels(base->dims(), desc.max_levels,
                                     opt_.force_levels);
    else
        levels = { base->dims() };

    hip_check(hipSetDevice(desc.device), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&own_stream_, hipStreamNonBlocking),
              "hipStreamCreate");
    stream_ = own_stream_;
    {
        const char* e = std::getenv("AQZ_NUMA");
        char bus[64] = { 0 };
        if (!(e && std::atoi(e) == 0) &&
            hipDeviceGetPCIBusId(bus, int(sizeof(bus)), desc.device) == hipSuccess)
            numa_cpus_ = numa_cpus_for_pci(bus, &numa_node_);
        (void)hipGetLastError();
    }

    const size_t n = base->ndims();
    const uint32_t B = opt_.max_batch_frames;
    DevBuf spacer;
    if (opt_.ring_spacer)
        spacer.alloc(opt_.ring_spacer, opt_.ring_malloc_flags);
    lv_.resize(levels.size());
    for (size_t k = 0; k < levels.size(); ++k) {
        StageLevel& L = lv_[k];
        L.dims = levels[k];
        if (k == 0)
            L.ad = std::move(base);
        else
            L.ad = std::make_unique<ArrayDimensions>(L.dims, desc.dtype);
        L.W = L.dims[n - 1].array_size_px;
        L.H = L.dims[n - 2].array_size_px;
        L.planes = L.dims[n - 3].array_size_px;
        if (k > 0)
            L.xy_shrinks = L.W < lv_[k - 1].W || L.H < lv_[k - 1].H;
        L.tw = L.dims[n - 1].chunk_size_px;
        L.th = L.dims[n - 2].chunk_size_px;
        L.ntx = parts_along(L.W, L.tw);
        L.nty = parts_along(L.H, L.th);
        L.bpc = L.ad->bytes_per_chunk();
        L.n_chunks = L.ad->number_of_chunks_in_memory();
        const uint64_t F = L.ad->frames_per_chunk_layer();
        if (F == 0 || F > 0x7fffffffull)
            throw Error(9, "unsupported frames per chunk layer");
        L.F = uint32_t(F);
        L.pitch = L.bpc + opt_.chunk_pad; // bench option: chunks staggered
        L.slot_bytes = L.pitch * L.n_chunks;
        L.layer_bytes = L.bpc * L.n_chunks;
        L.n_slots = std::max<uint32_t>(opt_.layer_slots,
                                       (B - 1 + L.F - 1) / L.F + 1);
        L.slot_layer.assign(L.n_slots, -1);

        // per-frame chunk addressing table (periodic in frames_per_layer)
        L.h_tab_off.resize(L.F);
        L.h_tab_grp.resize(L.F);
        for (uint32_t fl = 0; fl < L.F; ++fl) {
            const uint64_t sf = L.ad->transpose_frame_id(fl);
            const uint32_t grp = L.ad->tile_group_offset(sf);
            L.h_tab_grp[fl] = grp;
            L.h_tab_off[fl] = uint64_t(grp) * L.pitch + L.ad->chunk_internal_offset(sf);
        }
        const uint64_t P = uint64_t(L.n_slots) * L.F;
        if (P > 0x7fffffffull)
            throw Error(9, "chunk-layer ring period too large");
        L.period = uint32_t(P);
        if (!(k == 0 && opt_.skip_level0_split))
            arena_rings_ += (L.slot_bytes * L.n_slots + 0xffffull) & ~0xffffull;
        build_shard_order(L);
        L.tab_off.alloc(size_t(L.F) * 8);
        L.tab_grp.alloc(size_t(L.F) * 4);
        hip_check(hipMemcpy(L.tab_off.p, L.h_tab_off.data(), size_t(L.F) * 8,
                            hipMemcpyHostToDevice),
                  "hipMemcpy");
        hip_check(hipMemcpy(L.tab_grp.p, L.h_tab_grp.data(), size_t(L.F) * 4,
                            hipMemcpyHostToDevice),
                  "hipMemcpy");
    }

    // The chunk-layer rings.  Shipped: one arena holding every level's ring
    // back to back, mapped from 2 MiB virtual-memory pieces (hipMemCreate +
    // hipMemMap), when the rings reach 256 MiB.  The fused kernels ran in the
    // fast placement band on such memory in every configuration, box and
    // process tried, and in the slow one on hipMalloc'd rings, on pieces of
    // the rings' own sizes and on 1 GiB pieces (profiles/archive/r04_vmm_rings.txt;
    // DESIGN.md section 3).
    bool per_level = true;
    if (opt_.ring_arena || (opt_.ring_malloc_flags == 0 && arena_rings_ >= kArenaMinRings)) {
        try {
            arena_.alloc(arena_rings_ + opt_.ring_arena,
                         opt_.ring_malloc_flags ? opt_.ring_malloc_flags : kArenaFlags);
            set_ring_offset(0);
            per_level = false;
        } catch (const Error& e) {
            // out of memory is the caller's to see; a runtime without the
            // virtual-memory API gets the per-level rings (slower placement)
            if (e.status == 6 || opt_.ring_arena)
                throw;
            arena_ = DevBuf{};
            arena_fallback_ = true;
        }
    }
    if (per_level)
        for (size_t k = 0; k < lv_.size(); ++k)
            if (!(k == 0 && opt_.skip_level0_split))
                place_level(lv_[k]);
    spacer = DevBuf{}; // freed: only the rings' placement needed it

    // 2-D fast path: z never shrinks and XY shrinks at every level, so every
    // input frame emits exactly one frame per level (downsampler.cpp:358-399)
    fused_2d_ = true;
    for (size_t k = 1; k < lv_.size(); ++k)
        fused_2d_ &= !(lv_[k].planes < lv_[k - 1].planes) && lv_[k].xy_shrinks;
    n_fused_ = fused_2d_ ? std::min<uint32_t>(n_levels() - 1, kMaxFused) : 0;

    // 2x2x2 fast path: a regular z schedule (every z-halving level has an
    // even input plane count, so pairs are always (2j, 2j+1) of a stack and
    // never straddle stacks) and every level halving XY.
    if (!fused_2d_ && bpp_ <= 4 && n_levels() >= 2 &&
        n_levels() - 1 <= uint32_t(kMaxFused) && lv_[0].planes > 0) {
        bool ok = true;
        uint32_t nz = 0, zmask = 0;
        for (uint32_t k = 1; k < n_levels(); ++k) {
            ok &= lv_[k].xy_shrinks;
            if (lv_[k].planes < lv_[k - 1].planes) {
                ok &= lv_[k - 1].planes % 2 == 0 &&
                      lv_[k].planes * 2 == lv_[k - 1].planes;
                zmask |= 1u << k;
                ++nz;
            }
        }
        ok &= nz <= 3 && lv_[0].planes % (1u << nz) == 0;
        if (ok) {
            fused_3d_ = true;
            g3d_ = 1u << nz;
            zmask3d_ = zmask;
        }
    }
    // 64-row regions whenever LDS-cascaded levels (>= 3) exist: amortises
    // the per-region barriers of the cascade over 32 KiB of input
    {
        // 64-row regions amortise a region's fixed cost (tile setup, flag
        // flushes, the LDS cascade's barriers) over 32 KiB of input; the
        // fast path needs the region height to divide the chunk height.
        uint32_t tz = 0;
        while (tz < 6 && ((lv_[0].th >> tz) & 1u) == 0)
            ++tz;
        const uint32_t nf = fused_3d_ ? n_levels() - 1 : n_fused_;
        rh_log2_ = std::max<uint32_t>(std::max<uint32_t>(4, nf), tz);
        if (fused_3d_) {
            const uint32_t RW = uint32_t(512 / bpp_);
            fused_3d_ = lv_[0].W % RW == 0 && (lv_[0].H % (1u << rh_log2_)) == 0 &&
                        lv_[0].th % (1u << rh_log2_) == 0 &&
                        lv_[0].tw % uint32_t(16 / bpp_) == 0 &&
                        (1u << rh_log2_) <= uint32_t(kMaxRegionRows);
        }
    }
    // tuning (bench options only; the drop-in create leaves them at the
    // shipped values and no environment variable reaches them)
    knobs_ = opt_.knobs;
    xcd_rot_ = opt_.xcd_rot;
    nt_mode_ = opt_.nt_mode & 7u;
    if (const uint32_t v = opt_.region_rows_log2) {
        if (v >= std::max<uint32_t>(4, n_fused_) && (1u << v) <= uint32_t(kMaxRegionRows))
            rh_log2_ = v;
    }
    // XY-transposed storage order: the strip kernel reads the acquisition-
    // order frames itself (load_region_xy) when it takes the interior
    // regions (launch_interior's condition); otherwise transpose_frames
    // writes the storage-order frames first.  Knob 4096: always transpose.
    if (xy_ && fused_2d_) {
        const bool tail = n_levels() - 1 > n_fused_;
        xy_direct_ = bpp_ <= 4 && rh_log2_ == 6 && !(knobs_ & 128u) &&
                     (!tail || n_fused_ >= 5) && !(knobs_ & 4096u) &&
                     (uint64_t(acq_cols_) * bpp_) % 16 == 0;
    } else if (xy_ && fused_3d_) {
        // the 2x2x2 strip kernel reads acquisition-order planes itself
        // (launch_fused_pyramid_3d); batches that also need the generic
        // cascade take the transpose pass (run_batch)
        xy_direct_ = bpp_ <= 4 && rh_log2_ == 6 && n_levels() - 1 <= 4 &&
                     !(knobs_ & 256u) && !(knobs_ & 4096u) &&
                     (uint64_t(acq_cols_) * bpp_) % 16 == 0;
    }

    const Dim& d0 = lv_[0].dims[0];
    if (d0.array_size_px > 0) {
        max_frames_ = 1;
        for (size_t i = 0; i + 2 < n; ++i)
            max_frames_ *= lv_[0].dims[i].array_size_px;
    }
    // z-slab schedule: planes [begin, end) of every z stack
    if (opt_.z_slab_begin != 0 || opt_.z_slab_end != 0) {
        const uint64_t p0 = lv_[0].planes;
        const uint64_t b0 = opt_.z_slab_begin, e0 = opt_.z_slab_end;
        if (n < 4 || p0 == 0 || b0 >= e0 || e0 > p0)
            throw Error(1, "z slab needs a z dimension and 0 <= begin < end <= planes");
        if (opt_.first_frame % p0 != 0)
            throw Error(1, "with a z slab, first_frame must start a z stack");
        slab_len_ = e0 - b0;
        for (auto& L : lv_) {
            const uint64_t pk = L.planes;
            if ((b0 * pk) % p0 != 0 || (e0 * pk) % p0 != 0)
                throw Error(9, "z slab does not align with the z pyramid");
            slab_skip_.push_back(pk - (e0 - b0) * pk / p0);
        }
        opt_.first_frame += b0;
    }
    // z-slab sharding: this stage continues a stream at first_frame
    if (opt_.first_frame > 0) {
        const uint64_t p0 = std::max<uint32_t>(1, lv_[0].planes);
        for (auto& L : lv_) {
            const uint64_t pk = std::max<uint32_t>(1, L.planes);
            if ((opt_.first_frame * pk) % p0 != 0)
                throw Error(9, "first_frame does not align with the z pyramid");
            L.frames_written = opt_.first_frame * pk / p0;
            L.level_frame_count = uint32_t(L.frames_written);
        }
    }
    pend_.resize(lv_.size());
    for (int j = 0; j < 2; ++j) {
        hip_check(hipEventCreateWithFlags(&h2d_ev_[j], hipEventDisableTiming),
                  "hipEventCreate");
        hip_check(hipEventCreateWithFlags(&consume_ev_[j], hipEventDisableTiming),
                  "hipEventCreate");
    }
    // HIP runs its streams on at most GPU_MAX_HW_QUEUES hardware queues (4 by
    // default) per priority level; streams beyond that share a queue and then
    // run in submission order.  With the default stream, the compute and the
    // compression stream, the two PCIe streams made a fifth normal-priority
    // stream: compression waited for every queued D2H piece (e2e trace: 41 ->
    // 51 GB/s with 8 queues).  The PCIe streams take high priority, a queue
    // pool of their own; their work is DMA and small blits, so priority costs
    // the kernels nothing.
    {
        int least = 0, greatest = 0;
        hip_check(hipDeviceGetStreamPriorityRange(&least, &greatest),
                  "hipDeviceGetStreamPriorityRange");
        hip_check(hipStreamCreateWithPriority(&h2d_, hipStreamNonBlocking, greatest),
                  "hipStreamCreate");
        hip_check(hipStreamCreateWithPriority(&d2h_, hipStreamNonBlocking, greatest),
                  "hipStreamCreate");
        // compression streams: normal priority
        for (hipStream_t* cs : { &comp_, &comp_lo_ })
            hip_check(hipStreamCreateWithFlags(cs, hipStreamNonBlocking), "hipStreamCreate");
        // the smallest levels' layers (a few chunks: their codec kernels are
        // a handful of workgroups, pure latency) on a stream of the least
        // priority, whose hardware queue pool is not the normal one's, so
        // they run beside levels 0-2 instead of queueing behind them
        hip_check(hipStreamCreateWithPriority(&comp_lo2_, hipStreamNonBlocking, least),
                  "hipStreamCreate");
    }
    // AQZ_D2H_SDMA=1: the compressed frames' D2H on a DMA engine, with the
    // HSA agents of this device (matched by PCI location) and of the host
    if (const char* e = std::getenv("AQZ_D2H_SDMA"); e && std::atoi(e) != 0)
        sdma_d2h_ = find_hsa_agents(desc.device, &hsa_gpu_, &hsa_cpu_);
    for (auto& L : lv_) {
        hip_check(hipEventCreateWithFlags(&L.ops_ev, hipEventDisableTiming),
                  "hipEventCreate");
        if (!L.ring.p)
            continue;
        L.ready_ev.assign(L.n_slots, nullptr);
        L.copy_ev.assign(L.n_slots, nullptr);
        L.copy_pending.assign(L.n_slots, 0);
        for (uint32_t s = 0; s < L.n_slots; ++s) {
            hip_check(hipEventCreateWithFlags(&L.ready_ev[s], hipEventDisableTiming),
                      "hipEventCreate");
            hip_check(hipEventCreateWithFlags(&L.copy_ev[s], hipEventDisableTiming),
                      "hipEventCreate");
        }
        L.flag_bytes.alloc(size_t(L.n_slots) * L.n_chunks);
    }

    calibrate_placement();
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

// The chunk-layer ring of a level, its has_data words and its frame table.
// Zeroed: chunk padding (ragged tiles / intermediate dims, the reference's
// zero-initialised Chunk, chunk.cpp:8-15) is never written by any frame, so
// it stays zero for every layer that later occupies a slot; has_data words
// start at 0 (no tag).
void
Stage::place_level(StageLevel& L, uint8_t* at)
{
    if (at)
        L.ring.set_view(at, L.slot_bytes * L.n_slots);
    else
        L.ring.alloc(L.slot_bytes * L.n_slots, opt_.ring_malloc_flags & ~kRingsPlain);
    L.flags.alloc(size_t(L.n_chunks) * L.n_slots * 4);
    hip_check(hipMemsetAsync(L.ring.p, 0, L.ring.n, stream_), "hipMemsetAsync");
    hip_check(hipMemsetAsync(L.flags.p, 0, L.flags.n, stream_), "hipMemsetAsync");
    // frame -> (tiles, has_data) over one ring period
    std::vector<FrameRef> tab(L.period);
    for (uint64_t fid = 0; fid < L.period; ++fid) {
        const uint64_t slot = fid / L.F;
        tab[fid].tiles = L.ring.p + slot * L.slot_bytes + L.h_tab_off[fid % L.F];
        tab[fid].flags = reinterpret_cast<uint32_t*>(L.flags.p) + slot * L.n_chunks +
                         L.h_tab_grp[fid % L.F];
    }
    L.ref_table.alloc(size_t(L.period) * sizeof(FrameRef));
    hip_check(hipMemcpy(L.ref_table.p, tab.data(), size_t(L.period) * sizeof(FrameRef),
                        hipMemcpyHostToDevice),
              "hipMemcpy");
}

// Placement search (StageOptions::placement_tries > 1; the bench and the
// drop-in binding pass it).  The fused kernels' launch time depends on the
// physical memory the chunk-layer rings land in: on
// hipMalloc'd rings C2 runs 0.88-0.90 ms per 256-frame launch on every box,
// on the shipped arena of 2 MiB pieces 0.76-0.81 ms on most boxes and about
// 0.84-0.89 ms on a few.  The effect is not observable from user space, so
// it is timed, not predicted:
//   * candidate 0 is the rings as created; each candidate is timed on random
//     frames over `reps` launches after 2 warm-ups;
//   * the expectation is the timing launch's algorithmic bytes at the rate
//     of the copy-third probe (the stage's 1 : 4/3 bus shape, nontemporal)
//     streaming the same random frames into the candidate's own memory --
//     plain streaming does not see the placement bands (r04_probe_pieces);
//   * while the best candidate is more than kPlacementTolerance over it,
//     a fresh ring set of the same kind (a new arena of 2 MiB pieces, or new
//     per-level allocations) is made while the best is held, timed, and the
//     loser freed at once.
// Peak: two ring sets + the random frames (aqz_stage_estimate_memory).
// The kept placement is re-timed alone at the end (kept_ms_final).  Only
// for rings >= 256 MiB on the fused paths.
void
Stage::calibrate_placement()
{
    const uint32_t tries = opt_.placement_tries;
    const uint32_t reps = std::max<uint32_t>(1, opt_.placement_reps);
    uint64_t ring_bytes = 0, set_bytes = 0;
    std::vector<bool> has_ring(lv_.size());
    for (size_t k = 0; k < lv_.size(); ++k) {
        has_ring[k] = lv_[k].ring.p != nullptr;
        ring_bytes += lv_[k].ring.n;
        set_bytes += lv_[k].ring.n + lv_[k].flags.n + lv_[k].ref_table.n;
    }
    uint32_t n = opt_.max_batch_frames;
    if (fused_3d_ && !fused_2d_)
        n = n / g3d_ * g3d_;
    // XY stages search too when the strip kernels read acquisition order
    // themselves; with the separate transpose pass they keep the first
    if (tries <= 1 || n == 0 || !(fused_2d_ || fused_3d_) || (xy_ && !xy_direct_) ||
        ring_bytes < (uint64_t(256) << 20))
        return;
    const bool arena = arena_.p != nullptr;
    if (arena) // the rings are views: a ring set costs the whole arena
        set_bytes = set_bytes - ring_bytes + arena_.physical();
    const uint64_t fb0 = uint64_t(lv_[0].W) * lv_[0].H * bpp_;
    // the random source in the same kind of memory as the rings, so the
    // timing is the rings' placement and not the scratch source's
    DevBuf src;
    alloc_large(src, size_t(n) * fb0, arena);
    hip_check(hipMemsetAsync(src.p, 0, src.n, stream_), "hipMemsetAsync");
    hip_check(launch_fill_random(src.p, src.n, 0x5eedull, stream_), "fill launch");
    uint64_t live = memory_usage().device + src.n;
    uint64_t peak = live;
    hipEvent_t a = nullptr, b = nullptr;
    hip_check(hipEventCreate(&a), "hipEventCreate");
    hip_check(hipEventCreate(&b), "hipEventCreate");
    std::vector<uint64_t> fw0, lfc0;
    for (const auto& L : lv_) {
        fw0.push_back(L.frames_written);
        lfc0.push_back(L.level_frame_count);
    }
    constexpr uint32_t kWarm = 2;
    std::vector<uint64_t> emitted(lv_.size(), 0);
    auto restore = [&]() {
        for (size_t k = 0; k < lv_.size(); ++k) {
            lv_[k].frames_written = fw0[k];
            lv_[k].level_frame_count = uint32_t(lfc0[k]);
            lv_[k].slot_layer.assign(lv_[k].n_slots, -1);
        }
    };
    auto elapsed = [&]() {
        hip_check(hipEventSynchronize(b), "hipEventSynchronize");
        float ms = 0;
        hip_check(hipEventElapsedTime(&ms, a, b), "hipEventElapsedTime");
        return double(ms);
    };
    auto measure = [&]() {
        for (uint32_t w = 0; w < kWarm; ++w)
            run_batch(src.p, n);
        hip_check(hipEventRecord(a, stream_), "hipEventRecord");
        for (uint32_t r = 0; r < reps; ++r)
            run_batch(src.p, n);
        hip_check(hipEventRecord(b, stream_), "hipEventRecord");
        const double ms = elapsed() / reps;
        for (size_t k = 0; k < lv_.size(); ++k)
            emitted[k] = (lv_[k].frames_written - fw0[k]) / (kWarm + reps);
        restore();
        return ms;
    };
    // The copy-third probe over the random frames into the candidate's
    // memory (the arena, or the largest ring): every variant, best of 3
    // groups of 4 launches each; the best variant's bus GB/s.  A stage
    // without the level-0 split (1 read : 1/3 write) takes the read-third
    // probe, its own shape.
    const bool third_only = opt_.skip_level0_split;
    const double bus_per_read = third_only ? 4.0 / 3.0 : 7.0 / 3.0;
    auto probe = [&]() {
        DevBuf* dst = &arena_;
        if (!arena)
            for (auto& L : lv_)
                if (L.ring.n > dst->n)
                    dst = &L.ring;
        const uint64_t rd = probe_copy_third_read_bytes(src.n, dst->n);
        if (rd < (uint64_t(64) << 20))
            return 0.0;
        double best = 0;
        for (int v = 0; v < kPlacementProbeVariants; ++v) {
            hip_check(launch_probe_copy_third(src.p, dst->p, rd, stream_, v, third_only),
                      "probe launch");
            for (int g = 0; g < 3; ++g) {
                hip_check(hipEventRecord(a, stream_), "hipEventRecord");
                for (int r = 0; r < 4; ++r)
                    hip_check(launch_probe_copy_third(src.p, dst->p, rd, stream_, v, third_only),
                              "probe launch");
                hip_check(hipEventRecord(b, stream_), "hipEventRecord");
                const double ms = elapsed() / 4;
                if (ms > 0 && (best == 0 || ms < best))
                    best = ms;
            }
        }
        return best > 0 ? double(rd) * bus_per_read / (best * 1e-3) / 1e9 : 0.0;
    };
    struct Placement
    {
        DevBuf arena;
        std::vector<DevBuf> ring, flags, ref;
    };
    auto take = [&]() {
        Placement pl;
        pl.arena = std::move(arena_);
        for (auto& L : lv_) {
            pl.ring.push_back(std::move(L.ring));
            pl.flags.push_back(std::move(L.flags));
            pl.ref.push_back(std::move(L.ref_table));
        }
        return pl;
    };
    auto fresh = [&]() {
        if (arena) {
            // the same kind of memory as candidate 0 (the constructor's flags)
            arena_.alloc(arena_rings_ + opt_.ring_arena,
                         opt_.ring_malloc_flags ? opt_.ring_malloc_flags : kArenaFlags);
            place_rings_at(0);
        } else {
            for (size_t k = 0; k < lv_.size(); ++k)
                if (has_ring[k])
                    place_level(lv_[k]);
        }
    };
    PlacementReport rep;
    rep.reps = reps;
    rep.mode = arena ? 3u : 4u;
    Placement best;
    double best_ms = 0;
    try {
        for (uint32_t t = 0; t < tries; ++t) {
            if (t > 0) {
                fresh(); // the best so far is held: this set is other memory
                live += set_bytes;
                peak = std::max(peak, live);
            }
            const double ms = measure();
            rep.ms.push_back(ms);
            rep.probe_gbs.push_back(probe());
            if (t == 0) {
                for (size_t k = 0; k < lv_.size(); ++k)
                    rep.alg_bytes += emitted[k] * uint64_t(lv_[k].W) * lv_[k].H * bpp_ *
                                     (k == 0 ? (opt_.skip_level0_split ? 1 : 2) : 1);
                rep.probe_bus_gbs = rep.probe_gbs[0];
                if (rep.probe_bus_gbs > 0)
                    rep.expected_ms = double(rep.alg_bytes) / (rep.probe_bus_gbs * 1e9) * 1e3;
            }
            const bool better = t == 0 || ms < best_ms;
            Placement cur = take();
            if (better) {
                if (t > 0)
                    live -= set_bytes; // the old best, freed now
                best = std::move(cur);
                best_ms = ms;
                rep.kept = t;
            } else {
                cur = Placement{};
                live -= set_bytes;
            }
            rep.accepted = rep.expected_ms > 0 && !opt_.placement_never_accept &&
                           best_ms <= (1.0 + kPlacementTolerance) * rep.expected_ms;
            rep.stop = rep.accepted ? 1u
                       : (rep.expected_ms == 0 && !opt_.placement_never_accept) ? 3u
                                                                               : 2u;
            if (rep.accepted || t + 1 == tries ||
                (rep.expected_ms == 0 && !opt_.placement_never_accept))
                break;
        }
    } catch (const Error& e) {
        if (e.status != 6 || rep.ms.empty()) // out of memory: keep the best so far
            throw;
        (void)hipGetLastError();
        rep.stop = 4;
    }
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    {
        Placement cur = take(); // a candidate placed but not measured (OOM)
    }
    arena_ = std::move(best.arena);
    for (size_t k = 0; k < lv_.size(); ++k) {
        lv_[k].ring = std::move(best.ring[k]);
        lv_[k].flags = std::move(best.flags[k]);
        lv_[k].ref_table = std::move(best.ref[k]);
    }
    rep.kept_ms_final = measure();
    rep.peak_device = peak;
    placement_ = rep;
    // the calibration wrote frames and has_data tags: back to zero
    for (auto& L : lv_) {
        if (!L.ring.p)
            continue;
        hip_check(hipMemsetAsync(L.ring.p, 0, L.ring.n, stream_), "hipMemsetAsync");
        hip_check(hipMemsetAsync(L.flags.p, 0, L.flags.n, stream_), "hipMemsetAsync");
    }
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

void
Stage::grant_access(int device)
{
    if (!arena_.p || !arena_.vmm_span)
        return; // hipMalloc'd memory: peer access covers it
    std::lock_guard<std::mutex> lk(access_mu_);
    if (std::find(granted_.begin(), granted_.end(), device) != granted_.end())
        return;
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = device;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    hip_check(hipMemSetAccess(arena_.p, arena_.vmm_span, &acc, 1), "hipMemSetAccess");
    granted_.push_back(device);
}

// every level's ring (has_data words, frame table) placed in the arena at
// offset, levels back to back, each 64 KiB aligned
void
Stage::place_rings_at(uint64_t offset)
{
    uint64_t at = offset;
    for (size_t k = 0; k < lv_.size(); ++k) {
        StageLevel& L = lv_[k];
        if (!(k == 0 && opt_.skip_level0_split)) {
            place_level(L, arena_.p + at);
            at += (L.slot_bytes * L.n_slots + 0xffffull) & ~0xffffull;
        }
    }
}

void
Stage::set_ring_offset(uint64_t offset)
{
    if (!arena_.p)
        throw Error(1, "the stage has no ring arena (bench option ring_arena_bytes)");
    if (offset % 256 || offset + arena_rings_ > arena_.n)
        throw Error(1, "ring offset outside the arena's slack (or not 256-B aligned)");
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    place_rings_at(offset);
    for (auto& L : lv_) {
        L.frames_written = 0;
        L.level_frame_count = 0;
        L.slot_layer.assign(L.n_slots, -1);
    }
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

void
Stage::replace_rings(uint32_t mask)
{
    synchronize();
    for (size_t k = 0; k < lv_.size() && k < 32; ++k) {
        StageLevel& L = lv_[k];
        if (!((mask >> k) & 1u) || !L.ring.p)
            continue;
        held_.push_back(std::move(L.ring));
        held_.push_back(std::move(L.flags));
        held_.push_back(std::move(L.ref_table));
        place_level(L);
    }
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

Stage::~Stage()
{
    // host compression jobs read pinned inputs and wait on events: finish
    // them before anything is freed (the pool drains its queue)
    zpool_.reset();
    // other stages' imports still reading this stage's rings
    for (auto& L : lv_)
        for (auto& v : L.peer_ev)
            for (const auto& e : v)
                (void)hipEventSynchronize(e.get());
    if (stream_)
        (void)hipStreamSynchronize(stream_);
    for (hipStream_t s : { h2d_, comp_, comp_lo_, comp_lo2_, d2h_ })
        if (s) {
            (void)hipStreamSynchronize(s);
            (void)hipStreamDestroy(s);
        }
    for (int j = 0; j < 2; ++j)
        for (hipEvent_t e : { h2d_ev_[j], consume_ev_[j] })
            if (e)
                (void)hipEventDestroy(e);
    for (size_t i = inflight_head_; i < inflight_.size(); ++i)
        if (inflight_[i].first)
            free_ev_.push_back(inflight_[i].first);
    for (const Ticket& t : tickets_) {
        if (t.ev)
            free_ev_.push_back(t.ev);
        if (t.sig.handle) {
            // a DMA-engine copy still in flight must land before its
            // buffers go
            while (hsa_signal_wait_scacquire(t.sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                             HSA_WAIT_STATE_BLOCKED) > 0) {
            }
            free_sig_.push_back(t.sig);
        }
    }
    for (hipEvent_t e : free_ev_)
        (void)hipEventDestroy(e);
    for (hsa_signal_t g : free_sig_)
        (void)hsa_signal_destroy(g);
    for (auto& L : lv_) {
        if (L.ops_ev)
            (void)hipEventDestroy(L.ops_ev);
        for (hipEvent_t e : L.ready_ev)
            if (e)
                (void)hipEventDestroy(e);
        for (hipEvent_t e : L.copy_ev)
            if (e)
                (void)hipEventDestroy(e);
        for (hipEvent_t e : L.comp_ev)
            if (e)
                (void)hipEventDestroy(e);
        for (hipEvent_t e : L.cdone_ev)
            if (e)
                (void)hipEventDestroy(e);
        for (hipEvent_t e : L.zin_ev)
            if (e)
                (void)hipEventDestroy(e);
    }

    for (auto& pr : ev_pairs_) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    for (hipEvent_t e : mark_ev_)
        if (e)
            (void)hipEventDestroy(e);
    if (ext_ev_)
        (void)hipEventDestroy(ext_ev_);
    if (own_stream_)
        (void)hipStreamDestroy(own_stream_);
}

const std::vector<Dim>&
Stage::level_dims(uint32_t level) const
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    return lv_[level].dims;
}

LevelLayout
Stage::layout(uint32_t level) const
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    const StageLevel& L = lv_[level];
    return LevelLayout{ L.bpc,   L.n_chunks,
                        L.n_slots, L.F,
                        uint64_t(L.W) * L.H * bpp_, L.W,
                        L.H,     L.pitch };
}

void
Stage::set_stream(hipStream_t s)
{
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    stream_ = s ? s : own_stream_;
}

uint64_t
Stage::frames_written(uint32_t level) const
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    return lv_[level].frames_written;
}

void
Stage::synchronize()
{
    hip_check(hipStreamSynchronize(h2d_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(comp_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(comp_lo_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(comp_lo2_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(d2h_), "hipStreamSynchronize");
    retire_consumed(true);
}

void
Stage::note_consumed(hipStream_t s, uint64_t frames)
{
    appended_ += frames;
    if (!s) {
        // consumed already; later events cannot fire before earlier ones do
        if (inflight_head_ == inflight_.size())
            consumed_ = appended_;
        else
            inflight_.emplace_back(nullptr, appended_);
        return;
    }
    hipEvent_t e;
    if (free_ev_.empty()) {
        hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    } else {
        e = free_ev_.back();
        free_ev_.pop_back();
    }
    hip_check(hipEventRecord(e, s), "hipEventRecord");
    inflight_.emplace_back(e, appended_);
    retire_consumed(false);
}

void
Stage::retire_consumed(bool wait)
{
    while (inflight_head_ < inflight_.size()) {
        auto& [e, n] = inflight_[inflight_head_];
        if (e) {
            if (wait) {
                hip_check(hipEventSynchronize(e), "hipEventSynchronize");
            } else {
                const hipError_t q = hipEventQuery(e);
                if (q == hipErrorNotReady)
                    break;
                hip_check(q, "hipEventQuery");
            }
            free_ev_.push_back(e);
        }
        consumed_ = n;
        ++inflight_head_;
    }
    if (inflight_head_ == inflight_.size()) {
        inflight_.clear();
        inflight_head_ = 0;
    }
}

uint64_t
Stage::frames_consumed()
{
    retire_consumed(false);
    return consumed_;
}

// Blocks on the consumption events (no spin) until `frames` level-0 frames
// of the appended sources have been read.
void
Stage::wait_consumed(uint64_t frames)
{
    if (frames > appended_)
        throw Error(1, "wait_consumed beyond the frames appended");
    while (consumed_ < frames && inflight_head_ < inflight_.size()) {
        auto& [e, n] = inflight_[inflight_head_];
        if (e) {
            hip_check(hipEventSynchronize(e), "hipEventSynchronize");
            free_ev_.push_back(e);
        }
        consumed_ = n;
        ++inflight_head_;
    }
    retire_consumed(false);
}

// Hand-off tickets: every copy_*_async call records one event on the
// hand-off stream after its copies; ticket i (1-based, issue order) is
// complete once that event is.  The D2H stream is in order, so tickets
// complete in order.
uint64_t
Stage::issue_ticket()
{
    hipEvent_t e;
    if (free_ev_.empty()) {
        hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    } else {
        e = free_ev_.back();
        free_ev_.pop_back();
    }
    hip_check(hipEventRecord(e, d2h_), "hipEventRecord");
    tickets_.push_back(Ticket{ e, hsa_signal_t{ 0 } });
    ++tickets_issued_;
    // retire what has landed, so a caller that never asks does not hold one
    // live event per copy for the stage's lifetime
    (void)copies_completed();
    return tickets_issued_;
}

// a DMA-engine copy's ticket: complete when its signal reaches 0
uint64_t
Stage::issue_ticket(hsa_signal_t sig)
{
    tickets_.push_back(Ticket{ nullptr, sig });
    ++tickets_issued_;
    (void)copies_completed();
    return tickets_issued_;
}

uint64_t
Stage::copies_completed(bool wait_all, uint64_t until)
{
    while (!tickets_.empty() && tickets_done_ < tickets_issued_) {
        const Ticket t = tickets_.front();
        const bool wait = wait_all || tickets_done_ < until;
        if (t.sig.handle) {
            if (wait) {
                while (hsa_signal_wait_scacquire(t.sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                                 HSA_WAIT_STATE_BLOCKED) > 0) {
                }
            } else if (hsa_signal_load_scacquire(t.sig) > 0) {
                break;
            }
            free_sig_.push_back(t.sig);
        } else {
            if (wait) {
                hip_check(hipEventSynchronize(t.ev), "hipEventSynchronize");
            } else {
                const hipError_t q = hipEventQuery(t.ev);
                if (q == hipErrorNotReady)
                    break;
                hip_check(q, "hipEventQuery");
            }
            free_ev_.push_back(t.ev);
        }
        tickets_.pop_front();
        ++tickets_done_;
    }
    return tickets_done_;
}

void
Stage::wait_copies()
{
    hip_check(hipStreamSynchronize(comp_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(comp_lo_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(comp_lo2_), "hipStreamSynchronize");
    hip_check(hipStreamSynchronize(d2h_), "hipStreamSynchronize");
    (void)copies_completed(true); // every ticket has landed
}

void
Stage::append(const void* frames, uint64_t n_frames, int mem)
{
    if (n_frames == 0)
        return;
    if (!frames)
        throw Error(1, "null frames");
    finalized_ = false;
    const uint64_t fbytes = uint64_t(lv_[0].W) * lv_[0].H * bpp_;
    uint64_t n_ok = n_frames;
    if (max_frames_ > 0) {
        uint64_t room = max_frames_ - std::min(max_frames_, lv_[0].frames_written);
        if (slab_len_) {
            // frame ids jump over the other slabs' planes: count room in this
            // stage's own frames, (z stacks left) * slab - frames of this slab
            const uint64_t p0 = lv_[0].planes;
            const uint64_t stack = lv_[0].frames_written / p0;
            const uint64_t stacks = max_frames_ / p0;
            room = stack < stacks ? (stacks - stack) * slab_len_ - slab_done_ : 0;
        }
        n_ok = std::min(n_ok, room);
    }
    const auto* src = static_cast<const uint8_t*>(frames);
    const uint32_t B = opt_.max_batch_frames;
    for (uint64_t done = 0; done < n_ok;) {
        uint32_t b = uint32_t(std::min<uint64_t>(B, n_ok - done));
        if (slab_len_) // a batch never straddles two slabs
            b = uint32_t(std::min<uint64_t>(b, slab_len_ - slab_done_));
        const uint8_t* p = src + done * fbytes;
        if (mem == kMemDevice) {
            run_batch(p, b);
        } else {
            // Double buffer: batch i+1's host copy and H2D (on h2d_) overlap
            // batch i's kernels.  A pageable source is first copied into the
            // pinned staging buffer (the one copy ZarrStream_append makes,
            // frame.queue.cpp:37-39) and may be reused once append returns.
            // A pinned source is DMA'd directly and read asynchronously:
            // frames_consumed() says when its bytes may be overwritten.
            const int j = stage_idx_;
            stage_idx_ ^= 1;
            const size_t nbytes = size_t(b) * fbytes;
            alloc_large(d_stage_[j], size_t(B) * fbytes, opt_.codec.vmm);
            const uint8_t* hsrc = p;
            if (mem != kMemHostPinned) {
                h_stage_[j].alloc(size_t(B) * fbytes);
                hip_check(hipEventSynchronize(h2d_ev_[j]), "hipEventSynchronize");
                if (!pool_)
                    pool_ = std::make_unique<CopyPool>(copy_workers(), numa_cpus_);
                pool_->copy(h_stage_[j].p, p, nbytes);
                hsrc = h_stage_[j].p;
            }
            if (consume_rec_[j]) // kernels of the batch before last read d_stage_[j]
                hip_check(hipStreamWaitEvent(h2d_, consume_ev_[j], 0),
                          "hipStreamWaitEvent");
            memcpy_pieces(d_stage_[j].p, hsrc, nbytes, hipMemcpyHostToDevice, h2d_);
            hip_check(hipEventRecord(h2d_ev_[j], h2d_), "hipEventRecord");
            if (mem == kMemHostPinned)
                note_consumed(h2d_, b);
            hip_check(hipStreamWaitEvent(stream_, h2d_ev_[j], 0), "hipStreamWaitEvent");
            run_batch(d_stage_[j].p, b);
            hip_check(hipEventRecord(consume_ev_[j], stream_), "hipEventRecord");
            consume_rec_[j] = true;
        }
        if (mem == kMemDevice)
            note_consumed(stream_, b);
        else if (mem != kMemHostPinned)
            note_consumed(nullptr, b); // copied into staging before return
        done += b;
        if (slab_len_ && (slab_done_ += b) == slab_len_) {
            // next stack's slab: skip the planes other stages own
            for (size_t k = 0; k < lv_.size(); ++k) {
                lv_[k].frames_written += slab_skip_[k];
                lv_[k].level_frame_count += uint32_t(slab_skip_[k]);
            }
            slab_done_ = 0;
        }
    }
    if (n_ok < n_frames)
        throw Error(12, "append beyond the array's bounded extent");
}

void
Stage::run_batch(const uint8_t* dsrc, uint32_t n)
{
    // 2x2x2 pyramids: how many frames the fused kernel takes (whole z
    // groups, no carried partial plane), the rest go to the generic cascade
    uint32_t n3 = 0;
    if (!fused_2d_ && fused_3d_) {
        bool idle = lv_[0].frames_written % g3d_ == 0 &&
                    reinterpret_cast<uintptr_t>(dsrc) % 16 == 0;
        for (const auto& pd : pend_)
            idle &= !pd.has;
        if (idle)
            n3 = n / g3d_ * g3d_;
    }
    const bool direct = xy_direct_ && reinterpret_cast<uintptr_t>(dsrc) % 16 == 0 &&
                        (fused_2d_ || n3 == n);
    if (xy_ && !direct) {
        xbuf_.alloc(size_t(opt_.max_batch_frames) * acq_rows_ * acq_cols_ * bpp_);
        hip_check(launch_transpose_frames(dsrc, xbuf_.p, acq_rows_, acq_cols_, n,
                                          uint32_t(bpp_), stream_),
                  "transpose launch");
        dsrc = xbuf_.p;
        xy_src_ = false;
    } else {
        xy_src_ = xy_;
    }
    std::pair<hipEvent_t, hipEvent_t>* ev = nullptr;
    if (timing_) {
        if (ev_used_ == ev_pairs_.size()) {
            hipEvent_t a, b;
            hip_check(hipEventCreate(&a), "hipEventCreate");
            hip_check(hipEventCreate(&b), "hipEventCreate");
            ev_pairs_.emplace_back(a, b);
        }
        ev = &ev_pairs_[ev_used_++];
        hip_check(hipEventRecord(ev->first, stream_), "hipEventRecord");
    }
    if (fused_2d_) {
        run_fused(dsrc, n);
    } else {
        if (n3 > 0)
            run_fused3d(dsrc, n3);
        if (n3 < n)
            run_generic(dsrc + uint64_t(n3) * lv_[0].W * lv_[0].H * bpp_, n - n3);
    }
    if (ev)
        hip_check(hipEventRecord(ev->second, stream_), "hipEventRecord");
}

void
Stage::run_fused3d(const uint8_t* dsrc, uint32_t n)
{
    const uint32_t nl = n_levels();
    std::vector<uint32_t> nk(nl);
    for (uint32_t k = 0, z = 0; k < nl; ++k) {
        z += (zmask3d_ >> k) & 1u;
        nk[k] = n >> z;
        enter_layers(lv_[k], lv_[k].frames_written, nk[k]);
    }
    FusedParams p = fused_params(dsrc, n, nl - 1, rh_log2_, false);
    if (!p.fast_ok || p.nbx_in * p.nby_in != p.nbx * p.nby)
        throw Error(5, "2x2x2 fast path preconditions do not hold");
    p.G = g3d_;
    p.zmask = zmask3d_;
    hip_check(launch_fused_pyramid_3d(desc_.dtype, desc_.method, p, stream_),
              "fused_pyramid_3d launch");
    for (uint32_t k = 0; k < nl; ++k) {
        lv_[k].frames_written += nk[k];
        lv_[k].level_frame_count += nk[k];
    }
}

void
Stage::enter_layer(StageLevel& L, uint64_t layer)
{
    // A fresh layer needs no clearing: has_data words are generation-tagged
    // and the chunk padding was zeroed at allocation.  A hand-off copy still
    // reading the slot must finish before the slot is written again.
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (!L.copy_pending.empty() && L.copy_pending[slot]) {
        hip_check(hipStreamWaitEvent(stream_, L.copy_ev[slot], 0), "hipStreamWaitEvent");
        L.copy_pending[slot] = 0;
    }
    if (!L.peer_ev.empty()) {
        // another stage's import of the slot, on any device
        std::lock_guard<std::mutex> lk(access_mu_);
        for (const auto& e : L.peer_ev[slot])
            hip_check(hipStreamWaitEvent(stream_, e.get(), 0), "hipStreamWaitEvent");
        L.peer_ev[slot].clear();
    }
    L.slot_layer[slot] = int64_t(layer);
}

void
Stage::enter_layers(StageLevel& L, uint64_t first_fid, uint64_t n)
{
    if (n == 0 || !L.ring.p)
        return;
    for (uint64_t layer = first_fid / L.F; layer <= (first_fid + n - 1) / L.F;
         ++layer)
        enter_layer(L, layer);
}

LevelGeom
Stage::geom(StageLevel& L, uint64_t fid0, bool tiles, uint8_t* scratch) const
{
    LevelGeom g{};
    g.W = L.W;
    g.H = L.H;
    g.tw = L.tw;
    g.th = L.th;
    g.ntx = L.ntx;
    g.dtw = make_fastdiv(L.tw);
    g.dth = make_fastdiv(L.th);
    g.bpc = L.pitch;
    g.slot_bytes = L.slot_bytes;
    g.n_chunks = L.n_chunks;
    g.n_slots = L.n_slots;
    g.frames_per_layer = L.F;
    g.fid0_mod = uint32_t(fid0 % L.F);
    g.slot0 = uint32_t((fid0 / L.F) % L.n_slots);
    g.base = (tiles && L.ring.p) ? L.ring.p : nullptr;
    g.flags = reinterpret_cast<uint32_t*>(L.flags.p);
    g.tab_off = reinterpret_cast<const uint64_t*>(L.tab_off.p);
    g.tab_grp = reinterpret_cast<const uint32_t*>(L.tab_grp.p);
    g.scratch = scratch;
    return g;
}

void
Stage::tile_addr(const StageLevel& L, uint64_t fid, uint64_t* off,
                 uint32_t* flag_off, uint32_t* tag) const
{
    const uint64_t slot = (fid / L.F) % L.n_slots;
    *off = slot * L.slot_bytes + L.h_tab_off[fid % L.F];
    *flag_off = uint32_t(slot * L.n_chunks + L.h_tab_grp[fid % L.F]);
    if (tag)
        *tag = uint32_t(fid / L.period + 1);
}

FusedParams
Stage::fused_params(const uint8_t* dsrc, uint32_t n, uint32_t n_fused,
                    uint32_t rh_log2, bool tail)
{
    const StageLevel& L0 = lv_[0];
    FusedParams p{};
    p.src = dsrc;
    p.src_stride = uint64_t(L0.W) * L0.H * bpp_;
    p.xy = xy_src_ ? 1u : 0u;
    p.n_frames = n;
    p.n_fused = n_fused;
    p.rh_log2 = rh_log2;
    const uint32_t RW = uint32_t(512 / bpp_);
    p.nbx = parts_along(L0.W, RW);
    p.nby = parts_along(L0.H, 1u << rh_log2);
    // (xy: the acquisition rows, H[0] pixels, are the ones loaded as vectors)
    p.vec_rows = ((uint64_t(p.xy ? L0.H : L0.W) * bpp_) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dsrc) % 16 == 0)
                   ? 1
                   : 0;
    // (the interior kernel addresses a frame's tiles with 32-bit offsets)
    bool small_layers = true;
    for (uint32_t k = 0; k <= n_fused; ++k)
        small_layers = small_layers && lv_[k].slot_bytes < (uint64_t(1) << 32);
    p.fast_ok = (p.vec_rows && small_layers && L0.th % (1u << rh_log2) == 0 &&
                 L0.tw % uint32_t(16 / bpp_) == 0 && !(tail && n_fused <= 2))
                  ? 1
                  : 0;
    p.nt = nt_mode_;
    p.knobs = knobs_;
    p.nbx_in = p.fast_ok ? L0.W / RW : 0;
    p.nby_in = p.fast_ok ? L0.H >> rh_log2 : 0;
    // XCD-contiguous region order pays on large launches (A/B: C2 -4.5%,
    // C5 -3.5%, C3 even) and not on small ones (C1 +4%)
    p.xcd_order = (uint64_t(n) * p.nbx_in * p.nby_in >= 8192 && !(knobs_ & 64u)) ? 1 : 0;
    p.xcd_rot = (knobs_ >> 16) ? (knobs_ >> 16) : xcd_rot_; // knob bits 16-31: A/B
    p.xskew = (knobs_ & 2048u) ? 1u : 0u;                    // launcher sets the mask
    p.d_nreg_in = make_fastdiv(std::max<uint32_t>(1, p.nbx_in * p.nby_in));
    p.d_nbx_in = make_fastdiv(std::max<uint32_t>(1, p.nbx_in));
    p.tw = L0.tw;
    p.th = L0.th;
    p.dtw = make_fastdiv(L0.tw);
    p.dth = make_fastdiv(L0.th);
    p.bpc = L0.pitch;
    for (uint32_t k = 0; k <= n_fused; ++k) {
        StageLevel& L = lv_[k];
        if (L.pitch != p.bpc || L.tw != p.tw || L.th != p.th)
            throw Error(5, "chunk shape differs between levels");
        p.W[k] = L.W;
        p.H[k] = L.H;
        p.ntx[k] = L.ntx;
        if (L.ring.p) {
            if (n > L.period)
                throw Error(5, "batch longer than the ring period");
            p.lr[k].table = reinterpret_cast<const FrameRef*>(L.ref_table.p);
            p.lr[k].period = L.period;
            p.lr[k].r0 = uint32_t(L.frames_written % L.period);
            p.lr[k].tag0 = uint32_t(L.frames_written / L.period + 1);
        }
    }
    if (tail) {
        StageLevel& L = lv_[n_fused];
        L.scratch.alloc(size_t(opt_.max_batch_frames) * L.W * L.H * bpp_);
        p.scratch = L.scratch.p;
        p.scratch_level = n_fused;
    }
    return p;
}

void
Stage::run_fused(const uint8_t* dsrc, uint32_t n)
{
    const uint32_t nl = n_levels();
    const bool tail = nl - 1 > n_fused_;
    for (uint32_t k = 0; k < nl; ++k)
        enter_layers(lv_[k], lv_[k].frames_written, n);

    const FusedParams p = fused_params(dsrc, n, n_fused_, rh_log2_, tail);

    hip_check(launch_fused_pyramid(desc_.dtype, desc_.method, p, stream_),
              "fused_pyramid launch");

    // levels deeper than the fused depth: one generic step per level
    for (uint32_t k = n_fused_ + 1; k < nl; ++k) {
        StageLevel& L = lv_[k];
        StageLevel& P = lv_[k - 1];
        const bool more = k + 1 < nl;
        if (more)
            L.scratch.alloc(size_t(opt_.max_batch_frames) * L.W * L.H * bpp_);
        hip_check(hipEventSynchronize(L.ops_ev), "hipEventSynchronize");
        L.h_ops.alloc(size_t(opt_.max_batch_frames + 1) * sizeof(LevelOp));
        L.d_ops.alloc(size_t(opt_.max_batch_frames + 1) * sizeof(LevelOp));
        auto* ops = reinterpret_cast<LevelOp*>(L.h_ops.p);
        const uint64_t pfb = uint64_t(P.W) * P.H * bpp_;
        const uint64_t lfb = uint64_t(L.W) * L.H * bpp_;
        for (uint32_t f = 0; f < n; ++f) {
            LevelOp& o = ops[f];
            o = LevelOp{};
            o.a = P.scratch.p + f * pfb;
            o.a_scale = L.xy_shrinks ? 1 : 0;
            o.scratch_out = more ? L.scratch.p + f * lfb : nullptr;
            tile_addr(L, L.frames_written + f, &o.tile_off, &o.flag_off, &o.tag);
            o.has_tile = 1;
        }
        hip_check(hipMemcpyAsync(L.d_ops.p, ops, size_t(n) * sizeof(LevelOp),
                                 hipMemcpyHostToDevice, stream_),
                  "hipMemcpyAsync");
        hip_check(hipEventRecord(L.ops_ev, stream_), "hipEventRecord");
        LevelParams lp{};
        lp.Wp = P.W;
        lp.Hp = P.H;
        lp.g = geom(L, L.frames_written, true, nullptr);
        lp.ops = reinterpret_cast<const LevelOp*>(L.d_ops.p);
        lp.n_ops = n;
        hip_check(launch_level(desc_.dtype, desc_.method, lp, stream_),
                  "level launch");
    }
    for (uint32_t k = 0; k < nl; ++k) {
        lv_[k].frames_written += n;
        lv_[k].level_frame_count += n;
    }
}

const uint8_t*
Stage::frame_ptr(uint32_t level, uint32_t index, const uint8_t* dsrc) const
{
    const StageLevel& L = lv_[level];
    const uint64_t fb = uint64_t(L.W) * L.H * bpp_;
    if (level == 0)
        return dsrc + index * fb;
    return L.scratch.p + index * fb;
}

void
Stage::run_generic(const uint8_t* dsrc, uint32_t n)
{
    const uint32_t nl = n_levels();
    const size_t nd = lv_[0].dims.size();
    (void)nd;
    // level 0 tile split: the fused kernel with no pyramid levels
    if (!opt_.skip_level0_split) {
        enter_layers(lv_[0], lv_[0].frames_written, n);
        const FusedParams p = fused_params(dsrc, n, 0, 4, false);
        hip_check(launch_fused_pyramid(desc_.dtype, desc_.method, p, stream_),
                  "level-0 split launch");
    }
    lv_[0].frames_written += n;

    // Host simulation of the cascade (downsampler.cpp:306-401) -> ops/level.
    struct HostOp
    {
        int a_kind; // 0 frame of level k-1 in batch, 1 carried partial
        uint32_t a_index;
        bool a_scale;
        int has_b;
        uint32_t b_index;
        bool b_scale;
        int out; // 0 scratch slot, 1 partial store
        uint32_t out_index;
        uint64_t fid;
    };
    std::vector<std::vector<HostOp>> ops(nl);
    std::vector<uint32_t> nout(nl, 0);
    for (uint32_t i = 0; i < n; ++i) {
        ++lv_[0].level_frame_count;
        uint32_t cur = i; // index of the current frame at level k-1
        for (uint32_t k = 1; k < nl; ++k) {
            StageLevel& L = lv_[k];
            StageLevel& P = lv_[k - 1];
            bool average = L.planes < P.planes;
            if (P.planes % 2 != 0 && P.level_frame_count % P.planes == 0)
                average = false;
            const bool xy = L.xy_shrinks;
            Pending& pd = pend_[k];
            if (average) {
                if (pd.has) {
                    HostOp o{};
                    o.a_kind = pd.kind;
                    o.a_index = pd.index;
                    o.a_scale = pd.kind == 0 ? pd.scale : false;
                    o.has_b = 1;
                    o.b_index = cur;
                    o.b_scale = xy;
                    o.out = 0;
                    o.out_index = nout[k]++;
                    o.fid = L.frames_written++;
                    ops[k].push_back(o);
                    ++L.level_frame_count;
                    pd.has = false;
                    cur = o.out_index;
                } else {
                    pd.has = true;
                    pd.kind = 0;
                    pd.index = cur;
                    pd.scale = xy;
                    break;
                }
            } else {
                HostOp o{};
                o.a_kind = 0;
                o.a_index = cur;
                o.a_scale = xy;
                o.has_b = 0;
                o.out = 0;
                o.out_index = nout[k]++;
                o.fid = L.frames_written++;
                ops[k].push_back(o);
                ++L.level_frame_count;
                cur = o.out_index;
            }
        }
    }
    // an unpaired plane produced in this batch is carried in a partial buffer
    std::vector<int> store_into(nl, -1);
    for (uint32_t k = 1; k < nl; ++k) {
        Pending& pd = pend_[k];
        if (pd.has && pd.kind == 0) {
            const int dst = lv_[k].carried == 0 ? 1 : 0;
            HostOp o{};
            o.a_kind = 0;
            o.a_index = pd.index;
            o.a_scale = pd.scale;
            o.out = 1;
            o.out_index = uint32_t(dst);
            ops[k].push_back(o);
            store_into[k] = dst;
        }
    }

    // Execute level by level.
    for (uint32_t k = 1; k < nl; ++k) {
        StageLevel& L = lv_[k];
        StageLevel& P = lv_[k - 1];
        if (ops[k].empty())
            continue;
        const uint64_t lfb = uint64_t(L.W) * L.H * bpp_;
        const bool more = k + 1 < nl;
        if (more && nout[k] > 0)
            L.scratch.alloc(size_t(opt_.max_batch_frames) * lfb);
        if (store_into[k] >= 0)
            L.partial[store_into[k]].alloc(lfb);
        const size_t nops = ops[k].size();
        hip_check(hipEventSynchronize(L.ops_ev), "hipEventSynchronize");
        L.h_ops.alloc(size_t(opt_.max_batch_frames + 1) * sizeof(LevelOp));
        L.d_ops.alloc(size_t(opt_.max_batch_frames + 1) * sizeof(LevelOp));
        auto* dops = reinterpret_cast<LevelOp*>(L.h_ops.p);
        for (size_t j = 0; j < nops; ++j) {
            const HostOp& h = ops[k][j];
            LevelOp& o = dops[j];
            o = LevelOp{};
            o.a = h.a_kind == 0 ? frame_ptr(k - 1, h.a_index, dsrc)
                                : L.partial[L.carried].p;
            o.a_scale = h.a_scale ? 1 : 0;
            o.b = h.has_b ? frame_ptr(k - 1, h.b_index, dsrc) : nullptr;
            o.b_scale = h.b_scale ? 1 : 0;
            if (h.out == 0) {
                o.scratch_out = more ? L.scratch.p + h.out_index * lfb : nullptr;
                if (L.ring.p) {
                    enter_layer(L, h.fid / L.F);
                    tile_addr(L, h.fid, &o.tile_off, &o.flag_off, &o.tag);
                    o.has_tile = 1;
                }
            } else {
                o.scratch_out = L.partial[h.out_index].p;
            }
        }
        (void)P;
        hip_check(hipMemcpyAsync(L.d_ops.p, dops, nops * sizeof(LevelOp),
                                 hipMemcpyHostToDevice, stream_),
                  "hipMemcpyAsync");
        hip_check(hipEventRecord(L.ops_ev, stream_), "hipEventRecord");
        LevelParams lp{};
        lp.Wp = P.W;
        lp.Hp = P.H;
        lp.g = geom(L, 0, true, nullptr);
        lp.ops = reinterpret_cast<const LevelOp*>(L.d_ops.p);
        lp.n_ops = uint32_t(nops);
        hip_check(launch_level(desc_.dtype, desc_.method, lp, stream_),
                  "level launch");
    }
    for (uint32_t k = 1; k < nl; ++k) {
        if (store_into[k] >= 0) {
            lv_[k].carried = store_into[k];
            pend_[k].kind = 1;
        }
    }
}

void
Stage::copy_layer(uint32_t level, uint64_t layer, void* dst, size_t cap,
                  uint8_t* has_data, size_t has_data_cap, int mem)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    if (!L.ring.p)
        throw Error(1, "level 0 is not split on the device by this stage");
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (L.slot_layer[slot] != int64_t(layer))
        throw Error(3, "chunk layer not resident");
    if (dst && cap < L.layer_bytes)
        throw Error(2, "destination too small for a chunk layer");
    synchronize();
    if (dst) {
        copy_chunks(dst, L.ring.p + slot * L.slot_bytes, L.bpc, L.pitch, L.n_chunks,
                    kind_from(kMemDevice, mem), stream_);
        hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    }
    if (has_data) {
        if (has_data_cap < L.n_chunks)
            throw Error(2, "has_data too small");
        std::vector<uint32_t> f(L.n_chunks);
        hip_check(hipMemcpy(f.data(), L.flags.p + size_t(slot) * L.n_chunks * 4,
                            size_t(L.n_chunks) * 4, hipMemcpyDeviceToHost),
                  "hipMemcpy");
        const uint32_t tag = uint32_t(layer / L.n_slots + 1);
        for (uint32_t c = 0; c < L.n_chunks; ++c)
            has_data[c] = f[c] == tag ? 1 : 0;
    }
}

void
Stage::copy_layer_async(uint32_t level, uint64_t layer, void* dst, size_t cap,
                        uint8_t* has_data, size_t has_data_cap)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    if (!L.ring.p)
        throw Error(1, "level 0 is not split on the device by this stage");
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (L.slot_layer[slot] != int64_t(layer))
        throw Error(3, "chunk layer not resident");
    if (dst && cap < L.layer_bytes)
        throw Error(2, "destination too small for a chunk layer");
    if (has_data && has_data_cap < L.n_chunks)
        throw Error(2, "has_data too small");
    // after every kernel enqueued so far; the slot's next layer waits for it
    hip_check(hipEventRecord(L.ready_ev[slot], stream_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(d2h_, L.ready_ev[slot], 0), "hipStreamWaitEvent");
    if (dst)
        copy_chunks(dst, L.ring.p + slot * L.slot_bytes, L.bpc, L.pitch, L.n_chunks,
                    hipMemcpyDefault, d2h_);
    if (has_data) {
        uint8_t* fb = L.flag_bytes.p + size_t(slot) * L.n_chunks;
        hip_check(launch_flags_to_bytes(
                    reinterpret_cast<const uint32_t*>(L.flags.p) + size_t(slot) * L.n_chunks,
                    fb, L.n_chunks, uint32_t(layer / L.n_slots + 1), d2h_),
                  "flags launch");
        hip_check(hipMemcpyAsync(has_data, fb, L.n_chunks, hipMemcpyDefault, d2h_),
                  "hipMemcpyAsync");
    }
    hip_check(hipEventRecord(L.copy_ev[slot], d2h_), "hipEventRecord");
    L.copy_pending[slot] = 1;
    last_ticket_ = issue_ticket();
}

void
Stage::band_geometry(uint32_t level, int32_t* supported, uint32_t* n_bands,
                     uint64_t* frames_per_band, uint32_t* chunks_per_band) const
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    const ArrayDimensions& ad = *lv_[level].ad;
    const bool ok = ad.supports_dim1_banding();
    if (supported)
        *supported = ok ? 1 : 0;
    if (n_bands)
        *n_bands = ok ? ad.dim1_band_count() : 1;
    if (frames_per_band)
        *frames_per_band = ok ? ad.frames_per_dim1_band() : lv_[level].F;
    if (chunks_per_band)
        *chunks_per_band = ok ? ad.chunks_per_dim1_band() : lv_[level].n_chunks;
}

// Array::flush_completed_bands_ (array.cpp:873-908) hands band b of a layer
// -- the chunk slots [b*cpb, (b+1)*cpb), dim 1 being the slowest chunk index
// of a layer -- to compression once frames [b*fpb, (b+1)*fpb) of the layer
// are written.  Same ordering rules as copy_layer_async.
void
Stage::copy_band_async(uint32_t level, uint64_t layer, uint32_t band, void* dst,
                       size_t cap, uint8_t* has_data, size_t has_data_cap)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    if (!L.ring.p)
        throw Error(1, "level 0 is not split on the device by this stage");
    int32_t ok = 0;
    uint32_t nb = 1, cpb = L.n_chunks;
    uint64_t fpb = L.F;
    band_geometry(level, &ok, &nb, &fpb, &cpb);
    if (band >= nb)
        throw Error(3, "band out of range");
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (L.slot_layer[slot] != int64_t(layer))
        throw Error(3, "chunk layer not resident");
    // the trailing band of a ragged dim 1 is complete with its layer
    // (flush_layer_remainder_, array.cpp:863-871, 884-886)
    const uint64_t band_end = std::min<uint64_t>((uint64_t(band) + 1) * fpb, L.F);
    if (!finalized_ && L.frames_written < layer * L.F + band_end)
        throw Error(3, "band not complete");
    if (dst && cap < L.bpc * cpb)
        throw Error(2, "destination too small for a band");
    if (has_data && has_data_cap < cpb)
        throw Error(2, "has_data too small");
    const uint32_t c0 = band * cpb;
    hip_check(hipEventRecord(L.ready_ev[slot], stream_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(d2h_, L.ready_ev[slot], 0), "hipStreamWaitEvent");
    if (dst)
        copy_chunks(dst, L.ring.p + slot * L.slot_bytes + uint64_t(c0) * L.pitch, L.bpc,
                    L.pitch, cpb, hipMemcpyDefault, d2h_);
    if (has_data) {
        uint8_t* fb = L.flag_bytes.p + size_t(slot) * L.n_chunks + c0;
        hip_check(launch_flags_to_bytes(reinterpret_cast<const uint32_t*>(L.flags.p) +
                                          size_t(slot) * L.n_chunks + c0,
                                        fb, cpb, uint32_t(layer / L.n_slots + 1), d2h_),
                  "flags launch");
        hip_check(hipMemcpyAsync(has_data, fb, cpb, hipMemcpyDefault, d2h_),
                  "hipMemcpyAsync");
    }
    hip_check(hipEventRecord(L.copy_ev[slot], d2h_), "hipEventRecord");
    L.copy_pending[slot] = 1;
    last_ticket_ = issue_ticket();
}

void
Stage::wait_stream(hipStream_t s)
{
    if (!ext_ev_)
        hip_check(hipEventCreateWithFlags(&ext_ev_, hipEventDisableTiming),
                  "hipEventCreate");
    hip_check(hipEventRecord(ext_ev_, s), "hipEventRecord");
    hip_check(hipStreamWaitEvent(stream_, ext_ev_, 0), "hipStreamWaitEvent");
}

Footprint
Stage::memory_usage() const
{
    Footprint f;
    for (const StageLevel& L : lv_) {
        f.device += L.ring.n + L.flags.n + L.tab_off.n + L.tab_grp.n + L.ref_table.n +
                    L.scratch.n + L.partial[0].n + L.partial[1].n + L.d_ops.n +
                    L.flag_bytes.n + L.shard_order.n;
        f.pinned += L.h_ops.n;
        for (const DevBuf& b : L.cframes)
            f.device += b.n;
        for (const DevBuf& b : L.coffsets)
            f.device += b.n;
        for (const PinnedBuf& b : L.h_coffsets)
            f.pinned += b.n;
        for (const PinnedBuf& b : L.h_zin)
            f.pinned += b.n;
        for (const PinnedBuf& b : L.h_zhas)
            f.pinned += b.n;
        f.device += L.d_zshuf.n;
        if (L.comp)
            f.device += L.comp->device_bytes();
    }
    for (int j = 0; j < 2; ++j) {
        f.device += d_stage_[j].n;
        f.pinned += h_stage_[j].n;
    }
    f.device += xbuf_.n;
    if (arena_.p) { // the rings are views: the arena's pieces beyond them
        uint64_t views = 0;
        for (const StageLevel& L : lv_)
            views += L.ring.view ? L.ring.n : 0;
        f.device += arena_.physical() - std::min<uint64_t>(views, arena_.physical());
    }
    return f;
}

// The constructor's geometry without allocating: every buffer at the size
// the stage may grow it to (staging for a host source, per-level scratch and
// z partials for the generic cascade, the transposition buffer).
Footprint
Stage::estimate_memory(const ArrayDesc& desc, const StageOptions& opt_in)
{
    StageOptions opt = opt_in;
    if (opt.layer_slots == 0)
        opt.layer_slots = 2;
    if (opt.max_batch_frames == 0)
        opt.max_batch_frames = 64;
    const size_t bpp = bytes_of_type(desc.dtype);
    ArrayDimensions base(desc.dims, desc.dtype, desc.storage_order);
    const auto levels = desc.multiscale
                          ? make_pyramid_levels(base.dims(), desc.max_levels,
                                                opt.force_levels)
                          : std::vector<std::vector<Dim>>{ base.dims() };
    const size_t n = base.ndims();
    const uint64_t B = opt.max_batch_frames;
    Footprint f;
    uint64_t ring_bytes = 0, set_bytes = 0; // the placement search's unit
    uint64_t arena_rings = 0;               // the rings 64 KiB aligned
    for (size_t k = 0; k < levels.size(); ++k) {
        ArrayDimensions ad(levels[k], desc.dtype);
        const uint64_t W = levels[k][n - 1].array_size_px;
        const uint64_t H = levels[k][n - 2].array_size_px;
        const uint64_t bpc = ad.bytes_per_chunk();
        const uint64_t nc = ad.number_of_chunks_in_memory();
        const uint64_t F = std::max<uint64_t>(1, ad.frames_per_chunk_layer());
        const uint64_t slots = std::max<uint64_t>(opt.layer_slots, (B - 1 + F - 1) / F + 1);
        const uint64_t lfb = W * H * bpp;
        if (!(k == 0 && opt.skip_level0_split)) {
            const uint64_t ring = (bpc + opt.chunk_pad) * nc * slots;
            const uint64_t set = ring + nc * slots * 4 + slots * F * sizeof(FrameRef);
            f.device += set;        // ring, has_data words, frame table
            f.device += nc * slots; // has_data bytes
            ring_bytes += ring;
            set_bytes += set;
            arena_rings += (ring + 0xffffull) & ~0xffffull;
        }
        f.device += F * 12 + nc * 4; // tab_off + tab_grp, shard order
        if (k > 0) {
            f.device += B * lfb + 2 * lfb;                       // scratch, z partials
            f.device += (B + 1) * sizeof(LevelOp);               // d_ops
            f.pinned += (B + 1) * sizeof(LevelOp);               // h_ops
        }
    }
    const uint64_t fb0 = uint64_t(levels[0][n - 1].array_size_px) *
                         levels[0][n - 2].array_size_px * bpp;
    // the shipped ring arena: the rings 64 KiB aligned, rounded up to whole
    // pieces (2 MiB; an upper bound of 1 GiB for the bench's other pieces)
    const bool arena =
      opt.ring_arena || (opt.ring_malloc_flags == 0 && arena_rings >= kArenaMinRings);
    uint64_t arena_phys = 0;
    if (arena) {
        const uint64_t G = opt.ring_malloc_flags ? uint64_t(1) << 30 : uint64_t(2) << 20;
        arena_phys = (arena_rings + opt.ring_arena + G - 1) / G * G;
        f.device += arena_phys - ring_bytes;
    }
    // Two transients that never overlap: the creation-time placement search
    // (calibrate_placement: its random frames and a second ring set, freed
    // before the constructor returns), and what the first appends allocate
    // (H2D staging for host sources, the XY transposition buffer).  The
    // bound holds the larger.
    uint64_t steady = 2 * B * fb0; // H2D staging (host sources)
    f.pinned += 2 * B * fb0;       // pageable -> pinned staging
    if (base.needs_xy_transposition())
        steady += B * fb0;
    uint64_t creation = 0;
    if (opt.placement_tries > 1 && ring_bytes >= (uint64_t(256) << 20)) {
        const uint64_t src = arena && B * fb0 >= (uint64_t(64) << 20)
                               ? (B * fb0 + (uint64_t(2) << 20) - 1) >> 21 << 21
                               : B * fb0;
        creation = src + (arena ? set_bytes - ring_bytes + arena_phys : set_bytes);
    }
    f.device += std::max(steady, creation);
    return f;
}

void
Stage::device_layer(uint32_t level, uint64_t layer, void** chunks,
                    uint32_t** flags)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (!L.ring.p || L.slot_layer[slot] != int64_t(layer))
        throw Error(3, "chunk layer not resident");
    if (chunks)
        *chunks = L.ring.p + slot * L.slot_bytes;
    if (flags)
        *flags = reinterpret_cast<uint32_t*>(L.flags.p) + size_t(slot) * L.n_chunks;
}

// ---- shard packing ------------------------------------
uint32_t
crc32c(const uint8_t* p, size_t n)
{
    static const auto table = [] {
        std::vector<uint32_t> t(256);
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k)
                c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
            t[i] = c;
        }
        return t;
    }();
    uint32_t c = 0xFFFFFFFFu;
    for (size_t i = 0; i < n; ++i)
        c = table[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return c ^ 0xFFFFFFFFu;
}

void
shard_table(const uint64_t* offsets, const uint64_t* extents, uint32_t n, uint8_t* out)
{
    for (uint32_t i = 0; i < n; ++i)
        for (int b = 0; b < 8; ++b) {
            out[16 * i + b] = uint8_t(offsets[i] >> (8 * b));
            out[16 * i + 8 + b] = uint8_t(extents[i] >> (8 * b));
        }
    const uint32_t crc = crc32c(out, size_t(n) * 16);
    for (int b = 0; b < 4; ++b)
        out[size_t(n) * 16 + b] = uint8_t(crc >> (8 * b));
}

// Shard-major order of a level's chunks (Array::compress_and_flush_data_
// walks shards, array.cpp:777-803; Shard::write_chunk appends each chunk at
// the shard's running file offset, shard.cpp:55-112).  Without sharding
// (a shard size of 0) the order is the chunk order.
void
Stage::build_shard_order(StageLevel& L)
{
    const uint32_t n = L.n_chunks;
    L.h_order.resize(n);
    L.h_shard.assign(n, 0);
    L.h_internal0.assign(n, 0);
    for (uint32_t c = 0; c < n; ++c)
        L.h_order[c] = c;
    bool sharded = true;
    for (const Dim& d : L.ad->dims())
        sharded = sharded && d.shard_size_chunks > 0;
    if (sharded) {
        L.chunks_per_shard = L.ad->chunks_per_shard();
        L.n_shards = L.ad->number_of_shards();
        L.layers_per_shard = std::max<uint32_t>(1, L.ad->chunk_layers_per_shard());
        L.internal_stride = L.chunks_per_shard / L.layers_per_shard;
        for (uint32_t c = 0; c < n; ++c) {
            L.h_shard[c] = L.ad->shard_index_for_chunk(c);
            L.h_internal0[c] = L.ad->shard_internal_index(c);
        }
        std::stable_sort(L.h_order.begin(), L.h_order.end(), [&](uint32_t a, uint32_t b) {
            return L.h_shard[a] != L.h_shard[b] ? L.h_shard[a] < L.h_shard[b]
                                                : L.h_internal0[a] < L.h_internal0[b];
        });
    } else {
        L.chunks_per_shard = 1;
        L.n_shards = n;
        L.layers_per_shard = 1;
        L.internal_stride = 0;
        for (uint32_t c = 0; c < n; ++c)
            L.h_shard[c] = c;
    }
    L.shard_order.alloc(size_t(n) * 4);
    hip_check(hipMemcpy(L.shard_order.p, L.h_order.data(), size_t(n) * 4,
                        hipMemcpyHostToDevice),
              "hipMemcpy");
}

void
Stage::compressed_entries(uint32_t level, uint64_t layer, ChunkEntry* out, size_t n)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    const uint32_t slot = L.n_slots ? uint32_t(layer % L.n_slots) : 0;
    if (L.comp_layer.empty() || L.comp_layer[slot] != int64_t(layer))
        throw Error(3, "layer was not compressed (or its slot was reused)");
    if (n < L.n_chunks)
        throw Error(2, "entries too small");
    const uint64_t* off;
    if (L.comp_host[slot]) {
        HostLayerJob& j = *L.zjob[slot];
        j.wait();
        if (j.status)
            throw Error(j.status, "zstd compression failed");
        off = j.offsets.data();
    } else {
        hip_check(hipEventSynchronize(L.comp_ev[slot]), "hipEventSynchronize");
        off = reinterpret_cast<const uint64_t*>(L.h_coffsets[slot].p);
    }
    const uint32_t cl = uint32_t(layer % L.layers_per_shard);
    for (uint32_t i = 0; i < L.n_chunks; ++i) {
        const uint32_t c = L.h_order[i];
        out[i] = ChunkEntry{ c, L.h_shard[c], L.h_internal0[c] + cl * L.internal_stride, 0,
                             off[i], off[i + 1] - off[i] };
    }
}

void
Stage::shard_geometry(uint32_t level, uint32_t* chunks_per_shard, uint32_t* n_shards,
                      uint32_t* layers_per_shard) const
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    const StageLevel& L = lv_[level];
    if (chunks_per_shard)
        *chunks_per_shard = L.chunks_per_shard;
    if (n_shards)
        *n_shards = L.n_shards;
    if (layers_per_shard)
        *layers_per_shard = L.layers_per_shard;
}

// ---- device compression of resident layers ----------
Compressor::Compressor(uint64_t chunk_bytes, uint32_t typesize, const Compression& c,
                       const CodecTuning& tune)
  : c_(c)
  , tune_(tune)
  , nbytes_(chunk_bytes)
  , typesize_(typesize)
{
    if (c.codec < 1 || c.codec > 3)
        throw Error(4, "unknown codec");
    if (c.codec != 3 && (c.shuffle < 0 || c.shuffle > 2 || c.clevel < 0 || c.clevel > 9))
        throw Error(1, "invalid compression settings");
    // stock zstd: levels 0-22, no shuffle (validate_compression_settings,
    // zarr.stream.cpp:139-153)
    if (c.codec == 3 && (c.clevel < 0 || c.clevel > 22 || c.shuffle != 0))
        throw Error(1, "invalid zstd settings: level 0-22 and no shuffle");
    if (chunk_bytes == 0 || chunk_bytes > 0x7fffffefull || typesize == 0 ||
        typesize > 255)
        throw Error(1, "chunk size outside the blosc1 limits");
    if (c.codec == 1)
        g_ = make_blosc_geom(uint32_t(chunk_bytes), typesize, uint32_t(c.shuffle));
    store_only_ = c.codec != 3 && c.clevel == 0;
}

// Hash slices of the far-candidate pass for a compression setting (0: no
// far pass).  zstd level L (blosc clevel c is zstd level 2c - 1,
// zarr.common.cpp:117-126 -> c-blosc's zstd wrapper; plain zstd level 0 is
// libzstd's default, 3):
//   plain zstd   L 1-2: none (unit-local parse); 3-6: 4 slices (2^17
//                entries); >= 7: 8 slices (2^18)
//   blosc-zstd   bitshuffle, L >= 3: 1 slice (a bit plane of a u16 block
//                matches the previous plane 16 KiB back: camera 1.914 ->
//                1.983, c-blosc clevel 5 1.974); byte shuffle: none (its
//                planes lose from longer matches: camera 1.891 -> 1.845)
// (tools/zstd_lab.cpp far=..., farbatch=4096)
// The far pass's range split is sized for the MI355X's 256 CUs as a
// constant, not read from the device: the ranges (and so a chunk's frame
// bytes) then follow from the layer geometry alone, the same for a stage
// and a standalone compressor on any device.  Every choice decodes to the
// same chunk.
constexpr uint64_t kFarRangeCus = 256;

uint32_t
zstd_far_slices(const Compression& c, uint32_t typesize)
{
    (void)typesize;
    if (c.codec == 3) {
        const int zl = c.clevel == 0 ? 3 : c.clevel;
        return zl >= 7 ? 8u : zl >= 3 ? 4u : 0u;
    }
    if (c.codec == 2 && c.shuffle == 2 && c.clevel >= 2)
        return 1u;
    return 0u;
}

uint64_t
Compressor::scratch_bytes(const Compression& c, uint64_t chunk_bytes, uint32_t typesize,
                          uint32_t n_chunks)
{
    const uint64_t n = n_chunks;
    const bool store_only = c.codec != 3 && c.clevel == 0;
    uint64_t b = n * 4 + n + n * 8; // fsize, mode, cstart
    if (c.codec == 1) {
        const BloscGeom g = make_blosc_geom(uint32_t(chunk_bytes), typesize, uint32_t(c.shuffle));
        const uint64_t ns = n * g.spc;
        return b + (store_only ? 1 : ns * g.slot) + ns * 8;
    }
    uint64_t seg = chunk_bytes, nseg1 = 1;
    if (c.codec == 2) {
        const ZstdBloscGeom g = make_zstd_blosc_geom(uint32_t(chunk_bytes), typesize);
        seg = g.blocksize;
        nseg1 = g.nblocks;
    }
    const uint64_t nseg = n * nseg1, bps = (seg + zstd::kBlock - 1) / zstd::kBlock;
    const uint32_t gl =
      zstd_huf_group_log2(c.codec == 2 ? uint32_t(c.shuffle) : 0u, typesize, uint32_t(seg),
                          c.clevel);
    const uint64_t nblk = nseg * bps, ngrp = nseg * ((bps + (1u << gl) - 1) >> gl);
    b += nseg * 4; // spos
    if (c.codec == 2 && !store_only && (c.shuffle == 2 || (c.shuffle == 1 && typesize > 1)))
        b += n * chunk_bytes; // shuffled input
    if (store_only)
        return b;
    if (zstd_far_slices(c, typesize))
        b += nseg * seg * 4; // far candidates
    const uint64_t nu = nblk * kZSubBlocks;
    b += nu * kZSub + nu * kZSubSeq * 8 + 4 * nu * 4;              // parse units
    b += nblk * (1 + 4 + 4 + 4 + 256 * 4 + 1 + 4 + 4 + zstd::kBlock); // per block
    b += nseg * (192 * 4 + sizeof(ZstdSeqSeg) + 4 + 1 + 4);         // per segment
    b += ngrp * (sizeof(ZstdSegTable) + 4) + sizeof(zstd::SeqTables);
    return b;
}

void
Compressor::run(const uint8_t* chunks, uint64_t pitch, uint32_t n_chunks,
                const uint32_t* flags, uint32_t tag, uint8_t* out, uint64_t* offsets,
                hipStream_t stream, const uint32_t* order)
{
    if (c_.codec != 1) {
        run_zstd(chunks, pitch, n_chunks, flags, tag, out, offsets, stream, order);
        return;
    }
    const uint64_t ns = uint64_t(n_chunks) * g_.spc;
    alloc_large(scratch_, store_only_ ? 1 : ns * g_.slot, tune_.vmm);
    ssize_.alloc(ns * 4);
    spos_.alloc(ns * 4);
    fsize_.alloc(size_t(n_chunks) * 4);
    mode_.alloc(n_chunks);
    cstart_.alloc(size_t(n_chunks) * 8);
    BloscParams p{};
    p.g = g_;
    p.chunks = chunks;
    p.pitch = pitch;
    p.n_chunks = n_chunks;
    p.flags = flags;
    p.tag = tag;
    p.scratch = scratch_.p;
    p.ssize = reinterpret_cast<uint32_t*>(ssize_.p);
    p.spos = reinterpret_cast<uint32_t*>(spos_.p);
    p.fsize = reinterpret_cast<uint32_t*>(fsize_.p);
    p.mode = mode_.p;
    p.offsets = offsets;
    p.cstart = reinterpret_cast<uint64_t*>(cstart_.p);
    p.order = order;
    p.out = out;
    p.store_only = store_only_ ? 1 : 0;
    hip_check(launch_blosc_lz4(p, stream), "blosc-lz4 launch");
}

// blosc-zstd: one zstd frame per blosc block of the (device-shuffled)
// chunk; zstd: one frame per chunk (aqz_codec.hh ZstdParams).
void
Compressor::run_zstd(const uint8_t* chunks, uint64_t pitch, uint32_t n_chunks,
                     const uint32_t* flags, uint32_t tag, uint8_t* out, uint64_t* offsets,
                     hipStream_t stream, const uint32_t* order)
{
    const bool blosc = c_.codec == 2;
    ZstdParams p{};
    p.chunks = chunks;
    p.pitch = pitch;
    p.n_chunks = n_chunks;
    p.nbytes = uint32_t(nbytes_);
    p.typesize = typesize_;
    p.shuffle = blosc ? uint32_t(c_.shuffle) : 0;
    p.blosc = blosc ? 1 : 0;
    p.store_only = store_only_ ? 1 : 0;
    p.flags = flags;
    p.tag = tag;
    if (blosc) {
        const ZstdBloscGeom g = make_zstd_blosc_geom(uint32_t(nbytes_), typesize_);
        p.seg_bytes = g.blocksize;
        p.nseg = g.nblocks;
    } else {
        p.seg_bytes = uint32_t(nbytes_);
        p.nseg = 1;
    }
    p.bps = (p.seg_bytes + zstd::kBlock - 1) / zstd::kBlock;
    p.hgrp_log2 = zstd_huf_group_log2(p.shuffle, typesize_, p.seg_bytes, c_.clevel);
    p.ngrp = (p.bps + (1u << p.hgrp_log2) - 1) >> p.hgrp_log2;
    // The level chooses how far back matches reach (zstd_far_slices): the
    // unit-local parse at the fast levels, the far candidates above them.
    // A parse history (matches into the 12 / 28 KiB before a unit, loaded and
    // hashed per unit) is kept only as a tuning knob: the far candidates
    // reach every earlier unit at a fraction of its cost.
    p.phist = tune_.phist;
    // a match must save the bits of a sequence: ~12 with the fitted tables
    // of unshuffled data, 16 on shuffled planes (tools/zstd_lab.cpp sweep)
    p.match_bits = uint32_t(blosc ? zstd::kMatchBits : zstd::kMatchBitsFitted);
    p.fit = tune_.fit;
    p.src = chunks;
    p.src_pitch = pitch;
    // parse variants for A/B timing (bits 1/2/4/8; the frames stay valid)
    p.dbg = tune_.parse & 15u;
    const bool shuffle = blosc && !store_only_ &&
                         (c_.shuffle == 2 || (c_.shuffle == 1 && typesize_ > 1));
    if (shuffle) {
        alloc_large(zin_, size_t(n_chunks) * nbytes_, tune_.vmm);
        ShuffleParams sp{ chunks, pitch, n_chunks, flags, tag, p.nbytes, typesize_,
                          uint32_t(c_.shuffle), p.seg_bytes, p.nseg, zin_.p };
        hip_check(launch_shuffle_blocks(sp, stream), "shuffle launch");
        p.src = zin_.p;
        p.src_pitch = nbytes_;
    }
    const uint64_t nseg = uint64_t(n_chunks) * p.nseg, nblk = nseg * p.bps;
    // LZ matches unless tuned off (literals only: the serial model's
    // byte-exact mode, tests/test_gpu_zstd.py)
    p.match = tune_.match ? 1 : 0;
    if (!store_only_) {
        if (!seqt_.p) {
            zstd::SeqTables t;
            if (!zstd::build_seq_tables(t))
                throw Error(10, "zstd sequence tables");
            seqt_.alloc(sizeof(t));
            hip_check(hipMemcpy(seqt_.p, &t, sizeof(t), hipMemcpyHostToDevice), "hipMemcpy");
        }
        // far candidates (zstd_far) in place of a parse history, where a
        // history pays: zstd_far_slices (the level), 4-byte aligned segments
        p.far_slices = zstd_far_slices(c_, typesize_);
        // a blosc block (256 KiB) needs no more than 2^13 entries (bitshuffle
        // camera 1.972 -> 1.969, tools/zstd_lab.cpp far=13), a quarter of the
        // LDS: twice the workgroups per CU
        p.far_log = blosc ? 13u : kFarLog;
        p.far_tb = p.far_slices ? zstd_far_tag_bits(p.seg_bytes, p.far_slices, p.far_log) : 0;
        bool far = p.match && p.far_tb != 0 && (reinterpret_cast<uintptr_t>(p.src) & 3u) == 0 &&
                   (p.src_pitch & 3u) == 0 && (p.seg_bytes & 3u) == 0;
        far = far && tune_.far != 0;
        if (far) {
            alloc_large(far_, nseg * p.seg_bytes * 4, tune_.vmm);
            p.far = reinterpret_cast<uint32_t*>(far_.p);
            p.phist = 0; // the far candidates cover every earlier unit
            // A layer of few segments (the small levels' layers) walks each
            // segment in parallel ranges, each at least as long as its
            // warm-up: a range first inserts the 1 MiB and the two chunk
            // planes before it, so its positions miss only candidates
            // further back than that (the sequential walk of one segment per
            // slice is 2048 dependent steps for 8 MiB, whatever the layer's
            // size).  Layers that fill the device keep one range.
            const uint64_t wgs = nseg * p.far_slices;
            const uint64_t steps = (uint64_t(p.seg_bytes) + kZSub - 1) / kZSub;
            const uint64_t cus = kFarRangeCus;
            const uint64_t warm = std::max<uint64_t>(kFarWarm, (2 * plane_bytes_ + kZSub - 1) / kZSub);
            p.far_warm = uint32_t(std::min<uint64_t>(warm, steps));
            p.far_ranges = 1;
            while (tune_.ranges && p.far_ranges < 8 && wgs * p.far_ranges * 2 <= cus &&
                   steps / (2u * p.far_ranges) >= warm)
                p.far_ranges *= 2;
        }
        far_ranges_ = far ? p.far_ranges : 0;
        if (p.match) {
            const uint64_t nu = nblk * kZSubBlocks;
            alloc_large(lits_, nu * kZSub, tune_.vmm);
            alloc_large(seqs_, nu * kZSubSeq * 8, tune_.vmm);
            snseq_.alloc(nu * 4);
            snlit_.alloc(nu * 4);
            stail_.alloc(nu * 4);
            sval_.alloc(nu * 4);
        }
        const uint64_t ngrp = nseg * p.ngrp;
        bltype_.alloc(nblk);
        bseqb_.alloc(nblk * 4);
        bnlit_.alloc(nblk * 4);
        bnseq_.alloc(nblk * 4);
        hist_.alloc(nblk * 256 * 4);
        scount_.alloc(nseg * 192 * 4);
        sqt_.alloc(nseg * sizeof(ZstdSeqSeg));
        scarrier_.alloc(nseg * 4);
        bkind_.alloc(nblk);
        bpay_.alloc(nblk * 4);
        bpos_.alloc(nblk * 4);
        alloc_large(scratch_, nblk * zstd::kBlock, tune_.vmm);
        tab_.alloc(ngrp * sizeof(ZstdSegTable));
        carrier_.alloc(ngrp * 4);
        sraw_.alloc(nseg);
        ssize_.alloc(nseg * 4);
    }
    spos_.alloc(nseg * 4);
    fsize_.alloc(size_t(n_chunks) * 4);
    mode_.alloc(n_chunks);
    cstart_.alloc(size_t(n_chunks) * 8);
    p.seqt = reinterpret_cast<const zstd::SeqTables*>(seqt_.p);
    p.lits = lits_.p;
    p.seqs = reinterpret_cast<uint64_t*>(seqs_.p);
    p.snseq = reinterpret_cast<uint32_t*>(snseq_.p);
    p.snlit = reinterpret_cast<uint32_t*>(snlit_.p);
    p.stail = reinterpret_cast<uint32_t*>(stail_.p);
    p.sval = reinterpret_cast<uint32_t*>(sval_.p);
    p.bltype = bltype_.p;
    p.bseqb = reinterpret_cast<uint32_t*>(bseqb_.p);
    p.bnlit = reinterpret_cast<uint32_t*>(bnlit_.p);
    p.hist = reinterpret_cast<uint32_t*>(hist_.p);
    p.bnseq = reinterpret_cast<uint32_t*>(bnseq_.p);
    p.scount = reinterpret_cast<uint32_t*>(scount_.p);
    p.sqt = reinterpret_cast<ZstdSeqSeg*>(sqt_.p);
    p.scarrier = reinterpret_cast<uint32_t*>(scarrier_.p);
    p.bkind = bkind_.p;
    p.bpay = reinterpret_cast<uint32_t*>(bpay_.p);
    p.bpos = reinterpret_cast<uint32_t*>(bpos_.p);
    p.scratch = scratch_.p;
    p.tab = reinterpret_cast<ZstdSegTable*>(tab_.p);
    p.carrier = reinterpret_cast<uint32_t*>(carrier_.p);
    p.ssize = reinterpret_cast<uint32_t*>(ssize_.p);
    p.sraw = sraw_.p;
    p.spos = reinterpret_cast<uint32_t*>(spos_.p);
    p.fsize = reinterpret_cast<uint32_t*>(fsize_.p);
    p.mode = mode_.p;
    p.order = order;
    p.offsets = offsets;
    p.cstart = reinterpret_cast<uint64_t*>(cstart_.p);
    p.out = out;
    hip_check(launch_zstd(p, stream), "zstd launch");
}

void
Stage::ensure_comp_slots(StageLevel& L)
{
    if (!L.cframes.empty())
        return;
    L.cframes.resize(L.n_slots);
    L.coffsets.resize(L.n_slots);
    L.h_coffsets.resize(L.n_slots);
    L.comp_ev.assign(L.n_slots, nullptr);
    L.cdone_ev.assign(L.n_slots, nullptr);
    L.cdone_pending.assign(L.n_slots, 0);
    L.cdone_ticket.assign(L.n_slots, 0);
    L.comp_layer.assign(L.n_slots, -1);
    L.h_zin.resize(L.n_slots);
    L.h_zhas.resize(L.n_slots);
    L.zin_ev.assign(L.n_slots, nullptr);
    L.zjob.resize(L.n_slots);
    L.comp_host.assign(L.n_slots, 0);
    for (uint32_t s = 0; s < L.n_slots; ++s) {
        hip_check(hipEventCreateWithFlags(&L.comp_ev[s], hipEventDisableTiming),
                  "hipEventCreate");
        hip_check(hipEventCreateWithFlags(&L.cdone_ev[s], hipEventDisableTiming),
                  "hipEventCreate");
        hip_check(hipEventCreateWithFlags(&L.zin_ev[s], hipEventDisableTiming),
                  "hipEventCreate");
    }
}

// the zstd codecs run on the device unless AQZ_ZSTD_HOST=1 (device shuffle
// + host libzstd pool, aqz_hostzstd.hh)
static bool
zstd_on_host()
{
    const char* s = std::getenv("AQZ_ZSTD_HOST");
    return s && std::atoi(s) != 0;
}

// host threads for the zstd codecs (AQZ_ZSTD_THREADS)
static unsigned
zstd_workers()
{
    if (const char* s = std::getenv("AQZ_ZSTD_THREADS"))
        return unsigned(std::max(1, std::atoi(s)));
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return std::min(16u, std::max(1u, hw - 1));
}

// blosc-zstd and plain zstd (aqz_hostzstd.hh): on the compression stream,
// after the kernels that wrote the layer, the layer's blocks are shuffled
// on the device (blosc-zstd with a shuffle) and the chunks go D2H with their
// has_data bytes; the host pool compresses as soon as they have landed.
void
Stage::compress_layer_host(StageLevel& L, uint32_t slot, uint64_t layer,
                           const Compression& c)
{
    // level 0's layers compress on comp_; the small layers of the other
    // levels on comp_lo_ / comp_lo2_, overlapping level 0's (their kernels are few
    // workgroups and latency-bound)
    const hipStream_t cs = comp_stream(L);
    const ZstdLib& z = ZstdLib::get();
    if (!z.ok)
        throw Error(4, "libzstd.so.1 is not available: no zstd codecs");
    if (c.codec == 2 && (c.shuffle < 0 || c.shuffle > 2 || c.clevel < 0 || c.clevel > 9))
        throw Error(1, "invalid blosc compression settings");
    if (c.codec == 3 && (c.clevel < -131072 || c.clevel > z.max_clevel()))
        throw Error(1, "invalid zstd level");
    if (L.bpc > 0x7fffffefull)
        throw Error(1, "chunk size outside the blosc1 limits");
    ensure_comp_slots(L);
    if (!zpool_)
        zpool_ = std::make_unique<TaskPool>(zstd_workers(), numa_cpus_);
    if (L.zjob[slot])
        L.zjob[slot]->wait(); // its inputs and frames are about to be reused
    else
        L.zjob[slot] = std::make_shared<HostLayerJob>();
    // device frames of an earlier blosc-lz4 use of the slot may still be
    // on their way out
    if (L.cdone_ticket[slot]) {
        // the slot's frames left on a DMA engine: the host waits for them
        (void)copies_completed(false, L.cdone_ticket[slot]);
        L.cdone_ticket[slot] = 0;
    }
    if (L.cdone_pending[slot]) {
        hip_check(hipStreamWaitEvent(cs, L.cdone_ev[slot], 0), "hipStreamWaitEvent");
        L.cdone_pending[slot] = 0;
    }
    L.h_zin[slot].alloc(L.layer_bytes);
    L.h_zhas[slot].alloc(L.n_chunks);
    hip_check(hipEventRecord(L.ready_ev[slot], stream_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(cs, L.ready_ev[slot], 0), "hipStreamWaitEvent");
    const uint8_t* chunks = L.ring.p + slot * L.slot_bytes;
    const auto* flags = reinterpret_cast<const uint32_t*>(L.flags.p) + size_t(slot) * L.n_chunks;
    const uint32_t tag = uint32_t(layer / L.n_slots + 1);
    const bool shuffle = c.codec == 2 && (c.shuffle == 2 || (c.shuffle == 1 && bpp_ > 1));
    if (shuffle) {
        const ZstdBloscGeom g = make_zstd_blosc_geom(uint32_t(L.bpc), uint32_t(bpp_));
        L.d_zshuf.alloc(L.layer_bytes);
        ShuffleParams sp{ chunks, L.pitch, L.n_chunks, flags, tag, uint32_t(L.bpc),
                          uint32_t(bpp_), uint32_t(c.shuffle), g.blocksize, g.nblocks,
                          L.d_zshuf.p };
        hip_check(launch_shuffle_blocks(sp, cs), "shuffle launch");
        memcpy_pieces(L.h_zin[slot].p, L.d_zshuf.p, L.layer_bytes, hipMemcpyDeviceToHost,
                      cs);
    } else {
        copy_chunks(L.h_zin[slot].p, chunks, L.bpc, L.pitch, L.n_chunks,
                    hipMemcpyDeviceToHost, cs);
    }
    uint8_t* fb = L.flag_bytes.p + size_t(slot) * L.n_chunks;
    hip_check(launch_flags_to_bytes(flags, fb, L.n_chunks, tag, cs), "flags launch");
    hip_check(hipMemcpyAsync(L.h_zhas[slot].p, fb, L.n_chunks, hipMemcpyDeviceToHost, cs),
              "hipMemcpyAsync");
    hip_check(hipEventRecord(L.zin_ev[slot], cs), "hipEventRecord");
    // the ring slot is rewritten only after this D2H
    hip_check(hipEventRecord(L.copy_ev[slot], cs), "hipEventRecord");
    L.copy_pending[slot] = 1;

    HostLayerJob& j = *L.zjob[slot];
    j.codec = c.codec;
    j.clevel = c.clevel;
    j.shuffle = c.codec == 2 ? c.shuffle : 0;
    j.typesize = uint32_t(bpp_);
    j.bpc = L.bpc;
    j.n_chunks = L.n_chunks;
    j.chunks = L.h_zin[slot].p;
    j.has_data = L.h_zhas[slot].p;
    j.order = L.h_order;
    const ZstdBloscGeom g = make_zstd_blosc_geom(uint32_t(L.bpc), uint32_t(bpp_));
    j.frame_cap = std::max<uint64_t>(z.compress_bound(L.bpc),
                                     L.bpc + 16 + 8ull * g.nblocks + 64);
    j.tmp.resize(size_t(j.frame_cap) * L.n_chunks);
    host_zstd_compress(*zpool_, L.zjob[slot],
                       [ev = L.zin_ev[slot]] { (void)hipEventSynchronize(ev); });
    L.comp_layer[slot] = int64_t(layer);
    L.comp_host[slot] = 1;
}

void
Stage::compress_layer(uint32_t level, uint64_t layer, const Compression& c)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    // level 0's layers compress on comp_; the small layers of the other
    // levels on comp_lo_ / comp_lo2_, overlapping level 0's (their kernels are few
    // workgroups and latency-bound)
    const hipStream_t cs = comp_stream(L);
    if (!L.ring.p)
        throw Error(1, "level 0 is not split on the device by this stage");
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (L.slot_layer[slot] != int64_t(layer))
        throw Error(3, "chunk layer not resident");
    if ((c.codec == 2 || c.codec == 3) && zstd_on_host()) {
        compress_layer_host(L, slot, layer, c);
        return;
    }
    if (!L.comp || L.comp_cfg.codec != c.codec || L.comp_cfg.clevel != c.clevel ||
        L.comp_cfg.shuffle != c.shuffle) {
        hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize");
        hip_check(hipStreamSynchronize(d2h_), "hipStreamSynchronize");
        L.comp = std::make_unique<Compressor>(L.bpc, uint32_t(bpp_), c, opt_.codec);
        L.comp->set_plane_bytes(uint64_t(L.tw) * L.th * bpp_);
        L.comp_cfg = c;
    }
    ensure_comp_slots(L);
    if (L.zjob[slot]) // the slot last ran on the host: its inputs are in use
        L.zjob[slot]->wait();
    L.comp_host[slot] = 0;
    // the slot's previous frames may still be on their way to the host
    if (L.cdone_ticket[slot]) {
        // the slot's frames left on a DMA engine: the host waits for them
        (void)copies_completed(false, L.cdone_ticket[slot]);
        L.cdone_ticket[slot] = 0;
    }
    if (L.cdone_pending[slot]) {
        hip_check(hipStreamWaitEvent(cs, L.cdone_ev[slot], 0), "hipStreamWaitEvent");
        L.cdone_pending[slot] = 0;
    }
    const uint64_t cap = Compressor::max_bytes(L.bpc, L.n_chunks);
    if (L.cframes[slot].n < cap)
        hip_check(hipStreamSynchronize(cs), "hipStreamSynchronize"); // realloc below
    alloc_large(L.cframes[slot], cap, opt_.codec.vmm);
    L.coffsets[slot].alloc((size_t(L.n_chunks) + 1) * 8);
    L.h_coffsets[slot].alloc((size_t(L.n_chunks) + 1) * 8);
    // after every kernel enqueued so far; the slot's next layer waits for it.
    // Compression runs on its own stream: it overlaps the D2H of the frames
    // of earlier layers on the hand-off stream.
    hip_check(hipEventRecord(L.ready_ev[slot], stream_), "hipEventRecord");
    hip_check(hipStreamWaitEvent(cs, L.ready_ev[slot], 0), "hipStreamWaitEvent");
    L.comp->run(L.ring.p + slot * L.slot_bytes, L.pitch, L.n_chunks,
                reinterpret_cast<const uint32_t*>(L.flags.p) + size_t(slot) * L.n_chunks,
                uint32_t(layer / L.n_slots + 1), L.cframes[slot].p,
                reinterpret_cast<uint64_t*>(L.coffsets[slot].p), cs,
                reinterpret_cast<const uint32_t*>(L.shard_order.p));
    hip_check(hipMemcpyAsync(L.h_coffsets[slot].p, L.coffsets[slot].p,
                             (size_t(L.n_chunks) + 1) * 8, hipMemcpyDeviceToHost, cs),
              "hipMemcpyAsync");
    hip_check(hipEventRecord(L.comp_ev[slot], cs), "hipEventRecord");
    hip_check(hipEventRecord(L.copy_ev[slot], cs), "hipEventRecord");
    L.copy_pending[slot] = 1;
    L.comp_layer[slot] = int64_t(layer);
}

void
Stage::compressed_offsets(uint32_t level, uint64_t layer, uint64_t* offsets, size_t n)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    const uint32_t slot = L.n_slots ? uint32_t(layer % L.n_slots) : 0;
    if (L.comp_layer.empty() || L.comp_layer[slot] != int64_t(layer))
        throw Error(3, "layer was not compressed (or its slot was reused)");
    if (n < size_t(L.n_chunks) + 1)
        throw Error(2, "offsets too small");
    if (L.comp_host[slot]) {
        HostLayerJob& j = *L.zjob[slot];
        j.wait();
        if (j.status)
            throw Error(j.status, "zstd compression failed");
        std::memcpy(offsets, j.offsets.data(), (size_t(L.n_chunks) + 1) * 8);
        return;
    }
    hip_check(hipEventSynchronize(L.comp_ev[slot]), "hipEventSynchronize");
    std::memcpy(offsets, L.h_coffsets[slot].p, (size_t(L.n_chunks) + 1) * 8);
}

bool
Stage::compression_done(uint32_t level, uint64_t layer)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    const uint32_t slot = L.n_slots ? uint32_t(layer % L.n_slots) : 0;
    if (L.comp_layer.empty() || L.comp_layer[slot] != int64_t(layer))
        throw Error(3, "layer was not compressed (or its slot was reused)");
    if (L.comp_host[slot])
        return L.zjob[slot]->finished();
    const hipError_t q = hipEventQuery(L.comp_ev[slot]);
    if (q == hipErrorNotReady)
        return false;
    hip_check(q, "hipEventQuery");
    return true;
}

void
Stage::copy_compressed_async(uint32_t level, uint64_t layer, void* dst, size_t cap)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    const uint32_t slot = L.n_slots ? uint32_t(layer % L.n_slots) : 0;
    if (L.comp_layer.empty() || L.comp_layer[slot] != int64_t(layer))
        throw Error(3, "layer was not compressed (or its slot was reused)");
    if (L.comp_host[slot]) {
        // host frames: gathered into dst (host memory) right away
        HostLayerJob& j = *L.zjob[slot];
        j.wait();
        if (j.status)
            throw Error(j.status, "zstd compression failed");
        if (cap < j.offsets[L.n_chunks])
            throw Error(2, "destination too small for the compressed layer");
        j.gather(static_cast<uint8_t*>(dst));
        last_ticket_ = issue_ticket(); // complete as soon as it is issued
        return;
    }
    hip_check(hipEventSynchronize(L.comp_ev[slot]), "hipEventSynchronize");
    const uint64_t total =
      reinterpret_cast<const uint64_t*>(L.h_coffsets[slot].p)[L.n_chunks];
    if (cap < total)
        throw Error(2, "destination too small for the compressed layer");
    if (sdma_d2h_ && pinned_host(dst)) {
        // one copy on a DMA engine (the compression has finished: the event
        // above), no blit kernel beside the codec kernels; the next
        // compression into this slot waits for its ticket (compress_layer).
        // A DMA engine reads or writes page-locked memory only: pageable or
        // device destinations take the HIP copy below.
        hsa_signal_t sig{ 0 };
        if (free_sig_.empty()) {
            if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
                throw Error(5, "hsa_signal_create failed");
        } else {
            sig = free_sig_.back();
            free_sig_.pop_back();
            hsa_signal_store_screlease(sig, 1);
        }
        if (total == 0) {
            hsa_signal_store_screlease(sig, 0);
        } else if (hsa_amd_memory_async_copy(dst, hsa_cpu_, L.cframes[slot].p, hsa_gpu_, total,
                                             0, nullptr, sig) != HSA_STATUS_SUCCESS) {
            free_sig_.push_back(sig);
            throw Error(5, "hsa_amd_memory_async_copy failed");
        }
        last_ticket_ = issue_ticket(sig);
        L.cdone_ticket[slot] = last_ticket_;
        return;
    }
    memcpy_pieces(dst, L.cframes[slot].p, total, hipMemcpyDefault, d2h_);
    hip_check(hipEventRecord(L.copy_ev[slot], d2h_), "hipEventRecord");
    hip_check(hipEventRecord(L.cdone_ev[slot], d2h_), "hipEventRecord");
    L.copy_pending[slot] = 1;
    L.cdone_pending[slot] = 1;
    last_ticket_ = issue_ticket();
}

void
Stage::import_frames(Stage* src, uint32_t level, uint64_t layer, uint32_t first,
                     uint32_t count)
{
    if (level >= lv_.size())
        throw Error(3, "level out of range");
    StageLevel& L = lv_[level];
    if (!L.ring.p)
        throw Error(1, "level 0 is not split on the device by this stage");
    if (uint64_t(first) + count > L.F)
        throw Error(3, "frames outside the chunk layer");
    StageLevel* S = nullptr;
    if (src) {
        if (src->lv_.size() != lv_.size())
            throw Error(1, "stages of different pyramids");
        S = &src->lv_[level];
        if (S->bpc != L.bpc || S->n_chunks != L.n_chunks || S->F != L.F ||
            S->n_slots != L.n_slots || S->pitch != L.pitch || !S->ring.p)
            throw Error(1, "stages of different chunk geometry");
        if (S->slot_layer[layer % S->n_slots] != int64_t(layer))
            throw Error(3, "source chunk layer not resident");
        if (src->desc_.device != desc_.device) {
            // peer reads over xGMI; enabled once per device pair
            const hipError_t e = hipDeviceEnablePeerAccess(src->desc_.device, 0);
            if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                hip_check(e, "hipDeviceEnablePeerAccess");
            (void)hipGetLastError();
            src->grant_access(desc_.device);
        }
    }
    if (count == 0)
        return;
    const uint32_t slot = uint32_t(layer % L.n_slots);
    if (L.slot_layer[slot] != int64_t(layer))
        enter_layer(L, layer); // this stage wrote none of the layer's frames yet
    if (src) {
        // after every kernel src enqueued so far (the frames it wrote)
        hip_check(hipEventRecord(S->ready_ev[slot], src->stream_), "hipEventRecord");
        hip_check(hipStreamWaitEvent(stream_, S->ready_ev[slot], 0), "hipStreamWaitEvent");
    }
    const uint32_t tile_bytes = L.th * L.tw * uint32_t(bpp_);
    hip_check(launch_import_frames(
                L.ring.p + slot * L.slot_bytes, S ? S->ring.p + slot * S->slot_bytes : nullptr,
                reinterpret_cast<const uint64_t*>(L.tab_off.p),
                reinterpret_cast<const uint32_t*>(L.tab_grp.p), first, count, L.ntx * L.nty,
                L.pitch, tile_bytes,
                reinterpret_cast<uint32_t*>(L.flags.p) + size_t(slot) * L.n_chunks,
                S ? reinterpret_cast<const uint32_t*>(S->flags.p) + size_t(slot) * S->n_chunks
                  : nullptr,
                uint32_t(layer / L.n_slots + 1), stream_),
              "import launch");
    if (src) {
        // src's slot holds the layer until the copy has read it: an event of
        // this stage's device on this stream, for src's stream to wait on
        // before it reuses the slot (src->copy_ev is src's device's event
        // and may not be recorded here)
        hipEvent_t e = nullptr;
        hip_check(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        std::shared_ptr<ihipEvent_t> ev(e, [](hipEvent_t x) { (void)hipEventDestroy(x); });
        hip_check(hipEventRecord(e, stream_), "hipEventRecord");
        std::lock_guard<std::mutex> lk(src->access_mu_);
        if (S->peer_ev.empty())
            S->peer_ev.resize(S->n_slots);
        S->peer_ev[slot].push_back(std::move(ev));
    }
}

void
Stage::finalize()
{
    for (auto& L : lv_) {
        if (!L.ring.p)
            continue;
        const uint64_t fw = L.frames_written;
        // (a z-slab stage's frame id may already point past its last slab,
        // into a layer it never entered: nothing to flush there)
        if (fw % L.F == 0 || L.slot_layer[(fw / L.F) % L.n_slots] != int64_t(fw / L.F))
            continue;
        const uint64_t end = (fw / L.F + 1) * L.F;
        for (uint64_t fid = fw; fid < end; ++fid) {
            uint64_t off;
            uint32_t fo;
            tile_addr(L, fid, &off, &fo, nullptr);
            hip_check(launch_zero_frame_tiles(L.ring.p + off, L.pitch,
                                              L.ntx * L.nty,
                                              uint32_t(uint64_t(L.tw) * L.th * bpp_),
                                              stream_),
                      "zero launch");
        }
    }
    finalized_ = true;
    synchronize();
}

static unsigned
split_workers()
{
    if (const char* s = std::getenv("AQZ_SPLIT_THREADS"))
        return unsigned(std::max(0, std::atoi(s)));
    // 16 threads in all: a GPU's share of a node's cores (the reference
    // splits with OpenMP over all of them, array.cpp:575)
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    return std::min(15u, hw / 2);
}

void
Stage::split_level0_rows(const void* frame, uint64_t frame_id, uint32_t row_begin,
                         uint32_t row_end, void* frame_copy, uint32_t chunk0, void* dst,
                         size_t cap, uint8_t* has_data, size_t has_data_cap) const
{
    const StageLevel& L = lv_[0];
    if (!frame || !dst || !has_data)
        throw Error(1, "null frame, destination or has_data");
    const uint64_t n = std::min<uint64_t>(cap / L.bpc, has_data_cap);
    if (n == 0 || chunk0 >= L.n_chunks)
        throw Error(1, "destination holds no chunk of the layer");
    split_rows(split_geom(*L.ad, frame_id), static_cast<const uint8_t*>(frame), row_begin,
               row_end, static_cast<uint8_t*>(dst), chunk0,
               uint32_t(std::min<uint64_t>(n, L.n_chunks - chunk0)), has_data,
               static_cast<uint8_t*>(frame_copy));
}

void
Stage::split_level0_host(const void* frames, uint64_t n, uint64_t first, uint32_t chunk0,
                         void* dst, size_t cap, uint8_t* has_data, size_t has_data_cap)
{
    if (n == 0)
        return;
    if (!frames)
        throw Error(1, "null frames");
    const StageLevel& L = lv_[0];
    // one layer's frames: another layer's would land on the same chunks
    if (first / L.F != (first + n - 1) / L.F)
        throw Error(1, "the frames span two chunk layers");
    const uint64_t fbytes = uint64_t(L.W) * L.H * bpp_;
    // tasks of 64 rows (256 KiB of a 2048-px u16 frame), frame-major
    constexpr uint32_t kRows = 64;
    const uint32_t per_frame = parts_along(L.H, kRows);
    if (!split_pool_)
        split_pool_ = std::make_unique<SplitPool>(split_workers(), numa_cpus_);
    const auto* src = static_cast<const uint8_t*>(frames);
    split_pool_->run(size_t(n) * per_frame, [&](size_t i) {
        const uint64_t f = i / per_frame;
        const uint32_t r0 = uint32_t(i % per_frame) * kRows;
        split_level0_rows(src + f * fbytes, first + f, r0, std::min(L.H, r0 + kRows), nullptr,
                          chunk0, dst, cap, has_data, has_data_cap);
    });
}

void
Stage::enable_timing(bool on)
{
    synchronize();
    timing_ = on;
    ev_used_ = 0;
    timed_ms_ = 0;
    timed_launches_ = 0;
}

void
Stage::timing(double* total_ms, uint64_t* launches)
{
    synchronize();
    for (size_t i = 0; i < ev_used_; ++i) {
        float ms = 0;
        hip_check(hipEventElapsedTime(&ms, ev_pairs_[i].first,
                                      ev_pairs_[i].second),
                  "hipEventElapsedTime");
        timed_ms_ += ms;
        ++timed_launches_;
    }
    ev_used_ = 0;
    if (total_ms)
        *total_ms = timed_ms_;
    if (launches)
        *launches = timed_launches_;
}

// One timing event pair on the stream the kernels are launched on: the bench
// brackets its whole timed region with it (a pair per launch adds gaps).
void
Stage::mark(int which)
{
    if (which != 0 && which != 1)
        throw Error(1, "timing mark must be 0 (begin) or 1 (end)");
    if (!mark_ev_[which])
        hip_check(hipEventCreate(&mark_ev_[which]), "hipEventCreate");
    hip_check(hipEventRecord(mark_ev_[which], stream_), "hipEventRecord");
}

double
Stage::marked_ms()
{
    if (!mark_ev_[0] || !mark_ev_[1])
        throw Error(1, "timing marks not recorded");
    hip_check(hipEventSynchronize(mark_ev_[1]), "hipEventSynchronize");
    float ms = 0;
    hip_check(hipEventElapsedTime(&ms, mark_ev_[0], mark_ev_[1]), "hipEventElapsedTime");
    return ms;
}

const char*
Stage::dominant_kernel() const
{
    if (fused_2d_) {
        // launch_interior's choice (aqz_kernels.hip) for this stage's launches
        const bool tail = n_levels() - 1 > n_fused_;
        const bool strip = bpp_ <= 4 && rh_log2_ == 6 && !(knobs_ & 128u) &&
                           (!tail || n_fused_ >= 5);
        if (xy_)
            return xy_direct_ ? "fused_pyramid_strip (XY load)"
                              : (strip ? "transpose_frames + fused_pyramid_strip"
                                       : "transpose_frames + fused_pyramid");
        return strip ? "fused_pyramid_strip" : "fused_pyramid";
    }
    if (fused_3d_) { // launch_fused_pyramid_3d's choice
        const bool strip = rh_log2_ == 6 && n_levels() - 1 <= 4 && !(knobs_ & 256u);
        const bool pair = strip && !(knobs_ & 2u) && (zmask3d_ & 2u) && g3d_ % 2 == 0 &&
                          nt_mode_ != 0;
        const char* k = pair    ? "fused_pyramid_strip3d_pair"
                        : strip ? "fused_pyramid_strip3d"
                                : "fused_pyramid_3d";
        if (xy_ && xy_direct_) // the pair kernel reads XY only under knob 65536
            return pair && (knobs_ & 65536u) ? "fused_pyramid_strip3d_pair (XY load)"
                                             : "fused_pyramid_strip3d (XY load)";
        if (xy_)
            return pair       ? "transpose_frames + fused_pyramid_strip3d_pair"
                   : strip    ? "transpose_frames + fused_pyramid_strip3d"
                              : "transpose_frames + fused_pyramid_3d";
        return k;
    }
    return "level_kernel";
}

// ===========================================================================
// GpuDownsampler
// ===========================================================================
GpuDownsampler::GpuDownsampler(const ArrayDesc& desc)
  : dtype_(desc.dtype)
  , method_(desc.method)
  , device_(desc.device)
{
    bpp_ = bytes_of_type(desc.dtype); // throws on invalid dtype
    if (!method_valid(desc.method))
        throw Error(1, "Invalid downsampling method: " +
                         std::to_string(desc.method));
    ArrayDimensions ad(desc.dims, desc.dtype, desc.storage_order);
    levels_ = make_pyramid_levels(ad.dims(), desc.max_levels);
    const size_t n = ad.ndims();
    lv_.resize(levels_.size());
    for (size_t k = 0; k < levels_.size(); ++k) {
        Lv& L = lv_[k];
        L.W = levels_[k][n - 1].array_size_px;
        L.H = levels_[k][n - 2].array_size_px;
        L.planes = levels_[k][n - 3].array_size_px;
        L.xy_shrinks = k > 0 && (L.W < lv_[k - 1].W || L.H < lv_[k - 1].H);
    }
    hip_check(hipSetDevice(device_), "hipSetDevice");
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking),
              "hipStreamCreate");
}

GpuDownsampler::~GpuDownsampler()
{
    if (stream_) {
        (void)hipStreamSynchronize(stream_);
        (void)hipStreamDestroy(stream_);
    }
}

const std::vector<Dim>&
GpuDownsampler::level_dims(uint32_t level) const
{
    if (level >= levels_.size())
        throw Error(3, "level out of range");
    return levels_[level];
}

void
GpuDownsampler::add_frame(const void* frame, size_t nbytes, int mem)
{
    // downsampler.cpp:306-401
    const uint64_t fb0 = uint64_t(lv_[0].W) * lv_[0].H * bpp_;
    if (!frame || nbytes < fb0)
        throw Error(1, "Expecting at least " + std::to_string(fb0) + " bytes");
    hip_check(hipSetDevice(device_), "hipSetDevice");
    input_.alloc(fb0);
    hip_check(hipMemcpyAsync(input_.p, frame, fb0, kind_from(mem, kMemDevice),
                             stream_),
              "hipMemcpyAsync");
    ++lv_[0].count;

    // Plan this frame's cascade on the host, then run one launch per level.
    std::vector<LevelOp> ops;
    std::vector<uint32_t> op_level;
    const uint8_t* cur = input_.p;
    for (uint32_t k = 1; k < lv_.size(); ++k) {
        Lv& L = lv_[k];
        Lv& P = lv_[k - 1];
        const uint64_t lfb = uint64_t(L.W) * L.H * bpp_;
        L.cur.alloc(lfb);
        L.pending.alloc(lfb);
        L.partial.alloc(lfb);
        bool average = L.planes < P.planes;
        if (P.planes % 2 != 0 && P.count % P.planes == 0)
            average = false;
        LevelOp o{};
        if (average && !L.has_partial) {
            // partial_scaled_frames_.emplace + break (:386-389)
            o.a = cur;
            o.a_scale = L.xy_shrinks;
            o.scratch_out = L.partial.p;
            ops.push_back(o);
            op_level.push_back(k);
            L.has_partial = true;
            break;
        }
        if (average) {
            o.a = L.partial.p; // earlier plane, already XY-scaled
            o.b = cur;
            o.b_scale = L.xy_shrinks;
            L.has_partial = false;
        } else {
            o.a = cur;
            o.a_scale = L.xy_shrinks;
        }
        o.scratch_out = L.cur.p;
        ops.push_back(o);
        op_level.push_back(k);
        // emplace_downsampled_frame_ (:599-605): a waiting frame is kept,
        // the count advances regardless
        ++L.count;
        if (!L.has_pending) {
            std::swap(L.cur, L.pending);
            L.has_pending = true;
            cur = L.pending.p;
        } else {
            cur = L.cur.p;
        }
    }
    if (!ops.empty()) {
        d_op_.alloc(ops.size() * sizeof(LevelOp));
        hip_check(hipMemcpyAsync(d_op_.p, ops.data(), ops.size() * sizeof(LevelOp),
                                 hipMemcpyHostToDevice, stream_),
                  "hipMemcpyAsync");
        for (size_t j = 0; j < ops.size(); ++j) {
            const uint32_t k = op_level[j];
            LevelParams lp{};
            lp.Wp = lv_[k - 1].W;
            lp.Hp = lv_[k - 1].H;
            lp.g.W = lv_[k].W;
            lp.g.H = lv_[k].H;
            lp.ops = reinterpret_cast<const LevelOp*>(d_op_.p) + j;
            lp.n_ops = 1;
            hip_check(launch_level(dtype_, method_, lp, stream_),
                      "level launch");
        }
    }
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
}

bool
GpuDownsampler::take_frame(uint32_t level, void* dst, size_t cap, int mem,
                           size_t* nbytes)
{
    // downsampler.cpp:403-414
    if (level == 0 || level >= lv_.size() || !lv_[level].has_pending)
        return false;
    Lv& L = lv_[level];
    const size_t fb = size_t(L.W) * L.H * bpp_;
    if (nbytes)
        *nbytes = fb;
    if (dst) {
        if (cap < fb)
            throw Error(2, "destination too small");
        hip_check(hipMemcpy(dst, L.pending.p, fb, kind_from(kMemDevice, mem)),
                  "hipMemcpy");
    }
    L.has_pending = false;
    return true;
}

const char*
GpuDownsampler::method_name() const
{
    return downsampling_method_name(method_);
}

std::string
GpuDownsampler::metadata_json() const
{
    return downsampling_metadata_json(method_);
}

// Downsampler::downsampling_method (downsampler.cpp:422-438)
const char*
downsampling_method_name(int32_t method)
{
    switch (method) {
        case 0:
            return "decimate";
        case 1:
            return "local_mean";
        case 2:
            return "local_min";
        case 3:
            return "local_max";
        default:
            throw Error(1, "Invalid downsampling method: " + std::to_string(method));
    }
}

// Downsampler::get_metadata (downsampler.cpp:440-485) as nlohmann's
// json::dump() serialises it: compact, object keys sorted.  Byte-compared
// with the compiled reference (tests/test_metadata_cpu.py).
std::string
downsampling_metadata_json(int32_t method)
{
    switch (method) {
        case 1:
            return "{\"description\":\"The fields in the metadata describe how "
                   "to reproduce this multiscaling in scikit-image. The method "
                   "and its parameters are given here.\",\"kwargs\":{\"cval\":"
                   "\"0\",\"factors\":\"(2, 2)\"},\"method\":\"skimage."
                   "transform.downscale_local_mean\",\"version\":\"0.25.2\"}";
        case 0:
            return "{\"args\":[\"(slice(0, None, 2), slice(0, None, 2))\"],"
                   "\"description\":\"Subsampling by taking every 2nd "
                   "pixel/voxel (top-left corner of each 2x2 block). "
                   "Equivalent to numpy array slicing with stride 2.\","
                   "\"method\":\"np.ndarray.__getitem__\",\"version\":"
                   "\"2.2.6\"}";
        case 2:
            return "{\"description\":\"Minimum pooling over 2x2 blocks. "
                   "Equivalent to reshaping into blocks and taking numpy.min "
                   "along block dimensions.\",\"kwargs\":{\"func\":\"np.min\"},"
                   "\"method\":\"skimage.measure.block_reduce\",\"version\":"
                   "\"0.25.2\"}";
        case 3:
            return "{\"description\":\"Maximum pooling over 2x2 blocks. "
                   "Equivalent to reshaping into blocks and taking numpy.max "
                   "along block dimensions.\",\"kwargs\":{\"func\":\"np.max\"},"
                   "\"method\":\"skimage.measure.block_reduce\",\"version\":"
                   "\"0.25.2\"}";
        default:
            throw Error(1, "Invalid downsampling method: " + std::to_string(method));
    }
}

} // namespace aqz
