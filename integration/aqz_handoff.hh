// aqz_handoff.hh -- the consumer-thread side of the MI355X stage for one
// multiscale array, independent of zarr::Array so that it runs (and is
// tested, tests/native/handoff_replay.cpp) without the reference library.
//
// It replaces, for a multiscale array, what the reference's consumer thread
// does per frame (MultiscaleArray::write_frame, multiscale.array.cpp:57-74,
// 291-325, and Array::write_frame, array.cpp:153-223):
//
//   * frames are copied into one of two pinned batch buffers; a full batch
//     is appended asynchronously (aqz_stage_append reads pinned memory by
//     DMA) and the buffer is refilled only after aqz_stage_wait_consumed
//     says the stage has read it -- the frame queue's buffer swap
//     (frame.queue.cpp:48-73) without a spin;
//   * every complete unit of every level -- a dim-1 band where
//     Array::flush_completed_bands_ applies (array.cpp:873-908), else a
//     chunk layer -- is copied D2H asynchronously into a ring of pinned host
//     buffers (aqz_stage_copy_band_async / aqz_stage_copy_layer_async);
//   * a unit whose copy has landed (aqz_stage_copies_completed: hand-off
//     tickets complete in issue order) is installed into the caller's chunk
//     buffers and committed -- the tail of Array::write_frame that triggers
//     flush / rollover (array.cpp:196-219) -- strictly in frame order per
//     level.  Nothing waits for a copy except to reuse its host buffer.
#pragma once

#include "aqz_gpu.h"

#include <algorithm>
#include <cstring>
#include <deque>
#include <vector>

namespace aqz_binding {

// Where handed-off units go (GpuArray in the reference binding).
struct HandoffSink
{
    virtual ~HandoffSink() = default;
    // chunk slots [c0, c0 + n) of level's current layer: n chunks of
    // bytes_per_chunk bytes and their has_data bytes
    virtual void install(uint32_t level, const uint8_t* chunks, const uint8_t* has_data,
                         uint32_t c0, uint32_t n) = 0;
    // `frames` more frames of level are in its chunk buffers; flush = false
    // only for the zero-filled partial last unit (Array::close_ flushes it)
    virtual aqz_status commit(uint32_t level, uint64_t frames, bool flush) = 0;
};

class Handoff
{
  public:
    // host_slots: pinned unit buffers per level (>= 1; 2-3 keep the D2H of
    // one unit in flight while an earlier one is installed)
    Handoff(aqz_stage* st, uint64_t frame_bytes, uint32_t batch, uint32_t host_slots,
            HandoffSink& sink)
      : st_(st)
      , frame_bytes_(frame_bytes)
      , batch_(batch)
      , sink_(sink)
    {
        host_slots = std::max<uint32_t>(1, host_slots);
        for (int j = 0; j < 2; ++j)
            status_ = worse(status_, aqz_host_alloc(size_t(batch_) * frame_bytes_,
                                                    reinterpret_cast<void**>(&buf_[j])));
        const uint32_t nl = aqz_stage_n_levels(st_);
        levels_.resize(nl);
        for (uint32_t l = 0; l < nl && status_ == AQZ_STATUS_SUCCESS; ++l) {
            Level& L = levels_[l];
            status_ = worse(status_, aqz_stage_level_layout(st_, l, &L.lay));
            int32_t banded = 0;
            status_ = worse(status_, aqz_stage_band_geometry(st_, l, &banded, &L.n_bands,
                                                             &L.frames_per_band,
                                                             &L.chunks_per_band));
            L.banded = banded != 0;
            L.unit = L.banded ? L.frames_per_band : L.lay.frames_per_layer;
            L.slots.resize(host_slots);
            for (Slot& s : L.slots) {
                status_ = worse(status_, aqz_host_alloc(unit_bytes(L),
                                                        reinterpret_cast<void**>(&s.chunks)));
                status_ = worse(status_, aqz_host_alloc(L.chunks_per_band,
                                                        reinterpret_cast<void**>(&s.has)));
            }
        }
    }

    ~Handoff()
    {
        // a unit still in flight must land before its buffer is freed
        (void)aqz_stage_wait_copies(st_);
        for (Level& L : levels_)
            for (Slot& s : L.slots) {
                aqz_host_free(s.chunks);
                aqz_host_free(s.has);
            }
        for (uint8_t* b : buf_)
            aqz_host_free(b);
    }

    Handoff(const Handoff&) = delete;
    Handoff& operator=(const Handoff&) = delete;

    aqz_status status() const { return status_; }
    uint64_t frames_accepted() const { return accepted_; }

    // pinned host bytes held (batch buffers + unit rings)
    size_t host_bytes() const
    {
        size_t n = 2 * size_t(batch_) * frame_bytes_;
        for (const Level& L : levels_)
            n += L.slots.size() * (unit_bytes(L) + L.chunks_per_band);
        return n;
    }

    // One level-0 frame (frame_bytes bytes).  Appends a full batch.
    aqz_status write_frame(const void* frame)
    {
        if (status_ != AQZ_STATUS_SUCCESS)
            return status_;
        if (n_batched_ == 0) {
            // refill only once the stage has read this buffer's last batch
            const aqz_status s = aqz_stage_wait_consumed(st_, end_[cur_]);
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
        }
        std::memcpy(buf_[cur_] + size_t(n_batched_) * frame_bytes_, frame, frame_bytes_);
        ++n_batched_;
        ++accepted_;
        if (n_batched_ == batch_)
            return append_batch_();
        return AQZ_STATUS_SUCCESS;
    }

    // MultiscaleArray::close_ (multiscale.array.cpp:112-135): the partial
    // batch, the zero-filled partial last layer of every level (chunk.cpp:
    // 8-15), every remaining unit installed.
    aqz_status close()
    {
        if (status_ != AQZ_STATUS_SUCCESS)
            return status_;
        aqz_status s = append_batch_();
        if (s != AQZ_STATUS_SUCCESS)
            return s;
        s = aqz_stage_finalize(st_);
        if (s != AQZ_STATUS_SUCCESS)
            return status_ = s;
        s = issue_(true);
        if (s != AQZ_STATUS_SUCCESS)
            return status_ = s;
        return retire_(true);
    }

  private:
    struct Slot
    {
        uint8_t* chunks = nullptr;
        uint8_t* has = nullptr;
        bool busy = false;
    };
    struct Level
    {
        aqz_level_layout lay{};
        bool banded = false;
        uint32_t n_bands = 1, chunks_per_band = 0;
        uint64_t frames_per_band = 0, unit = 0;
        uint64_t issued = 0; // frames of this level handed off (copies issued)
        std::vector<Slot> slots;
        uint32_t next = 0;
    };
    struct Unit
    {
        uint32_t level, slot, band;
        uint64_t frames;
        bool flush;
        uint64_t ticket;
    };

    static aqz_status worse(aqz_status a, aqz_status b)
    {
        return a != AQZ_STATUS_SUCCESS ? a : b;
    }
    static size_t unit_bytes(const Level& L)
    {
        return size_t(L.lay.bytes_per_chunk) * L.chunks_per_band;
    }

    aqz_status append_batch_()
    {
        if (n_batched_ == 0)
            return AQZ_STATUS_SUCCESS;
        const aqz_status s =
          aqz_stage_append(st_, buf_[cur_], n_batched_, AQZ_MEM_HOST_PINNED);
        if (s != AQZ_STATUS_SUCCESS)
            return status_ = s;
        end_[cur_] = accepted_;
        cur_ ^= 1;
        n_batched_ = 0;
        const aqz_status h = issue_(false);
        if (h != AQZ_STATUS_SUCCESS)
            return status_ = h;
        return retire_(false);
    }

    // Copy every complete unit of every level D2H (final: the partial last
    // one too) into a free host buffer of its level.
    aqz_status issue_(bool final)
    {
        for (uint32_t l = 0; l < levels_.size(); ++l) {
            Level& L = levels_[l];
            const uint64_t written = aqz_stage_frames_written(st_, l);
            while (L.issued + L.unit <= written || (final && L.issued < written)) {
                Slot& slot = L.slots[L.next];
                while (slot.busy) { // its unit has not been installed yet
                    const aqz_status s = retire_one_(true);
                    if (s != AQZ_STATUS_SUCCESS)
                        return s;
                }
                const uint64_t F = L.lay.frames_per_layer;
                const uint64_t layer = L.issued / F;
                const uint32_t band = L.banded ? uint32_t((L.issued % F) / L.unit) : 0;
                aqz_status s;
                if (L.banded)
                    s = aqz_stage_copy_band_async(st_, l, layer, band, slot.chunks,
                                                  unit_bytes(L), slot.has, L.chunks_per_band);
                else
                    s = aqz_stage_copy_layer_async(st_, l, layer, slot.chunks, unit_bytes(L),
                                                   slot.has, L.chunks_per_band);
                if (s != AQZ_STATUS_SUCCESS)
                    return s;
                const uint64_t n = std::min(L.unit, written - L.issued);
                pending_.push_back(Unit{ l, L.next, band, n, n == L.unit,
                                         aqz_stage_last_ticket(st_) });
                slot.busy = true;
                L.issued += n;
                L.next = (L.next + 1) % uint32_t(L.slots.size());
            }
        }
        return AQZ_STATUS_SUCCESS;
    }

    // Install the oldest pending unit (wait: block until its copy landed;
    // else only if it has).  Tickets complete in issue order, so pending_ is
    // retired in frame order per level.
    aqz_status retire_one_(bool wait)
    {
        if (pending_.empty())
            return AQZ_STATUS_SUCCESS;
        const Unit u = pending_.front();
        if (wait) {
            const aqz_status s = aqz_stage_wait_ticket(st_, u.ticket);
            if (s != AQZ_STATUS_SUCCESS)
                return s;
        } else if (aqz_stage_copies_completed(st_) < u.ticket) {
            return AQZ_STATUS_SUCCESS;
        }
        pending_.pop_front();
        Level& L = levels_[u.level];
        Slot& slot = L.slots[u.slot];
        sink_.install(u.level, slot.chunks, slot.has, u.band * L.chunks_per_band,
                      L.chunks_per_band);
        slot.busy = false;
        return sink_.commit(u.level, u.frames, u.flush);
    }

    aqz_status retire_(bool wait_all)
    {
        while (!pending_.empty()) {
            const uint64_t before = pending_.size();
            const aqz_status s = retire_one_(wait_all);
            if (s != AQZ_STATUS_SUCCESS)
                return status_ = s;
            if (pending_.size() == before) // the oldest copy is still in flight
                break;
        }
        return AQZ_STATUS_SUCCESS;
    }

    aqz_stage* st_;
    const uint64_t frame_bytes_;
    const uint32_t batch_;
    HandoffSink& sink_;
    aqz_status status_ = AQZ_STATUS_SUCCESS;
    uint8_t* buf_[2] = { nullptr, nullptr };
    uint64_t end_[2] = { 0, 0 }; // frames accepted when each buffer was appended
    int cur_ = 0;
    uint32_t n_batched_ = 0;
    uint64_t accepted_ = 0;
    std::vector<Level> levels_;
    std::deque<Unit> pending_;
};

} // namespace aqz_binding
