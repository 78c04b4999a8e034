// estimate_host -- aqz_binding::estimate_memory (integration/aqz_handoff.hh)
// on the CPU: the drop-in's host and device bytes for one multiscale array,
// as the binding would add them to ZarrStreamSettings_estimate_max_memory_
// usage (acquire.zarr.cpp:216-314).  Needs libaqz_gpu.so, no GPU.
//
//   estimate_host < JOBS      one job per line:
//     ndims {type size chunk shard} x ndims dtype batch host_slots codec
//     clevel shuffle n_stages max_batch_frames layer_slots placement_tries
//   stdout: one line per job: host_bytes device_bytes (or "error STATUS")
#include "aqz_handoff.hh"

#include <cstdio>
#include <vector>

int
main()
{
    unsigned nd = 0;
    while (std::scanf("%u", &nd) == 1) {
        std::vector<aqz_dimension> d(nd);
        for (auto& x : d)
            if (std::scanf("%d %u %u %u", &x.type, &x.array_size_px, &x.chunk_size_px,
                           &x.shard_size_chunks) != 4)
                return 2;
        int dtype = 0, codec = 0, clevel = 0, shuffle = 0;
        unsigned batch = 0, slots = 0, stages = 0, max_batch = 0, layer_slots = 0, tries = 0;
        if (std::scanf("%d %u %u %d %d %d %u %u %u %u", &dtype, &batch, &slots, &codec, &clevel,
                       &shuffle, &stages, &max_batch, &layer_slots, &tries) != 10)
            return 2;
        aqz_array_desc desc{ d.data(), d.size(), dtype, 1, 1, 0, nullptr, 0 };
        aqz_stage_options opt{};
        opt.max_batch_frames = max_batch;
        opt.layer_slots = layer_slots;
        opt.placement_tries = tries;
        aqz_binding::HandoffOptions ho;
        ho.batch_frames = batch;
        ho.host_slots = slots;
        ho.comp = aqz_compression{ codec, clevel, shuffle };
        aqz_binding::MemoryEstimate m{};
        const aqz_status s = aqz_binding::estimate_memory(desc, opt, ho, stages, &m);
        if (s != AQZ_STATUS_SUCCESS)
            std::printf("error %d\n", int(s));
        else
            std::printf("%llu %llu\n", (unsigned long long)m.host_bytes,
                        (unsigned long long)m.device_bytes);
    }
    return 0;
}
