// wg_internal.hpp — host-side internals shared by the engine's translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wireglider_amd.h"

namespace wg {

// Launch geometry, read once from the environment (WG_L4_BLOCKS, ...; the
// accepted values are capi.hip's knob table, shared with wg_tune_set); the
// defaults are the measured best on MI355X.
struct Tune {
    uint64_t l4_blocks;   // grid cap for the wave-per-packet checksum kernels
    uint32_t l4_nt;       // 1: non-temporal packet loads
    uint32_t l4_small;    // descriptor-batch kernel: 5 split roles (default), 0 wave-per-packet
    uint32_t l4_small_uniform;  // 2: uniform batches with segment_size <= 64 a lane per segment; 0 the wave kernel
    uint64_t gso_blocks;  // grid cap for the GSO split kernel (one block per super-buffer)
    uint32_t gso_waves;   // waves per block (1, 2, 4, 8)
    uint32_t gso_split;   // blocks per super-buffer (grid y)
    uint32_t gso_groups;  // blocks per super-buffer, consecutive in the flat grid (one-shot waves)
    uint32_t gso_spw;     // segments per wave step: 0 one at a time, 1 ping-pong pipeline, 2-4 issued together
    uint32_t encap_spw;   // the same for the encap step's headers-only split
    uint32_t verify_small;  // 7 per-call choice (default), 0 wave kernel, 6 compacting path, 8 walking kernel
    uint32_t verify_auto_t;  // verify_small = 7: compacting path when >= this many of 64 sampled packets are small
    uint32_t verify_k2min;   // compacting path: minimum blocks of the long kernel
    uint32_t host_chunk_mb;  // host-memory pipeline chunk size, MiB
    uint32_t host_d2h;    // host pipeline downloads into pinned memory by a store kernel (bit 1 encap messages, bit 2 every decap plaintext chunk, bit 4 decap plaintext chunks < 24 MiB)
    uint32_t l4_unroll;   // split kernel: loads in flight per lane on a long packet's rest (4, 8)
    uint64_t l4_coop;     // descriptor batches of n <= l4_coop: a block of l4_coop_waves waves per packet (0: never)
    uint32_t l4_coop_waves;  // waves per packet in that mode (2, 4, 8, 16)
    uint32_t aead_k;      // AEAD: consecutive ChaCha20 blocks per lane (0 = 2 or 3 per batch, 2, 3)
    uint32_t aead_stage;  // AEAD encrypt: messages assembled in LDS, written out in whole lines (1)
    uint32_t encap_parts; // wg_encap_batch: slices split on a side stream under the previous slice's AEAD (1 = off)
    uint32_t encap_synth; // wg_encap_batch: the AEAD builds eligible segments' headers, the split skips them
    uint32_t gso_ablate;  // GSO A/B variants (1 non-temporal stores, 32 no XCD swizzle; both correct)
    uint32_t lane_coop;   // split kernel's lane role: 1 small packets' chunks loaded by the wave together (default), 0 per lane
};

// A snapshot of the knobs: a copy of the current immutable table, read
// lock-free (wg_tune_set may run concurrently on another host thread and
// publishes a new table; capi.hip).
Tune tune();

// Debugging aid: with WG_DEBUG_SYNC=1 in the environment, synchronise the
// stream after a launch and report a failing kernel by name on stderr.
// Returns false when the kernel failed.
bool debug_sync(hipStream_t st, const char *kernel);

// wg_gso_split's three launches (gso.hip); hdr_only = wg_encap_batch's
// headers-only split (segment headers written, payload left in the input);
// synth (non-null): its super-buffers that pass syn_eligible and whose
// messages fit these bounds (encap_fit) are not split at all (the encap
// AEAD writes their headers); list (nullable, 4 * (n + 1) bytes of device
// scratch): the plan kernel lists the rest and the split walks only those.
struct EncapFit {
    uint32_t msg_cap, max_segments, max_segment_size;
};
int gso_split_launch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                     wg_gso_result *dev_res, bool hdr_only, hipStream_t st, const EncapFit *synth = nullptr,
                     uint32_t *list = nullptr);

// wg_encap_batch with a device-resident counter base (aead.hip): counters
// start at counter0 + *dev_base (nullable: 0) and *dev_total gets *dev_base +
// this call's messages, so the host path chains its chunks on the device.
int encap_batch_launch(uint8_t *dev_in, const wg_gso_desc *dev_desc, uint64_t n, uint8_t *dev_out,
                       wg_gso_result *dev_gso_res, const uint8_t key[32], uint32_t receiver_index, uint64_t counter0,
                       const uint64_t *dev_msg_offset, uint32_t msg_cap, uint32_t max_segments,
                       uint32_t max_segment_size, uint8_t *dev_msgs, wg_encap_result *dev_res, uint32_t *dev_work,
                       uint64_t *dev_total, const uint64_t *dev_base, hipStream_t st);

}  // namespace wg
