// rt_device.h — parameters shared by the host launcher (rt_host.cpp) and the HIP kernels
// (rt_kernel.hip). Plain POD records (HIP vector types only), included by both sides.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_consts.h"

namespace rt {

// Work decomposition:
//   pixel enumeration i in [0, n_pixels): the rows of this render (y = row_offset + rr*row_stride),
//     in 64-pixel tiles (2^tile_lw x 64/2^tile_lw) while W and the row count allow, row-major
//     for the remainder;
//   a work item is one sample of one pixel: a lane traces it and stores its colour to the
//     sample's slot [s - sample_begin][i]. The reference averages samples with libstdc++'s
//     blocked reduce (<numeric>:443-460), ((c0+c1)+(c2+c3)) per block of 4, blocks in order,
//     then the spp%4 tail one by one; accumulate_kernel replays that order over the slots.
//     One-sample items keep every lane's unit of work short, so the launch drains evenly
//     (a multi-sample item on a deep path holds its wave long after the queues are dry).
//   items of one launch (a "pass"): samples [sample_begin, sample_end) x all pixels, item I ->
//     sample sample_begin + I / n_pixels, pixel I % n_pixels; passes start on multiples of 4.
//     Blocks of 64 consecutive items are dealt from 8 queues (queue q owns the q-th eighth of
//     the blocks) in guided chunks, one per-queue atomic ticket each.
// Per-render constants used only where a sample or an item starts (the kernel re-reads them
// from the kernarg segment at each use; see render_kernel).
struct FrameConsts {
    float org[3], llc[3], hor[3], ver[3];
    float lens, fW, fH;
    uint32_t corrected, W, spp;
    uint32_t inc_data_lo, inc_data_hi, inc_cam_lo, inc_cam_hi;
    uint32_t row_offset, row_stride, tiled_rows, tiles_x, n_pixels, sample_begin;
    UDiv div_W, div_tiles_x, div_n_pixels;
    uint32_t tile_lw;  // log2 of the tile width (3..6): tiles of 2^lw x 64/2^lw pixels
    float rW, rH;       // RN(1 / width), RN(1 / height)
    uint32_t div_fast;  // bit 0 / 1: x / width, x / height by rW / rH + one FMA correction is exact
    uint32_t n_pairs;   // sample pairs per pixel in this pass (KParams::n_pair_items / n_pixels)
};

// Sample pairs. The reference sums a pixel's samples as ((c0+c1)+(c2+c3)) per
// block of 4 (libstdc++ reduce): the pair sums c0+c1 and c2+c3 are all the accumulation needs of a
// block. A pass's full blocks are dealt as pair items — one lane traces samples 2j and 2j+1 of a
// pixel one after the other, parking c_2j in its LDS words, and stores RN(c_2j + c_2j+1) to
// the pair's slot (12 B per two samples); the pass's tail samples (spp % 4) stay single items.
// A main-launch lane keeps one word for its item: the item's slot (= its item index: pair items
// first, then the tail's single samples) in the low bits, these flags above; the pixel and the
// sample are re-derived from it where a sample starts.
constexpr uint32_t kItSlot = (1u << 29) - 1u;
constexpr uint32_t kItSecond = 1u << 31;     // tracing the pair's second sample
constexpr uint32_t kItFirstDeep = 1u << 30;  // the pair's first sample went to the deep queue
constexpr uint32_t kItRestart = 1u << 29;    // start the pair's second sample next iteration
// the deep queue's pair link of a path (DeepQueue::link): its role in the top two bits, the
// partner path's queue index below (both samples of a pair queued)
constexpr uint32_t kRoleSingle = 0u;       // a single sample: its colour is the slot's
constexpr uint32_t kRolePartnerDone = 1u;  // the partner's colour is in the pair's slot: add to it
constexpr uint32_t kRoleBothFirst = 2u;    // both samples queued; this is the first
constexpr uint32_t kRoleBothSecond = 3u;   // both samples queued; this is the second
constexpr uint32_t kLinkIndex = 0x3fffffffu;

// The deep queue of one workspace (structure of arrays, 8 regions of rcap paths): f =
// [9][8 rcap] floats {o.xyz, d.xyz, attenuation.xyz} of the next segment, the data-stream state,
// the sample's slot index, the path's hint sphere, its pair link and the both-deep arrival word
// (60 B per path). Region r is appended to by workgroups r mod 8; its counters sit in
// the workspace's queue-counter block, line r: word kDeepCount = paths appended (may exceed
// rcap: lanes past it keep their path), word kDeepDeal = the deep launch's dealing counter;
// they are reset with the queue counters.
struct DeepQueue {
    float *f;
    uint64_t *rng;
    uint32_t *slot;
    uint32_t *hid;           // the dielectric sphere the path last hit (its hint), ~0 = none
    uint32_t *ctr;           // the workspace's queue-counter block (8 x kQueueStride words)
    uint32_t *link;          // pair link (role << 30 | partner's index, kRole*)
    uint32_t *meet;          // both-deep pairs: arrivals at the first's index (0 between passes)
    uint32_t rcap;
    uint8_t *px;             // [n_pixels] 1: some sample of the pixel went to the queue (cleared by
                             // the accumulation that reads it)
};

struct KParams {
    FrameConsts fc;
    // camera basis (rt_camera)
    float org[3], llc[3], hor[3], ver[3];
    float lens;
    uint32_t corrected;
    // frame
    uint32_t W, H, spp, max_depth;
    uint32_t row_offset, row_stride, num_rows;
    uint32_t full_frame;
    uint64_t inc_data, inc_cam;  // PCG increments: ((2*seed) << 1) | 1 and ((2*seed+1) << 1) | 1
    // decomposition
    uint32_t n_pixels, tiles_x, tiled_rows;  // tiled_rows: rows covered by 64-pixel tiles (0 = untiled)
    uint32_t tile_lw;                       // log2 of the tile width (3: 8x8, 4: 16x4, 5: 32x2, 6: 64x1)
    uint32_t sample_begin, sample_end;      // this launch's samples
    uint32_t n_items;
    uint32_t n_slots;        // the pass's slots (bounds check): its slot rows x n_pixels (items may be fewer)
    uint32_t n_pair_items;   // items [0, n_pair_items) are sample pairs (FrameConsts::n_pairs x n_pixels),
                             // the rest single tail samples; the slot of item I is slot I either way
    uint32_t n_blocks;       // guided dealing: ceil(n_items / 64) blocks, 1/8 per queue
    float guided_l2b;        // log2(beta) < 0 of the guided dealing (rt_kernel.hip refill)
    // scene
    uint32_t n_spheres, n_materials;
    // scene blob, staged whole into LDS: [geo: n_geo float4 {cx, cy, cz, fl(r*r)}]
    // [sidx: n_geo u32 original indices, padded to 16 B][clusters: n_clusters x 2 float4].
    // geo = the always-tested list (n_always spheres, padded to 4) then each cluster's members
    // (padded to 8); padding entries have r*r = -inf and never hit.
    const float4 *blob;
    uint32_t blob_units;     // 16-byte units
    uint32_t n_geo, n_always, n_clusters, clus_offset;
    uint32_t n_supers, supers_offset;  // level 2: groups of kSuperClusters (8) consecutive clusters, 2 float4 each
    uint32_t use_root;       // level 3: one box over all clusters at supers_offset + 2 n_supers
    uint32_t iso;            // isolated-sphere shortcut of the walk (rt_kernel.hip hint_candidate)
    uint32_t transpose_max;  // clusters requested by at most this many lanes (<= 16) are tested transposed
    uint32_t fast_roots;     // scene and camera within 2^19 of the origin: short exact root forms (rt_kernel.hip RayDiv)
    float clus_pad;          // max over clusters of 1e-3 * (|C|_1 + |e|_1) + 1e-6 (per-ray pad adds 1e-3 |o|_1)
    // shading records in the blob at shade_offset, indexed by original sphere index:
    // {cx, cy, cz, r}, {albedo rgb, param} x n_spheres, then n_spheres kind bytes (16-B padded)
    uint32_t shade_offset;
    uint32_t lds_units;      // blob units staged in LDS: all of it, or the part before shade_offset
    uint32_t shade_lds;      // 1: shading records read from LDS, 0: from the global blob
    // outputs / workspace
    float *slots;            // [sample_end - sample_begin][n_pixels][3]
    uint32_t *queue_ctr;     // [8 x kQueueStride]: one counter per 256-B line
    unsigned long long *segments;  // optional [3]: segments, sphere tests, cluster box tests
    unsigned long long *dbg;       // [kDbgWords] diagnostics (V_STATS_LDS only)
    // deep-path split: a path that has traced deep_depth segments leaves the
    // launch through the deep queue (whole state, stream order unchanged) and a second launch
    // of the same kernel (deep_mode = the split depth) deals the queued paths densely over its lanes.
    DeepQueue deep;
    uint32_t deep_depth;     // 0: no split (and always 0 in the deep launch)
    uint32_t deep_mode;      // the deep launch: the split depth (its paths resume there); 0 otherwise
    uint32_t deep_prio;      // the deep launch's waves at the highest issue priority (s_setprio 3)
    uint32_t deep_static;    // the deep launch deals chunk j to wave j mod (waves of the grid), no atomics
    // instrumented kernel only (V_STATS_LDS): hint_candidate's neighbour slots formed without the
    // lane's own bound (the form before fd383c3), so that the bounds check sees stale words
    uint32_t diag_unbounded_nb;
    // Dealing order. The pixel enumeration is permuted by 64-pixel blocks:
    // position i holds pixel (block_perm[i / 64] * 64 + i % 64) of the natural enumeration
    // (identity when block_perm is null), and a pass's slots are [sample][position]. The
    // positions form n_groups groups [grp_pix[g], grp_pix[g + 1]): the lead tiles, the others,
    // the sky tiles. Group g's grp_items[g] items (sample-major over its positions, item J =
    // sample J / ng, position grp_pix[g] + J % ng) are dealt from 8 queues, queue q owning the q-th
    // eighth of its grp_blocks[g] blocks of 64; every wave deals group g from every queue before it
    // takes group g + 1. One group (natural order): item J = slot J.
    const uint32_t *block_perm;
    uint32_t n_groups;          // 1: natural order, 3: tile classes
    uint32_t grp_pix[4];
    uint32_t grp_items[3];
    uint32_t grp_blocks[3];     // (natural order: n_blocks, the last one possibly partial)
    UDiv div_grp[3];            // division by group g's position count
};

// V_STATS_LDS: every lane-computed index into the scene blob, the slots and the deep queue is
// checked against its bound before use; the first violation is recorded in dbg[kDbgError] as
// code << 32 | index (and the access is made at index 0 instead), rt_scene_debug_counters turns
// it into RT_ERR_DEVICE
constexpr uint32_t kDbgError = 15;
enum BoundsCode : uint32_t {
    BC_NONE = 0, BC_HINT_NB = 1, BC_SHADE = 2, BC_SLOT = 3, BC_DEEP_APPEND = 4, BC_DEEP_ITEM = 5,
    BC_DEEP_HINT = 6, BC_MEMBERS = 7, BC_DEEP_PX = 8
};

struct KAccum {
    const float *slots;      // [n_samples][n_pixels][3], first sample a multiple of 4; paired: the
                             // pass's 2 n_blocks pair sums, then its n_samples - 4 n_blocks tail samples
    uint32_t paired;
    float *acc;              // [n_pixels][3] running sum between passes
    float *out;              // final f32 RGB
    uint8_t *out_u8;         // optional gamma/u8 output (same layout)
    uint32_t n_pixels, n_samples;
    uint32_t n_blocks;       // full blocks of 4 among this pass's samples (the rest is the tail)
    uint32_t first, last, spp;
    uint32_t W, tiles_x, tiled_rows, row_offset, row_stride, full_frame, tile_lw;
    // frames in flight: thread 0 adds the render's internal segment counters to the caller's
    // and zeroes them
    unsigned long long *seg_from;
    unsigned long long *seg_to;
    // the render's queue counters, zeroed here for the next render on this workspace
    uint32_t *queue_reset;
    uint32_t queue_words;
    // deep-path split: a region appended past deep_rcap (paths left in the main launch) makes
    // the thread that resets its counter write deep_key (the render's camera key) to *deep_over,
    // host memory the library reads on later calls (no split for that camera on this scene)
    unsigned long long *deep_over;
    unsigned long long deep_key;
    uint32_t deep_rcap;
    const uint32_t *block_perm;  // the pass's permuted enumeration (KParams::block_perm), or null
    // positions from sky_pos0 on are the sky kernel's (n_pixels: none): skipped by every pass but
    // the last, whose accumulation divides their sums (at their sample-0 slots) by spp
    uint32_t sky_pos0;
    // split passes accumulate in two parts: part 1 (after the main launch, beside the deep one)
    // the pixels none of whose samples went to the deep queue, part 2 (after the deep launch)
    // the others, clearing their flags; part 3 (caller stream only): every pixel, clearing the
    // flags; part 0 (unsplit pass): every pixel
    uint8_t *deep_px;
    uint32_t part;
};

// RT_FLAG_CUDA_COMPAT: the semantics of the reference's CUDA variant (src/CUDA/cuda_impl.cu),
// see compat_kernel. One lane owns one pixel (its xorshift32 engine is sequential over the
// pixel's samples), lanes refill from a per-wave cursor over 64-pixel chunks.
struct KCompat {
    float org[3], llc[3], hor[3], ver[3];
    uint32_t W, H, spp, max_depth;
    uint32_t row_offset, row_stride, num_rows, full_frame;
    uint32_t seed;           // added to the pixel index x + y W (the reference: 0)
    uint32_t n_spheres, n_pixels, n_chunks;
    const float4 *shade;     // per sphere: {cx, cy, cz, r}, {albedo, param}, then n kind bytes
    float *out;
    uint32_t *ctr;
    unsigned long long *segments;  // optional [3]: segments, sphere tests, 0
};

// The sky kernel: every sample of the pixels of the tiles proven to send every
// primary ray to the sky, one thread per pixel, its samples summed in the reference's blocked
// order (main.cxx:205); sky position i's sum (not yet divided by spp) goes to sums[i - pos0].
struct KSky {
    FrameConsts fc;                // the frame (all of its samples: fc.spp; fc.sample_begin unused)
    const uint32_t *block_perm;
    uint32_t pos0, n_pix;          // the sky positions [pos0, pos0 + n_pix) of the enumeration
    float *sums;
    unsigned long long *segments;  // optional: adds n_pix * spp segments (no sphere test)
};

// The wavefront variant's ray queue (structure of arrays, capacity cap rays): f = [9][cap]
// floats {o.xyz, d.xyz, attenuation.xyz}, then the data-stream state, the item index (slot) and
// the segment count of each ray; count = rays in the queue.
struct RayQueue {
    float *f;
    uint64_t *rng;
    uint32_t *item, *depth, *count;
};
struct KWave {
    KParams p;
    RayQueue in, out;        // wave_gen_kernel writes `out`; wave_bounce_kernel reads `in`
    uint32_t cap;            // queue capacity (rays)
    uint32_t item_begin, n_chunk;  // wave_gen_kernel: items [item_begin, item_begin + n_chunk)
};

// queue counters sit on separate 256-byte lines so the 8 queues' atomics do not serialise
constexpr uint32_t kQueueStride = 64;
constexpr uint32_t kDeepDeal = 16;   // word of queue q's line (the deep launch deals while the queue counter is idle)
constexpr uint32_t kDeepCount = 32;  // word of queue q's line, in its second 128-B half

// V_STATS_LDS diagnostics buffer: 16 counters, then {start, exit, iterations, hw id | refills}
// per wave
constexpr uint32_t kDbgWaves = 65536;
// then kDbgEvents block-execution counters (rt_scene_debug_events)
constexpr uint32_t kDbgEvents = 32;
constexpr size_t kDbgEvBase = 16 + 4 * static_cast<size_t>(kDbgWaves);
constexpr size_t kDbgWords = kDbgEvBase + kDbgEvents;

enum Variant : int { V_EXACT_LDS = 0, V_EXACT_SCALAR = 1, V_FAST_LDS = 2, V_STATS_LDS = 3 };

} // namespace rt
