// rt_device.h — parameters shared by the host launcher (rt_host.cpp) and the HIP kernels
// (rt_kernel.hip). Plain POD records (HIP vector types only), included by both sides.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rt {

// Work decomposition:
//   pixel enumeration i in [0, n_pixels): the rows of this render (y = row_offset + rr*row_stride),
//     in 8x8 tiles while both W and the row count allow, row-major for the remainder;
//   slots: the reference averages samples with libstdc++'s blocked reduce (<numeric>:443-460):
//     ((c0+c1)+(c2+c3)) per block of 4, blocks added in order, then the spp%4 tail one by one.
//     Slot k < G4 = spp/4 holds the block sum of samples 4k..4k+3; slot G4+j holds tail sample
//     4*G4+j. A work item = (pixel, a group of up to K consecutive block slots) or (pixel, one
//     tail slot): one lane traces the group's 4K samples (or the tail sample) back to back and
//     writes each block's sum to its own slot, so the summation order does not depend on K.
//   items of one launch: slots [slot_begin, slot_end) x all pixels; per pixel, in this order,
//     n_groups block groups (slot_begin + g*K .. min(+K, group_end)), then the split blocks
//     [group_end, group_end + n_split4/4) one sample per item, then the tail slots from
//     tail_base. Item I -> ls = I / n_pixels, pixel I % n_pixels. The split blocks come last so
//     the launch drains on short items (a long item on a deep path keeps its wave, and the
//     CU, running after the queues are dry); their 4 samples land in n_split4 extra slots
//     after the n_local regular ones and accumulate_kernel forms ((c0+c1)+(c2+c3)) from them.
//     Chunks of 64 consecutive items are dealt from 8 queues (chunk c belongs to queue c % 8)
//     by per-queue atomic counters.
// Per-render constants used only where a sample or an item starts (the kernel re-reads them
// from the kernarg segment at each use; see render_kernel).
// Exact unsigned division by a per-render invariant d (Granlund-Montgomery, "round-up with
// add"): q = (t + ((n - t) >> 1)) >> (l - 1), t = mulhi(n, m), for every 32-bit n.
struct UDiv {
    uint32_t m, l;   // l = ceil(log2 d) (>= 1), m = floor(2^32 (2^l - d) / d) + 1; d = 1: l = 0
};

struct FrameConsts {
    float org[3], llc[3], hor[3], ver[3];
    float lens, fW, fH;
    uint32_t corrected, W, spp;
    uint32_t inc_data_lo, inc_data_hi, inc_cam_lo, inc_cam_hi;
    uint32_t row_offset, row_stride, tiled_rows, tiles_x, n_pixels, g4, slot_begin, kblk;
    uint32_t n_groups, group_end, tail_base, n_split4, n_local, pad_[3];
    UDiv div_W, div_tiles_x, div_n_pixels;
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
    uint32_t n_pixels, tiles_x, tiled_rows;  // tiled_rows: rows covered by 8x8 tiles (0 = untiled)
    uint32_t g4, n_slots;                   // full blocks of 4, total slots
    uint32_t slot_begin, slot_end;          // this launch's slots
    uint32_t kblk;                          // block slots per work item (K >= 1)
    uint32_t n_split;                       // last blocks of the pass traced one sample per item
    uint32_t n_items, n_chunks;
    // scene
    uint32_t n_spheres, n_materials;
    // scene blob, staged whole into LDS: [geo: n_geo float4 {cx, cy, cz, fl(r*r)}]
    // [sidx: n_geo u32 original indices, padded to 16 B][clusters: n_clusters x 2 float4].
    // geo = the always-tested list (n_always, multiple of 8) then each cluster's members
    // (padded to 8); padding entries have r*r = -inf and never hit.
    const float4 *blob;
    uint32_t blob_units;     // 16-byte units
    uint32_t n_geo, n_always, n_clusters, clus_offset;
    uint32_t n_clusters_real;  // n_clusters counts never-entered padding boxes (multiple of 4)
    uint32_t n_supers, supers_offset;  // level 2: groups of 4 consecutive clusters, 2 float4 each
    float clus_pad;          // max over clusters of 1e-3 * (|C|_1 + |e|_1) + 1e-6 (per-ray pad adds 1e-3 |o|_1)
    // per-sphere hit record joined with its material, indexed by original sphere index:
    // {cx, cy, cz, r}, {albedo rgb, param}, {kind, 0, 0, 0}
    const float4 *hitrec;
    // outputs / workspace
    float *slots;            // [slot_end - slot_begin][n_pixels][3]
    uint32_t *queue_ctr;     // [8]
    unsigned long long *segments;  // optional [3]: segments, sphere tests, cluster box tests
    unsigned long long *dbg;       // [kDbgWords] diagnostics (V_STATS_LDS only)
};

struct KAccum {
    const float *slots;      // [n_local_slots + 4 n_split][n_pixels][3]
    float *acc;              // [n_pixels][3] running sum between passes
    float *out;              // final f32 RGB
    uint8_t *out_u8;         // optional gamma/u8 output (same layout)
    uint32_t n_pixels, n_local_slots;
    uint32_t split_local, n_split;  // local slots [split_local, +n_split) are summed from 4 samples
    uint32_t first, last, spp;
    uint32_t W, tiles_x, tiled_rows, row_offset, row_stride, full_frame;
};

// V_STATS_LDS diagnostics buffer: 16 counters, then {start, exit, iterations, hw id | refills}
// per wave
constexpr uint32_t kDbgWaves = 65536;
constexpr size_t kDbgWords = 16 + 4 * static_cast<size_t>(kDbgWaves);

enum Variant : int { V_EXACT_LDS = 0, V_EXACT_SCALAR = 1, V_FAST_LDS = 2, V_STATS_LDS = 3 };

} // namespace rt
