/*
 * rt_api.h — C-ABI boundary of the MI355X-native path tracer (librt_mi355x.so).
 *
 * This header is the drop-in boundary for the reference's accelerated render path.
 * The reference (Alabuta/RaytracingInOneWeekend) binds its accelerated renderer as
 *
 *     extern void cuda_impl(std::uint32_t width, std::uint32_t height,
 *                           std::vector<math::u8vec3> &image_texels);      // src/main.cxx:18
 *
 * defined at src/CUDA/cuda_impl.cu:384-453 and called once at src/main.cxx:114. That
 * entry has C++ linkage, hardcodes scene/camera/spp/depth and throws on error. The
 * entry points below replace it with a C ABI: plain pointers and sizes, POD records,
 * an int status (0 = RT_OK), no exceptions across the boundary, caller-owned host
 * buffers. The literal `cuda_impl`-shaped C++ drop-in lives in rt_render_impl.hpp.
 *
 * Semantics follow the reference CPU render path (src/main.cxx:120-215 with
 * src/raytracer.hxx, src/camera.hxx, src/math.hxx); the CUDA variant's own semantics
 * (src/CUDA/cuda_impl.cu) are selected with RT_FLAG_CUDA_COMPAT or rt_render_cuda_impl.
 *
 * Threading: every call is synchronous unless its name ends in _device; calls on one
 * rt_scene come from one host thread. Device calls on one rt_scene may use different
 * streams: a call on a new stream is ordered after the previous call's work. Errors: a negative status; rt_last_error() returns a
 * thread-local message for the last failing call on this thread.
 */
#ifndef RT_API_H
#define RT_API_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_API_VERSION 2  /* 2: rt_options (resource bounds and A/B toggles), rt_scene_usage */

/* ---- status codes ---------------------------------------------------------------- */
enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID = -1,     /* bad argument (null pointer, zero size, bad index)       */
    RT_ERR_DEVICE = -2,      /* HIP runtime error (no device, launch/alloc failure)     */
    RT_ERR_CAPACITY = -3,    /* caller buffer too small                                 */
    RT_ERR_UNSUPPORTED = -4, /* feature not available in this build / on this host     */
    RT_ERR_COMM = -5,        /* RCCL failure in the multi-GPU path                      */
    RT_ERR_IO = -6           /* file could not be opened or written (rt_write_ppm)       */
};

/* ---- scene records ----------------------------------------------------------------
 * rt_sphere replaces primitives::sphere {math::vec3 center; float radius;
 * std::size_t material_index;} (src/primitives.hxx:6-17). A negative radius is legal
 * and flips the normal (hollow bubble, src/main.cxx:129; src/raytracer.hxx:71).      */
typedef struct rt_sphere {
    float center[3];
    float radius;
    uint32_t material;
} rt_sphere;

/* rt_material replaces material::types = std::variant<lambert, metal, dielectric>
 * (src/material.hxx:12-51). `param` is metal::roughness or dielectric::refraction_index
 * (unused for lambert).                                                               */
enum rt_material_kind { RT_LAMBERT = 0, RT_METAL = 1, RT_DIELECTRIC = 2 };
typedef struct rt_material {
    uint32_t kind;
    float albedo[3];
    float param;
} rt_material;

/* ---- camera -----------------------------------------------------------------------
 * Precomputed basis of raytracer::camera (src/camera.hxx:24-44); build it with
 * rt_camera_init() so the host arithmetic matches the reference constructor bit for bit.
 * mode RT_CAMERA_REFERENCE reproduces camera::ray() (src/camera.hxx:46-57) as shipped,
 * whose direction omits "- origin"; RT_CAMERA_CORRECTED subtracts the origin.        */
enum rt_camera_mode { RT_CAMERA_REFERENCE = 0, RT_CAMERA_CORRECTED = 1 };
typedef struct rt_camera {
    float origin[3];
    float lower_left_corner[3];
    float horizontal[3];
    float vertical[3];
    float lens_radius;
    uint32_t mode;
} rt_camera;

/* ---- render parameters ------------------------------------------------------------
 * width/height: FULL image size (u = x/width, v = y/height as src/main.cxx:192,195).
 * spp: samples per pixel (app::data::sampling_number, src/main.cxx:23).
 * max_depth: bounce limit (raytracer::data::bounces_number = 64, src/raytracer.hxx:20).
 * seed: RNG seed. Each (pixel, sample) owns two PCG32 streams keyed by
 *       key = (y*width + x)*spp + s — data stream seq 2*seed, camera stream seq 2*seed+1 —
 *       so any row partition renders the same bits.
 * Rows rendered: y_i = row_offset + i*row_stride for i in [0, num_rows). num_rows = 0
 *       means "all rows of the stride pattern below height".
 * Output layout: row-major RGB f32, 3 floats per pixel. With RT_FLAG_FULL_FRAME the
 *       output is indexed by the global row y (buffer of height*width*3 floats);
 *       otherwise rows are packed in render order (num_rows*width*3 floats).          */
enum rt_flags {
    RT_FLAG_FULL_FRAME = 1u << 0, /* write rows at their global position             */
    RT_FLAG_FAST_MATH = 1u << 1,  /* FMA-contracted kernel, stated tolerance          */
    RT_FLAG_SCALAR_SCENE = 1u << 2, /* A/B: brute force, spheres via the scalar cache   */
    RT_FLAG_BRUTE_FORCE = 1u << 3,  /* test every sphere (no cluster culling); same bits */
    RT_FLAG_CUDA_COMPAT = 1u << 4,  /* semantics of the reference's CUDA variant instead of its
                                       CPU path: src/CUDA/cuda_impl.cu (see rt_render_cuda_impl) */
    RT_FLAG_WAVEFRONT = 1u << 5     /* A/B: the wavefront variant (one launch per segment, ray
                                       queues in HBM) instead of the persistent megakernel;
                                       same bits, cluster culling; rt_options.wave_queue_rays
                                       bounds a chunk (2^25 rays, 52 B each, two queues)       */
};
typedef struct rt_params {
    uint32_t width, height;
    uint32_t spp, max_depth;
    uint64_t seed;
    uint32_t row_offset, row_stride, num_rows;
    uint32_t flags;
} rt_params;

typedef struct rt_stats {
    uint64_t primaries;  /* pixel-samples traced (W*rows*spp)                          */
    uint64_t segments;   /* hit_world() calls = ray segments traced                    */
    uint64_t sphere_tests; /* ray-sphere tests executed (lane level)                   */
    uint64_t box_tests;  /* cluster AABB tests executed (lane level)                    */
    double kernel_ms;    /* render kernel time (HIP events)                            */
    double wall_ms;      /* whole call: upload + kernel + download                     */
} rt_stats;

/* ---- library ----------------------------------------------------------------------- */
int rt_version(void);
const char *rt_last_error(void);
int rt_device_count(int *count);

/* ---- options: resource bounds and same-bits variants of a scene ---------------------
 * rt_options_default() fills the library defaults; change fields, then pass the record to
 * rt_scene_create_ex / rt_multi_create_ex, or make it the process default
 * (rt_set_default_options) for scenes created without one: rt_scene_create, the synchronous
 * renders (rt_render_f32, rt_render_rgb8, rt_render_multi_*) and rt_multi_create.
 * The environment variable RT_OPTIONS ("key=value,key=value", keys as the field names, the
 * diag bits as ieee_roots=1 ...; rt_options_parse) is applied over the defaults once, at the
 * library's first use, so an unmodified caller (the reference's main() with the drop-in) can
 * be A/B-tested. Every value is checked: RT_ERR_INVALID names the field. No option changes
 * a rendered bit (every variant is the reference's arithmetic); they trade memory and speed. */
typedef struct rt_options {
    uint32_t size;                  /* sizeof(rt_options): the record's revision              */
    uint32_t render_streams;        /* frames in flight: internal render streams. 0 = auto
                                       (GPU_MAX_HW_QUEUES - 1, within 2..7), 1 = every kernel
                                       on the caller's stream, 2..8                           */
    uint32_t workspaces_per_stream; /* sample-slot workspaces per render stream, 1..2 (2)     */
    uint32_t deep_split;            /* paths past this many segments finish in a second, dense
                                       launch; 0 = no split, 1..1024 (8)      */
    uint64_t max_pass_bytes;        /* slot workspace of one pass (12 B per pixel and sample):
                                       12 B .. 2 GiB (2 GiB); frames above it run in passes    */
    uint64_t max_workspace_bytes;   /* cap on the scene's device workspaces (slots, deep-path
                                       queues, multi-pass sums, wavefront queues); 0 = none.
                                       Over it, workspaces per stream go to 1, then passes
                                       shrink (to 4 samples), then streams go; RT_ERR_CAPACITY
                                       if one 4-sample pass on the caller's stream does not fit */
    uint64_t deep_min_items;        /* a pass issued while no other render runs (a lone frame)
                                       is split only from this many samples (2^25); passes
                                       issued beside other renders are split at any size       */
    uint32_t cluster_size;          /* spheres per culling cluster, 4..64, a multiple of 4 (16);
                                       read when the scene is created                         */
    uint32_t transpose_max;         /* clusters requested by at most this many lanes run as
                                       (ray, member) pairs over the wave, 0..16 (16)           */
    uint32_t wave_queue_rays;       /* RT_FLAG_WAVEFRONT: rays per chunk, >= 64 (2^25)        */
    uint32_t diag;                  /* rt_diag bits (0)                                        */
    uint64_t ring_pass_bytes;       /* with frames in flight: slot workspace of a pass issued
                                       beside other renders, 0 or 12 B .. 2 GiB (384 MiB); the
                                       frame's samples are cut into equal passes of a multiple
                                       of 4 within it, if they hold 32 samples or more. A frame
                                       issued alone that fits max_pass_bytes runs in one pass in
                                       a workspace of its own. 0 = passes of max_pass_bytes     */
} rt_options;
enum rt_diag {
    RT_DIAG_IEEE_ROOTS = 1u << 0,      /* the IEEE sqrt/division sequences for every root     */
    RT_DIAG_NO_SHORTCUT = 1u << 1,     /* no walk shortcut for rays in glass balls            */
    RT_DIAG_NO_NEIGHBOURS = 1u << 2,   /* the shortcut for isolated balls only                */
    RT_DIAG_NO_ROOT_BOX = 1u << 3,     /* no level-3 box gate before the cluster walk         */
    RT_DIAG_SHADE_LDS = 1u << 4,       /* shading records forced into LDS ...                 */
    RT_DIAG_SHADE_GLOBAL = 1u << 5,    /* ... or into global memory (default: by occupancy)   */
    RT_DIAG_STATS = 1u << 6,           /* the instrumented kernel (rt_scene_debug_*)           */
    RT_DIAG_STATS_DEEP_ONLY = 1u << 7, /* with STATS: count the deep launch alone             */
    RT_DIAG_VERBOSE = 1u << 8,         /* print every launch's plan to stderr                 */
    RT_DIAG_STANDIN_TRANSPORT = 1u << 9, /* rt_multi with every rank on one device: the RCCL
                                          gather code path, RCCL replaced by stream-ordered
                                          device copies (tests of that path on one GPU)       */
    RT_DIAG_UNBOUNDED_NB = 1u << 10,    /* with STATS: the walk shortcut's neighbour slots formed
                                          without the lane's own bound (the pre-fd383c3 form),
                                          for the bounds check to report (rt_scene_debug_counters) */
    RT_DIAG_NO_PAIRS = 1u << 11,        /* one sample per item and slot, under a cap too        */
    RT_DIAG_PAIRS = 1u << 12,           /* sample pairs for passes in flight without a cap
                                          (otherwise taken only under max_workspace_bytes)    */
    RT_DIAG_IN_FLIGHT = 1u << 13,       /* every pass planned as if issued beside other renders
                                          (partial grid, ring pass, pairs if asked): tests of
                                          that plan that must not depend on timing             */
    RT_DIAG_NATURAL_ORDER = 1u << 14,   /* items dealt in the pixels' natural tile order (no
                                          tile classes, no sky path)           */
    RT_DIAG_NO_SKY = 1u << 15,          /* tile classes order the dealing, but the tiles proven
                                          to send every primary ray to the sky are dealt last by
                                          the main launch (traced) instead of the sky kernel   */
    RT_DIAG_LONE_UNSPLIT = 1u << 16,    /* a lone pass dealt by tile classes is not split (its
                                          trapped paths start in its first items)              */
    RT_DIAG_SKY_SERIAL = 1u << 17       /* a lone pass's sky kernel after its main and deep
                                          launches on their stream (not beside them)           */
};
int rt_options_default(rt_options *out);
/* Applies "key=value[,key=value...]" (fields above; diag bits as ieee_roots, no_shortcut,
 * no_neighbours, no_root_box, shade_lds, shade_global, stats, stats_deep_only, verbose,
 * standin_transport = 0/1) to *inout; RT_ERR_INVALID on an unknown key or a bad value.   */
int rt_options_parse(const char *text, rt_options *inout);
/* The options of scenes created without explicit ones (NULL: the library defaults).      */
int rt_set_default_options(const rt_options *options);
int rt_get_default_options(rt_options *out);

/* ---- host-side scene / camera construction ----------------------------------------- */
/* raytracer::camera ctor, src/camera.hxx:24-44 (aperture -> lens_radius = aperture/2). */
int rt_camera_init(const float position[3], const float lookat[3], const float up[3],
                   float aspect, float vfov_degrees, float aperture, float focus_distance,
                   uint32_t mode, rt_camera *out);
/* The reference's default camera for a width x height image: src/main.cxx:179-183.     */
int rt_camera_default(uint32_t width, uint32_t height, uint32_t mode, rt_camera *out);
/* Simple scene, src/main.cxx:120-129: 5 spheres, 4 materials.                          */
int rt_scene_simple(rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres,
                    rt_material *materials, uint32_t material_cap, uint32_t *n_materials);
/* The CUDA variant's hardcoded scene, src/CUDA/cuda_impl.cu:425-437: 5 spheres, 4 materials. */
int rt_scene_cuda(rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres,
                  rt_material *materials, uint32_t material_cap, uint32_t *n_materials);
/* The CUDA variant's camera, src/CUDA/cuda_impl.cu:371-375 (origin 0, look -z, vFOV 88,
 * focus 1; its rays carry no lens offset, camera.hxx:48-50).                            */
int rt_camera_cuda(uint32_t width, uint32_t height, rt_camera *out);
/* Huge random scene: simple scene + the generator of src/main.cxx:131-177 driven by
 * std::mt19937{seed} (the reference seeds from std::random_device). Namespace typo
 * fixed; a "type 3" draw pushes no material (as shipped), so such a sphere aliases the
 * next pushed material and trailing ones are resolved by one default material
 * (material::types{} = lambert{albedo 1}). Pass null buffers to query the counts.     */
int rt_scene_huge(uint32_t seed, rt_sphere *spheres, uint32_t sphere_cap, uint32_t *n_spheres,
                  rt_material *materials, uint32_t material_cap, uint32_t *n_materials);

/* The dealing order of the pass that camera + params describe on this scene:
 * its 64-pixel blocks (8x8 tiles, then row-major blocks of leftover rows) as dealt, perm[i] =
 * the natural block of dealing position i; n_lead blocks first (a primary ray can meet a
 * cluster's box), n_sky blocks last (every primary ray proven to meet no sphere: those samples
 * skip the closest-hit test). n_blocks = 0: the pass keeps the natural order (its pixel count is
 * not a multiple of 64). cap = 0 queries the counts. Host-only (no device needed).            */
int rt_tile_order(const rt_sphere *spheres, uint32_t n_spheres, const rt_material *materials,
                  uint32_t n_materials, const rt_camera *camera, const rt_params *params,
                  uint32_t *perm, uint32_t cap, uint32_t *n_blocks, uint32_t *n_lead, uint32_t *n_sky);

/* ---- synchronous host-buffer renders (the cuda_impl replacement) ------------------- */
/* These keep one device context per device between calls (the scene on the device, its
 * workspaces, the frame buffers), keyed by the scene's records and the process-default
 * options: a repeated call with the same scene renders without rebuilding anything, as the
 * reference's main() calls its entry once per frame (src/main.cxx:114). Another scene or
 * other default options rebuild it. Calls are serialised within the process.
 * rt_release_cached frees every such context (its device memory and streams).           */
int rt_release_cached(void);
/* Linear (pre-gamma) averaged RGB, f32. rgb_out: see rt_params output layout.          */
int rt_render_f32(const rt_sphere *spheres, uint32_t n_spheres,
                  const rt_material *materials, uint32_t n_materials,
                  const rt_camera *camera, const rt_params *params,
                  float *rgb_out, rt_stats *stats);
/* Gamma 1/2.2 + (uint8)(255*c) epilogue (src/main.cxx:39-45,77-85) fused on device.    */
int rt_render_rgb8(const rt_sphere *spheres, uint32_t n_spheres,
                   const rt_material *materials, uint32_t n_materials,
                   const rt_camera *camera, const rt_params *params,
                   uint8_t *rgb_out, rt_stats *stats);
/* Row-interleaved split over ngpu devices of this process (device i renders rows
 * y ≡ i mod ngpu), gathered to device 0 with RCCL over xGMI, then copied to rgb_out
 * (full frame, height*width*3 floats). ngpu <= 0 uses every visible device. One-shot:
 * builds and tears down an rt_multi context (below) around the frame.                 */
int rt_render_multi_f32(const rt_sphere *spheres, uint32_t n_spheres,
                        const rt_material *materials, uint32_t n_materials,
                        const rt_camera *camera, const rt_params *params, int ngpu,
                        float *rgb_out, rt_stats *stats);
/* The same with the gamma/u8 epilogue (src/main.cxx:39-45,77-85) run on every rank's tile
 * before the gather: 3 bytes per pixel cross xGMI instead of 12 (height*width*3 bytes).  */
int rt_render_multi_rgb8(const rt_sphere *spheres, uint32_t n_spheres,
                         const rt_material *materials, uint32_t n_materials,
                         const rt_camera *camera, const rt_params *params, int ngpu,
                         uint8_t *rgb_out, rt_stats *stats);

/* app::save_to_file (src/main.cxx:87-101): binary PPM "P6\n<width> <height>\n255\n"
 * followed by width*height RGB texels, row 0 first. RT_ERR_IO if the file cannot be
 * written (the reference throws "bad file").                                           */
int rt_write_ppm(const char *path, const uint8_t *rgb, uint32_t width, uint32_t height);

/* The literal replacement of the reference's accelerated entry point
 *     void cuda_impl(uint32_t width, uint32_t height, std::vector<u8vec3> &image_texels)
 * (src/main.cxx:18, defined src/CUDA/cuda_impl.cu:384-453): its scene and camera, 48 spp,
 * 32 bounces, one xorshift32 engine per pixel seeded with the pixel index, gamma 1/2.2 and
 * (uint8)(255 c). rgb_out: width*height*3 bytes, row 0 = top. Synchronous.
 * With RT_FLAG_CUDA_COMPAT in rt_params any scene/camera/spp/depth renders with those
 * semantics (seed is added to the pixel index; the camera's lens radius is not used).   */
int rt_render_cuda_impl(uint32_t width, uint32_t height, uint8_t *rgb_out);

/* ---- device-resident API (inputs resident in HBM, async on a caller stream) -------- */
typedef struct rt_scene rt_scene;
/* Uploads the scene to `device` (packed SoA).                   */
int rt_scene_create(const rt_sphere *spheres, uint32_t n_spheres,
                    const rt_material *materials, uint32_t n_materials, int device,
                    rt_scene **out);
/* The same with explicit options (NULL: the process default, rt_set_default_options).   */
int rt_scene_create_ex(const rt_sphere *spheres, uint32_t n_spheres,
                       const rt_material *materials, uint32_t n_materials, int device,
                       const rt_options *options, rt_scene **out);
int rt_scene_destroy(rt_scene *scene);
/* Enqueue one render for `stream` (a hipStream_t, or NULL for the null stream).
 * d_rgb: device buffer laid out as rt_params says. d_segments: optional device u64[3]
 * that accumulates {segments, sphere tests, cluster box tests} (zero it first). No
 * host sync (a call whose workspaces must grow, or be re-cut under max_workspace_bytes,
 * synchronises the device once, before enqueuing). The render kernels rotate over the
 * scene's internal render streams (rt_options.render_streams: by default the process's
 * hardware queues - 1, i.e. 3 at HIP's default GPU_MAX_HW_QUEUES=4 and at most 7) with
 * rt_options.workspaces_per_stream slot workspaces each, so consecutive frames overlap; they
 * read only the scene and the by-value arguments, and the writes to d_rgb / d_segments are
 * enqueued on `stream`, so results appear in stream order.                                   */
int rt_render_device(rt_scene *scene, const rt_camera *camera, const rt_params *params,
                     float *d_rgb, void *stream, uint64_t *d_segments);
/* Device memory a scene holds and how its renders are cut (after the last render call).  */
typedef struct rt_scene_usage {
    uint64_t device_bytes;     /* every device allocation of the scene                       */
    uint64_t workspace_bytes;  /* of which workspaces (bounded by max_workspace_bytes)       */
    uint32_t render_streams;   /* streams the last render rotated over (1: caller's only)    */
    uint32_t workspaces;       /* slot workspaces in use                                     */
    uint32_t pass_samples;     /* samples per pass of the last render                        */
    uint32_t static_lds_bytes; /* the culled render kernel's static LDS per workgroup        */
    uint32_t max_lds_bytes;    /* the device's LDS per workgroup                              */
    uint32_t deep_launch;      /* the last render's last deep-path launch: waves per workgroup
                                  (4: beside other renders; 8: a lone pass, shading records in
                                  LDS) | 16 when it dealt its chunks statically; 0 = none      */
    uint32_t pair_passes;      /* passes of the last render that stored sample pairs          */
    uint32_t split_passes;     /* passes of the last render with a deep-path launch           */
    uint32_t lead_tiles;       /* the last pass: 64-pixel tiles dealt first (a primary can meet
                                  a dielectric sphere), 0 = natural order      */
    uint32_t sky_tiles;        /* the last pass: tiles whose primaries are proven to reach the
                                  sky (dealt last, no closest-hit test)                        */
} rt_scene_usage;
int rt_scene_usage_get(const rt_scene *scene, rt_scene_usage *out);
/* Spans (ms, HIP events) of the render kernels of the most recent calls of
 * rt_render_device on this scene, oldest first: entry i runs from the start event of the
 * call's first pass to the end event of its last pass. Consecutive calls' launches run
 * side by side (frames in flight), so a span also covers time the GPU spent on other
 * calls' renders and accumulations: it is a latency, not a per-frame cost. Writes up to
 * `max` entries, *n = entries written. Waits for those calls to finish.                 */
int rt_scene_kernel_times(rt_scene *scene, uint32_t max, float *ms, uint32_t *n);
/* Diagnostics: with RT_DIAG_STATS in the scene's options, its renders use an
 * instrumented kernel (identical output) that tallies: [0] wave loop iterations,
 * [1] wave refill rounds, [2] wave / [3] lane sphere blocks with a positive discriminant,
 * [4] wave / [5] lane root evaluations, [6] segments, [7] wave-level blocks of 8 cluster
 * members executed, [8..12] shader-clock cycles summed over waves per loop region
 * (refill, sample start + rejection loop, closest hit, shading, fold), [13] items dealt (the
 * deep launch: queued paths), [14] ~(earliest wave
 * start, 100 MHz clock), [15] the bounds check's first violation, code << 32 | index
 * (rt_device.h BoundsCode; 0 = none). Copies them out; reset zeroes. Returns RT_ERR_DEVICE
 * (the message names the index) when [15] is set: the instrumented kernel checks every
 * lane-computed index into the scene, the sample slots and the deep queue before using it. */
int rt_scene_debug_counters(rt_scene *scene, uint64_t out[16], int reset);
/* Diagnostics: per-wave records of the last instrumented render launch, out[4w .. 4w+3] for
 * wave w of the grid = {time the wave found every queue dry, exit} (100 MHz realtime
 * clock), (shader-clock cycles in the loop << 32 | refill rounds << 16 | loop iterations),
 * and (hardware CU id << 48 | iterations after dry (a deep launch: iterations in which the wave
 * walked the clusters) << 32 | low 32 bits of the wave's start on
 * the realtime clock); at most max_waves records, *n = records written (0 without
 * RT_DIAG_STATS).                                                                            */
int rt_scene_debug_timeline(rt_scene *scene, uint64_t *out, uint32_t max_waves, uint32_t *n);
/* Diagnostics: with RT_DIAG_STATS, how often each block of the render loop ran, counted once
 * per wave per execution, summed over the instrumented launches since the last reset: [0] loop
 * iterations, [1] refill trips, [2] sample starts, [3] rejection attempts, [4] lens rays done,
 * [5] scatters done, [6] root-box passes, [7] level-2 boxes walked, [8] level-2 boxes passed,
 * [9] clusters requested, [10] transposed member tests, [11] their rounds, [12] their far-root
 * passes, [13] per-lane member tests, [14] sky, [15] hit shading, [16] lambert, [17] unit
 * direction (metal/dielectric), [18] dielectric, [19] sample stores, [20] metal absorptions,
 * [21] live lanes summed over iterations, [22] iterations after the item queues ran dry, [23]
 * live lanes summed over those, [24] lanes that skipped the walk (shortcut), [25] iterations
 * whose walk no lane needed, [26..29] iterations whose walk 1, 2, 3-4, 5-8 lanes needed.                                        */
int rt_scene_debug_events(rt_scene *scene, uint64_t out[32], int reset);
/* Enqueue the gamma/u8 epilogue over n_pixels RGB f32 texels.                          */
int rt_epilogue_rgb8_device(const float *d_rgb, uint8_t *d_out, uint64_t n_pixels,
                            void *stream);

/* ---- persistent multi-GPU context (row tiles over ranks, gather over xGMI) ----------
 * Rank r of n_ranks renders rows y = r, r + n, ... of every frame on device devices[r]
 * (devices = NULL: rank r on device r) into a packed tile; tiles are gathered to rank 0's
 * device with RCCL send/recv when every rank has its own device, and de-interleaved into
 * the caller's frame. Scenes, streams and communicators are built once here; tiles and the
 * gather buffer are allocated on first use of a frame size. Ranks that share a device with
 * rank 0 ("virtual ranks", e.g. devices = {0, 0, 0, 0}: an N-way split rehearsed on one
 * GPU) move their tiles with device copies instead of RCCL; the result is the same frame.
 * A device list is either all distinct or all equal to devices[0]; a mix is RT_ERR_INVALID. */
typedef struct rt_multi rt_multi;
enum rt_output_format { RT_OUTPUT_F32 = 0, RT_OUTPUT_RGB8 = 1 };
int rt_multi_create(const rt_sphere *spheres, uint32_t n_spheres,
                    const rt_material *materials, uint32_t n_materials,
                    const int *devices, int n_ranks, rt_multi **out);
/* The same with explicit options for every rank's scene (NULL: the process default).     */
int rt_multi_create_ex(const rt_sphere *spheres, uint32_t n_spheres,
                       const rt_material *materials, uint32_t n_materials,
                       const int *devices, int n_ranks, const rt_options *options,
                       rt_multi **out);
int rt_multi_destroy(rt_multi *ctx);
/* n_ranks, and whether the gather runs over RCCL (1) or device copies (0).              */
int rt_multi_info(const rt_multi *ctx, int *n_ranks, int *uses_rccl);
/* Enqueue one full frame (params' row fields and RT_FLAG_FULL_FRAME are ignored; the
 * other flags apply on every rank) into d_out on rank 0's device: height*width*3 floats
 * (RT_OUTPUT_F32) or bytes (RT_OUTPUT_RGB8). Rank 0 renders on `stream` (a stream of rank
 * 0's device) and the frame is complete in `stream` order; other ranks run on their own
 * streams. No host synchronisation, except when a frame is larger than any before it
 * (buffers grow). Frames stream: each rank overlaps consecutive renders as
 * rt_render_device does. One host thread per context.                                   */
int rt_multi_render_device(rt_multi *ctx, const rt_camera *camera, const rt_params *params,
                           uint32_t format, void *d_out, void *stream);
/* Synchronous host-buffer frames through a context (full frame, row 0 = top); stats sum
 * every rank's counters, kernel_ms spans the frame on rank 0's device.                   */
int rt_multi_render_f32(rt_multi *ctx, const rt_camera *camera, const rt_params *params,
                        float *rgb_out, rt_stats *stats);
int rt_multi_render_rgb8(rt_multi *ctx, const rt_camera *camera, const rt_params *params,
                         uint8_t *rgb_out, rt_stats *stats);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* RT_API_H */
