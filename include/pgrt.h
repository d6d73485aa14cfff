/* pgrt.h -- C ABI of the MI355X-native Whitted trace path (libpgrt.so).
 *
 * This is the drop-in boundary for the reference renderer src/pg/pg1_embree.  It replaces
 * two reference interfaces (see INTEGRATION.md for the binding a maintainer adds):
 *
 *  (1) virtual Color4f SimpleGuiDX11::get_pixel(int x, int y, float t)
 *        simpleguidx11.h:27, overridden at raytracer.h:32, implemented raytracer.cpp:396-437,
 *        called per pixel by SimpleGuiDX11::Producer (simpleguidx11.cpp:105-118).
 *      -> pgrt_render(): one call renders the whole frame (or a tile rect) into an RGBA float
 *         framebuffer with the Producer's layout (row-major, top-down, 4 floats per pixel,
 *         simpleguidx11.cpp:109-115).  The reference's get_pixel(x,y) is then a load from it.
 *
 *  (2) the Embree 3.11 scene / query API used by Raytracer::LoadScene and get_ray_hit
 *        rtcNewScene/rtcNewGeometry/rtcSetNewGeometryBuffer/rtcCommitScene (raytracer.cpp:71-127)
 *        rtcIntersect1 (raytracer.cpp:146; src/libs/embree/include/embree3/rtcore_scene.h:96)
 *      -> pgrt_set_scene(): host arrays in, LBVH built on the device (Embree disappears);
 *         pgrt_intersect_closest(): batched closest-hit query with rtcIntersect1 semantics.
 *
 * Conventions: every entry point returns PGRT_OK (0) or a negative PGRT_ERR_* code; no C++
 * exception crosses the ABI; pgrt_last_error(ctx) describes the last failure on that context.
 * One host thread per context; calls on one context are not reentrant.  Pointers are plain
 * host pointers unless the name says _device.  Sizes are element counts.
 */
#ifndef PGRT_H_
#define PGRT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGRT_ABI_VERSION 3 /* 2 (round 5): pgrt_config carries its size (checked) and host_export;
                              3 (round 6): pgrt_config.peer_wait_ms */

#define PGRT_OK 0
#define PGRT_ERR_INVALID_ARGUMENT (-1)
#define PGRT_ERR_HIP (-2)
#define PGRT_ERR_OUT_OF_MEMORY (-3)
#define PGRT_ERR_NO_SCENE (-4)
#define PGRT_ERR_NO_CAMERA (-5)
#define PGRT_ERR_RCCL (-6)
#define PGRT_ERR_IO (-7)
#define PGRT_ERR_NO_DEVICE (-8)

/* Material kinds (MTL "shader" key, objloader.cpp:135-138; only 4 is special-cased,
 * raytracer.cpp:293-294).  Any other value shades with the Phong branch. */
#define PGRT_MATERIAL_DIELECTRIC 4

/* Index of refraction of air; rays start in air (material.h:15, raytracer.cpp:416). */
#define PGRT_IOR_AIR 1.000293f

/* Jitter modes for the stratified sample offsets r1,r2 (raytracer.cpp:407-410) and the lens
 * offsets (PinHoleCamera.cpp:77-81).  The reference seeds std::mt19937 from the wall clock,
 * which is not reproducible; these modes are counter-based and deterministic. */
/* render modes: the reference's recursive Whitted trace (raytracer.cpp:237-437), or the path
 * tracer of its README "To do" list (README.md:17-21; semantics in DESIGN.md §2 "Path tracing"):
 * one continuation ray per hit -- a cosine-weighted diffuse bounce off Phong/Lambert materials,
 * reflection OR refraction of a dielectric chosen with the reference's Fresnel-like R -- and
 * next-event estimation with hard shadow rays from the hit point to every light */
#define PGRT_MODE_WHITTED 0
#define PGRT_MODE_PATH 1

#define PGRT_JITTER_NONE 0            /* r1 = r2 = 0, lens offset 0 */
#define PGRT_JITTER_HASH 1            /* independent hashed uniforms per (pixel, sample) */
#define PGRT_JITTER_HASH_CORRELATED 2 /* lens uniforms == jitter uniforms, as when both
                                         reference generators get the same microsecond seed */

typedef struct pgrt_ctx pgrt_ctx;

/* Material (material.h:34-125); fields the trace path reads. */
typedef struct pgrt_material {
    float diffuse[3];  /* Kd (RGB) */
    float specular[3]; /* Ks (RGB) */
    float shininess;   /* Ns */
    float ior;         /* Ni */
    int type;          /* "shader" */
    int diffuse_tex;   /* index into pgrt_scene_desc.textures, -1 = none (map_Kd) */
} pgrt_material;

/* Decoded texture: raw BGR(A) bytes, top-down rows, `pitch` bytes per row, `bpp` bytes per
 * pixel -- the layout Texture::Texture produces with FreeImage_ConvertToRawBits
 * (texture.cpp:43-47). */
typedef struct pgrt_texture {
    int width, height, pitch, bpp;
    const unsigned char* data;
} pgrt_texture;

/* Point light (LightSource.h; the ambient term is unused by the trace path). */
typedef struct pgrt_light {
    float position[3];
    float diffuse[3];
    float specular[3];
} pgrt_light;

/* Scene: de-indexed triangles (3 vertices per triangle, raytracer.cpp:96-120), the global
 * triangle index is (surface offset + Embree primID) in surface attach order.  The library
 * copies everything to HBM; the caller keeps ownership of the arrays. */
typedef struct pgrt_scene_desc {
    int num_triangles;        /* >= 0; 0 = an empty scene: every ray misses (the environment) */
    const float* positions;   /* 9*N: v0.xyz v1.xyz v2.xyz          (vertex buffer)      */
    const float* normals;     /* 9*N: per-vertex normals           (attribute slot 0)   */
    const float* uvs;         /* 6*N: per-vertex (u,v)             (attribute slot 1)   */
    const int* material_ids;  /* N:   index into materials          (geometry user data) */
    int num_materials;
    const pgrt_material* materials;
    int num_textures;
    const pgrt_texture* textures;
    int env_texture;          /* SphericalMap texture (index into textures), -1 = black */
    int num_lights;
    const pgrt_light* lights;
} pgrt_scene_desc;

/* PinHoleCamera(width, height, fov_y, view_from, view_at) (PinHoleCamera.cpp:5-29). */
typedef struct pgrt_camera {
    int width, height;
    float fov_y; /* radians */
    float from[3], at[3], up[3];
} pgrt_camera;

/* Per-frame parameters.  Reference values: spp_side 3, max_level 7, dof 1, focal 200,
 * aperture 5, gamma 0.5 (raytracer.cpp:398-400,282; UI default :450,464-465). */
typedef struct pgrt_render_params {
    int spp_side;         /* S: S*S stratified samples per pixel */
    int max_level;        /* d: rays at level >= d are intersected but shaded black (:282) */
    int dof;              /* 0: pinhole generate_ray(x,y), 1: thin-lens generate_ray(...,f,a) */
    float focal_distance; /* DoF focal distance */
    float aperture;       /* DoF square aperture side */
    float gamma_level;    /* Raytracer::gamma exponent (applied twice) */
    int jitter;           /* PGRT_JITTER_* */
    uint32_t seed;
    uint32_t frame;
    int rect_x, rect_y, rect_w, rect_h; /* sub-rectangle; rect_w==0 -> full frame */
    int profile;          /* 0 off, 1 per-stage HIP-event timing, 2 + traversal counters */
    int mode;             /* PGRT_MODE_WHITTED (0, the reference's trace) or PGRT_MODE_PATH */
} pgrt_render_params;

typedef struct pgrt_stats {
    uint64_t rays_primary, rays_shadow, rays_reflect, rays_refract;
    uint64_t node_visits, tri_tests; /* only with profile == 2 */
    double ms_total;                 /* host wall time of the call */
    /* profile >= 1: ms_trace = every closest-hit launch (level queues + the shadow queue);
     * ms_shadow = the shadow-queue launch alone (a part of ms_trace); ms_combine = the finish
     * kernel (shadow resolve + bottom-up combine + sample accumulation + gamma).
     * Distributed frames: ms_gather = device time of the ncclGather (including the wait for the
     * slowest rank) + rank 0's tile unpack, ms_resolve = the unpack alone (asynchronous frames,
     * reported by pgrt_render_wait); the synchronous pgrt_render_distributed* report the host
     * wall time of gather + unpack as ms_gather. */
    double ms_raygen, ms_trace, ms_shade, ms_shadow, ms_combine, ms_resolve, ms_gather;
    int trace_launches;              /* launches of the closest-hit kernel in ms_trace */
    int levels;                      /* trace levels executed */
    int overflow_retries;            /* queue re-sizings this call */
    uint64_t wide_node_visits;       /* profile == 2: 8-wide (80-B) node visits; node_visits
                                        counts the binary (64-B) ones */
    uint64_t shade_hits;             /* profile == 2 (Whitted): shaded rays that hit a triangle
                                        (the others sample the environment map) */
    uint64_t shade_textured_hits;    /* ... of which sampled a diffuse texture (map_Kd) */
} pgrt_stats;

typedef struct pgrt_bvh_info {
    int num_triangles, num_nodes, max_depth;
    double build_ms;
    float scene_lo[3], scene_hi[3];
    size_t device_bytes;
    int builder;          /* PGRT_BVH_LBVH or PGRT_BVH_PLOC (default) */
    int build_iterations; /* PLOC merge iterations */
    int width;            /* traversal layout: 2 (binary, default) or 8 (quantized 8-wide) */
    int num_references;   /* BVH leaf entries: triangles plus early-split-clipping duplicates */
    float split_beta;     /* split budget used (extra references / triangles), 0 = off */
} pgrt_bvh_info;

/* Context configuration (pgrt_get_config / pgrt_set_config).  Every choice here changes speed
 * only: frames and hit records are bit-identical for every value (the closest hit is
 * order-independent, tests/test_gpu_parity.py).  Zero-initialised fields mean "default". */
#define PGRT_BVH_LBVH 1           /* Karras 2012 LBVH over 63-bit Morton codes */
#define PGRT_BVH_PLOC 2           /* PLOC clustering over the Morton order + SAH leaf collapse */
#define PGRT_PACKETS_AUTO 0       /* per level, from the measured packet efficiency (default) */
#define PGRT_PACKETS_OFF (-1)     /* every level one lane per ray */
#define PGRT_HOST_EXPORT_KERNEL 1 /* host frames: per-slot export kernels into page-locked memory */
#define PGRT_HOST_EXPORT_COPY (-1) /* host frames: one device-to-host copy after the frame */
#define PGRT_HOST_EXPORT_SPLIT 2  /* host frames: after the frame, a share by an XCD-0 blit kernel and
                                     the rest by one DMA copy, concurrently */
typedef struct pgrt_config {
    unsigned size;        /* sizeof(pgrt_config) of the caller's pgrt.h: pgrt_get_config fills it, and
                             pgrt_set_config rejects any other value (a caller built against another
                             layout fails loudly instead of writing fields into the wrong places) */
    int bvh_builder;      /* 0 = PGRT_BVH_PLOC (default), PGRT_BVH_LBVH; applied by pgrt_set_scene */
    int bvh_width;        /* 0 or 2: binary traversal layout (default); 8: quantized 8-wide for
                             every queue.  The 8-wide layout is always built for small queues. */
    float split_beta;     /* early split clipping budget (extra references / triangles), 0 off */
    int packet_levels;    /* PGRT_PACKETS_AUTO, PGRT_PACKETS_OFF, or k >= 1: levels 0..k-1 traced
                             as wave packets, deeper levels one lane per ray */
    int group_max;        /* queues of <= group_max rays: 8 lanes per ray over the 8-wide BVH;
                             0 = default (400k synchronous, 100k with frames in flight), -1 never */
    long long max_batch_rays;  /* level-0 rays per sample batch (0 = 32M); smaller values split a
                                  frame's samples into more batches (queue memory vs launches) */
    int max_batches_in_flight; /* sample batches queued across frames in flight (0 = no bound) */
    int rank0_share_a, rank0_share_b; /* distributed frames: rank 0 renders a tiles for every b of
                                         another rank (1..64 each; 0 = the default deal of
                                         pgrt_tile_share; pgrt_tune_distribution sets them) */
    int packet_budget;    /* bounce levels traced as wave packets: a wave still traversing after this
                             many node / triangle steps hands its rays (with their closest hits so
                             far) to the 8-lanes-per-ray kernel; 0 = default (64 steps for one-frame
                             batches of scenes up to 262144 triangles, 256 otherwise), -1 = no budget */
    int subtree_level;    /* Whitted levels >= k evaluated as whole ray trees, one launch (every ray of
                             level k traces and shades its reflection / refraction / shadow rays
                             depth first, as the reference's recursive trace does): 0 = default
                             (one-frame batches of scenes up to 262144 triangles: from level 2 for
                             synchronous frames, from level 3 with frames in flight;
                             one launch per level otherwise), -1 = one launch per level, k >= 1 =
                             from level k */
    int call_order;     /* frames in flight: 1 = each call's level-0 trace waits for the previous
                             call's level-0 shade (the bulk work of the calls in submission order,
                             their latency-bound deeper levels overlapping the next call's bulk);
                             -1 = calls share the GPU freely; 0 = default: ordered for scenes above
                             262144 triangles (C5 -7 %; the avenger's C2 / C3 lose when ordered,
                             profiles/r3/ab_r3ab_call_order.txt) */
    int tile_order;     /* synchronous one-frame renders (two pipeline slots): 0 = default, the tiles
                             whose primary rays hit a dielectric in the previous frame of the same
                             size form the first slot, so the deep reflection / refraction levels
                             (the frame's critical path) start after a short level 0 while the
                             other slot's level 0 still runs; -1 = tiles dealt round-robin */
    int host_export;    /* frames into page-locked host memory (pgrt_render,
                             pgrt_render_frames_host_async): 0 = default -- each pipeline slot exports
                             its finished tiles with a small blit kernel as soon as that slot is done
                             (a synchronous frame's bulk slot crosses PCIe while its deep-tile slot
                             still renders; a call in flight right after its frames); PGRT_HOST_EXPORT_KERNEL = export kernels always;
                             PGRT_HOST_EXPORT_COPY = one DMA copy after every frame (pageable
                             destinations always take the copy); PGRT_HOST_EXPORT_SPLIT = after every
                             frame, part of the bytes by a blit kernel on XCD 0 and the rest by a
                             DMA copy at the same time */
    int peer_wait_ms;   /* distributed frames (rank 0): how long to wait for the peers' tiles of one
                             gather before giving up -- the communicator is then aborted
                             (ncclCommAbort), the call and every later distributed call return
                             PGRT_ERR_RCCL, and pgrt_destroy still returns; 0 = default 120000 */
} pgrt_config;

/* ---- context ---- */
const char* pgrt_version(void);
int pgrt_device_count(int* count);
int pgrt_create(int hip_device, pgrt_ctx** out);
/* Single-process multi-device context (SURVEY §8b `pgrt_create(const int* hip_device_ids, int
 * n_devices, ...)`; the reference is one process with one Producer thread,
 * simpleguidx11.cpp:86-128): rank r renders its image tiles (the deal of pgrt_tile_count_ex
 * with the context's share) on hip_device_ids[r], and every frame is gathered into rank 0's
 * output over RCCL communicators the context creates itself (ncclCommInitAll; one host thread
 * posts every rank's sends / receives in one ncclGroupStart / ncclGroupEnd).  Ranks listed on
 * the same device exchange their tiles by device copies instead (RCCL takes one rank per device).
 * n_devices in [1, 16].  Every pgrt_* call on the returned context applies to all ranks:
 * set_scene (the same deterministic build on each device), set_camera, set_config,
 * set_frames_in_flight, synchronize, destroy; pgrt_render / pgrt_render_device /
 * pgrt_render_frames_device, their _async forms and the pgrt_render_distributed* calls render
 * whole frames (no render rect) into a buffer on hip_device_ids[0]; stats count the rays of
 * every rank, device times are the slowest rank's.  The batch queries (pgrt_intersect_closest,
 * pgrt_occluded), pgrt_render_accumulate and pgrt_render_tiles_device run on rank 0's device;
 * host-output frames (pgrt_render_frames_host_async) and pgrt_comm_init are not available. */
int pgrt_create_devices(const int* hip_device_ids, int n_devices, pgrt_ctx** out);
void pgrt_destroy(pgrt_ctx* ctx);
const char* pgrt_last_error(const pgrt_ctx* ctx);
/* The BVH fields take effect at the next pgrt_set_scene, the others at the next frame
 * (pending frames complete first). */
int pgrt_get_config(const pgrt_ctx* ctx, pgrt_config* cfg);
int pgrt_set_config(pgrt_ctx* ctx, const pgrt_config* cfg);

/* ---- scene / camera (replaces Raytracer::LoadScene's Embree upload, raytracer.cpp:71-127,
 *      and the PinHoleCamera ctor, PinHoleCamera.cpp:5-29) ---- */
/* Limits: the traversal and shading kernels address BVH nodes, triangle records and texels by
 * 32-bit byte offsets, so every BVH / triangle array stays below 4 GiB (~53 M triangle references,
 * split duplicates included) and the texel pool too; larger scenes return
 * PGRT_ERR_INVALID_ARGUMENT with a message. */
int pgrt_set_scene(pgrt_ctx* ctx, const pgrt_scene_desc* scene);
int pgrt_bvh_get_info(const pgrt_ctx* ctx, pgrt_bvh_info* info);
int pgrt_set_camera(pgrt_ctx* ctx, const pgrt_camera* cam);

/* ---- frame (replaces get_pixel for every pixel of the Producer loop) ---- */
int pgrt_render(pgrt_ctx* ctx, const pgrt_render_params* p, float* rgba_host, pgrt_stats* st);
/* Same, output left in device memory (rgba_device: W*H*4 floats, or rect_w*rect_h*4). */
int pgrt_render_device(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device,
                       pgrt_stats* st);
/* Device buffer helpers for callers without their own allocator (bench, tests). */
int pgrt_device_alloc(pgrt_ctx* ctx, size_t bytes, void** out);
int pgrt_device_free(pgrt_ctx* ctx, void* ptr);
int pgrt_copy_to_host(pgrt_ctx* ctx, void* dst_host, const void* src_device, size_t bytes);
int pgrt_synchronize(pgrt_ctx* ctx);

/* ---- frame sink (replaces the Producer's endless re-render, simpleguidx11.cpp:86-128, with a
 *      progressive average): each call renders one frame (use a new params.frame per call so the
 *      jitter / lens samples differ), adds it to a device running sum in call order and writes
 *      the running mean (W*H*4 floats, or the rect) to mean_host when not NULL.  *frames receives
 *      the number of frames in the sum.  A different frame size or pgrt_accumulate_reset restarts. */
int pgrt_accumulate_reset(pgrt_ctx* ctx);
int pgrt_render_accumulate(pgrt_ctx* ctx, const pgrt_render_params* p, float* mean_host, int* frames,
                           pgrt_stats* st);

/* ---- frames in flight (asynchronous frames) ----
 * pgrt_render_device_async enqueues a frame and returns at once with a ticket; up to n frames
 * (pgrt_set_frames_in_flight, 1..16, default 1) run concurrently, each on its own pipeline
 * streams, so one frame's latency-bound deep Whitted levels overlap the next frame's wide levels.
 * Submitting when n frames are pending first completes the oldest.  pgrt_render_wait(ticket)
 * completes every frame up to that ticket and returns its statistics (ms_total = submit to
 * completion); a ticket stays valid until its frame set is reused n submissions later.  The
 * framebuffer of a pending frame must not be read or reused.  Frames are bit-identical to
 * pgrt_render_device.  The synchronous entry points complete pending frames first.  profile must
 * be 0 for asynchronous frames. */
int pgrt_set_frames_in_flight(pgrt_ctx* ctx, int n);
int pgrt_render_device_async(pgrt_ctx* ctx, const pgrt_render_params* p, void* rgba_device,
                             unsigned long long* ticket);
int pgrt_render_wait(pgrt_ctx* ctx, unsigned long long ticket, pgrt_stats* st);
/* Batched frames: one call renders nframes (1..64) consecutive frames of the same camera and
 * params, frame f with jitter frame index p->frame + f, into rgba_device + f * (frame floats)
 * (W*H*4 floats per frame, or the rect's w*h*4).  Every launch covers all nframes frames, so
 * small frames fill the GPU and pay the per-launch latency once per call instead of once per
 * frame.  Each frame is bit-identical to pgrt_render_device with params.frame = p->frame + f.
 * One ticket completes all nframes frames; its statistics are the sums over them. */
int pgrt_render_frames_device_async(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes,
                                    void* rgba_device, unsigned long long* ticket);
/* Synchronous form of the batched frames (profile allowed: stage timings cover all nframes). */
int pgrt_render_frames_device(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes,
                              void* rgba_device, pgrt_stats* st);
/* Batched frames to a HOST framebuffer (the reference's Producer hands every finished frame to
 * the host-side D3D texture, APP/simpleguidx11.cpp:105-124): frames are rendered into a device
 * staging buffer owned by the frame in flight, then the nframes * W*H*4 floats move into
 * rgba_host behind them (pgrt_config.host_export: by default a copy kernel on XCD 0), so the PCIe
 * transfer of one call overlaps the rendering of
 * the calls in flight behind it.  rgba_host must stay valid until the ticket is waited for; pinned
 * memory from pgrt_host_alloc makes the copy truly asynchronous (pageable memory works but takes
 * one synchronous DMA copy).  Same pixels as pgrt_render_frames_device. */
int pgrt_render_frames_host_async(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes,
                                  float* rgba_host, unsigned long long* ticket);
/* Page-locked host memory for framebuffers (pgrt_render, pgrt_render_frames_host_async). */
int pgrt_host_alloc(pgrt_ctx* ctx, size_t bytes, void** out);
int pgrt_host_free(pgrt_ctx* ctx, void* ptr);

/* ---- batched closest-hit query with rtcIntersect1 semantics ----
 * rays: n x 8 floats {org.xyz, tnear, dir.xyz, tfar}; hits: n x 4 {t, u, v, prim} where prim
 * is the global triangle index stored as int32 bits, -1 on a miss (t = tfar, u = v = 0). */
int pgrt_intersect_closest(pgrt_ctx* ctx, const float* rays, int n, float* hits);
/* The same query on structure-of-arrays streams (SURVEY.md §8b's soa_rays / soa_hits; Embree's
 * rtcIntersectNp layout): rays_soa = 8 arrays of n floats (org x, y, z, tnear, dir x, y, z,
 * tfar), hits_soa = 4 arrays of n floats (t, u, v, primID as int bits, -1 = miss). */
int pgrt_intersect_closest_soa(pgrt_ctx* ctx, const float* rays_soa, int n, float* hits_soa);

/* ---- batched occlusion query with rtcOccluded1 semantics (rtcore_scene.h:120; Embree marks an
 * occluded ray by setting tfar = -inf): occluded[i] = 1 when ANY triangle is hit with t in
 * (tnear, tfar], else 0.  Same ray layout as pgrt_intersect_closest; the traversal stops at the
 * first accepted triangle. */
int pgrt_occluded(pgrt_ctx* ctx, const float* rays, int n, int* occluded);

/* ---- multi-GPU image tiles (one process per GPU, RCCL over xGMI) ----
 * Tiles are tile_size x tile_size, numbered row-major and dealt to ranks in rounds of
 * a + b*(world-1) tiles: rank 0 gets a, every other rank b (min(a,b) sub-rounds of one tile per
 * rank, then the remaining b-a tiles of ranks 1.. or a-b tiles of rank 0), so rank 0 renders a/b
 * of another rank's share -- less when its unpack of every gathered frame costs more, more when
 * the gather into it over xGMI is the bound (pgrt_tune_distribution).  pgrt_tile_share reports the
 * default (a, b) for a world size (PGRT_RANK0_SHARE="a/b" overrides; a == b is the round-robin
 * deal t -> rank t % world).  pgrt_tile_index maps local tile j of rank to its
 * tile index (error past the rank's last tile); pgrt_tile_count is the rank's tile count. */
int pgrt_tile_count(int width, int height, int tile_size, int rank, int world);
int pgrt_tile_index(int width, int height, int tile_size, int rank, int world, int j);
int pgrt_tile_share(int world, int* a, int* b);
int pgrt_tile_rect(int width, int height, int tile_size, int tile_index, int rect[4]);
/* Unpack a rank-major gathered tile buffer (every rank's tiles in its local order, each tile
 * tile_size^2 * 4 floats, ranks back to back with exactly pgrt_tile_count tiles each) into a
 * W x H RGBA framebuffer.  Host reference of the device unpack. */
int pgrt_unpack_tiles_host(int width, int height, int tile_size, int world,
                           const float* gathered, float* rgba);
/* The tail of a rank's distributed send (two ints after its tiles): its flag (0 ok,
 * 1 the rank's queues overflowed -- it re-renders and sends again, 2 it gave up) and the frame's
 * sequence number (>= 1).  pgrt_gather_tail forms it as the device does; pgrt_gather_tail_verdict
 * is rank 0's reading of one gather's tails (flags[r], seqs[r] for r < world; seqs[r] == 0: rank r
 * not received in this gather, rank 0's own entry ignored): PGRT_OK with regather[r] = 1 for the
 * ranks whose tiles must be received again, PGRT_ERR_RCCL when a rank sent another frame's tiles
 * (the ranks did not submit / wait in the same order), PGRT_ERR_OUT_OF_MEMORY when a rank gave up;
 * *bad_rank names that rank.  The distributed frames run exactly this logic; host-only (the
 * world-2 gloo test drives it). */
int pgrt_gather_tail(int overflow, int poison, unsigned seq, int tail[2]);
int pgrt_gather_tail_verdict(const int* flags, const unsigned* seqs, int world, unsigned expect_seq, int* regather,
                             int* bad_rank);
/* The same three with an explicit share (rank 0 renders a tiles for every b of another rank,
 * 1..64 each; a = b = 0: the default share) -- the deal of a context whose pgrt_config sets
 * rank0_share_a / rank0_share_b. */
int pgrt_tile_count_ex(int width, int height, int tile_size, int rank, int world, int a, int b);
int pgrt_tile_index_ex(int width, int height, int tile_size, int rank, int world, int a, int b, int j);
int pgrt_unpack_tiles_host_ex(int width, int height, int tile_size, int world, int a, int b,
                              const float* gathered, float* rgba);
int pgrt_comm_unique_id(char id[128]);
int pgrt_comm_init(pgrt_ctx* ctx, int world, int rank, const char id[128]); /* world <= 16 */
/* The communicator's rank count and this context's rank as RCCL reports them (ncclCommCount /
 * ncclCommUserRank); without a communicator the context's world / rank (1 / 0 by default). */
int pgrt_comm_info(const pgrt_ctx* ctx, int* nranks, int* rank);
/* Rank-local half of the distributed render, for callers that gather with their own
 * communicator: render the tiles of `rank` (of `world`) of the camera image into a tile-compact
 * device buffer.  The deal is the CONTEXT's: with a = pgrt_config.rank0_share_a and
 * b = pgrt_config.rank0_share_b (pgrt_get_config; pgrt_tune_distribution sets them), size the
 * buffer as pgrt_tile_count_ex(W, H, 64, rank, world, a, b) * 64 * 64 * 4 floats; local tile j is
 * tile pgrt_tile_index_ex(W, H, 64, rank, world, a, b, j) (edge tiles are padded).  Only when
 * a = b = 0 (the default) are these pgrt_tile_count / pgrt_tile_index. */
int pgrt_render_tiles_device(pgrt_ctx* ctx, const pgrt_render_params* p, int rank, int world,
                             void* tiles_device, pgrt_stats* st);
/* Device form of pgrt_unpack_tiles_host_ex for callers that gather pgrt_render_tiles_device
 * buffers themselves: tiles_device is rank-major (exactly pgrt_tile_count_ex tiles per rank,
 * RGBA tiles), rgba_device W*H*4 floats.  Synchronous. */
int pgrt_unpack_tiles_device(pgrt_ctx* ctx, int width, int height, int world, int a, int b,
                             const void* tiles_device, void* rgba_device);
/* Collective (every rank calls it with the same arguments): measure the distributed batched
 * frames (p, nframes per call into rgba_device as pgrt_render_frames_distributed_device_async)
 * for rank-0 shares a/8 = 4/8 .. 32/8 -- `calls` timed calls each, the slowest rank's wall time
 * (ncclAllReduce max) decides -- and keep the fastest in the context's pgrt_config
 * (rank0_share_a/b, returned in *a, *b).  With one rank it returns 1/1 and does nothing. */
int pgrt_tune_distribution(pgrt_ctx* ctx, const pgrt_render_params* p, int nframes,
                           void* rgba_device, int calls, int* a, int* b);
/* Render this rank's tiles, gather them on rank 0 (grouped ncclSend / ncclRecv of each rank's
 * exact tile list), unpack on device.
 * rgba_host (rank 0 only, may be NULL elsewhere): W*H*4 floats. */
int pgrt_render_distributed(pgrt_ctx* ctx, const pgrt_render_params* p, float* rgba_host,
                            pgrt_stats* st);
/* Same, framebuffer left on rank 0's device (W*H*4 floats). */
int pgrt_render_distributed_device(pgrt_ctx* ctx, const pgrt_render_params* p,
                                   void* rgba_device, pgrt_stats* st);
/* Asynchronous form (frames in flight, see pgrt_render_device_async): the gather of a frame is
 * enqueued when it completes (pgrt_render_wait or a later submission) and overlaps the frames
 * still in flight.  Every rank must submit and wait in the same order. */
int pgrt_render_distributed_device_async(pgrt_ctx* ctx, const pgrt_render_params* p,
                                         void* rgba_device, unsigned long long* ticket);
/* Batched distributed frames (see pgrt_render_frames_device_async): each rank renders its tiles
 * of nframes frames in one pass, one ncclGather moves all of them, rank 0 unpacks frame f into
 * rgba_device + f * W*H*4 floats. */
int pgrt_render_frames_distributed_device_async(pgrt_ctx* ctx, const pgrt_render_params* p,
                                                int nframes, void* rgba_device,
                                                unsigned long long* ticket);

/* ---- scene ingest (LoadOBJ / LoadMTL, objloader.cpp:53-507; host only) ----
 * Texture files named by map_Kd are NOT decoded here: their paths are reported so the caller
 * decodes them (FreeImage is not available) and fills pgrt_texture entries. */
typedef struct pgrt_obj pgrt_obj;
int pgrt_obj_load(const char* obj_path, int flip_yz, pgrt_obj** out);
void pgrt_obj_free(pgrt_obj* obj);
const char* pgrt_obj_error(void);
/* Fills desc with pointers owned by obj (textures/env/lights left empty for the caller). */
int pgrt_obj_scene(const pgrt_obj* obj, pgrt_scene_desc* desc);
int pgrt_obj_counts(const pgrt_obj* obj, int* num_surfaces, int* num_materials,
                    int* num_textures);
const char* pgrt_obj_texture_path(const pgrt_obj* obj, int i);
const char* pgrt_obj_material_name(const pgrt_obj* obj, int i);
int pgrt_obj_surface_range(const pgrt_obj* obj, int i, int* first_triangle, int* count);

/* ---- diagnostics of the last pgrt_render* call (traversal counters need profile == 2):
 *      per level L, rays traced at L and shadow rays emitted at L, with their BVH node visits
 *      and triangle tests (sum and the maximum of one ray).  Returns the levels filled. ---- */
typedef struct pgrt_level_diag {
    uint64_t rays, shadow_rays;
    uint64_t visits, tests, max_visits, max_tests;
    uint64_t shadow_visits, shadow_tests, shadow_max_visits, shadow_max_tests;
    uint64_t max_wave_iterations; /* binary traversal: node steps + leaf rounds of the longest
                                     wave (lower bound) -- the latency chain of the level */
    uint64_t max_ray_ticks;       /* longest single-ray traversal, 100 MHz wall-clock ticks */
    uint64_t stack_spills;        /* traversal stack pushes past the LDS part (global memory) */
    uint64_t max_stack;           /* deepest traversal stack of one ray */
    uint64_t longest_ray[6];      /* the longest ray: visits, tests, leaf rounds, node-phase,
                                     leaf-phase and node-load shader cycles / 64 */
    uint64_t wide_visits;         /* the part of visits that were 8-wide nodes */
    double ms_trace, ms_shade;    /* this level's launches (profile >= 1 on the call; summed
                                     over sample batches) */
    uint64_t packet_steps_hit;    /* levels traced as wave packets (sampled blocks): lane-steps
                                     at which the lane's ray hit a child box of the wave's node */
    uint64_t packet_steps_live;   /* ... and live lane-steps; hit / live = packet utilisation */
} pgrt_level_diag;
int pgrt_frame_diag(const pgrt_ctx* ctx, pgrt_level_diag* out, int max_levels);

/* ---- launch timeline (device clock; no rocprof, no HIP events) ----
 * While enabled, every kernel of every later frame (synchronous and asynchronous calls alike)
 * stamps the device wall clock (s_memrealtime, 100 MHz) in each of its waves at entry and exit;
 * when the call is collected, each launch becomes one record: the first wave's start and the last
 * wave's end.  The stamps cost one 16-B store per wave; the kernels, grids and streams are those
 * of an unrecorded frame.  pgrt_timeline_read returns the records collected so far (oldest first,
 * at most max) and removes them; *n receives the count returned.  Enabling or disabling completes
 * pending frames first. */
#define PGRT_TL_RAYGEN 0        /* k_raygen */
#define PGRT_TL_TRACE_PKT 1     /* wave-packet closest hit (level 0 generates its rays) */
#define PGRT_TL_TRACE 2         /* one lane per ray */
#define PGRT_TL_TRACE_8G 3      /* 8 (4) lanes per ray over the 8-wide BVH */
#define PGRT_TL_TRACE_RESUME 4  /* 8 lanes per ray, the deferred rays of a budgeted packet launch */
#define PGRT_TL_TRACE_SHADOW 5  /* the shadow queue */
#define PGRT_TL_SHADE 6
#define PGRT_TL_COMBINE 7
#define PGRT_TL_FINISH 8
#define PGRT_TL_EXPORT 9        /* frame counters to the host */
#define PGRT_TL_UNPACK 10
#define PGRT_TL_PATH_SHADE 11
#define PGRT_TL_PATH_RESOLVE 12
#define PGRT_TL_SUBTREE 13      /* the deep levels as one launch (pgrt_config.subtree_level) */
#define PGRT_TL_HOST_EXPORT 14  /* a slot's finished tiles to a page-locked host framebuffer */
#define PGRT_TL_DROPPED 15      /* marker: this call had more waves than the stamp buffer holds (4M);
                                   its later launches are not recorded */
typedef struct pgrt_timeline_rec {
    uint64_t ticket;     /* the call (the ticket an asynchronous call returned; synchronous calls count too) */
    int slot;            /* pipeline slot (stream) of the call */
    int kind;            /* PGRT_TL_* */
    int level;           /* queue level, -1 = none */
    int waves;           /* waves that stamped */
    uint64_t start, end; /* device wall clock ticks (100 MHz): first wave in, last wave out */
    uint32_t wave_p50, wave_p90, wave_max; /* wave durations (ticks): median, 90th percentile, longest */
    uint32_t last_in;    /* ticks from start to the last wave's entry (launch fill / tail split) */
} pgrt_timeline_rec;
int pgrt_timeline_enable(pgrt_ctx* ctx, int on);
int pgrt_timeline_read(pgrt_ctx* ctx, pgrt_timeline_rec* out, int max, int* n);

/* ---- test hook: evaluates the shared math of pgrt_detmath.h on the device.  in: n (a,b)
 *      pairs; out: n x 8 {sqrtf(a), a/b, powf(a,b), expf(a), atan2f(a,b), asinf(a),
 *      1/sqrtf(a), (float)pow((double)a,(double)b)} ---- */
int pgrt_selftest_math(pgrt_ctx* ctx, const float* in_pairs, int n, float* out8);
/* ---- test hook: the kernels' sRGB expand / compress (mix_srgb, utils.cpp:204-241) against their
 *      exact pg_pow_d form on every float whose bit pattern is in [first_bits, first_bits + count):
 *      mismatches[0] / [1] = inputs where expand / compress differ (bitwise) ---- */
int pgrt_selftest_srgb(pgrt_ctx* ctx, uint32_t first_bits, uint32_t count, uint64_t* mismatches);

#ifdef __cplusplus
}
#endif

#endif /* PGRT_H_ */
