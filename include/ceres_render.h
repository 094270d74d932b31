/* ceres_render.h -- C ABI of the MI355X-native CERES hot path (libceres_hip.so).
 *
 * The reference has no C ABI, plugin registry or FFI: its hot path is the header-only
 * template `render()` (include/render.hpp:86-156 in iracigt/ceres-raytracer) plus the
 * host-side scene preparation its callers run first (static.cpp:76-107, anim.cpp:38-65).
 * Every entry point below replaces one of those reference interfaces; the reference
 * file:line is cited per function.  Plain pointers and sizes only -- no C++ or torch
 * types -- so it can be bound from C, C++, ctypes, cgo, JNI ...
 *
 * Data layouts (all little-endian, fp32 unless stated), identical to the reference's
 * in-memory structures so a caller can hand its own arrays over unchanged:
 *   tri48   n_tri  x {p0[3], e1[3], e2[3], n[3]}        = bvh::Triangle<float> (triangle.hpp:17-37)
 *   norm36  n_tri  x {n0[3], n1[3], n2[3]}              = std::array<Vector3,3> (obj_norms.hpp:113-115)
 *   nodes32 n_nodes x {bounds[6], u32 count, u32 first} = bvh::Bvh<float>::Node (bvh.hpp:25-30)
 *   prim64  n_tri  x u64                                = Bvh::primitive_indices (bvh.hpp:94)
 *   pixels  3*W*H  floats, row j = 0 at the BOTTOM       (render.hpp:107)
 *   rgb8    3*W*H  bytes = the P6 body, rows top-down, truncating quantiser (static.cpp:135-147)
 *
 * Errors: functions return 0 on success and a negative ceres_status on failure;
 * ceres_last_error() describes the last failure of the calling thread.  The product
 * path has NO CPU fallback: without a usable gfx950 device every render call fails.
 * Threading: a ceres_scene is not thread-safe; use one scene per thread (or lock).
 */
#ifndef CERES_RENDER_H
#define CERES_RENDER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    CERES_OK = 0,
    CERES_EINVAL = -1,      /* bad argument (null pointer, zero size, malformed BVH) */
    CERES_EIO = -2,         /* file could not be read / malformed OBJ index (obj_norms.hpp:90) */
    CERES_ENOMEM = -3,      /* host or device allocation failed */
    CERES_EHIP = -4,        /* HIP runtime error (no device, launch failure, ...) */
    CERES_ESTACK = -5,      /* traversal stack overflow (single_ray_traverser.hpp:29 assert) */
    CERES_EUNSUPPORTED = -6
} ceres_status;

typedef enum {
    CERES_MODE_FULL = 0,     /* primary + shadow + smooth shading (render.hpp:104-153) */
    CERES_MODE_PRIMARY = 1,  /* primary rays only; pixel = |normalize(tri.n)| (render.hpp:123-125) */
    CERES_MODE_ROBUST = 0x10, /* OR-ed flag: traverse with the library's RobustNodeIntersector
                                (node_intersectors.hpp:54-79) instead of render()'s FastNodeIntersector;
                                float scenes only */
    CERES_MODE_QBVH4 = 0x20, /* OR-ed flag (full mode, float, not with ROBUST): shadow rays traverse
                                a COMPRESSED BVH4 -- 64-B nodes, child boxes quantised to 8 bits per
                                bound, rounded outwards -- instead of the exact 128-B one.  Not
                                bit-exact: a box can only grow, so every leaf the reference reaches
                                is still tested, but a grazing shadow ray may also meet a triangle
                                the reference's slab tests never reach (a lit pixel turns dark).
                                Held to the SURVEY section 7 budget (+-1 LSB, <= 1e-5 of pixels),
                                never the default (node_intersectors.hpp:35-47,83-103). */
    CERES_MODE_FMA = 0x40    /* OR-ed flag: the arithmetic of the reference as its own CMake build
                                compiles it (CMakeLists.txt:11-13, g++ -O3 -mavx2 -mfma, where GCC
                                contracts a*b+c into FMA): an explicit fmaf at exactly the sites GCC
                                fuses (primary direction render.hpp:111, Moller-Trumbore
                                triangle.hpp:98-109, hit point :129-133, normalize/cross/dot
                                vector.hpp:134-167, shading render.hpp:48-81; the list with the
                                compiler evidence is oracle/contraction_sites.txt).  Bit-identical to
                                _ref/ref_render (the reference-flag build) given a scene prepared with
                                CERES_ARITH_FMA; without it, bit-identical to the -ffp-contract=off
                                build.  Combines with ROBUST, QBVH4 and PRIMARY. */
} ceres_mode;

/* Arithmetic of the host scene preparation (the *_arith calls below): CERES_ARITH_EXACT is the
 * reference compiled without contraction, CERES_ARITH_FMA the reference's own CMake build (the
 * triangle normals cross(e1, e2), the rotation, the vertex-normal normalisation, the SAH costs,
 * the camera basis and the orbit Transform all contract there, so that build's scene differs
 * bit-wise from the exact one: pair it with CERES_MODE_FMA renders). */
#define CERES_ARITH_EXACT 0
#define CERES_ARITH_FMA   1

typedef struct ceres_scene ceres_scene;

/* Per-render counters.  rays/hits are exactly render()'s return pair (render.hpp:102,115,
 * 119,138,148,155) widened to 64 bit.  The traversal counters are filled only when the
 * scene was created with CERES_SCENE_STATS (they follow single_ray_traverser.hpp:132-135,
 * except that shadow rays stop at the first occluder -- any-hit, result-identical). */
typedef struct {
    uint64_t rays;            /* primary + shadow traversals */
    uint64_t hits;            /* primary hits + occluded shadow rays */
    uint64_t primary_rays, shadow_rays;
    uint64_t node_pairs;      /* traversal_steps, all rays */
    uint64_t tri_tests;       /* intersections, all rays */
    double   ms;              /* device time of the render (HIP events), host-buffer API only */
} ceres_stats;

/* Row partition across ranks; world = 1 renders the whole frame.
 * bands = 0: rows are dealt in blocks of `row_block` rows, block b to rank b % world; local row k
 *   of a rank is global row j = ((k / row_block) * world + rank) * row_block + k % row_block.
 * bands = 1: frame f of the call (0-based) is cut into `world` contiguous bands of `row_block`
 *   rows (the last one shorter; row_block * world >= height) and the rank renders band
 *   (rank + f) mod world: local row k is global row j = band * row_block + k, every frame has
 *   row_block local rows, those with j >= height are not rendered (their RGB8 positions, the
 *   first ones of the frame's buffer, are not written).  Rotating the band from frame to frame
 *   keeps ranks balanced over a batch; a band is a contiguous slice of the frame's PPM body, so
 *   an owner rank can receive it in place (no un-interleave). */
typedef struct {
    uint32_t row_block, rank, world;
    uint32_t bands;
} ceres_tiling;

/* ---- host-side scene preparation (what static.cpp / anim.cpp run before render()) ---- */

/* obj::load_from_file<float> (obj_norms.hpp:120-127 / load_from_stream :57-118): v/f lines,
 * fan triangulation, area-weighted left-handed vertex normals.  *tri48 / *norm36 are
 * malloc'd (free with ceres_free).  An unreadable file yields n_tri = 0 like the reference. */
int ceres_obj_load(const char* path, float** tri48, float** norm36, size_t* n_tri);
/* Procedural heightfield mesh of the C5 configuration (n x n vertices, 2(n-1)^2 triangles,
 * SURVEY.md §8(d)); same arrays as ceres_obj_load. */
int ceres_proc_mesh(int n, float** tri48, float** norm36, size_t* n_tri);
/* rotate_triangles<Axis> (render.hpp:24-44); axis 0/1/2 = x/y/z.  In place. */
int ceres_rotate_triangles(float* tri48, size_t n_tri, int axis, float degrees);
/* compute_bounding_boxes_and_centers + BinnedSahBuilder<Bvh,16>::build (utilities.hpp:142-171,
 * binned_sah_builder.hpp:39-234).  *nodes32 (n_nodes x 32 B) / *prim64 malloc'd. */
int ceres_bvh_build(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64);
/* The same BinnedSahBuilder<Bvh,16> build on the GPU: identical topology,
 * boxes and primitive_indices as ceres_bvh_build (node numbering is breadth-first for the top,
 * then subtree-contiguous, as the reference's own numbering is OpenMP-timing dependent).
 * ceres_bvh_build_gpu: host buffers in/out, same outputs as ceres_bvh_build, on HIP `device`.
 * ceres_bvh_build_device: d_tri48 in device memory; d_nodes32 holds 2*n_tri-1 nodes (8 u32 each),
 * d_prim32 n_tri u32; stream-ordered on `stream` (a hipStream_t), returns once *n_nodes is known. */
int ceres_bvh_build_gpu(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64,
                        int device);
int ceres_bvh_build_device(const float* d_tri48, size_t n_tri, uint32_t* d_nodes32, uint32_t* d_prim32,
                           size_t* n_nodes, void* stream);
/* obj::load_from_stream on the GPU: the reference loader's exact triangles
 * and face-order normal sums (obj_norms.hpp:57-118), numbers via glibc-exact strtof/strtol.
 * ceres_obj_load_gpu: same contract as ceres_obj_load (file read on the host, parsed on HIP
 * `device`, malloc'd outputs).  ceres_obj_parse_device: device text in; *d_tri48 / *d_norm36
 * are device arrays (free with ceres_device_free), NULL when the mesh is empty.  A face
 * referencing a missing vertex (the reference's assert, obj_norms.hpp:90) returns CERES_EIO. */
int ceres_obj_load_gpu(const char* path, float** tri48, float** norm36, size_t* n_tri, int device);
int ceres_obj_parse_device(const char* d_text, size_t len, float** d_tri48, float** d_norm36, size_t* n_tri,
                           void* stream);
/* rotate_triangles<Axis> on device triangles (cos/sin of the angle taken on the host). */
int ceres_rotate_triangles_device(float* d_tri48, size_t n_tri, int axis, float degrees, void* stream);
void ceres_device_free(void* d_ptr);
/* The GPU scene preparation above in a chosen arithmetic (CERES_ARITH_EXACT = the calls above,
 * CERES_ARITH_FMA = the reference's CMake build: contracted triangle normals, vertex-normal
 * normalisation, rotation and SAH costs; bit-identical to the *_arith host calls below). */
int ceres_bvh_build_gpu_arith(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64,
                              int device, int arith);
int ceres_bvh_build_device_arith(const float* d_tri48, size_t n_tri, uint32_t* d_nodes32, uint32_t* d_prim32,
                                 size_t* n_nodes, void* stream, int arith);
int ceres_obj_load_gpu_arith(const char* path, float** tri48, float** norm36, size_t* n_tri, int device, int arith);
int ceres_obj_parse_device_arith(const char* d_text, size_t len, float** d_tri48, float** d_norm36, size_t* n_tri,
                                 void* stream, int arith);
int ceres_rotate_triangles_device_arith(float* d_tri48, size_t n_tri, int axis, float degrees, void* stream, int arith);
/* Camera basis of render.hpp:91-97: out = {dir[3], image_u*w[3], image_v*w*ratio[3]}. */
int ceres_camera_basis(const float eye[3], const float dir[3], const float up[3], float fov_deg,
                       size_t width, size_t height, float out9[9]);
/* The camera/sun orbit of anim.cpp:76-88 (Transform::rotate, transform.hpp:67-112): per frame,
 * eye, dir and sun are rotated by step_deg about `axis` (up is not); rotate_first = 1 rotates
 * before frame 0 like anim.cpp, 0 starts at the given pose.  Writes n_frames x basis12
 * ({eye, dir, image_u, image_v}, as ceres_camera_basis), n_frames x sun3 and, when dir3 is
 * not NULL, n_frames x the rotated (un-normalised) camera dir. */
int ceres_orbit_cameras(const float eye[3], const float dir[3], const float up[3], const float sun[3],
                        float fov_deg, size_t width, size_t height, const float axis[3], float step_deg,
                        uint32_t n_frames, int rotate_first, float* basis12, float* sun3, float* dir3);
void ceres_free(void* p);
/* The six steps above in a chosen arithmetic, arith = CERES_ARITH_EXACT (= the calls above) or
 * CERES_ARITH_FMA (the reference's own CMake build: obj_norms.hpp's normals, the Triangle
 * constructor's cross product, rotate_triangles, the SAH costs of binned_sah_builder.hpp:98-109,179,
 * the camera basis and Transform contract as GCC contracts them; oracle/contraction_sites.txt). */
int ceres_obj_load_arith(const char* path, float** tri48, float** norm36, size_t* n_tri, int arith);
int ceres_proc_mesh_arith(int n, float** tri48, float** norm36, size_t* n_tri, int arith);
int ceres_rotate_triangles_arith(float* tri48, size_t n_tri, int axis, float degrees, int arith);
int ceres_bvh_build_arith(const float* tri48, size_t n_tri, uint32_t** nodes32, size_t* n_nodes, uint64_t** prim64,
                          int arith);
int ceres_camera_basis_arith(const float eye[3], const float dir[3], const float up[3], float fov_deg,
                             size_t width, size_t height, float out9[9], int arith);
int ceres_orbit_cameras_arith(const float eye[3], const float dir[3], const float up[3], const float sun[3],
                              float fov_deg, size_t width, size_t height, const float axis[3], float step_deg,
                              uint32_t n_frames, int rotate_first, float* basis12, float* sun3, float* dir3, int arith);

/* ---- double precision (render<double>, anim.cpp's -d mode, anim.cpp:146-155) ----
 * The same host steps with Scalar = double: bvh::Triangle<double> (96 B), tri_norms as
 * 3 x Vector3<double> (72 B), bvh::Bvh<double>::Node (6 doubles + 2 x u64 = 64 B); OBJ
 * coordinates are strtof floats widened to double (obj_norms.hpp:78-80). */
int ceres_obj_load_f64(const char* path, double** tri96, double** norm72, size_t* n_tri);
int ceres_proc_mesh_f64(int n, double** tri96, double** norm72, size_t* n_tri);
int ceres_rotate_triangles_f64(double* tri96, size_t n_tri, int axis, double degrees);
int ceres_bvh_build_f64(const double* tri96, size_t n_tri, uint64_t** nodes64, size_t* n_nodes, uint64_t** prim64);
int ceres_camera_basis_f64(const double eye[3], const double dir[3], const double up[3], double fov_deg,
                           size_t width, size_t height, double out9[9]);
int ceres_orbit_cameras_f64(const double eye[3], const double dir[3], const double up[3], const double sun[3],
                            double fov_deg, size_t width, size_t height, const double axis[3], double step_deg,
                            uint32_t n_frames, int rotate_first, double* basis12, double* sun3, double* dir3);
/* The same double steps in a chosen arithmetic (CERES_ARITH_FMA: anim.cpp -d as the reference's
 * CMake build compiles it, -O3 -mavx2 -mfma; pair with CERES_MODE_FMA renders). */
int ceres_obj_load_f64_arith(const char* path, double** tri96, double** norm72, size_t* n_tri, int arith);
int ceres_proc_mesh_f64_arith(int n, double** tri96, double** norm72, size_t* n_tri, int arith);
int ceres_rotate_triangles_f64_arith(double* tri96, size_t n_tri, int axis, double degrees, int arith);
int ceres_bvh_build_f64_arith(const double* tri96, size_t n_tri, uint64_t** nodes64, size_t* n_nodes,
                              uint64_t** prim64, int arith);
int ceres_camera_basis_f64_arith(const double eye[3], const double dir[3], const double up[3], double fov_deg,
                                 size_t width, size_t height, double out9[9], int arith);
int ceres_orbit_cameras_f64_arith(const double eye[3], const double dir[3], const double up[3], const double sun[3],
                                  double fov_deg, size_t width, size_t height, const double axis[3], double step_deg,
                                  uint32_t n_frames, int rotate_first, double* basis12, double* sun3, double* dir3,
                                  int arith);

/* ---- device scene ---- */

#define CERES_SCENE_STATS 1u   /* flag: build the kernels' traversal-statistics variant */
#define CERES_SCENE_FIRST_ORDER 2u  /* flag: order the shadow BVH4's inner children for walks that take the
                                     * first passing child, and walk single frames in that order (automatic
                                     * for scenes whose nearest-first stack would cost waves, e.g. C5) */

/* Upload a scene to HIP device `device` (re-laid for the GPU: sibling-pair 64-B node records,
 * triangles permuted into leaf order).  The caller keeps ownership of its host arrays; they
 * may be freed after the call.  Returns NULL on failure (see ceres_last_error).
 * Replaces the (bvh, triangles, tri_norms) arguments of render() (render.hpp:87-88).
 * Limits (CERES_EUNSUPPORTED): below 2^32 triangles and nodes; the shadow-ray BVH4 packs each
 * child in one word, so triangle slots / BVH4 records stay below 2^27.  Leaves of any size are
 * accepted: BinnedSahBuilder leaves hold up to 16 triangles, but a node whose centroids cannot be
 * split (coincident triangles, the depth cap) stays one bigger leaf; the shadow BVH4 stores a
 * leaf of more than 31 triangles as a node of equal-box pieces. */
ceres_scene* ceres_scene_create(const float* tri48, size_t n_tri, const float* norm36,
                                const void* nodes32, size_t n_nodes, const uint64_t* prim64,
                                int device, uint32_t flags);
/* The same scene from arrays already in HBM of `device`: d_tri48 / d_norm36 as
 * above, the BVH as n_nodes x 32-B nodes with u32 primitive_indices (ceres_bvh_build_device's
 * output).  The GPU layout is built on the GPU (records numbered differently from
 * ceres_scene_create; the traversal and every image are identical).  Ordered on `stream`
 * (a hipStream_t; NULL = the scene's own); the caller keeps its buffers. */
ceres_scene* ceres_scene_create_device(const float* d_tri48, size_t n_tri, const float* d_norm36,
                                       const uint32_t* d_nodes32, size_t n_nodes, const uint32_t* d_prim32,
                                       int device, uint32_t flags, void* stream);
/* Double-precision scene (render<double>, anim.cpp -d): tri96 / norm72 / nodes64 / prim64 as
 * produced by the _f64 host calls (or the reference's own Bvh<double>).  Render it with
 * ceres_render_f64 / ceres_render_records_f64; the float render calls reject it. */
ceres_scene* ceres_scene_create_f64(const double* tri96, size_t n_tri, const double* norm72, const void* nodes64,
                                    size_t n_nodes, const uint64_t* prim64, int device, uint32_t flags);
void ceres_scene_destroy(ceres_scene* scene);
/* depth of the BVH (levels below the root) and the traversal-stack entries the kernels use */
int ceres_scene_info(const ceres_scene* scene, uint32_t* depth, uint32_t* stack_entries,
                     size_t* n_pairs, size_t* device_bytes);
/* shadow-BVH4 traversal-stack bounds: nearest-first walks (any child order) and walks that take
 * the first passing child (after the host's inner-child ordering; device-built scenes: equal) */
int ceres_scene_shadow_stacks(const ceres_scene* scene, uint32_t* nearest_first, uint32_t* first_passing);

/* ---- the hot path ---- */

/* render<float>() (render.hpp:86-156) on host buffers: uploads nothing but the camera,
 * renders on the device, copies back.  pixels (3*W*H floats) and/or rgb8 (3*W*H bytes, PPM
 * body) may be NULL.  basis12 = {eye[3], dir[3], image_u[3], image_v[3]} as produced by
 * ceres_camera_basis (so libm stays on the host and is pinned by fixtures). */
int ceres_render_f32(ceres_scene* scene, const float basis12[12], const float sun[3], int mode,
                     float* pixels, uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats);

/* Device-resident variant for benchmarks and multi-GPU drivers: all output pointers are
 * DEVICE pointers on the scene's device, work is enqueued on `stream` (a hipStream_t, NULL =
 * default stream) and NOT synchronised.  Launches of one scene may be in flight on several
 * streams at once (bench.py does) as long as only one of them at a time passes d_counters.  Outputs cover only this rank's rows (ceres_tiling):
 * d_pixels = 3*W*local_rows floats (local row-major, local row 0 first) or NULL;
 * d_rgb8 = 3*W*local_rows bytes with local row k stored at position local_rows-1-k (so for
 * world = 1 it is exactly the PPM body) or NULL.  d_counters (8 x u64, zeroed by this call)
 * receives {rays, hits, primary_rays, shadow_rays, node_pairs, tri_tests, 0, 0}; may be NULL. */
int ceres_render_device(ceres_scene* scene, const float basis12[12], const float sun[3], int mode,
                        size_t width, size_t height, const ceres_tiling* tiling,
                        float* d_pixels, uint8_t* d_rgb8, uint64_t* d_counters, void* stream);
/* A batch of `frames` (1..64) frames of one scene in ONE launch pair -- the render() call
 * that anim.cpp:93-110 makes once per orbit frame, batched.  basis12 = frames x 12 floats
 * (eye, dir, iu, iv per frame), sun3 = frames x 3 floats.  Frame f of the batch occupies
 * d_pixels[f*3*W*local_rows ...] / d_rgb8[f*3*W*local_rows ...], each laid out exactly as
 * ceres_render_device's; counters are summed over the batch.  Every frame keeps its own
 * camera and sun, and its pixels are bit-identical to a single-frame render. */
int ceres_render_batch_device(ceres_scene* scene, uint32_t frames, const float* basis12,
                              const float* sun3, int mode, size_t width, size_t height,
                              const ceres_tiling* tiling, float* d_pixels, uint8_t* d_rgb8,
                              uint64_t* d_counters, void* stream);
/* Multi-GPU frame assembly (device pointers, async on `stream`): d_gathered holds `world`
 * rank buffers, rank r at byte offset r * rank_stride_bytes, each = that rank's d_rgb8 output
 * of a ceres_render_batch_device call with tiling {row_block, r, world} (F frames back to
 * back).  Writes F PPM bodies (F x 3*W*H bytes) to d_out.  This is the un-interleave after the
 * RCCL gather to rank 0; the reference renders on one host (render.hpp:104). */
int ceres_assemble_rgb8(const uint8_t* d_gathered, size_t rank_stride_bytes, uint8_t* d_out, uint32_t frames,
                        size_t width, size_t height, uint32_t row_block, uint32_t world, void* stream);
/* number of HIP devices visible to this process (negative CERES_E* on error) */
int ceres_device_count(void);
/* render<float>() of one frame split over `world` GPUs in ONE process (`./render --gpus N`):
 * scenes[r] (distinct scene objects, one per rank, each on its own device -- or several on one
 * device for testing) renders rows {row_block, r, world}; the RGB8 rows move peer-to-peer
 * (xGMI) to scenes[0]'s device and are assembled there.  pixels / rgb8 are HOST buffers as in
 * ceres_render_f32 (either may be NULL, not both); the frame is identical to a one-GPU render.
 * stats->ms = wall time of the whole call (render + gather + copy back). */
int ceres_render_multi_f32(ceres_scene* const* scenes, uint32_t world, uint32_t row_block,
                           const float basis12[12], const float sun[3], int mode, float* pixels,
                           uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats);
/* The same un-interleave for PACKED rank buffers (an all-to-all's receive buffer): rank r's
 * `frames` x n_r rows start right after rank r-1's, n_r = ceres_tiling_local_rows of rank r. */
int ceres_assemble_rgb8_packed(const uint8_t* d_gathered, uint8_t* d_out, uint32_t frames, size_t width,
                               size_t height, uint32_t row_block, uint32_t world, void* stream);
/* Per-pixel hit records of one render (host buffers, W*H entries each, pixel = j*W + i):
 * prim = ORIGINAL triangle index of the primary hit or -1 (render.hpp:120), tuv = {t, u, v}
 * of that hit (triangle.hpp:95-115 convention), shadow = -1 (no shadow ray), 0 (lit) or
 * 1 (occluded).  A G-buffer output for parity checks and downstream users. */
int ceres_render_records(ceres_scene* scene, const float basis12[12], const float sun[3], int mode,
                         size_t width, size_t height, int32_t* prim, float* tuv, int8_t* shadow,
                         ceres_stats* stats);
/* rows a rank owns under a tiling */
size_t ceres_tiling_local_rows(size_t height, const ceres_tiling* tiling);
/* render<double>() (render.hpp:86-156 with Scalar = double): pixels = 3*W*H doubles (bottom row
 * first) and/or the RGB8 PPM body, basis12 / sun in double.  Records: t/u/v as doubles. */
int ceres_render_f64(ceres_scene* scene, const double basis12[12], const double sun[3], int mode,
                     double* pixels, uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats);
int ceres_render_records_f64(ceres_scene* scene, const double basis12[12], const double sun[3], int mode,
                             size_t width, size_t height, int32_t* prim, double* tuv, int8_t* shadow,
                             ceres_stats* stats);

/* Per-launch device timing: while enabled, every render records HIP events around its one
 * kernel (ceres_fused, or ceres_primary in primary-only mode) on the stream it was launched on.
 * ceres_scene_read_timing synchronises, returns the summed kernel durations (ms; shadow_ms is
 * always 0: primary and shadow rays run in the same kernel) and the number of renders since the
 * last read, and resets. */
int ceres_scene_set_timing(ceres_scene* scene, int enable);
int ceres_scene_read_timing(ceres_scene* scene, double* kernel_ms, double* shadow_ms, uint64_t* renders);

/* Diagnostic: per-wavefront records of the last full-mode render of a CERES_SCENE_STATS scene
 * (one 8x8 tile per wavefront), 8 x u64 each: {start, after the primary rays, end
 * (s_memrealtime, 100 MHz), longest primary chain (node pairs), shadow-loop trips, primary hits,
 * the wavefront's primary node pairs, its shadow node pairs}.  Synchronises the device. */
int ceres_scene_wave_log(ceres_scene* scene, uint64_t* out, size_t max_waves, size_t* n_waves);

/* Diagnostic (round 6): the bytes the kernels' own fetch sites moved on `device` since the last
 * reset -- out[8] = {64-B sibling-pair records by vector loads (per lane), BVH4 records by vector
 * loads (per lane), BVH4 records through the scalar cache (per wavefront), triangles by vector
 * loads (per lane), triangles through the scalar cache (per wavefront), shading fetches (hit
 * triangle, orig index, vertex normals), framebuffer stores, tile-order entries}.  Only the
 * counting build (`make count`: libceres_hip_count.so, compiled with -DCERES_COUNTING=1) tallies;
 * the product library returns CERES_EUNSUPPORTED.  Synchronises the device; reset != 0 zeroes the
 * tally afterwards.  No reference counterpart: it prices the build against the reference's
 * Statistics (single_ray_traverser.hpp:132-135). */
int ceres_fetch_counters(int device, uint64_t out[8], int reset);

/* ---- the CPU path (./render --cpu) ----
 * render<float>() on host cores, chosen explicitly -- no call falls back to it.  The scene is the
 * product's layout built on the host (sibling-pair records, leaf-ordered triangles) from the same
 * arrays ceres_scene_create takes; the render walks it in the reference's order
 * (single_ray_traverser.hpp:68-126, shadow rays traced closest-hit like render.hpp:135-136) with
 * the arithmetic of the gfx950 kernels, so images, rays and hits equal the reference's in both
 * arithmetics (CERES_MODE_FMA or not), with CERES_MODE_ROBUST / CERES_MODE_PRIMARY as on the GPU
 * (CERES_MODE_QBVH4: CERES_EUNSUPPORTED).  pixels (3*W*H floats, render.hpp:107 layout) and/or rgb8
 * (the PPM body) may be NULL; stats->node_pairs / tri_tests are the reference's Statistics
 * (single_ray_traverser.hpp:132-135) over all rays, stats->ms the wall time.  threads <= 0: the
 * OpenMP default.  Replaces render<float>() (render.hpp:86-156) for a caller without a GPU. */
typedef struct ceres_cpu_scene ceres_cpu_scene;
ceres_cpu_scene* ceres_cpu_scene_create(const float* tri48, size_t n_tri, const float* norm36, const void* nodes32,
                                        size_t n_nodes, const uint64_t* prim64);
void ceres_cpu_scene_destroy(ceres_cpu_scene* scene);
int ceres_render_cpu_f32(const ceres_cpu_scene* scene, const float basis12[12], const float sun[3], int mode,
                         float* pixels, uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats, int threads);
/* render<double> (anim.cpp -d) on host cores: the double arrays of ceres_scene_create_f64, the
 * reference's mixed precision (double rays and traversal, float shading helpers; render64.hip);
 * CERES_MODE_ROBUST is float-only (CERES_EUNSUPPORTED). */
ceres_cpu_scene* ceres_cpu_scene_create_f64(const double* tri96, size_t n_tri, const double* norm72, const void* nodes64,
                                            size_t n_nodes, const uint64_t* prim64);
int ceres_render_cpu_f64(const ceres_cpu_scene* scene, const double basis12[12], const double sun[3], int mode,
                         double* pixels, uint8_t* rgb8, size_t width, size_t height, ceres_stats* stats, int threads);

/* 64-bit content hash of a byte range (multithreaded; deterministic for a given byte string) --
 * what the drop-in include/ceres/render.hpp uses to honour render.hpp:86-156's per-call reading
 * of the caller's triangles / tri_norms / BVH while uploading a scene only when they change. */
uint64_t ceres_content_hash(const void* p, size_t bytes);

/* Launch-geometry introspection for the roofline accounting in bench.py (kernel names as
 * they appear in rocprofv3 traces). */
const char* ceres_kernel_names(void);

const char* ceres_last_error(void);
/* "ceres-mi355x <version> (gfx950) src <16 hex>": the last field is the sha256 of the sources the
 * library was built from (Makefile build_info.o), which bench.py checks against its own tree. */
const char* ceres_version(void);

#ifdef __cplusplus
}
#endif

#endif /* CERES_RENDER_H */
