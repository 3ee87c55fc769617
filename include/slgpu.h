/*
 * slgpu.h — C ABI of the MI355X (gfx950) structured-light reconstruction library.
 *
 * Drop-in boundary for the hot path of TtT609/Structured_Light_for_3D_Model_Replication.
 * The reference has no FFI: its boundary is the Python call surface, so each export below
 * replaces one reference function (cited), and the Python package
 * `structured_light_for_3d_model_replication_amd` binds these symbols with ctypes and keeps
 * the reference's signatures.
 *
 *   slg_decode_stats       <- mask thresholds of ProcessingLogic._gray_decode
 *                             (server/processing.py:59-78; Otsu / manual) and of
 *                             SLSystem.generate_cloud.gray_decode (server/sl_system.py:527-543;
 *                             95th-percentile / dynamic range)
 *   slg_decode             <- ProcessingLogic._gray_decode (server/processing.py:28-124) and
 *                             generate_cloud.gray_decode (server/sl_system.py:516-588)
 *   slg_triangulate        <- ProcessingLogic._reconstruct_point_cloud
 *                             (server/processing.py:127-234) and
 *                             generate_cloud.reconstruct_point_cloud (server/sl_system.py:592-661)
 *   slg_reconstruct        <- decode + triangulate of one view as run by
 *                             process_multi_ply._process_source (server/processing.py:286-298)
 *                             without materialising the correspondence maps
 *   slg_decode_triangulate <- the same without the stats launch (after slg_decode_stats)
 *   slg_reconstruct_batch  <- process_multi_ply(mode='batch') over view folders
 *                             (server/processing.py:314-334): many views, one stream
 *   slg_ply_write          <- ProcessingLogic._save_ply (server/processing.py:236-248), host side
 *   slg_ply_format         <- the same lines formatted on the device (batch pipeline)
 *   slg_png_gray8_size /   <- cv2.imread(f, 0) of an 8-bit grayscale capture frame
 *   slg_png_gray8_decode      (server/processing.py:59-60,98-99), host side fast path
 *   slg_rays_match_pinhole <- the `Nc.shape[1] == h*w` ray source test
 *                             (server/processing.py:143-156): tells whether the calibration's
 *                             Nc table equals the cam_K pinhole rays bit for bit, in which case
 *                             the kernels recompute rays instead of gathering 24 B/pixel.
 *
 * Conventions
 *   - All buffer pointers are DEVICE pointers owned by the caller (the library never
 *     allocates or frees caller memory); scratch lives in a caller-provided workspace of
 *     slg_workspace_bytes() bytes, zeroed once with slg_workspace_init().
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).  Every export only
 *     enqueues work (no host synchronisation), so calls can be captured into a hipGraph.
 *   - Return value: SLG_OK (0) or an SLG_ERR_* code; slg_last_error() returns a thread-local
 *     message for the last failing call on the calling thread.
 *   - Frames: uint8 [n_frames][frame_stride] planar stack in capture order (index 0 white,
 *     1 black, then (pattern, inverse) per column bit MSB-first, then per row bit starting
 *     at 2 + 2*ceil(log2(proj_cols))).  frame_stride % 8 == 0 and >= round_up(H*W, 8)
 *     (every frame row is readable in whole 8-byte words), base 8-byte aligned.
 *   - Points are written in ascending pixel order (np.where(mask) order); row_mode 2 writes
 *     the column cloud then the row cloud, like np.hstack((P_col, P_row)).
 */
#ifndef SLGPU_H
#define SLGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SLG_ABI_VERSION 2

#define SLG_OK 0
#define SLG_ERR_INVALID 1      /* bad argument (message in slg_last_error) */
#define SLG_ERR_HIP 2          /* HIP runtime / launch error */
#define SLG_ERR_UNSUPPORTED 3  /* e.g. more than 15 code bits per axis */
#define SLG_ERR_NOT_ENOUGH 4   /* fewer than 4 frames (reference: ValueError) */
#define SLG_ERR_INDEX 5        /* odd trailing frame in the sl_system variant (IndexError) */

/* thresh_mode */
#define SLG_THRESH_OTSU 0        /* processing.py:63-72 */
#define SLG_THRESH_MANUAL 1      /* processing.py:73-76 */
#define SLG_THRESH_PERCENTILE 2  /* sl_system.py:534-540 */

/* variant */
#define SLG_VARIANT_PROCESSING 0 /* ProcessingLogic._gray_decode: first-n bits, rescaled */
#define SLG_VARIANT_SLSYSTEM 1   /* generate_cloud.gray_decode: all bits, break on missing */

/* ray_mode */
#define SLG_RAYS_TABLE 0         /* gather Nc[:, idx] (processing.py:143-144) */
#define SLG_RAYS_PINHOLE 1       /* recompute from cam_K (processing.py:145-156) */

/* Limits (SLG_ERR_UNSUPPORTED otherwise): height*width < 1.43e9 and n_frames*frame_stride
 * < 4 GiB -- the kernels address frames and texture with 32-bit buffer offsets. */
typedef struct slg_capture {
  const uint8_t *frames;   /* device, [n_frames][frame_stride] */
  int64_t frame_stride;    /* bytes between frames (>= round_up(height*width, 8), % 8 == 0) */
  int32_t n_frames;        /* frames present (len(files)) */
  int32_t height;
  int32_t width;
  int32_t reserved;
  const uint8_t *texture;  /* device, [height*width][3] BGR (cv2.imread(files[0])), or NULL for a
                              gray capture: BGR = frame 0 replicated, what cv2.imread(files[0])
                              returns for an 8-bit gray PNG (no texture bytes are then read) */
} slg_capture;

typedef struct slg_decode_params {
  int32_t proj_cols;       /* n_cols  (processing.py:28) */
  int32_t proj_rows;       /* n_rows */
  int32_t n_sets_col;      /* processing variant only (processing.py:83) */
  int32_t n_sets_row;
  int32_t variant;         /* SLG_VARIANT_* */
  int32_t thresh_mode;     /* SLG_THRESH_* */
  double shadow_val;       /* manual: compared as double; pass float32-rounded values for */
  double contrast_val;     /* NumPy-2 weak-scalar semantics (the Python layer does this) */
} slg_decode_params;

typedef struct slg_calib {
  const double *rays;      /* device (3, height*width) C-contiguous, or NULL (SLG_RAYS_PINHOLE) */
  int32_t ray_mode;        /* SLG_RAYS_* */
  int32_t reserved;
  double fx, fy, cx, cy;   /* cam_K[0,0], cam_K[1,1], cam_K[0,2], cam_K[1,2] */
  double oc[3];            /* Oc (always 0 from calibrate_final, sl_system.py:355) */
  const double *col_planes;/* device (n_col_planes, 4) row-major = wPlaneCol.T */
  int32_t n_col_planes;
  int32_t reserved2;
  const double *row_planes;/* device (n_row_planes, 4) row-major = wPlaneRow.T */
  int32_t n_row_planes;
  int32_t reserved3;
  /* Optional (NULL: the kernels compute numer per point; same values either way): */
  const double *col_planes_num; /* device (2, n_col_planes, 2) "pair planes": [0][c] = (n0, n1),
                                 * [1][c] = (n2, numer), numer = ((n0*Oc0 + n1*Oc1) + n2*Oc2) + d
                                 * (processing.py:163-166), so a wave's neighbouring column codes
                                 * gather neighbouring 16-byte pairs */
  const double *row_planes_num; /* the same for the row planes (read by row_mode 2 only) */
} slg_calib;

typedef struct slg_tri_params {
  int32_t row_mode;        /* 0 col only, 1 epipolar filter, 2 col+row clouds (processing.py:174-234) */
  int32_t xyz_f64;         /* 1: XYZ float64 (bit-exact with the reference); 0: float32 */
  double epipolar_tol;     /* processing.py:199 */
} slg_tri_params;

typedef struct slg_maps {
  const int32_t *col;      /* device [height*width] */
  const int32_t *row;      /* device [height*width] (may be NULL for row_mode 0) */
  const uint8_t *mask;     /* device [height*width] bool */
  const uint8_t *texture;  /* device [height*width][3] BGR */
  int32_t height;
  int32_t width;
} slg_maps;

typedef struct slg_cloud {
  void *xyz;               /* device [capacity][3] float or double */
  uint8_t *bgr;            /* device [capacity][3] */
  int64_t *count;          /* device, 1 element: number of points written */
  int64_t capacity;        /* >= height*width (row_mode 0/1) or 2*height*width (row_mode 2) */
} slg_cloud;

int32_t slg_version(void);
const char *slg_last_error(void);
/* Digest of the sources and flags this library was built from (build.py: sha256 of every
 * source, the header and the compile flags); _native.lib() refuses a library whose digest does
 * not match the sources beside it. */
const char *slg_build_id(void);
/* The fused kernel's instance table, one line per instance ("<symbol>\t<0|1>\n", 1 = its device
 * code is in the library's gfx950 code object) into buf (cap bytes, NUL-terminated; truncated
 * lines are dropped).  Returns the number of instances missing, or -SLG_ERR_INVALID.  Launches
 * of a missing instance return SLG_ERR_UNSUPPORTED instead of reaching the HIP runtime, which
 * aborts on them.  Reads the library file only (no HIP call). */
int32_t slg_kernel_table(char *buf, int64_t cap);
/* The symbol of the fused kernel instance that the calling thread's last fused launch picked from
 * that table, into buf (cap bytes, NUL-terminated); "" when the thread has picked none, or its last
 * pick found no instance.  A test hook: the GPU suite checks that every instance of the table runs and
 * matches the oracle.  Host only (no HIP call). */
int32_t slg_last_kernel(char *buf, int64_t cap);

/* Workspace size for images of n_pixels (covers every mode). */
int64_t slg_workspace_bytes(int64_t n_pixels);
/* Zero a freshly allocated workspace (once; the kernels keep it consistent afterwards). */
int32_t slg_workspace_init(void *workspace, int64_t workspace_bytes, void *stream);

/* Resident jobs (jobs.ResidentJob): bind n_slices workspace slices (ws_stride apart) to one
 * packed output arena of capacity_points points.  From then on, whichever kernel sets a slice's
 * thresholds (stats, partials, a fused launch's finishing workgroups) also reserves the view's
 * region: atomicAdd(*cursor, need) with need = min(#white >= smin, #(white - black) >= cmin) x
 * points_per_valid (1: row_mode 0/1, 2: row_mode 2) -- an upper bound of the view's points -- so
 * no view can write past its region; no room left: the view stores nothing.  The fused launches
 * then take every bound slice's cloud (slg_cloud) as: xyz / bgr = the arena's base, capacity =
 * the arena's, count -> int64[2] = {points, first point index in the arena or -1 (no room: re-run
 * the view)}.  The caller zeroes *cursor (device int64) before each job; cursor NULL unbinds.
 * Asynchronous on `stream`. */
int32_t slg_workspace_set_arena(void *workspace, int64_t ws_stride, int32_t n_slices, int64_t *cursor,
                                int64_t capacity_points, int32_t points_per_valid, void *stream);

/* Histograms + thresholds of the valid mask into the workspace; also arms the workspace for
 * the next slg_decode / slg_reconstruct on the same stream. */
int32_t slg_decode_stats(const slg_capture *cap, const slg_decode_params *dp, void *workspace,
                         void *stream);

/* One view split over ranks by bands of rows ("single huge view"; its one exchange
 * step).  slg_decode_histograms writes the band's mask histograms, summed over the band, to
 * hist_out (device uint32[513]): Otsu -> [0..255] white, [256..511] clip(white - black, 0, 255)
 * (processing.py:63-72); percentile -> [0..255] black, [512] = max(white - black) + 256
 * (sl_system.py:534-540).  The ranks add [0..511] and take the max of [512] (RCCL all-reduce);
 * slg_thresholds_from_histograms then sets this band's workspace thresholds from the view's
 * totals (n_pixels = the whole view's, so the thresholds are the unsplit view's, bit for bit) and
 * arms it for slg_decode_triangulate of the band (n_band_pixels).  Manual thresholds need no
 * exchange: slg_decode_stats on the band.  Each band's cloud is its rows' points in pixel order,
 * so rank-ordered concatenation is the view's cloud (row_mode 2: every band's column cloud, then
 * every band's row cloud). */
int32_t slg_decode_histograms(const slg_capture *cap, const slg_decode_params *dp, void *workspace,
                              uint32_t *hist_out, void *stream);
int32_t slg_thresholds_from_histograms(const uint32_t *hist, int64_t n_pixels, const slg_decode_params *dp,
                                       void *workspace, int64_t n_band_pixels, void *stream);

/* Gray decode to correspondence maps (after slg_decode_stats on the same workspace). */
int32_t slg_decode(const slg_capture *cap, const slg_decode_params *dp, void *workspace,
                   int32_t *col_out, int32_t *row_out, uint8_t *mask_out, void *stream);

/* Ray-plane triangulation + ordered compaction from maps.  Arms the workspace itself. */
int32_t slg_triangulate(const slg_maps *maps, const slg_calib *calib, const slg_tri_params *tp,
                        void *workspace, const slg_cloud *out, void *stream);

/* Fused: stats + decode + triangulate + compaction of one view (maps never hit HBM). */
int32_t slg_reconstruct(const slg_capture *cap, const slg_decode_params *dp,
                        const slg_calib *calib, const slg_tri_params *tp, void *workspace,
                        const slg_cloud *out, void *stream);

/* The fused decode+triangulate launch alone (slg_reconstruct minus the stats launch): call
 * after slg_decode_stats on the same workspace and stream. */
int32_t slg_decode_triangulate(const slg_capture *cap, const slg_decode_params *dp,
                               const slg_calib *calib, const slg_tri_params *tp, void *workspace,
                               const slg_cloud *out, void *stream);

/* A batch of views of one geometry (turntable scan, scan farm; frame counts may differ):
 * per group of up to 16 views, one batched stats launch and ONE fused decode+triangulate launch
 * covering every view of the group (no host sync).  `workspace` holds n_views slices of
 * `ws_stride` bytes (>= slg_workspace_bytes, % 256 == 0), each initialised once; outs[v]
 * receives view v.  timing_events (optional: NULL, or 2 hipEvent_t / NULL entries per group of
 * 16 views) are recorded around each fused launch. */
int32_t slg_reconstruct_batch(const slg_capture *caps, int32_t n_views, const slg_decode_params *dp,
                              const slg_calib *calib, const slg_tri_params *tp, void *workspace,
                              int64_t ws_stride, const slg_cloud *outs, void *const *timing_events,
                              void *stream);

/* The two halves of slg_reconstruct_batch, so a caller can run the stats of the next batch on a
 * second stream while this batch's fused launch runs (each view's workspace slice must not be
 * shared between the two batches in flight). */
int32_t slg_decode_stats_batch(const slg_capture *caps, int32_t n_views, const slg_decode_params *dp,
                               void *workspace, int64_t ws_stride, void *stream);
int32_t slg_decode_triangulate_batch(const slg_capture *caps, int32_t n_views, const slg_decode_params *dp,
                                     const slg_calib *calib, const slg_tri_params *tp, void *workspace,
                                     int64_t ws_stride, const slg_cloud *outs, void *const *timing_events,
                                     void *stream);

/* Streaming turntable batches (thresh_mode OTSU only): the fused launch of batch k also
 * computes the Otsu histograms of batch k+2 (`next`, n_next <= n_views views, same geometry),
 * one 1 KB partial per 2048-pixel tile in each view's workspace slice; no separate pass over
 * the white/black frames of batch k+2 is needed.  Batch k+2 must then use the SAME workspace
 * slices as batch k, and slg_decode_stats_partials_batch on them (after this launch, before
 * batch k+2's fused launch; it may overlap batch k+1's) turns the partials into thresholds and
 * arms the slices for batch k+2.  Results are identical to slg_decode_stats_batch. */
int32_t slg_decode_triangulate_batch_next(const slg_capture *caps, int32_t n_views,
                                          const slg_decode_params *dp, const slg_calib *calib,
                                          const slg_tri_params *tp, void *workspace, int64_t ws_stride,
                                          const slg_cloud *outs, const slg_capture *next,
                                          int32_t n_next, void *const *timing_events, void *stream);
int32_t slg_decode_stats_partials_batch(int32_t n_views, int32_t height, int32_t width,
                                        const slg_decode_params *dp, void *workspace,
                                        int64_t ws_stride, void *stream);

/* The streaming turntable pipeline on ONE stream (what BatchReconstructor.run_pipelined
 * "fused" issues): slg_decode_triangulate_batch_next, plus `n_fin` views whose partials an
 * EARLIER launch on this stream carried (slices at fin_workspace + v * ws_stride) turned into
 * thresholds by finishing workgroups at the front of this launch's grid -- the work of
 * slg_decode_stats_partials_batch without its kernel or a second stream.  Batch k's launch
 * carries batch k+2 and finishes batch k+1; fin_workspace must not be this launch's own
 * workspace.  The finished batch must share this launch's geometry (height, width) and decode
 * parameters `dp` (its slices are read with them; nothing else identifies it).  ws_stride must
 * be >= slg_workspace_bytes and 256-aligned whenever n_views, n_next or n_fin exceeds 1.
 * Results are identical to slg_decode_stats_batch. */
int32_t slg_decode_triangulate_batch_carry(const slg_capture *caps, int32_t n_views,
                                           const slg_decode_params *dp, const slg_calib *calib,
                                           const slg_tri_params *tp, void *workspace, int64_t ws_stride,
                                           const slg_cloud *outs, const slg_capture *next,
                                           int32_t n_next, void *fin_workspace, int32_t n_fin,
                                           void *const *timing_events, void *stream);

/* Count (into *mismatches, device int64) the Nc entries that differ bitwise from the cam_K
 * pinhole rays; 0 means SLG_RAYS_PINHOLE reproduces the table exactly. */
int32_t slg_rays_match_pinhole(const double *rays, int32_t height, int32_t width, double fx,
                               double fy, double cx, double cy, int64_t *mismatches,
                               void *stream);

/* Colour captures (the phone path: canvas PNGs uploaded by frontend/App.tsx:234-247 and saved
 * as-is by server/server.py:86) on the device, from ONE upload of the decoded frames:
 * gray[f][i] = cv2.imread(f, 0) of rgb frame f (RGB or RGBA bytes, `channels` 3|4, frame f at
 * rgb + f * src_stride) into a frame stack of gray_stride, and, when bgr0 is not NULL, frame 0
 * as the BGR texture cv2.imread(files[0]) returns.  weights: libpng's rgb_to_gray fixed point
 * (PNG) or OpenCV's BGR2GRAY weights (BMP) -- restated from the libraries' published formulas,
 * parity unpinned (no OpenCV here).  Replaces the host conversion of frames.py. */
#define SLG_GRAY_PNG 0
#define SLG_GRAY_BMP 1
int32_t slg_rgb_to_gray(const uint8_t *rgb, int32_t channels, int64_t n_pixels, int64_t src_stride,
                        int32_t n_frames, uint8_t *gray, int64_t gray_stride, uint8_t *bgr0,
                        int32_t weights, void *stream);
/* Texture of a gray capture (cv2.imread(files[0]) of an 8-bit gray PNG: frame 0 replicated to
 * B, G, R) built on the device from the uploaded frame 0: no host replication, no extra upload. */
int32_t slg_gray_texture(const uint8_t *frame0, int64_t n_pixels, uint8_t *bgr, void *stream);

/* Host: write an ASCII PLY exactly as ProcessingLogic._save_ply does (processing.py:236-248):
 * header, then "%.4f %.4f %.4f R G B" per point (Python's correctly rounded formatting, BGR
 * swapped to RGB).  xyz/bgr are HOST arrays [n][3].  Formats on n_threads host threads
 * (<= 0: all cores).  Returns bytes written, or -SLG_ERR_* on failure. */
int64_t slg_ply_write(const char *path, const double *xyz, const uint8_t *bgr, int64_t n,
                      int32_t n_threads);

/* Device: the BODY of the same PLY (the lines after end_header), formatted on the GPU from a
 * DEVICE cloud (xyz float64 [n][3], bgr uint8 [n][3]) into DEVICE `text`, so a batch's clouds
 * leave HBM as the bytes to write (processing.py:245-248; byte-identical with slg_ply_write).
 * `text` holds slg_ply_format_bound(n) bytes, `ws` slg_ply_format_ws_bytes(n) bytes (device).
 * Asynchronous on `stream`; afterwards ws holds {int64 body_bytes; int32 bad; int32 pad}: bad
 * != 0 means a coordinate is NaN, infinite or >= 9.2e14 in magnitude, the body is not written,
 * and the caller formats on the host (slg_ply_write).  Returns 0 or SLG_ERR_*. */
int64_t slg_ply_format_bound(int64_t n);
int64_t slg_ply_format_ws_bytes(int64_t n);
int32_t slg_ply_format(const double *xyz, const uint8_t *bgr, int64_t n, char *text, void *ws, void *stream);

/* Host: frame ingest fast path for cv2.imread(f, 0) (processing.py:59-60,98-99) on 8-bit
 * grayscale, non-interlaced PNGs, where it is the identity on the stored samples.
 * slg_png_gray8_size returns 0 and the size for such a file, non-zero for any other file
 * (decode it the general way).  slg_png_gray8_decode fills out[height][width]; non-zero on a
 * CRC error, a truncated stream or a size mismatch.  Thread-safe (one call per decode thread). */
int32_t slg_png_gray8_size(const char *path, int32_t *width, int32_t *height);
int32_t slg_png_gray8_decode(const char *path, uint8_t *out, int64_t cap, int32_t width,
                             int32_t height);

/* Host: any other PNG (colour, gray + alpha, palette, 1-16 bits, Adam7) decoded to exactly what
 * OpenCV's PNG decoder returns: cv2.imread(f, 0) into gray[height][width] and / or cv2.imread(f)
 * into bgr[height][width][3] (either may be NULL; caps in bytes).  OpenCV converts through libpng
 * (png_set_strip_16, png_set_strip_alpha, png_set_palette_to_rgb, png_set_expand_gray_1_2_4_to_8,
 * then png_set_bgr / png_set_gray_to_rgb / png_set_rgb_to_gray(png, 1, 0.299, 0.587)); that
 * arithmetic -- gamma tables of gAMA / sRGB files included -- is restated, pinned byte for byte
 * to libpng 1.6.37 (tests/test_png_color.py), and the files whose colour handling libpng decides
 * from data not restated (iCCP profiles, duplicate / invalid / disagreeing gAMA and sRGB) go
 * through the system libpng itself.  info[7]: {width, height, colour type, bit depth, interlace,
 * restated (1) or libpng (0), decoded by libpng (1)}.  slg_png_info fills info[0..5] only.
 * Return 0, else non-zero (unreadable, corrupt or unsupported: cv2.imread would return None).
 * Thread-safe. */
int32_t slg_png_info(const char *path, int32_t *info /* [6] */);
int32_t slg_png_read(const char *path, uint8_t *gray, int64_t gray_cap, uint8_t *bgr, int64_t bgr_cap,
                     int32_t *info /* [7] */);

/* PNG decode on the device (the same cv2.imread of every used frame, for the batch file path):
 * the host only reads the file and checks its chunks, the GPU inflates and un-filters.
 * slg_png_zstream (host): for an 8-bit, non-interlaced PNG of colour type 0 (gray), 2 (RGB),
 * 4 (gray + alpha) or 6 (RGBA) -- a colour one only without gAMA / sRGB / iCCP chunks, whose
 * gray conversion (libpng's gamma path) is slg_png_read's -- copies the concatenated IDAT payload (the zlib stream) into
 * buf (cap bytes; needs zlen + 8, the file size + 8 always suffices) and fills info[4] =
 * {width, height, channels, zlen}; returns 0, else non-zero (any other file, a CRC error, cap
 * too small: decode it the general way).  Thread-safe.
 * slg_png_decode_device: decodes n frames (DEVICE descriptors `frames`, each naming DEVICE
 * buffers: z = the zlib stream as read by slg_png_zstream, 4-byte aligned and readable for
 * zlen + 8 bytes; raw = scratch of slg_png_raw_bytes(w, h, ch) bytes; out = the samples,
 * [height][out_pitch] rows of width * channels bytes).  status is DEVICE int32 [2 * n]:
 * status[2f] = 0 or SLG_PNG_E_* (a frame with a non-zero status is left unspecified and must
 * be decoded on the host), status[2f + 1] internal.  Asynchronous on `stream`; returns 0 or SLG_ERR_*. */
#define SLG_PNG_E_STREAM 1     /* not a valid zlib/deflate stream (or reads past zlen) */
#define SLG_PNG_E_SIZE 2       /* inflated size differs from height * (1 + width * channels) */
#define SLG_PNG_E_ADLER 3      /* Adler-32 of the inflated bytes differs from the stream's */
#define SLG_PNG_E_FILTER 4     /* a scanline filter type byte > 4 */
#define SLG_PNG_E_UNSUPPORTED 5 /* rows wider than the device un-filter takes (width * channels > 24576) */
typedef struct slg_png_frame {
  const uint8_t *z;        /* zlib stream (device) */
  int64_t zlen;
  uint8_t *raw;            /* scratch (device), slg_png_raw_bytes() */
  uint8_t *out;            /* samples (device) */
  int64_t out_pitch;       /* bytes between output rows (>= width * channels) */
  int32_t width, height, channels, reserved;
} slg_png_frame;
int32_t slg_png_zstream(const char *path, uint8_t *buf, int64_t cap, int32_t *info /* [4] */);
int64_t slg_png_raw_bytes(int32_t width, int32_t height, int32_t channels);
int32_t slg_png_decode_device(const slg_png_frame *frames, int32_t n, int32_t *status, void *stream);
/* A stream for the device PNG decode that leaves CUs free (hipExtStreamCreateWithCUMask): every
 * `reserve_every`-th CU of the current device is left out of its mask, so a long inflate launch
 * (one 50 KB-LDS wave per stream, ~225 ms) cannot occupy every CU and the batch pipeline's fused
 * launches of host-decoded views keep running beside it.  *stream = the hipStream_t; returns 0
 * or SLG_ERR_*.  slg_stream_destroy releases it. */
int32_t slg_stream_create_reserving(int32_t reserve_every, void **stream);
int32_t slg_stream_destroy(void *stream);

/* ---- Multi-GPU: the final point-cloud gather of a view-sharded scan.
 * Replaces nothing in the reference (its batch loop is serial, server/processing.py:314-334);
 * it is the one collective of the sharded path: after every rank has reconstructed its block
 * of turntable views, the clouds move to one rank over RCCL (xGMI), exact sizes only.
 * RCCL is resolved at run time (the librccl.so.1 already in the process, e.g. torch's).
 *   1. rank 0: slg_gather_unique_id(id); the caller distributes the 128 bytes (e.g. a
 *      torch.distributed broadcast);  every rank: slg_gather_init(&comm, n_ranks, rank, id),
 *      with its HIP device current;
 *   2. slg_gather_counts: all-gather of n_per_rank int64 counts per rank (device buffers,
 *      all_counts = [n_ranks][n_per_rank]); the caller reads them to size the root's buffer;
 *   3. slg_gatherv: rank r's send_bytes land at root's recv + sum(recv_bytes[:r]) (recv and the
 *      HOST array recv_bytes[n_ranks] are read on the root only); grouped point-to-point;
 *   4. slg_gather_destroy.  All calls enqueue on `stream` (hipStream_t). */
#define SLG_GATHER_ID_BYTES 128
typedef struct slg_gather_comm slg_gather_comm;
int32_t slg_gather_unique_id(uint8_t *id /* [SLG_GATHER_ID_BYTES] */);
int32_t slg_gather_init(slg_gather_comm **comm, int32_t n_ranks, int32_t rank, const uint8_t *id);
int32_t slg_gather_counts(slg_gather_comm *comm, const int64_t *counts, int32_t n_per_rank,
                          int64_t *all_counts, void *stream);
int32_t slg_gatherv(slg_gather_comm *comm, const void *send, int64_t send_bytes, void *recv,
                    const int64_t *recv_bytes, int32_t root, void *stream);
int32_t slg_gather_destroy(slg_gather_comm *comm);
/* Host only, no RCCL: the plan slg_gatherv follows.  On the root (rank == root): checks
 * recv_bytes (non-negative, recv_bytes[root] == send_bytes), writes offsets[n_ranks + 1] (rank
 * r lands at recv + offsets[r], offsets[n_ranks] = total) and recv_from[n_ranks] (1 = a
 * point-to-point receive from that peer; 0 for the root, whose own part is a device copy, and
 * for zero-byte peers).  On other ranks: recv_from[0] = 1 when the rank sends (send_bytes > 0),
 * offsets untouched.  Returns the number of point-to-point operations this rank issues, or a
 * negative SLG_ERR_* code (slg_last_error() says why). */
int32_t slg_gatherv_plan(int32_t n_ranks, int32_t rank, int32_t root, int64_t send_bytes,
                         const int64_t *recv_bytes, int64_t *offsets, int32_t *recv_from);

#ifdef __cplusplus
}
#endif

#endif /* SLGPU_H */
