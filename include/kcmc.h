/*
 * kcmc.h -- C ABI of the MI355X (gfx950) alignment hot path.
 *
 * Drop-in boundary for the per-frame hot path of VideoAligner
 * (reference: /root/reference/VideoAligner.py, cited as VA:<line>).  The reference
 * farms three per-frame functions out to a joblib process pool through
 * VideoAligner._parallelize (VA:460-471).  Each entry point below replaces one of
 * those per-frame calls with ONE batched call over all frames of a slab:
 *
 *   kcmc_match_frames      <- _get_frame_keypoints matching part (VA:194-214):
 *                             cv2.BFMatcher(crossCheck=False).knnMatch(des_t, des_q, k=2),
 *                             best-match reorder, ratio filter, median filter.
 *   kcmc_knn2_l2u8         <- cv2.BFMatcher().knnMatch(..., k=2) alone (VA:194-195).
 *   kcmc_consensus         <- _get_consensus_kps + _lookup_consensus_kps (VA:224-286),
 *                             host-only, reproducing CPython set/Counter ordering.
 *   kcmc_consensus_vote / _merge / _lookup  <- the same consensus in three parts, the
 *                             per-frame parts on the device (frame-sharded jobs exchange
 *                             only the O(n_tpl) votes).
 *   kcmc_ransac_rigid      <- _compute_euclidean_affine (VA:288-323), i.e. skimage 0.18.3
 *                             ransac(EuclideanTransform, 2, 2, max_trials, random_state).
 *   kcmc_warp_affine_u16   <- _apply_affine (VA:455-458): cv2.warpAffine(img, M, (W,H),
 *                             INTER_LINEAR), BORDER_CONSTANT 0, classic fixed-point path.
 *
 * Conventions
 *   - Plain pointers and sizes only.  Pointers named *_dev are device (HBM) pointers
 *     owned by the caller (e.g. torch ROCm tensors' data_ptr()); *_host are host
 *     pointers.  The library never frees caller memory.
 *   - Launch entry points are asynchronous on `stream` (a hipStream_t; NULL = the
 *     null stream) and perform no synchronisation.  The warp, float-matcher and
 *     detector entry points take a per-call workspace from the context's private
 *     stream-ordered memory pool (hipMallocFromPoolAsync / hipFreeAsync on `stream`);
 *     outside stream capture one block per stream is kept and reused in stream order.
 *     Under hipGraph capture the workspace is the graph's own allocation node (never
 *     the per-stream block), so the launches are capturable and a replay never touches
 *     memory that later eager calls may free.  kcmc_ransac_prepare allocates and
 *     synchronises.
 *   - Return value: KCMC_OK (0) or an error code; kcmc_last_error() returns the
 *     calling thread's last message.  Per-frame model failure is NOT an error: it is
 *     NaN in the output parameters, as in the reference (VA:321-322).
 *   - One kcmc_ctx per device; contexts are independent (no global mutable state
 *     except the thread-local error string).
 */
#ifndef KCMC_H_
#define KCMC_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KCMC_ABI_VERSION 2

enum {
  KCMC_OK = 0,
  KCMC_EINVAL = 1,       /* bad argument (maps to ValueError on the Python side) */
  KCMC_EHIP = 2,         /* HIP runtime / launch failure */
  KCMC_ENOMEM = 3,       /* allocation failure */
  KCMC_EUNSUPPORTED = 4, /* shape outside what the kernels implement */
  KCMC_EALIGN = 5        /* too few consensus keypoints (VideoAligner.AlignmentError, VA:241-244) */
};

typedef struct kcmc_ctx kcmc_ctx;
typedef void* kcmc_stream_t; /* hipStream_t */

int kcmc_abi_version(void);
const char* kcmc_last_error(void);

/* hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, stream): the pinned-host <-> device
 * transfers of a pipelined caller (e.g. kcmc_amd.pipeline) without a runtime binding of its own. */
int kcmc_memcpy_async(void* dst, const void* src, size_t bytes, kcmc_stream_t stream);

/* Create / destroy the per-device context (holds the uploaded RANSAC hypothesis
 * tables).  `device` is a HIP device ordinal. */
int kcmc_create(int device, kcmc_ctx** out);
int kcmc_destroy(kcmc_ctx* ctx);

/* ---------------------------------------------------------------- K1: matching
 * Brute-force k=2 nearest neighbours under OpenCV NORM_L2 on uint8 descriptors
 * (cv2.BFMatcher default normType, VA:194), batched over frames.
 *   des_tpl_dev [n_tpl, D] u8      template ("query" in OpenCV terms), shared
 *   des_q_dev   [P, D] u8          all frames' descriptors, frame f = rows
 *                                  q_off[f] .. q_off[f+1]-1 ("train" in OpenCV terms)
 *   q_off_dev   [n_frames+1] i32   CSR offsets (device)
 *   max_nq                          max_f (q_off[f+1]-q_off[f]) (host-known bound)
 *   out_idx_dev [n_frames, n_tpl, 2] i32   train index of best / second best (-1: none)
 *   out_dist_dev[n_frames, n_tpl, 2] f32   sqrtf of the exact integer SSD (FLT_MAX: none)
 * Ties go to the lower frame-keypoint index, as OpenCV's K-insertion does.
 * 1 <= D <= 64. */
int kcmc_knn2_l2u8(kcmc_ctx* ctx, const uint8_t* des_tpl_dev, int n_tpl, int D,
                   const uint8_t* des_q_dev, const int32_t* q_off_dev, int n_frames, int max_nq,
                   int32_t* out_idx_dev, float* out_dist_dev, kcmc_stream_t stream);

/* kcmc_knn2_l2u8 + VA:196-214 per frame:
 *   out_kp_ordered_dev [n_frames, n_tpl, 2] f64 = kp_q[best match] for every template row
 *   out_keep_bits_dev  [n_frames, ceil(n_tpl/32)] u32  bit i = template row i survived the
 *                      ratio filter (d0 < ratio*d1, in double) and the displacement filter
 *                      (d_lo*median <= |kp_t - kp_q| <= d_hi*median over ratio survivors)
 *   out_counts_dev     [n_frames, 4] i32 = the four numbers of the reference's per-frame
 *                      debug log (VA:215-221): len(kp_query) (== n_tpl after the reorder),
 *                      len(matches), #ratio survivors, #distance survivors.
 * kp_tpl_dev [n_tpl, 2] f64, kp_q_dev [P, 2] f64 (cv2 KeyPoint.pt promoted to f64).
 * Every frame must have >= 2 keypoints (the reference raises otherwise, VA:203). */
int kcmc_match_frames(kcmc_ctx* ctx, const uint8_t* des_tpl_dev, const double* kp_tpl_dev, int n_tpl,
                      int D, const uint8_t* des_q_dev, const double* kp_q_dev,
                      const int32_t* q_off_dev, int n_frames, int max_nq, double ratio, double d_lo,
                      double d_hi, int32_t* out_idx_dev, float* out_dist_dev,
                      double* out_kp_ordered_dev, uint32_t* out_keep_bits_dev,
                      int32_t* out_counts_dev, kcmc_stream_t stream);

/* VA:196-214 alone, on knn results of any of the matchers (out_idx / out_dist of
 * kcmc_knn2_l2u8 / _hamming / _l2f32): the outputs of kcmc_match_frames after its knn, so that
 * the filter can run on another stream than the knn (ordered after it by the caller). */
int kcmc_match_filter(kcmc_ctx* ctx, const int32_t* idx_dev, const float* dist_dev, const double* kp_tpl_dev,
                      const double* kp_q_dev, const int32_t* q_off_dev, int n_frames, int n_tpl, double ratio,
                      double d_lo, double d_hi, double* out_kp_ordered_dev, uint32_t* out_keep_bits_dev,
                      int32_t* out_counts_dev, kcmc_stream_t stream);

/* -------------------------------------------------- K1 opt-in: binary descriptors, NORM_HAMMING
 * BFMatcher(NORM_HAMMING).knnMatch(k=2): distance = number of differing bits (as a float),
 * ties to the lower frame index.  NOT the reference's matcher (VA:194 uses the default
 * NORM_L2, kcmc_knn2_l2u8); for binary ORB/BRIEF/AKAZE descriptors where Hamming is
 * wanted.  1 <= D <= 64 bytes, fewer than 2^21 rows per frame.  Arguments as
 * kcmc_knn2_l2u8 / kcmc_match_frames (the filters VA:196-214 are the same). */
int kcmc_knn2_hamming(kcmc_ctx* ctx, const uint8_t* des_tpl_dev, int n_tpl, int D, const uint8_t* des_q_dev,
                      const int32_t* q_off_dev, int n_frames, int max_nq, int32_t* out_idx_dev,
                      float* out_dist_dev, kcmc_stream_t stream);
int kcmc_match_frames_hamming(kcmc_ctx* ctx, const uint8_t* des_tpl_dev, const double* kp_tpl_dev, int n_tpl,
                              int D, const uint8_t* des_q_dev, const double* kp_q_dev, const int32_t* q_off_dev,
                              int n_frames, int max_nq, double ratio, double d_lo, double d_hi,
                              int32_t* out_idx_dev, float* out_dist_dev, double* out_kp_ordered_dev,
                              uint32_t* out_keep_bits_dev, int32_t* out_counts_dev, kcmc_stream_t stream);

/* -------------------------------------------------- K1 extension: float descriptors
 * BFMatcher(NORM_L2).knnMatch(k=2) on float32 descriptors (BASELINE config 5,
 * SIFT-style; the reference's AKAZE/BRISK descriptors are uint8, VA:22-25).  Distance:
 * dist = sqrtf((float)sum_k ((double)a_k - (double)b_k)^2) (sequential fp64 sum; OpenCV's
 * own float accumulation order is build-dependent), ties to the lower
 * frame index.  1 <= D <= 128.  Arguments as kcmc_knn2_l2u8 / kcmc_match_frames. */
int kcmc_knn2_l2f32(kcmc_ctx* ctx, const float* des_tpl_dev, int n_tpl, int D, const float* des_q_dev,
                    const int32_t* q_off_dev, int n_frames, int max_nq, int32_t* out_idx_dev,
                    float* out_dist_dev, kcmc_stream_t stream);
int kcmc_match_frames_f32(kcmc_ctx* ctx, const float* des_tpl_dev, const double* kp_tpl_dev, int n_tpl,
                          int D, const float* des_q_dev, const double* kp_q_dev,
                          const int32_t* q_off_dev, int n_frames, int max_nq, double ratio,
                          double d_lo, double d_hi, int32_t* out_idx_dev, float* out_dist_dev,
                          double* out_kp_ordered_dev, uint32_t* out_keep_bits_dev,
                          int32_t* out_counts_dev, kcmc_stream_t stream);

/* ------------------------------------------------------- host: keypoint consensus
 * VA:224-286 on the host, reproducing CPython 3 set/Counter iteration order exactly:
 *   keep_bits_host [n_frames, ceil(n_tpl/32)] u32 (output of kcmc_match_frames)
 *   out_consensus_host [n_kp_global] i32  template indices in Counter.most_common order
 *   out_votes_host     [n_kp_global] i32  their vote counts
 *   *out_n_consensus   number of entries written (<= n_kp_global)
 *   out_pt_off_host [n_frames+1] i32, out_pt_idx_host [n_frames * n_kp_global] i32:
 *       per-frame template indices of list(consensus_set.intersection(frame_set)),
 *       i.e. the RANSAC point order of VA:274.
 * Returns KCMC_EALIGN if fewer than n_min keypoints received any vote (VA:241-244). */
int kcmc_consensus(const uint32_t* keep_bits_host, int n_frames, int n_tpl, int n_kp_global,
                   int n_min, int32_t* out_consensus_host, int32_t* out_votes_host,
                   int* out_n_consensus, int32_t* out_pt_off_host, int32_t* out_pt_idx_host);
/* The same consensus (from all n_frames frames' bitmasks) with the per-frame lists of
 * frames [f_begin, f_end) only: out_pt_off_host [f_end - f_begin + 1] (starting at 0),
 * out_pt_idx_host [(f_end - f_begin) * n_kp_global].  A rank of a frame-sharded job
 * calls it with its own frame range after the bitmask all-gather, so that its host
 * work per step does not grow with the number of ranks. */
int kcmc_consensus_slice(const uint32_t* keep_bits_host, int n_frames, int n_tpl, int n_kp_global,
                         int n_min, int f_begin, int f_end, int32_t* out_consensus_host,
                         int32_t* out_votes_host, int* out_n_consensus, int32_t* out_pt_off_host,
                         int32_t* out_pt_idx_host);

/* ------------------------------------- keypoint consensus in three parts (VA:224-286)
 * The same consensus split so that each rank of a frame-sharded job works on its own
 * frames and exchanges O(n_tpl) numbers instead of every frame's bitmask:
 *   vote   (per rank)   votes [2, n_tpl] i64: row 0 = Counter count of every template over
 *                        the rank's frames (VA:239); row 1 = its first-occurrence key
 *                        (frame_base + f) << 32 | slot, f the first frame whose set holds it
 *                        and slot its position in that CPython set's table (iteration order),
 *                        INT64_MAX if no frame holds it.
 *   merge  (host)       counts summed over ranks, keys min'ed: Counter.most_common(n_kp_global)
 *                        (VA:240) and the iteration order of set(consensus) (VA:248).
 *   lookup (per rank)   list(consensus_set.intersection(frame_set)) per frame (VA:274) as the
 *                        CSR RANSAC point lists.
 * frame_base = global index of the rank's first frame (0 on one device). */
int kcmc_consensus_vote(kcmc_ctx* ctx, const uint32_t* keep_bits_dev, int n_frames, int n_tpl,
                        long long frame_base, int64_t* out_votes_dev, kcmc_stream_t stream);
int kcmc_consensus_vote_host(const uint32_t* keep_bits_host, int n_frames, int n_tpl, long long frame_base,
                             int64_t* out_votes_host);
/* votes_host [world, 2, n_tpl] (the ranks' vote outputs, any order).  out_consensus_host /
 * out_votes_host [n_kp_global] as kcmc_consensus; out_cons_pack_host [n_kp_global + ceil(n_tpl/32)]
 * i32: set(consensus)'s iteration order in [0, nc), its bitmask (u32 words) in [nc, nc + words)
 * -- the input of kcmc_consensus_lookup.  KCMC_EALIGN if fewer than n_min templates were voted. */
int kcmc_consensus_merge(const int64_t* votes_host, int world, int n_tpl, int n_kp_global, int n_min,
                         int32_t* out_consensus_host, int32_t* out_votes_host, int* out_n_consensus,
                         int32_t* out_cons_pack_host);
/* Device lookup: cons_pack_dev = kcmc_consensus_merge's pack (nc entries + bitmask words);
 * out_pt_off_dev [n_frames + 1], out_pt_idx_dev [n_frames * nc]; scratch_dev of at least
 * kcmc_consensus_lookup_scratch_bytes(n_frames, nc) bytes (the CPython set emulation tables
 * that do not fit in LDS; 0 bytes -- scratch_dev may be NULL -- while nc < 308). */
long long kcmc_consensus_lookup_scratch_bytes(int n_frames, int nc);
int kcmc_consensus_lookup(kcmc_ctx* ctx, const uint32_t* keep_bits_dev, int n_frames, int n_tpl,
                          const int32_t* cons_pack_dev, int nc, int32_t* out_pt_off_dev,
                          int32_t* out_pt_idx_dev, void* scratch_dev, kcmc_stream_t stream);
int kcmc_consensus_lookup_host(const uint32_t* keep_bits_host, int n_frames, int n_tpl,
                               const int32_t* cons_iter_host, int nc, int32_t* out_pt_off_host,
                               int32_t* out_pt_idx_host);

/* The boundary of a slab's RANSAC output for NaN-gap filling across ranks (VA:347-407):
 * params_dev [n_frames, E] f64 (E = 6 for [F,2,3], 9 for [F,3,3]); out_dev [2 + 2E] f64 =
 * (first frame without NaN or -1, last such frame or -1, its E params, the last one's E params). */
int kcmc_params_boundary(kcmc_ctx* ctx, const double* params_dev, int n_frames, int E, double* out_dev,
                         kcmc_stream_t stream);

/* --------------------------------------------------------------- K2: RANSAC
 * The seeded sample stream skimage 0.18.3 consumes: trial t of a frame with n points
 * uses np.random.RandomState(seed).choice(n, min_samples, replace=False) drawn t+1-th
 * (fit.py:791, 819-826), i.e. the first min_samples entries of the t-th legacy
 * MT19937 permutation.  out_host [trials, min_samples] i32.  Host only. */
int kcmc_hypothesis_table(int n, int trials, uint32_t seed, int min_samples, int32_t* out_host);

/* Build (host, cached per context) and upload the rigid (min_samples = 2) tables for
 * the point counts n_values_host[0..count) (each in [3, 65535]).  Allocates and
 * synchronises when a new count appears; call before kcmc_ransac_rigid with every
 * point count that frame batch will run RANSAC on. */
int kcmc_ransac_prepare(kcmc_ctx* ctx, const int32_t* n_values_host, int count, int trials, uint32_t seed);

/* Batched rigid RANSAC, one frame per workgroup.
 * Point k of frame f (k < N_f = pt_off[f+1]-pt_off[f]):
 *   pt_idx_dev == NULL: src = src_dev[pt_off[f]+k], dst = dst_dev[pt_off[f]+k]
 *   pt_idx_dev != NULL: q = pt_idx[pt_off[f]+k]; src = src_dev[f*src_frame_stride + q],
 *                       dst = dst_dev[q]        (src = kcmc_match_frames' kp_ordered,
 *                                                dst = template keypoints: VA:275-276)
 * src = frame keypoints, dst = template keypoints (VA:310).  Frames with
 * N_f < n_skip (VideoAligner.N_KP_FRAME_SKIP) or with no inlier get NaN params.
 *   out_params_dev   [n_frames, 2, 3] f64  model.params[:2], translation * spatial_rate
 *   out_inliers_dev  [P] u8                best hypothesis' inlier mask (skimage ransac's
 *                                          second return value), CSR like the points
 *   out_n_inliers_dev[n_frames] i32, out_best_trial_dev[n_frames] i32 (-1: none)
 * max_n >= every N_f; every N_f >= max(n_skip, 3) must have been prepared with the same
 * `trials` (kcmc_ransac_prepare); a missing table yields NaN for that frame and
 * n_inliers = -1. */
int kcmc_ransac_rigid(kcmc_ctx* ctx, const double* src_dev, const double* dst_dev,
                      const int32_t* pt_idx_dev, const int32_t* pt_off_dev, int src_frame_stride,
                      int n_frames, int max_n, int trials, double residual_threshold,
                      double spatial_rate, int n_skip, double* out_params_dev,
                      uint8_t* out_inliers_dev, int32_t* out_n_inliers_dev,
                      int32_t* out_best_trial_dev, kcmc_stream_t stream);

/* ------------------------------------------------- K2 extension: affine / projective
 * The reference only fits EuclideanTransform (VA:311).  BASELINE configs 3-5 need the
 * other scikit-image 0.18.3 models through the same ransac call (fit.py:621-881):
 *   KCMC_MODEL_AFFINE      ransac(..., AffineTransform,     min_samples=3, ...)
 *   KCMC_MODEL_PROJECTIVE  ransac(..., ProjectiveTransform, min_samples=4, ...)
 * with the same seeded sample stream (RandomState(seed).choice(N, min_samples, False)
 * per trial) and skimage's total-least-squares refit on the inliers
 * (_geometric.py:596-703). */
enum { KCMC_MODEL_EUCLIDEAN = 0, KCMC_MODEL_AFFINE = 1, KCMC_MODEL_PROJECTIVE = 2 };

/* kcmc_ransac_prepare for min_samples in {2, 3, 4} (2 is kcmc_ransac_prepare itself).
 * Every point count must exceed min_samples (skimage raises otherwise, fit.py:798). */
int kcmc_ransac_prepare_samples(kcmc_ctx* ctx, int min_samples, const int32_t* n_values_host, int count,
                                int trials, uint32_t seed);

/* Batched affine / projective RANSAC (model = KCMC_MODEL_AFFINE or _PROJECTIVE); points,
 * pt_idx/pt_off/src_frame_stride, outputs and NaN conventions as kcmc_ransac_rigid,
 * except:
 *   out_params_dev [n_frames, 3, 3] f64  model.params (affine: last row 0 0 1), scaled for
 *                                         spatial downsampling as S H S^-1, S = diag(r, r, 1)
 *                                         (affine: translation * r, like VA:320)
 * Frames with N_f < max(n_skip, min_samples + 1) get NaN.  Tables for every other N_f
 * must have been prepared with kcmc_ransac_prepare_samples(ctx, min_samples, ...). */
int kcmc_ransac_model(kcmc_ctx* ctx, int model, const double* src_dev, const double* dst_dev,
                      const int32_t* pt_idx_dev, const int32_t* pt_off_dev, int src_frame_stride,
                      int n_frames, int max_n, int trials, double residual_threshold,
                      double spatial_rate, int n_skip, double* out_params_dev,
                      uint8_t* out_inliers_dev, int32_t* out_n_inliers_dev,
                      int32_t* out_best_trial_dev, kcmc_stream_t stream);

/* ------------------------------------------------------------------ K3: warp
 * cv2.warpAffine(frame, M_f, (W, H), flags=INTER_LINEAR [| WARP_INVERSE_MAP]) for
 * every frame: src_dev/dst_dev [n_frames, H, W, C] u16 (C interleaved, C=1 for the
 * reference's grayscale stacks), M_dev [n_frames, 2, 3] f64 forward maps (inverted
 * in double exactly as OpenCV does unless inverse_map != 0).  Out-of-image taps
 * read 0.  Bit-exact to the classic OpenCV fixed-point algorithm on platforms
 * without FMA contraction. */
int kcmc_warp_affine_u16(kcmc_ctx* ctx, const uint16_t* src_dev, uint16_t* dst_dev,
                         const double* M_dev, int n_frames, int H, int W, int C, int inverse_map,
                         kcmc_stream_t stream);

/* cv2.warpPerspective(frame, M_f, (W, H), flags=INTER_LINEAR [| WARP_INVERSE_MAP]) for
 * every frame -- the warp of the homography extension (BASELINE config 5; the
 * reference's own warp is warpAffine, VA:458).  M_dev [n_frames, 3, 3] f64 forward maps,
 * inverted like cv::invert (closed-form 3x3) unless inverse_map != 0; classic
 * WarpPerspectiveInvoker fixed-point coordinates (per-block double evaluation, 1/32 px)
 * and the remapBilinear blend of kcmc_warp_affine_u16; out-of-image taps read 0. */
int kcmc_warp_perspective_u16(kcmc_ctx* ctx, const uint16_t* src_dev, uint16_t* dst_dev,
                              const double* M_dev, int n_frames, int H, int W, int C, int inverse_map,
                              kcmc_stream_t stream);

/* ------------------------------------------- f2: normalisation front end (VA:100-104)
 * brightest = np.percentile(images, 99.99) (VA:479-482) needs two order statistics of
 * the flattened uint16 stack; they come from two streaming 256-bin histogram passes:
 *   kcmc_histogram_u16(..., shift = 8, match = -1, ...)   counts of every value's high byte
 *   kcmc_histogram_u16(..., shift = 0, match = h, ...)    counts of the low byte of the values
 *                                                          whose high byte is h
 * out_hist_dev [256] u64 (overwritten).  src_dev 16-byte aligned, n elements. */
int kcmc_histogram_u16(kcmc_ctx* ctx, const uint16_t* src_dev, unsigned long long n, int shift, int match,
                       unsigned long long* out_hist_dev, kcmc_stream_t stream);

/* images_u8 = lut[images] for every element: the host evaluates the reference's
 * np.clip(v / brightest * 255, 0, 255).astype(uint8) (VA:484-492) once per uint16 value
 * (lut_dev [65536] u8); all buffers 16-byte aligned. */
int kcmc_lut_u16_to_u8(kcmc_ctx* ctx, const uint16_t* src_dev, unsigned long long n, const uint8_t* lut_dev,
                       uint8_t* dst_dev, kcmc_stream_t stream);

/* ------------------------------------------------------ f1: keypoint detection
 * The build's exact ORB-style detector (replaces the host OpenCV
 * detectAndCompute of VA:114-116 / VA:190-192, parity vs OpenCV unpinned): FAST-9
 * score > threshold, 3x3 NMS, the n_features largest integer-Harris responses
 * (harris_k), intensity-centroid orientation in 32 bins, steered BRIEF on a 5x5
 * binomial smoothing.  frames_dev [n_frames, H, W] u8 (e.g. kcmc_lut_u16_to_u8 output);
 * pattern_dev [32][512][2] i8 and bin_cs_dev [32][2] f64 from kcmc_amd/orb.py;
 * edge >= 16.  Outputs per frame, in candidate order (64x16 tiles row-major, raster
 * inside a tile): out_kp_dev [n_frames, n_features, 2] f64 (x, y),
 * out_des_dev [n_frames, n_features, 32] u8, out_count_dev [n_frames] i32. */
int kcmc_orb_detect(kcmc_ctx* ctx, const uint8_t* frames_dev, int n_frames, int H, int W, int threshold,
                    int n_features, double harris_k, int edge, const int8_t* pattern_dev,
                    const double* bin_cs_dev, double* out_kp_dev, uint8_t* out_des_dev,
                    int32_t* out_count_dev, kcmc_stream_t stream);

/* ----------------------------------------------------- f4: spatial downsample
 * cv2.pyrDown(frame, dstsize=(dst_w, dst_h)) of every uint8 frame (replaces the per-frame
 * host calls of VideoAligner._downsample, VA:501-503): 5x5 binomial (1,4,6,4,1)^2 / 256,
 * BORDER_REFLECT_101, (sum + 128) >> 8.  src_dev [n_frames, H, W] u8, dst_dev
 * [n_frames, dst_h, dst_w] u8, both 4-byte aligned.  KCMC_EINVAL (OpenCV's assertion)
 * unless |2 dst_w - W| <= 2 and |2 dst_h - H| <= 2. */
int kcmc_pyr_down_u8(kcmc_ctx* ctx, const uint8_t* src_dev, int n_frames, int H, int W, uint8_t* dst_dev,
                     int dst_h, int dst_w, kcmc_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* KCMC_H_ */
