/* omv.h — C ABI of the MI355X-native OpenMAVIS hot path (libomv_hip.so).
 *
 * Plain pointers and sizes only; no torch / OpenCV / Eigen types.  Every call is reentrant per
 * handle; a handle must not be used by two threads at once (the reference's extractors have the
 * same rule: one ORBextractor per camera thread, src/Frame.cc:1841-1862).  Device pointers are HIP
 * device memory; `stream` is a hipStream_t (NULL = the default stream).  Functions return an
 * omv_status; nothing throws across the ABI.
 *
 * Each entry point names the reference interface it replaces (file:line in the reference).
 */
#ifndef OMV_H
#define OMV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int omv_status;
#define OMV_OK 0
#define OMV_ERR_ARG 1          /* bad argument (NULL, size out of range)                        */
#define OMV_ERR_HIP 2          /* a HIP runtime call failed                                     */
#define OMV_ERR_CAPACITY 3     /* a device-side capacity was exceeded (reported, never silent)  */
#define OMV_ERR_NO_DEVICE 4    /* no HIP device visible: there is no CPU fallback               */

/* ------------------------------------------------------------------------------------------------
 * ORB extraction — replaces ORBextractor::ORBextractor (src/ORBextractor.cc:351-414) and
 * ORBextractor::operator() (include/ORBextractor.h:33-38, src/ORBextractor.cc:987-1071).
 * ---------------------------------------------------------------------------------------------- */
typedef struct omv_orb_params {
    int nfeatures;      /* ORBextractor.nFeatures                                  */
    float scale_factor; /* ORBextractor.scaleFactor (1.2)                          */
    int nlevels;        /* ORBextractor.nLevels (8)                                */
    int ini_th_fast;    /* ORBextractor.iniThFAST                                  */
    int min_th_fast;    /* ORBextractor.minThFAST                                  */
} omv_orb_params;

/* cv::KeyPoint fields the reference reads (pt, size, angle, response, octave); 24 bytes. */
typedef struct omv_kp {
    float x, y, size, angle, response;
    int32_t octave;
} omv_kp;

typedef struct omv_orb omv_orb;

/* Create an extractor for images of width x height (u8), batching up to max_images per call. */
omv_status omv_orb_create(const omv_orb_params *params, int width, int height, int max_images,
                          omv_orb **out);
omv_status omv_orb_destroy(omv_orb *orb);

/* Test hook (no reference counterpart): the device replica of libstdc++'s std::sort that the octree
 * uses for DistributeOctTree's compareNodes order (src/ORBextractor.cc:482-494, :629-632), on one
 * array of n <= 2048 (k1, k2) pairs with k1 >= 0, 0 <= k2 < 2^20 (device memory); perm receives the
 * original indices in sorted order. */
omv_status omv_selftest_node_sort(const int *k1, const int *k2, int n, int *perm, void *stream);

/* Upper bound on keypoints one image can produce (output row capacity N_max).  The reference can
 * return up to quota+2 keypoints per level (DistributeOctTree :673 stops at >= N). */
int omv_orb_max_keypoints(const omv_orb *orb);

/* The ORBextractor getters (include/ORBextractor.h:40-50): nlevels floats each, host memory. */
omv_status omv_orb_scale_tables(const omv_orb *orb, float *scale, float *inv_scale, float *sigma2,
                                float *inv_sigma2);

/* Batched ORBextractor::operator() over n_images device-resident images.
 *   images      device, image i at images + i*image_stride, rows `pitch` bytes apart
 *   lapping     host, 2 ints per image: [x0, x1] (vLappingArea)
 *   kps         device, [n_images][N_max] omv_kp
 *   desc        device, [n_images][N_max][32] u8
 *   n_out       device, [n_images] keypoint count (rows of kps/desc that are valid)
 *   mono_index  device, [n_images] return value of operator() (monoIndex)
 * Output order per image is the reference's: non-lapping keypoints from the front, lapping ones
 * from the back in reverse, level by level.  Asynchronous on `stream`. */
omv_status omv_orb_extract_batch(omv_orb *orb, int n_images, const uint8_t *images, size_t image_stride,
                                 size_t pitch, const int *lapping, omv_kp *kps, uint8_t *desc, int *n_out,
                                 int *mono_index, void *stream);

/* Synchronous host-memory convenience used by the ORBextractor::operator() adapter: stages one
 * image H2D, extracts, copies back.  Returns monoIndex in *mono_index and the count in *n_out. */
omv_status omv_orb_extract_host(omv_orb *orb, const uint8_t *image, size_t pitch, int lap0, int lap1,
                                omv_kp *kps, uint8_t *desc, int *n_out, int *mono_index);

/* Optional extra output of the following omv_orb_extract_batch calls: per output row (the omv_kp layout
 * [image][N_max]) OpenCV ORB's Harris response (orb.cpp HarrisResponses, blockSize 7, k 0.04) at the keypoint's
 * level position -- the north star's "Harris score".  The reference never computes it (its HARRIS_SCORE is a dead
 * enum, include/ORBextractor.h:24; KeyPoint::response stays FAST's cornerScore).  NULL (default) disables it. */
omv_status omv_orb_set_harris(omv_orb *orb, float *harris);

/* Device-side error word of the last batch (OMV_ERR_CAPACITY if a bound was hit); syncs the stream. */
omv_status omv_orb_last_error(omv_orb *orb);

/* Per-stage device time (HIP events on the launch stream) for measurement: stages are
 * 0 pyramid, 1 FAST cells, 2 octree, 3 orientation + GaussianBlur 7x7 at the samples + descriptor.  omv_orb_stage_ms
 * syncs, returns the accumulated milliseconds since the last reset and the number of timed batches. */
omv_status omv_orb_enable_timing(omv_orb *orb, int on);
omv_status omv_orb_stage_ms(omv_orb *orb, double *ms4, long long *calls, int reset);

/* Measurement: FAST candidates (the octree's input) and distributed keypoints of the last batch, summed over its
 * images (synchronous read-back). */
omv_status omv_orb_last_counts(omv_orb *orb, long long *n_candidates, long long *n_keypoints);

/* Debug/parity hooks: copy pyramid level `level` of image `img` of the last batch to host. */
omv_status omv_orb_debug_level(omv_orb *orb, int img, int level, uint8_t *out, int *w, int *h);

/* ------------------------------------------------------------------------------------------------
 * Hamming matching on multi-camera frames
 *
 * Frame layout (device): keypoints/descriptors padded per camera block, kps [frame][cam][kp_cap],
 * desc [frame][cam][kp_cap][32], n_kp [frame][cam] (the extractor's batched output as-is).  Block 0
 * is the left camera, block 1 the right camera, blocks >= 2 side cameras — the reference's
 * [L|R|SL|SR] concatenation (src/Frame.cc:1936-1939) generalised to n_cams.  A keypoint "slot" is
 * cam * kp_cap + i; per-slot arrays (kp_to_mp, occupancy) are [frame][n_cams * kp_cap].
 * ---------------------------------------------------------------------------------------------- */
typedef struct omv_frame_geom {
    int n_cams;
    float min_x, max_x;  /* Frame::mnMinX/mnMaxX (bounds of imLeft, shared by all cameras, Frame.cc:1875) */
    float min_y, max_y;
    int nlevels;
    float scale_factors[16]; /* Frame::mvScaleFactors                                              */
    /* GeometricCamera type per camera block (Frame::mpCamera, mpCamera2, ...): OMV_CAM_KB8 (0, the
     * zero-initialised default) or OMV_CAM_PINHOLE.  The projection searches project with it:
     * SearchByProjection(F, LastF) block 0 (ORBmatcher.cc:2022, :2134), Fuse / SearchByProjection(KF, Sim3) /
     * SearchByProjection(F, KF) the job's block (:1536, :1710, :710, :2443). */
    int cam_model[8];
} omv_frame_geom;

/* Local map points projected into a frame (the MapPoint fields SearchByProjection reads after
 * Frame::isInFrustum, src/ORBmatcher.cc:33-60).  Device SoA: per-point arrays are [frame][M],
 * per-camera arrays [frame][M][n_cams]. */
typedef struct omv_mp_view {
    const uint8_t *desc;      /* [M][32] MapPoint::GetDescriptor()                                  */
    const float *proj_x;      /* [M][n_cams] mTrackProjX / XR / XSL / XSR ...                       */
    const float *proj_y;      /* [M][n_cams]                                                        */
    const float *view_cos;    /* [M][n_cams] mTrackViewCos*                                         */
    const int32_t *level;     /* [M][n_cams] mnTrackScaleLevel* (-1 = none)                         */
    const uint8_t *in_view;   /* [M][n_cams] mbTrackInView*                                         */
    const float *track_depth; /* [M] mTrackDepth                                                    */
    const uint8_t *is_bad;    /* [M] MapPoint::isBad()                                              */
    const uint8_t *has_obs;   /* [M] Observations() > 0                                             */
} omv_mp_view;

typedef struct omv_matcher omv_matcher;

/* Workspace for up to max_frames frames of n_cams blocks x kp_cap keypoints and max_mps points. */
omv_status omv_matcher_create(int max_frames, int n_cams, int kp_cap, int max_mps, omv_matcher **out);
omv_status omv_matcher_destroy(omv_matcher *m);

/* Frame::AssignFeaturesToGrid (src/Frame.cc:541-582) for n_frames frames: per camera a 64x48 grid
 * (cell = ix*48 + iy) of ascending keypoint indices, kept in the handle for the searches below. */
omv_status omv_matcher_assign_grid(omv_matcher *m, int n_frames, const omv_frame_geom *geom, const omv_kp *kps,
                                   const int *n_kp, void *stream);
/* Copy one camera's grid to host: cell_start [64*48+1], idx [kp_cap]. Syncs. */
omv_status omv_matcher_grid_debug(omv_matcher *m, int frame, int cam, int32_t *cell_start, int32_t *idx);

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
 * (src/ORBmatcher.cc:23-340) on n_frames frames with the grid of the last assign_grid call.
 *   l2r / r2l     [frame][kp_cap] mvLeftToRightMatch / mvRightToLeftMatch (block-local indices, -1 none)
 *   kp_occ_init   [frame][slots] 1 where F.mvpMapPoints[slot] is already a point with observations
 *                 (may be NULL = none)
 *   kp_to_mp      [frame][slots] in/out: map point index assigned to each keypoint (F.mvpMapPoints)
 *   n_matches     [frame] the return value
 * Exactly the reference's sequential semantics: earlier points claim keypoints first, a failed
 * ratio test skips the point's remaining cameras, th scales only the left-camera window. */
omv_status omv_matcher_search_projection(omv_matcher *m, int n_frames, const omv_frame_geom *geom, const omv_kp *kps,
                                         const uint8_t *desc, const int *n_kp, const omv_mp_view *mps, int M, float th,
                                         int far_points, float th_far, float nnratio, const int32_t *l2r,
                                         const int32_t *r2l, const uint8_t *kp_occ_init, int32_t *kp_to_mp,
                                         int *n_matches, void *stream);

/* Lapping-area stereo candidates of Frame::ComputeMultiFishEyeMatches (src/Frame.cc:1461-1491):
 * knnMatch(k=2) of camera-0 rows [mono0, n0) against camera-1 rows [mono1, n1), Lowe ratio
 * d0 < ratio * d1.  Writes l2r/r2l [frame][kp_cap] (later left index wins a shared right keypoint).
 * The KannalaBrandt8::TriangulateMatches depth check that follows in the reference is not applied. */
omv_status omv_matcher_stereo_lapping(omv_matcher *m, int n_frames, const uint8_t *desc, const int *n_kp,
                                      const int *mono, double ratio, int32_t *l2r, int32_t *r2l, void *stream);

/* The depth check of Frame::ComputeMultiFishEyeMatches (src/Frame.cc:1488-1512) on the pairs
 * omv_matcher_stereo_lapping left in l2r: KannalaBrandt8::TriangulateMatches(mpCamera2, kpL, kpR,
 * mRlr, mtlr, sigma2[octL], sigma2[octR]) > 1e-4 keeps a pair (l2r / r2l [frame][kp_cap], the later
 * left index wins on r2l), writes mvDepth of the left keypoints (depth [frame][kp_cap], -1 elsewhere)
 * and mvStereo3Dpoints (p3d [frame][kp_cap][3]); failures clear l2r.  kps: [frame][n_cams][kp_cap]
 * (block 0 = left, 1 = right).  cams: host [2][8] (L, R); Rlr / tlr / level_sigma2: host. */
omv_status omv_matcher_stereo_triangulate(omv_matcher *m, int n_frames, int n_cams, int kp_cap, const omv_kp *kps,
                                          const int *n_kp, const int *mono, const float *cams, const float *Rlr,
                                          const float *tlr, const float *level_sigma2, int nlevels, int32_t *l2r,
                                          int32_t *r2l, float *depth, float *p3d, void *stream);

/* Device-side error word (OMV_ERR_CAPACITY if a bound was hit) since the last call; syncs. */
omv_status omv_matcher_last_error(omv_matcher *m);

/* Per-stage device time: 0 grid, 1 lapping knn, 2 projection candidates, 3 claim resolution. */
omv_status omv_matcher_enable_timing(omv_matcher *m, int on);
omv_status omv_matcher_stage_ms(omv_matcher *m, double *ms4, int reset);

/* cv::BFMatcher(NORM_HAMMING).knnMatch(k=2) (src/Frame.cc:1483) over n_pairs independent sets:
 * query [pair][q_cap][32] with nq[pair] rows, train [pair][t_cap][32] with nt[pair] rows.
 * idx2/dist2 [pair][q_cap][2]: two nearest train rows, first index wins ties; -1 / INT32_MAX when
 * fewer than 1 / 2 train rows exist. */
omv_status omv_bf_knn2(int n_pairs, const uint8_t *query, int q_cap, const int *nq, const uint8_t *train, int t_cap,
                       const int *nt, int32_t *idx2, int32_t *dist2, void *stream);

/* ORBmatcher::SearchByProjection(Frame &CurrentFrame, const Frame &LastFrame, th, bMono)
 * (src/ORBmatcher.cc:1985-2413, ComputeThreeMaxima :2537-2573): motion-model matching of the last
 * frame's tracked map points, multi-camera branch, generalised to n_cams blocks (block 1 searched at
 * Trl * x projected with the LEFT camera model, blocks >= 2 at the left projection — both as in the
 * reference), rotation-consistency filter when check_ori. */
typedef struct omv_se3f {          /* Sophus::SE3f: unit quaternion (x, y, z, w) and translation */
    float q[4];
    float t[3];
} omv_se3f;

typedef struct omv_last_frame {    /* device SoA per LastFrame keypoint slot s = cam * last_cap + i */
    const float *pos;              /* [frame][S][3] mvpMapPoints[s]->GetWorldPos()                  */
    const uint8_t *desc;           /* [frame][S][32] GetDescriptor()                                */
    const uint8_t *valid;          /* [frame][S] mvpMapPoints[s] && !mvbOutlier[s]                  */
    const uint8_t *has_obs;        /* [frame][S] Observations() > 0                                 */
    const omv_kp *kps;             /* [frame][S] LastFrame keypoint s (octave, angle)               */
    int S;                         /* slots per last frame (n_cams * last_cap), <= the matcher's max_mps */
} omv_last_frame;

/* cams: host [n_cams][8] camera parameters (block 0's, of type geom->cam_model[0], are used for every
 * projection, as the reference's CurrentFrame.mpCamera);
 * Tcw / Tlw: device [n_frames] current / last block-0 poses; Trl: host, block 1 from block 0;
 * kp_to_mp [frame][n_cams*kp_cap] in/out receives last-frame slots; n_matches [frame] (device). */
omv_status omv_matcher_search_last_frame(omv_matcher *m, int n_frames, const omv_frame_geom *geom, const omv_kp *kps,
                                         const uint8_t *desc, const int *n_kp, const float *cams, const omv_se3f *Tcw,
                                         const omv_se3f *Tlw, const omv_se3f *Trl, const omv_last_frame *last, float th,
                                         int bMono, float mb, int check_ori, const uint8_t *kp_occ_init,
                                         int32_t *kp_to_mp, int32_t *n_matches, void *stream);

/* ------------------------------------------------------------------------------------------------
 * Keyframe-side projection searches: map points projected into one camera block of a
 * keyframe (or frame) of the last omv_matcher_assign_grid batch and matched by Hamming distance in the
 * GetFeaturesInArea window.  One call runs a list of jobs; a job = (keyframe, camera block, pose, a run
 * of map points).  Modes:
 *   OMV_KF_FUSE       ORBmatcher::Fuse(KF, vpMapPoints, th, cameraID) (src/ORBmatcher.cc:1458-1647):
 *                     depth / IsInImage / distance-invariance / 60-degree viewing tests, PredictScale,
 *                     KeyFrame::GetFeaturesInArea (src/KeyFrame.cc:771-834), levels [pred-1, pred], the
 *                     chi2 reprojection gate (stereo 7.8 on block 0 where mvuRight >= 0, else 5.99), best
 *                     by (distance, window order) from 256, accepted at <= TH_LOW.  The caller applies
 *                     the Replace / AddObservation of each accepted (point, keypoint) in list order.
 *   OMV_KF_FUSE_SIM3  ORBmatcher::Fuse(KF, Scw, vpPoints, th, vpReplacePoint) (:1649-1769), one job per
 *                     camera block: no distance / viewing tests, no gate, best from INT_MAX.
 *   OMV_KF_SBP_SIM3   ORBmatcher::SearchByProjection(KF, Siw, vpPoints[, vpPointsKFs], vpMatched, th,
 *                     ratioHamming, cameraID) (:668-776, :778-893): keypoints matched before (kp_match
 *                     >= 0, initially and by earlier points of the job) are skipped, accepted at
 *                     <= TH_LOW * ratioHamming and claimed in kp_match.
 *   OMV_KF_SBP_FRAME  ORBmatcher::SearchByProjection(Frame&, KF, sAlreadyFound, th, ORBdist)
 *                     (:2415-2535): the "keyframe" of the job is the current frame (inclusive mnMinX..mnMaxX
 *                     bounds, Frame::GetFeaturesInArea with levels [pred-1, pred+1]), no viewing test,
 *                     claims in kp_match, accepted at <= ORBdist; with check_ori the rotation-histogram
 *                     filter (ComputeThreeMaxima, :2537-2573) un-claims matches outside the three top bins.
 * Jobs on the same keyframe / frame run in job order (claims carry over), others in parallel.  The
 * caller leaves out of a job's list the points the reference skips before projecting (isBad(),
 * IsInKeyFrame(pKF), spAlreadyFound / sAlreadyFound) and passes each job's camera pose as the
 * reference composes it (GetPose / GetRightPose / ..., SE3f(Siw.rotationMatrix(), Siw.translation() /
 * Siw.scale()), GetRelativePoseTrl() * Tlw, CurrentFrame.GetPose()).
 * ---------------------------------------------------------------------------------------------- */
enum { OMV_KF_FUSE = 0, OMV_KF_FUSE_SIM3 = 1, OMV_KF_SBP_SIM3 = 2, OMV_KF_SBP_FRAME = 3 };

typedef struct omv_kf_search_job {
    int kf;                /* keyframe / frame index in the assign_grid batch */
    int cam;               /* cameraID: the camera block searched */
    omv_se3f Tcw;          /* world -> camera block `cam` */
    float Ow[3];           /* that camera's centre (the distance / viewing tests) */
    int mp_start, mp_count;   /* the job's entries [mp_start, mp_start + mp_count) of mp_list; jobs tile
                                 mp_list in order */
} omv_kf_search_job;

typedef struct omv_kf_mps {        /* device map-point table */
    const float *pos;              /* [M][3] GetWorldPos()                                           */
    const float *normal;           /* [M][3] GetNormal()                                             */
    const float *min_dist;         /* [M] mfMinDistance (GetMinDistanceInvariance = 0.8f * it)      */
    const float *max_dist;         /* [M] mfMaxDistance (GetMaxDistanceInvariance = 1.2f * it)      */
    const uint8_t *desc;           /* [M][32] GetDescriptor()                                        */
} omv_kf_mps;

typedef struct omv_kf_search_params {
    int mode;                      /* OMV_KF_*                                                       */
    float th;                      /* window radius factor (th * mvScaleFactors[pred])                */
    float max_dist;                /* acceptance: best <= max_dist (TH_LOW, TH_LOW * ratio, ORBdist) */
    float bf;                      /* KeyFrame::mbf (OMV_KF_FUSE stereo gate)                         */
    const float *uright;           /* device [n_kf][kp_cap] mvuRight of block 0 (OMV_KF_FUSE) or NULL */
    float inv_level_sigma2[16];    /* mvInvLevelSigma2                                               */
    float log_scale_factor;        /* mfLogScaleFactor                                               */
    int n_levels;                  /* mnScaleLevels                                                  */
    float cams[8][8];              /* camera parameters per block (KB8 fx fy cx cy k1..k4 / Pinhole fx fy cx cy;
                                      the type is geom->cam_model[block])                             */
    int check_ori;                 /* OMV_KF_SBP_FRAME: mbCheckOrientation                           */
    const float *mp_angle;         /* device [n_entries]: pKF->mvKeysUn[i].angle per entry (check_ori) */
} omv_kf_search_params;

/* jobs: host [n_jobs] (validated, then copied to the handle); mp_list: device [n_entries] map-point table rows; kp_match: device
 * [n_kf][n_cams * kp_cap] slot claims (-1 free, else the claiming table row; in/out, claim modes only,
 * may be NULL otherwise); best_idx / best_dist: device [n_entries] — the chosen keypoint as the
 * keyframe's N-index (camera offset + index in its block; -1 if the point was rejected or nothing
 * qualified) and its distance (Fuse modes: the scan's best even above the threshold; claim modes: the
 * accepted match only); n_matches: device [n_jobs] the reference's return value per job. */
omv_status omv_matcher_search_kf(omv_matcher *m, int n_kf, const omv_frame_geom *geom, const omv_kp *kps,
                                 const uint8_t *desc, const int *n_kp, int n_jobs, const omv_kf_search_job *jobs,
                                 int n_entries, const int32_t *mp_list, const omv_kf_mps *mps,
                                 const omv_kf_search_params *p, int32_t *kp_match, int32_t *best_idx,
                                 int32_t *best_dist, int32_t *n_matches, void *stream);

/* ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, S12, th) (src/ORBmatcher.cc:1771-1983) for a list of
 * keyframe pairs of the last omv_matcher_assign_grid batch.  Side 1 of a job = the pKF1 keypoints i1 whose
 * map point the reference projects (GetMapPointMatches()[i1] set, !vbAlreadyMatched1[i1], !isBad()), as
 * (kp1 = i1, the N-index, mp1 = its map-point table row); side 2 likewise for pKF2.  Each side-1 point goes
 * through T1w then S21 into pKF2, each side-2 point through T2w then S12 into pKF1; both use the pinhole
 * formula with pKF1's fx fy cx cy (as the reference), IsInImage, the distance invariance on |p3Dc|,
 * PredictScale, KeyFrame::GetFeaturesInArea (camera block 0) at levels [pred-1, pred], the strict-< best,
 * kept at <= TH_HIGH; then the agreement check vnMatch2[vnMatch1[i1]] == i1.  A side's kp entries must be
 * distinct within a job. */
typedef struct omv_sim3f {         /* Sophus::Sim3f: RxSO3 quaternion (x, y, z, w; |q|^2 = scale), translation */
    float q[4];
    float t[3];
    float scale;                   /* S.scale() as the caller's Sophus computes it (q.squaredNorm())          */
} omv_sim3f;

typedef struct omv_sim3_job {
    int kf1, kf2;                  /* keyframes of the assign_grid batch                                       */
    omv_se3f T1w, T2w;             /* pKF1->GetPose(), pKF2->GetPose()                                         */
    omv_sim3f S12, S21;            /* S12 and S12.inverse()                                                    */
    float fx, fy, cx, cy;          /* pKF1->fx, fy, cx, cy                                                     */
    int start1, count1;            /* the job's run of the side-1 list (runs tile the list in order)          */
    int start2, count2;            /* the job's run of the side-2 list                                         */
} omv_sim3_job;

/* jobs: host [n_jobs]; kp1 / mp1: device [n1]; kp2 / mp2: device [n2]; mps: pos, min_dist, max_dist, desc
 * (normal unused); th: the radius factor; match12: device [n1] the pKF2 keypoint (N-index) matched to each
 * side-1 entry (vpMatches12[i1] = vpMapPoints2[match12]) or -1; n_found: device [n_jobs] the return value. */
omv_status omv_matcher_search_by_sim3(omv_matcher *m, int n_kf, const omv_frame_geom *geom, const omv_kp *kps,
                                      const uint8_t *desc, const int *n_kp, int n_jobs, const omv_sim3_job *jobs,
                                      int n1, const int32_t *kp1, const int32_t *mp1, int n2, const int32_t *kp2,
                                      const int32_t *mp2, const omv_kf_mps *mps, float th, float log_scale_factor,
                                      int n_levels, int32_t *match12, int32_t *n_found, void *stream);

/* ------------------------------------------------------------------------------------------------
 * Frame::isInFrustum (src/Frame.cc:736-826; the multi-camera isInFrustumChecks, :1529-1653) with
 * MapPoint::PredictScale (src/MapPoint.cc:624-637) and KannalaBrandt8::project(Vector3f)
 * (src/CameraModels/KannalaBrandt8.cpp:48-67), for every local map point of every frame — the loop
 * of Tracking::SearchLocalPoints.  Writes the projection fields SearchByProjection reads.
 * ---------------------------------------------------------------------------------------------- */
/* GeometricCamera subclasses (src/CameraModels): KannalaBrandt8 (KannalaBrandt8.cpp) and Pinhole (Pinhole.cpp) */
#define OMV_CAM_KB8 0
#define OMV_CAM_PINHOLE 1

typedef struct omv_rig {
    int n_cams;
    float cam[8][8];               /* KannalaBrandt8 mvParameters per camera block                 */
    float R_cl[8][9], t_cl[8][3];  /* camera block c from block 0: mTrl / mTsll / mTsrl (c=0: I, 0) */
    float t_lc[8][3];              /* translation of the inverse: mTlr / mTlsl / mTlsr (c=0: 0)     */
    float min_x, max_x, min_y, max_y;  /* mnMinX .. mnMaxY                                          */
    float log_scale_factor;        /* mfLogScaleFactor                                              */
    int n_levels;                  /* mnScaleLevels                                                 */
    int model[8];                  /* camera model per block: OMV_CAM_KB8 (0, the default of a
                                      zero-initialised rig) or OMV_CAM_PINHOLE (cam[c][0..3] = fx fy cx cy) */
} omv_rig;

typedef struct omv_frame_pose {   /* block-0 camera: mRcw, mtcw and the inverse mRwc, mOw */
    float Rcw[9], tcw[3], Rwc[9], Ow[3];
} omv_frame_pose;

typedef struct omv_mp_world {     /* device SoA, [frame][M] */
    const float *pos;              /* [M][3] GetWorldPos()                                          */
    const float *normal;           /* [M][3] GetNormal()                                            */
    const float *min_dist;         /* [M] mfMinDistance                                             */
    const float *max_dist;         /* [M] mfMaxDistance                                             */
} omv_mp_world;

typedef struct omv_mp_track {     /* outputs, same layout as omv_mp_view */
    float *proj_x, *proj_y;        /* [M][n_cams] -1 when not in view (reset like the reference)    */
    float *view_cos;               /* [M][n_cams] written when in view                              */
    int32_t *level;                /* [M][n_cams] predicted level, -1 when not in view              */
    uint8_t *in_view;              /* [M][n_cams]                                                   */
    float *track_depth;            /* [M] block-0 distance, written only when block 0 sees the point */
} omv_mp_track;

/* poses: device [n_frames]; n_in_view (optional, device [n_frames], accumulated): points for which
 * isInFrustum returned true. */
omv_status omv_frustum(int n_frames, const omv_frame_pose *poses, const omv_rig *rig, const omv_mp_world *mp, int M,
                       float viewing_cos_limit, const omv_mp_track *out, int32_t *n_in_view, void *stream);

/* ------------------------------------------------------------------------------------------------
 * Local inertial bundle adjustment — replaces the optimisation inside Optimizer::LocalInertialBA
 * (src/Optimizer.cc:2728-3385): EdgeMono / EdgeInertial / EdgeGyroRW / EdgeAccRW
 * (src/G2oTypes.cc, include/G2oTypes.h:283-633), g2o's Levenberg-Marquardt
 * (Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:61-169) with the landmark Schur
 * complement (block_solver.hpp:353-486).  The host adapter flattens the KeyFrame/MapPoint graph
 * (window selection, vertex ids, edge creation stay host-side, :2740-3267) into this problem and
 * writes the state back unless status == OMV_LBA_FAIL (the reference's FAIL guard, :3317-3321).
 * ---------------------------------------------------------------------------------------------- */
/* Per inertial edge: IMU::Preintegrated members in float, in this order:
 *   dR[9] dV[3] dP[3] JRg[9] JVg[9] JVa[9] JPg[9] JPa[9] b[6] (bax bay baz bwx bwy bwz) dT[1] C[225]
 * (3x3 / 15x15 row-major).  Information matrices are derived from C like EdgeInertial's ctor. */
#define OMV_PREINT_FLOATS 292
#define OMV_LBA_OK 0
#define OMV_LBA_FAIL 1   /* (2*err < err_end || isnan) && !bLarge: the reference discards the result */

typedef struct omv_lba_problem {
    int n_cams;
    const float *cam;          /* [n_cams][8] KannalaBrandt8 mvParameters: fx fy cx cy k1 k2 k3 k4 */
    const double *Rcb, *tcb;   /* [n_cams][9] row-major, [n_cams][3]: body -> camera (ImuCamPose) */
    const double *Rbc, *tbc;   /* [n_cams][9], [n_cams][3]: camera -> body */
    int n_kf;                  /* KeyFrame vertices; the first n_opt are optimisable, the rest fixed */
    int n_opt;
    const uint8_t *kf_imu;     /* [n_kf] KeyFrame::bImu: velocity / gyro / acc bias vertices exist */
    double *Rwb, *twb;         /* [n_kf][9], [n_kf][3] body pose (in/out) */
    double *Rcw, *tcw;         /* [n_kf][n_cams][9], [n_kf][n_cams][3] camera poses (in/out) */
    double *vel, *bg, *ba;     /* [n_kf][3] (in/out) */
    int n_pts;
    double *pts;               /* [n_pts][3] world points (in/out) */
    const float *pt_track_depth;   /* [n_pts] MapPoint::mTrackDepth (bClose = < 10 m, :3284) */
    int n_mono;
    const int32_t *mono_pt, *mono_kf, *mono_cam;   /* [n_mono] */
    const double *mono_obs;    /* [n_mono][2] keypoint (u, v) */
    const float *mono_inv_sigma2;  /* [n_mono] information = I * invSigma2 / uncertainty2 */
    int n_imu;                 /* inertial edges; each also carries one EdgeGyroRW and one EdgeAccRW */
    const int32_t *imu_kf1, *imu_kf2;
    const float *preint;       /* [n_imu][OMV_PREINT_FLOATS] */
    const uint8_t *imu_robust; /* Huber sqrt(16.92) on this inertial edge (last one / bRecInit) */
    const float *imu_info_scale;   /* 1, or 1e-2 on the last edge of the window (:2986) */
    /* EdgeStereo (include/G2oTypes.h:364-402, src/G2oTypes.cc:402-431): left-camera (cam 0)
     * observations with mvuRight >= 0 (Optimizer.cc:3108-3143): obs (u, v, u_R), information
     * I3 * invSigma2, Huber sqrt(7.815); u_R predicted as u - bf / z (ImuCamPose::ProjectStereo,
     * G2oTypes.cc:198-205).  n_stereo = 0 when there is no depth / right coordinate. */
    int n_stereo;
    const int32_t *stereo_pt, *stereo_kf;   /* [n_stereo] */
    const double *stereo_obs;  /* [n_stereo][3] (kpUn.pt.x, kpUn.pt.y, mvuRight); mvuRight >= 0 */
    const float *stereo_inv_sigma2;   /* [n_stereo] */
    float bf;                  /* KeyFrame::mbf (ImuCamPose::bf) */
    /* GeometricCamera type per camera: OMV_CAM_KB8 (cam = KannalaBrandt8 fx fy cx cy k1..k4) or
     * OMV_CAM_PINHOLE (cam = Pinhole fx fy cx cy, the rest ignored: Pinhole::project / projectJac,
     * src/CameraModels/Pinhole.cpp:18-24, :55-65).  NULL: every camera KannalaBrandt8. */
    const int32_t *cam_model;  /* [n_cams] */
} omv_lba_problem;

typedef struct omv_lba_opts {
    int opt_it;            /* 10, or 4 when bLarge */
    double lambda_init;    /* setUserLambdaInit: 1e0, or 1e-2 when bLarge */
    int max_trials;        /* maxTrialsAfterFailure (10) */
    int large;             /* bLarge: disables the FAIL guard */
} omv_lba_opts;

typedef struct omv_lba_result {
    float err, err_end;    /* activeRobustChi2 before / after optimize(), as floats like the reference */
    int status;            /* OMV_LBA_OK / OMV_LBA_FAIL */
    int iterations;        /* LM iterations run (solve() calls) */
    int trials;            /* LM trials (linear solves) in total */
    double lambda;         /* final lambda */
    double *mono_chi2;     /* optional [n_mono]: e->chi2() after optimize (may be NULL) */
    uint8_t *mono_outlier; /* optional [n_mono]: the :3282-3296 outlier test (may be NULL) */
    double *stereo_chi2;   /* optional [n_stereo] */
    uint8_t *stereo_outlier;   /* optional [n_stereo]: chi2 > 7.815 (:3299-3311) */
} omv_lba_result;

typedef struct omv_lba omv_lba;

/* Workspace for problems up to the given sizes (max_mono bounds the visual edges a handle holds:
 * EdgeMono + EdgeStereo; with sharding, the rank's share). */
omv_status omv_lba_create(int max_kf, int max_cams, int max_pts, int max_mono, int max_imu, omv_lba **out);
omv_status omv_lba_destroy(omv_lba *h);
/* Upload a problem (host arrays); the structure (point -> keyframe slots, reduced-system layout,
 * block fill pattern) is analysed on the host once here. */
omv_status omv_lba_set_problem(omv_lba *h, const omv_lba_problem *p);
/* Run the optimisation on the uploaded problem; on return the state arrays of `p` (Rwb, twb, Rcw,
 * tcw, vel, bg, ba, pts) hold the optimised state and `r` the outcome.  Synchronous. */
omv_status omv_lba_optimize(omv_lba *h, const omv_lba_opts *o, omv_lba_problem *p, omv_lba_result *r);
/* Residual/Jacobian evaluation at the uploaded state for parity: mono_err [n_mono][2],
 * mono_jx [n_mono][6] (2x3), mono_jp [n_mono][12] (2x6), imu_err [n_imu][9] (any may be NULL). */
omv_status omv_lba_evaluate(omv_lba *h, double *mono_err, double *mono_jx, double *mono_jp, double *imu_err);
/* The same for the EdgeStereo edges: err [n_stereo][3], jx [n_stereo][9] (3x3), jp [n_stereo][18] (3x6). */
omv_status omv_lba_evaluate_stereo(omv_lba *h, double *stereo_err, double *stereo_jx, double *stereo_jp);
/* Restore the state uploaded by the last set_problem (device-side copy; for re-runs and benchmarks). */
omv_status omv_lba_reset(omv_lba *h);
/* Per-stage device time of the last optimize: 0 linearise+build, 1 Schur, 2 reduced solve,
 * 3 back-substitution+update+errors; plus the number of trials.  On one rank the stages are timed only
 * with omv_lba_enable_timing(h, 1) (direct launches with events instead of the captured LM step). */
omv_status omv_lba_stage_ms(omv_lba *h, double *ms4, int *trials);
omv_status omv_lba_enable_timing(omv_lba *h, int on);
/* LM driver: 0 (default) keeps g2o's accept / reject / lambda / stop logic on the device (on one rank the steps
 * are captured hipGraphs of four; a sharded solve launches the same gated steps directly, its collectives called
 * in stream order), one control read-back per batch of steps; 1 runs it on the host with a read-back per trial.
 * Both make the same decisions (tests/test_lba_gpu.py). */
omv_status omv_lba_set_driver(omv_lba *h, int host_driven);
/* Host waits (stream synchronisations) of the last omv_lba_optimize's LM loop and its trial count: the device
 * driver waits once per batch of steps, never per trial. */
omv_status omv_lba_host_syncs(omv_lba *h, int *host_syncs, int *trials);

/* Landmark sharding across ranks: two exchanges per LM step, no host wait per step.
 * Call before omv_lba_set_problem.  Every rank then passes the SAME full problem; the handle keeps
 * the rank's contiguous share of the landmarks (in its landmark order) with their edges, and rank 0
 * alone evaluates the inertial / random-walk edges, adds lambda to the pose diagonal and the pose
 * part of computeScale.  Per trial the handle calls
 *     allreduce(ctx, buf, count, stream)   — in-place SUM of `count` doubles of device memory,
 * once on the partial Schur system [packed blocks | b | coef] and once on [chi2 of the current state (when
 * recomputed), chi2 of the trial, scale] (and once on optimize()'s initial chi2).  The call must be enqueued on
 * (or ordered after) `stream`;
 * it returns 0 on success.  ncclAllReduce(buf, buf, count, ncclFloat64, ncclSum, comm, stream)
 * is exactly that.  Every rank solves the identical reduced system; after omv_lba_optimize each
 * rank has written its own landmarks / edges (chi2, outlier) and all keyframes; err / err_end are
 * global.  world == 1 (the default) is the single-GPU path with no calls. */
typedef int (*omv_allreduce_fn)(void *ctx, double *buf, size_t count, void *stream);
omv_status omv_lba_set_comm(omv_lba *h, int rank, int world, omv_allreduce_fn allreduce, void *ctx);
/* Landmarks / visual edges this rank owns after set_problem, and (optional, [n_pts]) the caller
 * indices of its landmarks.  Any pointer may be NULL. */
omv_status omv_lba_shard(omv_lba *h, int32_t *n_pts, int32_t *n_mono, int32_t *pt_index);

/* ------------------------------------------------------------------------------------------------
 * ORBmatcher::SearchForTriangulation(KeyFrame*, KeyFrame*, vector<pair<size_t,size_t>>&, bOnlyStereo,
 * bCoarse) (src/ORBmatcher.cc:1131-1456) for multi-camera keyframes, with pCamera1->epipolarConstrain
 * dispatched on camera 1's type (:1380-1387): KannalaBrandt8::epipolarConstrain / TriangulateMatches /
 * unproject / Triangulate (src/CameraModels/KannalaBrandt8.cpp:219-229, 319-395, 96-126, 414-429;
 * Eigen::JacobiSVD<Matrix4f> restated; pCamera2's unprojectEig / project by its own type) or
 * Pinhole::epipolarConstrain (src/CameraModels/Pinhole.cpp:103-132: F12 = K1^-T [t12]x R12 K2^-1).  One workgroup per keyframe pair; pairs are independent (vbMatched2 is never set).
 * ---------------------------------------------------------------------------------------------- */
#define OMV_TRI_PAIRS 10   /* LL, LR, RL, RR, L-SL, SL-L, SL-SL, R-SR, SR-R, SR-SR (ORBmatcher.cc:1300-1392) */

/* A keyframe in the reference's concatenated keypoint order [L | R | SL | SR] (device pointers). */
typedef struct omv_kf_view {
    int n;                              /* KeyFrame::N */
    int n_left, n_right, n_sideleft;    /* NLeft, NRight, NSideLeft: camera of idx by range (0..3) */
    const omv_kp *kps;                  /* [n] mvKeys / mvKeysRight / mvKeysSideLeft / mvKeysSideRight by idx */
    const uint8_t *desc;                /* [n][32] mDescriptors */
    const uint8_t *has_mp;              /* [n] GetMapPoint(idx) != NULL */
    int n_nodes;                        /* DBoW2::FeatureVector: node ids ascending, CSR of keypoint indices */
    const uint32_t *node_id;            /* [n_nodes] */
    const int32_t *node_start;          /* [n_nodes + 1] */
    const int32_t *node_idx;
    float level_sigma2[16];             /* mvLevelSigma2 (host values) */
} omv_kf_view;

typedef struct omv_tri_pair {
    omv_kf_view kf1, kf2;
    /* R12 (row-major 3x3) | t12 of the camera pairs in OMV_TRI_PAIRS order: T1w * Tw2 composed with the
     * rig (Tll = T1w Tw2, Tlr = T1w Twr2, Trl = Tr1w Tw2, ...: ORBmatcher.cc:1157-1195). */
    float T[OMV_TRI_PAIRS][12];
    int32_t *match12;                   /* device [kf1.n]: vMatches12 (-1 = none); vMatchedPairs = (i, match12[i] >= 0) */
} omv_tri_pair;

/* cams: host [4][8] parameters of the rig's L, R, SL, SR cameras (both keyframes share the rig):
 * KannalaBrandt8 fx fy cx cy k1..k4 or Pinhole fx fy cx cy; cam_model: host [4] OMV_CAM_KB8 /
 * OMV_CAM_PINHOLE per camera, NULL = all KannalaBrandt8.  n_matches: device [n_pairs] (the return value).  The camera-pair transform of a pair of
 * cameras the reference does not list ((L,SR), (SR,L), (R,SL), (SL,R), (SL,SR), (SR,SL)) is whatever the
 * previous candidate of the scan assigned (the reference's R12/t12/pCamera1/pCamera2 persist across
 * iterations); before any assignment it is LL (the reference's R12/t12 are uninitialised there). */
/* Parity hook: KannalaBrandt8::unproject of kp1 (cams2[0]) and kp2 (cams2[1]), JacobiSVD<Matrix4f> V of
 * svd_in (row-major 4x4), TriangulateMatches(kp1, kp2, R12, t12, sigma, unc) on one device thread:
 * out31 = ray1[3] ray2[3] V[16] z p3D[3] x3D[3] uv1[2] (x3D / uv1: the triangulated point and its
 * projection into camera 1 even when a later check rejects it).  Host pointers; synchronous. */
omv_status omv_tri_debug(const float *cams2, const omv_kp *kp1, const omv_kp *kp2, const float *R12, const float *t12,
                         const float *svd_in, float sigma, float unc, float *out31);

omv_status omv_matcher_search_for_triangulation(omv_matcher *m, int n_pairs, const omv_tri_pair *pairs,
                                                const float *cams, const int32_t *cam_model, int only_stereo,
                                                int coarse, int check_ori, int32_t *n_matches, void *stream);

/* ------------------------------------------------------------------------------------------------
 * ORBmatcher::SearchByBoW — Hamming matching of the keypoints that share a vocabulary node (DBoW2
 * FeatureVector, node ids ascending), with the rotation-consistency filter (ComputeThreeMaxima):
 *   OMV_BOW_KF_FRAME  SearchByBoW(KeyFrame *pKF, Frame &F, vpMapPointMatches) (src/ORBmatcher.cc:349-666):
 *                     per keyframe keypoint with a map point, the best unmatched frame keypoint of each
 *                     camera block (L [0, Nleft), R, SL, SR by the frame's ranges; F.n_left = -1: one block),
 *                     left accepted at <= TH_LOW with the nnratio test, right / side blocks accepted at
 *                     <= TH_LOW (their ratio test is `|| true`) and only when the left best passed TH_LOW.
 *                     Called by Tracking::TrackReferenceKeyFrame / Relocalization.
 *   OMV_BOW_KF_KF     SearchByBoW(KeyFrame *pKF1, KeyFrame *pKF2, vpMatches12) (:1006-1129): per pKF1
 *                     keypoint with a map point the best unclaimed pKF2 keypoint with a map point (vbMatched2),
 *                     accepted at < TH_LOW with the nnratio test.  Called by LoopClosing's place recognition.
 * One wavefront per job; jobs are independent.  `kf.has_mp` / `other.has_mp` = GetMapPoint(idx) && !isBad().
 * ---------------------------------------------------------------------------------------------- */
enum { OMV_BOW_KF_FRAME = 0, OMV_BOW_KF_KF = 1 };

typedef struct omv_bow_job {
    omv_kf_view kf;         /* pKF / pKF1 (its kps give the keyframe keypoint angles, mvKeysUn order) */
    omv_kf_view other;      /* F (n_sideleft = -1: no side cameras) / pKF2 */
    int32_t *match;         /* device: OMV_BOW_KF_FRAME [other.n] vpMapPointMatches as the keyframe keypoint
                               index whose map point the frame keypoint received (-1 none);
                               OMV_BOW_KF_KF [kf.n] vpMatches12 as the pKF2 keypoint index (-1 none) */
} omv_bow_job;

/* jobs: host [n_jobs]; n_matches: device [n_jobs] (the reference's return value).  Up to 16384 keypoints
 * per view (OMV_ERR_CAPACITY beyond). */
omv_status omv_matcher_search_by_bow(omv_matcher *m, int n_jobs, const omv_bow_job *jobs, int mode, float nnratio,
                                     int check_ori, int32_t *n_matches, void *stream);
/* Diagnostic: the number of keyframe keypoints whose short candidate list ran out during the sequential walk
 * (the node was rescanned under the current claims), summed over every SearchByBoW call of the process. */
omv_status omv_matcher_bow_rescans(int64_t *total, int reset);

/* ORBmatcher::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (src/ORBmatcher.cc:
 * 895-1004): for every level-0 keypoint of F1 in order, Frame::GetFeaturesInArea(vbPrevMatched[i1], windowSize,
 * 0, 0) on F2's grid (the last omv_matcher_assign_grid batch, camera block 0: F2.mvKeysUn), the best candidate
 * whose previous match (vMatchedDistance) is strictly worse, accepted at <= TH_LOW with the nnratio test; a
 * better later F1 keypoint takes the F2 keypoint over; rotation-consistency filter; vbPrevMatched updated to the
 * matched F2 keypoints.  pairs: host [n_pairs][2] (F1, F2) frame indices of the batch; prev_matched: device
 * [n_pairs][kp_cap][2] in/out; matches12: device [n_pairs][kp_cap] (vnMatches12, -1 none); n_matches: device
 * [n_pairs].  F1's keypoints are frame pairs[i][0]'s block 0 (mvKeysUn). */
omv_status omv_matcher_search_for_initialization(omv_matcher *m, int n_pairs, const int32_t *pairs,
                                                 const omv_frame_geom *geom, const omv_kp *kps, const uint8_t *desc,
                                                 const int *n_kp, float *prev_matched, int window, float nnratio,
                                                 int check_ori, int32_t *matches12, int32_t *n_matches, void *stream);

/* ------------------------------------------------------------------------------------------------
 * Pose-inertial optimisation of tracked frames — replaces Optimizer::PoseInertialOptimizationLastKeyFrame
 * (src/Optimizer.cc:5021-5578): Gauss-Newton (4 rounds x 10 iterations, dense LDLT) over the frame's
 * VertexPose / VertexVelocity / VertexGyroBias / VertexAccBias with the last keyframe's vertices fixed;
 * EdgeMonoOnlyPose (G2oTypes.h:330-362, G2oTypes.cc:382-400) and EdgeStereoOnlyPose (:404-431,
 * :433-456) per matched keypoint, one EdgeInertial + EdgeGyroRW + EdgeAccRW; the outlier
 * classification between rounds (chi2 thresholds 12 / 7.5 / 5.991 / 5.991, stereo 15.6 / 9.8 / 7.815 /
 * 7.815, robust kernels dropped after round 3), the "recover not too bad points" pass, and the
 * marginal Hessian the reference stores in Frame::mpcpi.  A batch of frames runs in one launch
 * (one workgroup per frame).
 * ---------------------------------------------------------------------------------------------- */
typedef struct omv_pose_batch {
    int n_frames;
    /* rig (as omv_lba_problem): per camera KannalaBrandt8 parameters and body <-> camera */
    int n_cams;
    const float *cam;                   /* host [n_cams][8] */
    const double *Rcb, *tcb, *Rbc, *tbc;   /* host [n_cams][9] / [3] */
    float bf;                           /* Frame::mbf (EdgeStereoOnlyPose) */
    /* device: frame state (in/out) — ImuCamPose(Frame*) (G2oTypes.cc:74-133) */
    double *Rwb, *twb;                  /* [F][9], [F][3] */
    double *Rcw, *tcw;                  /* [F][n_cams][9], [F][n_cams][3] initial camera poses, updated */
    double *vel, *bg, *ba;              /* [F][3] */
    /* device: Frame::mpLastKeyFrame's vertices (fixed) */
    const double *kf_Rwb, *kf_twb, *kf_vel, *kf_bg, *kf_ba;
    const float *preint;                /* [F][OMV_PREINT_FLOATS] Frame::mpImuPreintegrated */
    /* device: visual edges, frame-major (edges of frame f: [start[f], start[f+1])) */
    const int32_t *mono_start;          /* [F+1] */
    const int32_t *mono_cam, *mono_kp;  /* camera index, keypoint index i of the frame (mvbOutlier[i]) */
    const double *mono_obs;             /* [E][2] */
    const float *mono_inv_sigma2;       /* [E] mvInvLevelSigma2[octave] / uncertainty2 */
    const float *mono_xw;               /* [E][3] MapPoint::GetWorldPos() */
    const uint8_t *mono_close;          /* [E] MapPoint::mTrackDepth < 10 (bClose) */
    const int32_t *stereo_start;        /* [F+1] (all zero: no stereo edges) */
    const int32_t *stereo_cam, *stereo_kp;
    const double *stereo_obs;           /* [S][3] (u, v, mvuRight) */
    const float *stereo_inv_sigma2, *stereo_xw;
    int kp_cap;                         /* per-frame stride of kp_outlier */
    int n_mono, n_stereo;               /* edge totals of the batch (mono_start[F], stereo_start[F]) */
    const int32_t *cam_model;           /* host [n_cams] OMV_CAM_KB8 / OMV_CAM_PINHOLE (as omv_lba_problem); NULL: KB8 */
} omv_pose_batch;

typedef struct omv_pose omv_pose;
omv_status omv_pose_create(int max_frames, int max_edges, omv_pose **out);
omv_status omv_pose_destroy(omv_pose *h);
/* PoseInertialOptimizationLastKeyFrame on every frame of the batch.  kp_outlier (device
 * [F][kp_cap], Frame::mvbOutlier of the keypoints that carry an edge; others untouched), n_good
 * (device [F], the return value nInitialCorrespondences - nBad), H (device [F][225] or NULL, the
 * 15x15 Hessian of ConstraintPoseImu: pose 0-5, v 6-8, bg 9-11, ba 12-14).  Asynchronous. */
omv_status omv_pose_inertial_last_kf(omv_pose *h, const omv_pose_batch *b, int rec_init, uint8_t *kp_outlier,
                                     int32_t *n_good, double *H, void *stream);

/* Optimizer::PoseInertialOptimizationLastFrame (src/Optimizer.cc:5580-6170): as above, but the previous
 * frame's four vertices are free (ids 4-7; the batch's kf_* fields hold Frame::mpPrevFrame's state and
 * `preint` is Frame::mpImuPreintegratedFrame), one EdgeInertial over all six vertex blocks, EdgeGyroRW /
 * EdgeAccRW between the two frames' biases with information from Frame::mpImuPreintegrated's C (the
 * last keyframe's preintegration, :5960-5971), and an EdgePriorPoseImu (G2oTypes.cc:748-785, Huber 5)
 * on the previous frame from its ConstraintPoseImu (pFp->mpcpi).  The mono chi2 threshold is 5.991 in all
 * four rounds (:5992).  H receives the frame's 15x15 block after Optimizer::Marginalize(H, 0, 14)
 * (:3388-3455, pseudo-inverse below 1e-6) — the matrix handed to the ConstraintPoseImu ctor (:6158-6164);
 * run omv_pose_constraint on it to obtain the stored prior.  The previous frame's state is not written
 * back (the reference discards it). */
typedef struct omv_pose_prior {
    const double *Rwb, *twb, *vel, *bg, *ba;   /* device [F][9] / [F][3]: ConstraintPoseImu Rwb, twb, vwb, bg, ba */
    const double *H;                           /* device [F][225]: ConstraintPoseImu::H (after its ctor) */
    const float *preint_kf;                    /* device [F][OMV_PREINT_FLOATS]: Frame::mpImuPreintegrated */
} omv_pose_prior;
omv_status omv_pose_inertial_last_frame(omv_pose *h, const omv_pose_batch *b, const omv_pose_prior *prior,
                                        int rec_init, uint8_t *kp_outlier, int32_t *n_good, double *H, void *stream);

/* Optimizer::PoseOptimization (src/Optimizer.cc:855-1278), the visual-only pose optimisation Tracking runs before the
 * IMU is initialised (Tracking.cc:2924) and in the visual-only configurations: one VertexSE3Expmap (SE3Quat Tcw of
 * camera 0, oplus = exp(dx) * T, se3quat.h:223-257), one unary edge per edge of the batch — mono edges
 * EdgeSE3ProjectXYZOnlyPose (camera 0) / ...ToBody / ...SLPoseToBody / ...SRPoseToBody (camera c through T_c0,
 * OptimizableTypes.cpp:30-171; Huber sqrt(5.991)), stereo edges EdgeStereoSE3ProjectXYZOnlyPose (camera 0 with
 * fx fy cx cy = cam[0][0..3] and bf, types_six_dof_expmap.cpp:339-404; Huber sqrt(7.815)) — and
 * Levenberg-Marquardt (optimization_algorithm_levenberg.cpp:61-169, tau 1e-5, 10 trials) with a dense LDLT: 4 rounds of
 * optimize(10), each from the initial pose, chi2 5.991 / 7.815 outlier classification between rounds, robust kernels
 * dropped after round 3, a single round below 10 edges.  Uses of `b`: n_frames, n_cams, cam, cam_model, bf, the
 * mono_* / stereo_* edge arrays (mono_close unused; stereo_cam ignored: camera 0), kp_cap, n_mono, n_stereo — the
 * inertial state / preintegration fields are ignored.  Edges follow the reference's creation rule: one edge per
 * keypoint (the conventional branch makes a keypoint with mvuRight >= 0 a stereo edge INSTEAD of a mono one).
 *   rig_q / rig_t   host [n_cams][4] (x y z w) / [3]: T_c0 = mTrl / mTsll / mTsrl as SE3Quat (entry 0 unused)
 *   pose_q / pose_t device [F][4] / [F][3] in/out: Frame::GetPose() as the SE3Quat the reference builds (:871-873);
 *                   out: the optimised estimate (unchanged below 3 edges)
 *   kp_outlier      device [F][kp_cap]: mvbOutlier of the edges' keypoints
 *   n_good          device [F]: the return value (nInitialCorrespondences - nBad; 0 below 3 edges)
 * One workgroup per frame; asynchronous. */
omv_status omv_pose_optimization(omv_pose *h, const omv_pose_batch *b, const double *rig_q, const double *rig_t,
                                 double *pose_q, double *pose_t, uint8_t *kp_outlier, int32_t *n_good, void *stream);

/* Kernel choice of the two calls above.  OMV_POSE_AUTO (default): up to 16 frames per call run on the grouped
 * kernel — one frame over `parts` workgroups (0: one per 126 (LastFrame) / 190 (LastKeyFrame) visual edges of the batch's
 * mean frame, at least ceil(edges of the whole batch / 1022) so that no frame's part can overflow, at most 48) that
 * exchange their normal-equation sums every Gauss-Newton iteration, the latency path of Tracking's one-frame call —
 * and larger batches (or a batch whose edges need more than 48 parts) on one workgroup per frame.  OMV_POSE_BATCH / OMV_POSE_GROUPED force one of them (GROUPED needs kp_cap <= 16384).
 * The grouped kernel reports a frame it could not run (more than 1024 visual edges in one workgroup's keypoint
 * range) with n_good = -1 and OMV_ERR_CAPACITY in omv_pose_last_error. */
#define OMV_POSE_AUTO 0
#define OMV_POSE_BATCH 1
#define OMV_POSE_GROUPED 2
omv_status omv_pose_set_mode(omv_pose *h, int mode, int parts);
/* Device error word of the calls since the last read (0, or OMV_ERR_CAPACITY / OMV_ERR_HIP from the grouped kernel);
 * resets it and synchronises `stream`. */
omv_status omv_pose_last_error(omv_pose *h, int32_t *err, void *stream);

/* The pose graph's visual edges of ONE frame from its map-point assignment, on the device — the edge-creation loop
 * of PoseInertialOptimizationLastKeyFrame / LastFrame (src/Optimizer.cc:5079-5330, :5640-5800) for the multi-camera
 * frame (bRight), so SearchByProjection's output feeds the optimisation without a host round trip: per keypoint slot
 * s = cam * kp_cap + i (the [L | R | SL | SR] order) with kp_to_mp[s] >= 0 an EdgeMonoOnlyPose of block cam (obs =
 * keypoint, invSigma2 = inv_level_sigma2[octave] (uncertainty2 = 1 for KannalaBrandt8 / Pinhole), Xw =
 * mp_pos[kp_to_mp[s]], bClose = mp_track_depth < 10), and with uright[s] > 0 also an EdgeStereoOnlyPose of that
 * block; both lists in slot order, counts in mono_start[1] / stereo_start[1] (start[0] = 0) — the omv_pose_batch edge
 * arrays of a one-frame batch (pass max_edges as its n_mono / n_stereo bound; the batch's kp_cap = n_cams * kp_cap).
 * kps / n_kp / kp_to_mp / mp_* / uright: device (uright [n_cams][kp_cap], omv_frame_uright's layout, or NULL = no
 * stereo edges); inv_level_sigma2: host [n_levels].  More than max_edges edges of a kind
 * raise OMV_ERR_CAPACITY in omv_pose_last_error.  Asynchronous. */
omv_status omv_pose_edges_from_matches(omv_pose *h, int n_cams, int kp_cap, const omv_kp *kps, const int *n_kp,
                                       const int32_t *kp_to_mp, const float *mp_pos, const float *mp_track_depth,
                                       const float *inv_level_sigma2, int n_levels, const float *uright, int max_edges,
                                       int32_t *mono_start, int32_t *mono_cam, int32_t *mono_kp, double *mono_obs,
                                       float *mono_inv_sigma2, float *mono_xw, uint8_t *mono_close, int32_t *stereo_start,
                                       int32_t *stereo_cam, int32_t *stereo_kp, double *stereo_obs,
                                       float *stereo_inv_sigma2, float *stereo_xw, void *stream);

/* ConstraintPoseImu ctor (include/G2oTypes.h:639-659) on n matrices: H <- (H + H) / 2 (= H), then its
 * symmetric eigen-decomposition with eigenvalues below 1e-12 zeroed, recomposed.  Device [n][225]
 * (H_out may alias H_in).  Asynchronous. */
omv_status omv_pose_constraint(int n, const double *H_in, double *H_out, void *stream);

/* ---- IMU preintegration ----
 * IMU::Preintegrated::IntegrateNewMeasurement (src/ImuTypes.cc:160-239) over n independent records, as
 * Tracking::PreintegrateIMU drives it (src/Tracking.cc:1675-1712).  Record r integrates the measurements
 * meas[start[r] .. start[r+1]) in order, each (ax ay az wx wy wz dt) with the interpolation of
 * PreintegrateIMU already applied, starting from its current state:
 *   preint  device [n][OMV_PREINT_FLOATS] in/out (dR dV dP JRg JVg JVa JPg JPa b dT C; Initialize() =
 *           identity dR, zeros elsewhere, b = the bias)
 *   avg     device [n][6] in/out avgA | avgW, or NULL
 *   start   device [n+1]; meas device [start[n]][7]
 *   Nga / NgaWalk  host [6]: the diagonals of IMU::Calib::Cov / CovWalk (Eigen::DiagonalMatrix<float, 6>,
 *                  include/ImuTypes.h:126; Tracking.cc:601 builds them from Ng*sf, Na*sf, Ngw/sf, Naw/sf). */
omv_status omv_imu_preintegrate(int n, float *preint, float *avg, const float *meas, const int32_t *start,
                                const float *Nga, const float *NgaWalk, void *stream);

/* ---- DBoW2 vocabulary transform ----
 * TemplatedVocabulary<FORB::TDescriptor, FORB>::transform(features, BowVector&, FeatureVector&, levelsup)
 * (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1127-1194, per feature :1217-1259) as Frame::ComputeBoW /
 * KeyFrame::ComputeBoW call it (src/KeyFrame.cc:207-214, levelsup 4), over a batch of descriptor sets.
 * The vocabulary tree is flattened in loadFromTextFile's node order (node 0 = root, :1338-1424). */
typedef struct omv_vocab {
    int n_nodes, n_words;
    int L;                         /* m_L (FeatureVector level = L - levelsup)                        */
    int scoring;                   /* DBoW2::ScoringType: 0 L1, 1 L2, 2 chi-square, 3 KL, 4 Bhattacharyya, 5 dot product */
    int weighting;                 /* DBoW2::WeightingType: 0 TF_IDF, 1 TF, 2 IDF, 3 BINARY            */
    const int32_t *child_start;    /* device [n_nodes + 1]: m_nodes[i].children as a CSR, file order  */
    const int32_t *child_ids;      /* device [child_start[n_nodes]]                                   */
    const uint8_t *desc;           /* device [n_nodes][32] node descriptors                           */
    const int32_t *word_id;        /* device [n_nodes] m_nodes[i].word_id (leaves)                    */
    const double *weight;          /* device [n_nodes] m_nodes[i].weight (idf; 0 = stopped word)      */
} omv_vocab;

/* n_sets sets of desc [set][cap][32] with n_desc[set] <= cap <= 16384 rows (mDescriptors row order).
 * Per feature (device [set][cap]): word, wval (the word's weight), node (FeatureVector node, -1 if the
 * descent ended above that level).  BowVector (device [set][cap]): bow_word ascending, bow_value, count in
 * bow_n [set].  FeatureVector (device): fv_node [set][cap] ascending, fv_start [set][cap + 1] (offsets
 * into fv_idx [set][cap]), count in fv_n [set].  Stopped words (weight <= 0) are left out of both, as in
 * the reference.  Asynchronous. */
omv_status omv_bow_transform(const omv_vocab *voc, int n_sets, const uint8_t *desc, int cap, const int *n_desc,
                             int levelsup, int32_t *word, double *wval, int32_t *node, int32_t *bow_word,
                             double *bow_value, int32_t *bow_n, int32_t *fv_node, int32_t *fv_start, int32_t *fv_idx,
                             int32_t *fv_n, void *stream);

/* ---- Frame construction tail (src/Frame.cc:1913-1939) ---- */

/* cv::fisheye::undistortPoints parameters of one camera block (GetDepthFromUndistortedPoints,
 * src/Frame.cc:1659-1734): origK / newK as float (fx, fy, cx, cy; the reference's cv::Mat_<float>),
 * dist_coeff as double (k1..k4). */
typedef struct omv_fisheye_undist {
    float K[4];
    double D[4];
    float newK[4];
} omv_fisheye_undist;

/* GetDepthFromUndistortedPoints for every keypoint of every camera block:
 * cv::fisheye::undistortPoints(kp.pt, origK, D, noArray(), newK) (OpenCV >= 4.5 semantics: at most
 * 10 Newton steps, eps 1e-8, theta clipped to pi/2, (-1e6, -1e6) for a flipped / unconverged theta),
 * then d = depth[cam](round(y), round(x)) (0 outside the image) and
 * u_right = kp.x - bf / d where 0 < d <= 20, else -1 (:1736-1763); the reference's mvuRight.
 * The first n_blocks (<= n_cams, <= 8) camera blocks of each frame are processed.
 *   kps / n_kp   device [frame][n_cams][kp_cap] / [frame][n_cams]
 *   depth        device float [frame][n_blocks][depth_h][depth_w] (the undistorted depth images)
 *   undist       host [n_blocks]: the block's parameters (the reference maps L, R, SL, SR to its
 *                cam_id 1, 0, 4, 3, :1916-1922)
 *   u_right      device float [frame][n_blocks][kp_cap]
 *   undist_xy    device float [frame][n_blocks][kp_cap][2] (the undistorted points) or NULL */
omv_status omv_frame_uright(int n_frames, int n_cams, int n_blocks, int kp_cap, const omv_kp *kps, const int *n_kp,
                            const float *depth, int depth_w, int depth_h, const omv_fisheye_undist *undist, float bf,
                            float *u_right, float *undist_xy, void *stream);

/* The cv::vconcat of Frame's per-camera keypoints / descriptors / mvuRight into the dense frame
 * arrays (mDescriptors = [L; R; SL; SR], :1936-1939; mvKeys order of the N-indexed vectors):
 * frame f's keypoints of its first n_blocks (<= n_cams) blocks land at rows [offset[f], offset[f] + N_f),
 * N_f = sum of n_kp[f][0..n_blocks).  uright_in: [frame][n_blocks][kp_cap] (omv_frame_uright's layout).
 *   offset       device int [n_frames + 1] (output; exclusive prefix of N_f, offset[n_frames] = total)
 *   kps_out / desc_out / uright_out   device [total] rows (uright_in / uright_out may be NULL) */
omv_status omv_frame_pack(int n_frames, int n_cams, int n_blocks, int kp_cap, const omv_kp *kps, const uint8_t *desc,
                          const float *uright_in, const int *n_kp, int *offset, omv_kp *kps_out, uint8_t *desc_out,
                          float *uright_out, void *stream);


/* ---- map-point refresh (LocalMapping.cc:338-339, :776-778, :897-898; MapPoint.cc:377) ----------------------------
 * MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:405-490) for a batch of map points: point p's descriptors are
 * rows desc_row[desc_start[p] .. desc_start[p+1]) of `desc` ([rows][32] u8) -- its observations' L / R / SL / SR rows
 * in the reference's mObservations (std::map) order, bad keyframes left out by the caller.  best_row[p] = the row of
 * the descriptor with the least median Hamming distance to the others (vDists[0.5 (N - 1)] of its sorted row, the
 * first on ties), -1 when the point has none (mDescriptor untouched); desc_out[p] (may be NULL) = that descriptor.
 * All pointers device. */
omv_status omv_mappoint_distinctive_descriptors(int n_points, const int32_t *desc_start, const int32_t *desc_row,
                                                const uint8_t *desc, int32_t *best_row, uint8_t *desc_out, void *stream);
/* MapPoint::UpdateNormalAndDepth (src/MapPoint.cc:503-588): per point its observation entries
 * obs_start[p] .. obs_start[p+1] with the entry camera centre obs_center[e] (float3: GetCameraCenter /
 * GetRightCameraCenter / GetSideLeftCameraCenter / GetSideRightCameraCenter of the keyframe, every entry -- the
 * reference does not skip bad keyframes here), its mWorldPos pos[p], the reference keyframe's camera centre
 * ref_center[p], mvScaleFactors[level] of the point's keypoint in it (ref_level_scale[p]) and
 * mvScaleFactors[nLevels - 1] (ref_max_scale[p]).  Out: mNormalVector, mfMinDistance, mfMaxDistance (float, the
 * reference's arithmetic order); a point without entries is left untouched.  All pointers device. */
omv_status omv_mappoint_normal_depth(int n_points, const int32_t *obs_start, const float *obs_center, const float *pos,
                                     const float *ref_center, const float *ref_level_scale, const float *ref_max_scale,
                                     float *normal, float *min_dist, float *max_dist, void *stream);


/* ---- LocalMapping::SearchInNeighbors' fuse sequence (src/LocalMapping.cc:837-889) ------------------------------------
 * The reference runs ORBmatcher::Fuse (ORBmatcher.cc:1458-1647) as a chain of calls that mutate the map between (and
 * within) calls: phase A fuses the current keyframe's map points (ONE snapshot of GetMapPointMatches(), :839) into every
 * target keyframe, camera block by camera block (:840-853); phase B fuses the target keyframes' map points (collected
 * AFTER phase A, non-bad, first occurrence, :859-881) into the current keyframe (:883-889).  Each accepted match either
 * AddObservation + AddMapPoint's, or Replace's the weaker of the two points (MapPoint.cc:316-380: observations moved,
 * the loser bad, the survivor's descriptor recomputed by ComputeDistinctiveDescriptors, :405-483).  A later point's
 * decision reads that state: isBad(), IsInKeyFrame(pKF), GetMapPoint(bestIdx), Observations() and -- through the
 * window search -- GetDescriptor().
 * Here the window searches of every (job, point) are evaluated on the device speculatively (one omv_matcher_search_kf
 * launch per phase), the decisions are walked in the reference's order on the host against the flattened graph, and an
 * entry whose point's descriptor changed since its evaluation (a Replace survivor) is re-evaluated on the device with
 * the recomputed descriptor before it is used (the recomputation itself on the device: the distinctive-descriptor
 * kernel over the observation rows the reference's ComputeDistinctiveDescriptors reads at that moment).  The result is
 * the reference's graph after phase B, plus the ordered edit log a caller replays with the reference's own methods.
 * Phase C (:891-900: ComputeDistinctiveDescriptors / UpdateNormalAndDepth of the current keyframe's points) is
 * omv_mappoint_* on the caller's side.
 * Keyframes are the n_kf frames of the matcher's last omv_matcher_assign_grid batch (C = geom->n_cams <= 4 camera blocks,
 * N-index = block offset + index in the block, NLeft / NRight / NSideLeft = n_kp[kf][0..2]), NUMBERED IN THE ORDER OF
 * THE MAP POINTS' std::map<KeyFrame*, ...> KEYS (observations are kept sorted by keyframe index). */
typedef struct omv_fuse_graph {
    /* keyframes (host) */
    int n_kf;
    const int32_t *n_blocks;            /* [n_kf] camera blocks Fuse runs on: 1 (NLeft == -1), 2, or 4 (side cameras) */
    const omv_se3f *Tcw;                /* [n_kf][C] GetPose / GetRightPose / GetSideLeftPose / GetSideRightPose */
    const float *Ow;                    /* [n_kf][C][3] the matching camera centres */
    const float *uright;                /* [n_kf][kp_cap] mvuRight of block 0 (host; AddObservation's nObs += 2 when
                                           the keyframe has one camera), or NULL */
    int32_t *kf_mps;                    /* [n_kf][C * kp_cap] in/out: mvpMapPoints by N-index (entries [0, N) of each
                                           keyframe's row): map-point index or -1 */
    /* map points (host): the snapshot of the points the keyframes reference */
    int n_mps;
    int32_t *bad;                       /* [n_mps] in/out isBad() */
    int32_t *n_obs;                     /* [n_mps] in/out Observations() (nObs) */
    int32_t *replaced;                  /* [n_mps] out: the point it was Replace'd by, or -1 */
    const int32_t *obs_start;           /* [n_mps + 1] in: mObservations rows, keyframe order */
    const int32_t *obs_kf;              /* [rows] keyframe index */
    const int32_t *obs_idx;             /* [rows][4] left / right / side-left / side-right N-index or -1 */
    /* out: the final mObservations (CSR with capacity), the edit log */
    int32_t *out_obs_start;             /* [n_mps + 1] */
    int32_t *out_obs_kf;                /* [obs_cap] */
    int32_t *out_obs_idx;               /* [obs_cap][4] */
    int obs_cap;
    int32_t *log;                       /* [log_cap][4]: {0, mp, kf, idx} AddObservation(pKF, idx) + pKF->AddMapPoint;
                                           {1, a, b, -1} a->Replace(b); in the reference's order */
    int log_cap;
    int32_t n_log;                      /* out: entries written (OMV_ERR_CAPACITY past log_cap / obs_cap) */
    int32_t n_reevaluated;              /* out: entries re-evaluated after a descriptor change (diagnostic) */
    int32_t n_device_calls;             /* out: device round trips (diagnostic) */
} omv_fuse_graph;

/* current: the current keyframe's index; targets: host [n_targets] vpTargetKFs in order; mps: the device map-point
 * table (pos / normal / min_dist / max_dist as GetWorldPos / GetNormal / mfMinDistance / mfMaxDistance; desc is
 * UPDATED IN PLACE to the final descriptors); p: omv_kf_search_params with mode OMV_KF_FUSE, th 3, max_dist TH_LOW
 * (50); geom / kps / desc / n_kp: the assign_grid batch (device).  n_fused: host [n_targets * C + C] per Fuse call,
 * phase A (target-major, block-minor) then phase B; calls the reference does not make (blocks past n_blocks) are 0.
 * Synchronous. */
omv_status omv_search_in_neighbors_fuse(omv_matcher *m, const omv_frame_geom *geom, const omv_kp *kps,
                                        const uint8_t *desc, const int *n_kp, int kp_cap, omv_fuse_graph *g,
                                        int current, int n_targets, const int32_t *targets, const omv_kf_mps *mps,
                                        const omv_kf_search_params *p, int32_t *n_fused, void *stream);

/* ---- LocalMapping::CreateNewMapPoints (src/LocalMapping.cc:395-783) ---------------------------------------------------
 * The reference walks the current keyframe's neighbours in order (:439).  Per neighbour pKF2: the baseline test
 * (:447-461: |Ow2 - Ow1| < pKF2->mb skips it when !mbMonocular; Ow1 is the PERSISTENT side-1 camera centre, see below),
 * SearchForTriangulation(mpCurrentKeyFrame, pKF2) (:468), and for every match (idx1, match12[idx1]) in idx1 order the
 * camera-pair state (listed pairs (0,0) (0,1) (1,0) (1,1) when both rigs have a second camera, (0,2) (2,0) (2,2) (1,3)
 * (3,1) (3,3) when they have four, :529-636; other pairs keep the previous match's state), parallax of the unprojected
 * rays, GeometricTools::Triangulate (JacobiSVD<Matrix4f>) or KeyFrame::UnprojectStereo, positive depth, reprojection
 * error in both keyframes, scale consistency; an accepted match creates a MapPoint and mpCurrentKeyFrame->AddMapPoint(
 * pMP, idx1) (:766-781) -- so every LATER neighbour's SearchForTriangulation skips idx1 (ORBmatcher.cc:1223-1227).
 * The state that crosses matches and neighbours: sophTcw1 / Ow1 (side 1's camera block, declared before the loop,
 * :419-424) persists across neighbours; pCamera1 / pCamera2 and side 2 reset per neighbour (:445, :470-474).  Float
 * arithmetic as the reference (no contraction; glibc atan2f / cosf / tanf restated).  Creating the MapPoint objects and
 * the graph updates (AddObservation, pKF2->AddMapPoint, ComputeDistinctiveDescriptors, UpdateNormalAndDepth) stay with
 * the caller (the last two: omv_mappoint_*); the current keyframe's has-map-point flags are updated here. */
typedef struct omv_cnmp_kf {
    omv_kf_view kf;                     /* kps by idx (mvKeysUn when NLeft == -1, else mvKeys / Right / SideLeft /
                                           SideRight by range), n_left = -1 for a single-camera keyframe, level_sigma2;
                                           desc / has_mp / nodes: read by omv_local_mapping_create_new_map_points'
                                           SearchForTriangulation (neighbours; the current keyframe's has_mp is the
                                           separate in/out array), unused by omv_create_new_map_points */
    const omv_kp *kps_raw;              /* [n] mvKeys for KeyFrame::UnprojectStereo (NULL: kf.kps) */
    float Tcw[4][12];                   /* GetPose / GetRightPose / GetSideLeftPose / GetSideRightPose: Rcw (row-major) | tcw */
    float Ow[4][3];                     /* GetCameraCenter / GetRightCameraCenter / GetSideLeft.. / GetSideRight.. */
    float Rwc[9], twc[3];               /* mRwc, mTwc.translation() (UnprojectStereo) */
    float fx, fy, cx, cy, invfx, invfy; /* the keyframe's fx fy cx cy invfx invfy */
    float mb, mbf;                      /* mb: also the neighbour's baseline threshold (:453) */
    const float *uright, *depth;        /* device [n] mvuRight / mvDepth (NULL: no stereo observations) */
    float scale_factors[16];            /* mvScaleFactors */
} omv_cnmp_kf;

typedef struct omv_cnmp_job {
    omv_cnmp_kf kf2;                    /* the neighbour */
    const int32_t *match12;             /* device [kf1.kf.n]: SearchForTriangulation's vMatches12 (-1 none; entries
                                           outside [0, kf2.kf.n) are ignored) */
    float *x3D;                         /* device [kf1.kf.n][3]: the new point of an accepted match */
    int32_t *status;                    /* device [kf1.kf.n]: 1 triangulated, 2 by UnprojectStereo (bPointStereo),
                                           0 rejected, no match, or the neighbour skipped by the baseline test */
} omv_cnmp_job;

/* The per-match geometry of CreateNewMapPoints for jobs whose match lists the caller obtained itself (e.g. the
 * single-camera stereo rigs SearchForTriangulation's device path does not cover).  Jobs run in order with the
 * reference's state chain: check_baseline = !mbMonocular (the baseline test against the persistent Ow1);
 * side1_state: device int32 in/out, side 1's camera block (sophTcw1 / Ow1) entering the first job and leaving the last
 * (0 = the current keyframe's left camera, the value at the top of CreateNewMapPoints; NULL: 0, not returned);
 * has_mp1: device [kf1.kf.n] or NULL, set to 1 at every accepted idx1 (:773).
 * EXACTNESS: a job's match12 must be the SearchForTriangulation result computed AFTER the previous jobs' AddMapPoint
 * (has_mp1), as the reference computes it per neighbour (:468).  A caller-driven loop passes one job per call
 * (SearchForTriangulation with kf1.has_mp = has_mp1, then this call with the same side1_state); several jobs in one
 * call are exact only when no accepted idx1 of an earlier job appears in a later job's list.
 * omv_local_mapping_create_new_map_points runs the whole loop on the device.
 * cams / cam_model: host [4][8] / [4] (the rig's L, R, SL, SR; NULL model = all KannalaBrandt8; others OMV_ERR_ARG);
 * n_cams: cameras of the rig (1: mpCamera2 == NULL, 2: L + R, 4: L R SL SR); inertial: mbInertial; far_points /
 * th_far_points: mbFarPoints / mThFarPoints; scale_factor: the current keyframe's mfScaleFactor (ratioFactor =
 * 1.5 scale_factor).  jobs: host array (n_jobs <= 64).  Asynchronous. */
omv_status omv_create_new_map_points(int n_jobs, const omv_cnmp_kf *kf1, const omv_cnmp_job *jobs, const float *cams,
                                     const int32_t *cam_model, int n_cams, int inertial, int far_points,
                                     float th_far_points, float scale_factor, int check_baseline,
                                     int32_t *side1_state, uint8_t *has_mp1, void *stream);

/* One neighbour of omv_local_mapping_create_new_map_points. */
typedef struct omv_cnmp_neighbour {
    omv_cnmp_kf kf2;                    /* kf2.kf: the full view SearchForTriangulation reads (kps, desc, has_mp =
                                           pKF2->GetMapPoint(idx2) != NULL, FeatureVector, level_sigma2) */
    float T[OMV_TRI_PAIRS][12];         /* the camera-pair transforms, as omv_tri_pair.T (keyframe 1 = current) */
    int skip;                           /* the caller's `continue` before the search: mbMonocular's median-depth
                                           ratio test (:455-461); the stereo baseline test is done here */
    int32_t *match12;                   /* device [kf1.kf.n] out: the neighbour's vMatches12 (all -1 when skipped) */
    float *x3D;                         /* device [kf1.kf.n][3] out, as omv_cnmp_job */
    int32_t *status;                    /* device [kf1.kf.n] out, as omv_cnmp_job */
} omv_cnmp_neighbour;

/* LocalMapping::CreateNewMapPoints' loop (:439-783) for a multi-camera rig (n_cams 2 or 4: the rigs
 * omv_matcher_search_for_triangulation covers), on the device with no host round trip between neighbours: per
 * neighbour in order, the baseline gate on the persistent Ow1, SearchForTriangulation(mpCurrentKeyFrame, pKF2,
 * bOnlyStereo = false, bCoarse = coarse) with the matcher's checkOri off (ORBmatcher matcher(0.6, false), :417) against
 * the current keyframe's has-map-point flags AS LEFT BY THE PREVIOUS NEIGHBOURS, then the per-match geometry, then
 * AddMapPoint(idx1) of the accepted matches.
 *   kf1        the current keyframe (kf1.kf: kps, desc, FeatureVector, level_sigma2, ranges; kf1.kf.has_mp ignored)
 *   has_mp1    device [kf1.kf.n] in/out: GetMapPoint(idx1) != NULL on entry, plus every accepted idx1 on return
 *   nb         host [n_nb] (n_nb <= 64) neighbours in vpNeighKFs order
 *   n_matches  device [n_nb]: SearchForTriangulation's return values (0 for a skipped neighbour)
 *   side1_state device int32 in/out or NULL (as omv_create_new_map_points): calls compose, so a caller that checks
 *              CheckNewKeyFrames() between neighbours (:440) runs one neighbour per call with the same has_mp1 /
 *              side1_state and gets the identical result
 * check_baseline = !mbMonocular; the other arguments as omv_create_new_map_points.  Synchronises `stream` once at the
 * end (the device error word: OMV_ERR_CAPACITY for a keyframe past SearchForTriangulation's limits). */
omv_status omv_local_mapping_create_new_map_points(omv_matcher *m, const omv_cnmp_kf *kf1, uint8_t *has_mp1, int n_nb,
                                                   const omv_cnmp_neighbour *nb, const float *cams,
                                                   const int32_t *cam_model, int n_cams, int inertial,
                                                   int check_baseline, int coarse, int far_points, float th_far_points,
                                                   float scale_factor, int32_t *n_matches, int32_t *side1_state,
                                                   void *stream);

#ifdef __cplusplus
}
#endif
#endif /* OMV_H */
