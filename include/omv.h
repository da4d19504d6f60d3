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

/* Device-side error word of the last batch (OMV_ERR_CAPACITY if a bound was hit); syncs the stream. */
omv_status omv_orb_last_error(omv_orb *orb);

/* Debug/parity hooks: copy pyramid level `level` of image `img` of the last batch to host. */
omv_status omv_orb_debug_level(omv_orb *orb, int img, int level, uint8_t *out, int *w, int *h);

/* ------------------------------------------------------------------------------------------------
 * Hamming matching
 * ---------------------------------------------------------------------------------------------- */

/* cv::BFMatcher(NORM_HAMMING).knnMatch(k=2) as used by Frame::ComputeMultiFishEyeMatches
 * (src/Frame.cc:1483): for each query row the two nearest train rows (first index wins ties).
 * Batched over n_pairs independent (query, train) sets laid out [pair][rows][32].
 *   idx2/dist2 device [n_pairs][q_cap][2]; -1 / INT32_MAX when fewer than 1 / 2 train rows. */
omv_status omv_bf_knn2(int n_pairs, const uint8_t *query, int q_cap, const int *nq, const uint8_t *train,
                       int t_cap, const int *nt, int32_t *idx2, int32_t *dist2, void *stream);

/* Camera-block view of one multi-camera Frame (the reference's Frame after the multi ctor,
 * src/Frame.cc:1767-1949): keypoints and descriptors concatenated [cam0|cam1|...] with per-camera
 * offsets, and per-camera 64x48 grids (AssignFeaturesToGrid, src/Frame.cc:541-582). */
typedef struct omv_frame_geom {
    int n_cams;          /* camera blocks: 0 = left, 1 = right, >=2 side cameras                */
    float min_x, max_x;  /* Frame::mnMinX/mnMaxX (bounds of imLeft, shared by all cameras)       */
    float min_y, max_y;
    int nlevels;
    float scale_factors[16]; /* Frame::mvScaleFactors                                            */
} omv_frame_geom;

/* Build the per-camera grids on device.  kps/desc are [frame][n_cams][kp_cap]; n_kp [frame][cam].
 * grid_start/grid_idx are device outputs sized by omv_grid_sizes(). */
void omv_grid_sizes(int n_frames, int n_cams, int kp_cap, size_t *start_ints, size_t *idx_ints);
omv_status omv_grid_build(int n_frames, const omv_frame_geom *geom, const omv_kp *kps, int kp_cap,
                          const int *n_kp, int32_t *grid_start, int32_t *grid_idx, void *stream);

/* Local map points projected into a frame (the fields SearchByProjection reads from MapPoint after
 * Frame::isInFrustum, src/ORBmatcher.cc:33-60; src/Frame.cc:736-826).  SoA, [frame][M] per field
 * except the per-camera arrays which are [frame][M][n_cams]. */
typedef struct omv_mp_view {
    const uint8_t *desc;      /* [M][32] MapPoint::GetDescriptor()                                */
    const float *proj_x;      /* [M][n_cams] mTrackProjX / XR / XSL / XSR ...                     */
    const float *proj_y;      /* [M][n_cams]                                                      */
    const float *view_cos;    /* [M][n_cams] mTrackViewCos*                                       */
    const int32_t *level;     /* [M][n_cams] mnTrackScaleLevel* (-1 = none)                       */
    const uint8_t *in_view;   /* [M][n_cams] mbTrackInView*                                       */
    const float *track_depth; /* [M] mTrackDepth                                                  */
    const uint8_t *is_bad;    /* [M] MapPoint::isBad()                                            */
    const uint8_t *has_obs;   /* [M] Observations() > 0                                           */
} omv_mp_view;

/* ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th, bFarPoints, thFarPoints)
 * (src/ORBmatcher.cc:23-340), batched over n_frames independent frames.
 *   kp_to_mp      device [frame][N_total] in/out: MapPoint index per keypoint (-1 = none), i.e.
 *                 F.mvpMapPoints as dense indices; entries >= 0 on entry whose point has
 *                 observations block the keypoint (the `Observations() > 0` test, :77-79) —
 *                 pass kp_occ_init for points outside this call's list.
 *   l2r / r2l     device [frame][N_cam0] / [frame][N_cam1] mvLeftToRightMatch/mvRightToLeftMatch
 *   n_matches     device [frame] return value.
 * Semantics are the reference's sequential ones (earlier map points claim keypoints first). */
omv_status omv_match_project(int n_frames, const omv_frame_geom *geom, const omv_kp *kps, const uint8_t *desc,
                             int kp_cap, const int *n_kp, const int32_t *grid_start, const int32_t *grid_idx,
                             const omv_mp_view *mps, int M, float th, int far_points, float th_far,
                             float nnratio, const int32_t *l2r, const int32_t *r2l, const uint8_t *kp_occ_init,
                             int32_t *kp_to_mp, int *n_matches, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* OMV_H */
