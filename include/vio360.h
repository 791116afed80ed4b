/*
 * vio360.h — C-ABI of the MI355X-native hot path of 93won/360_visual_inertial_odometry.
 *
 * Pure C, caller-owned host buffers, no Eigen/OpenCV/torch types.  Each entry point replaces
 * one reference interface (cited file:line, paths relative to the reference repo root):
 *
 *   vio_ba_solve          Optimizer::RunLocalBA / RunBA / RunFullBA / RunVIBA / SolvePnP
 *                         (src/optimization/Optimizer.h:107-177, Optimizer.cpp:83-966)
 *                         = Ceres::Solve(SPARSE/DENSE_SCHUR, LM) over BAFactor/PnPFactor/
 *                         InertialFactorFixedGravity (src/optimization/Factors.cpp:33-612,1299-1485)
 *                         plus the chi^2 outlier tagging that follows each solve.
 *   vio_ba_solve_batched  many independent windows in one launch (config 4 / §8e).
 *   erp_klt_track         cv::calcOpticalFlowPyrLK call in FeatureTracker::TrackOpticalFlow
 *                         (src/processing/FeatureTracker.cpp:228-251)
 *   erp_gftt              cv::goodFeaturesToTrack call in FeatureTracker::DetectNewFeatures
 *                         (src/processing/FeatureTracker.cpp:208-226)
 *   vio_mono_init_solve   Initializer::TryMonocularInitialization (src/processing/Initializer.cpp:47-291)
 *   vio_window_*          Estimator::CreateKeyframe window slide / TriangulateNewMapPoints
 *                         (src/processing/Estimator.cpp:637-804, 1141-1318)
 *   erp_rot_ransac        FeatureTracker::RejectOutliersRotationRANSAC / EstimateRotation /
 *                         ComputeRotationInliers (src/processing/FeatureTracker.cpp:253-379)
 *
 * The gather of a window from the Frame/MapPoint graph and the write-back rules are the host
 * adapter's job; this ABI sees only flat arrays.
 *
 * Return convention: 0 on success, negative errno-style code on an API error (bad argument,
 * HIP failure).  A numerical failure of the solver is NOT an API error: it is reported through
 * vio_ba_summary.success = 0, exactly like Ceres Solver::Summary::IsSolutionUsable().
 */
#ifndef VIO360_H_
#define VIO360_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VIO360_ABI_VERSION 4

/* ----------------------------------------------------------------------------------------- */
/* error codes                                                                                */
#define VIO_OK 0
#define VIO_EINVAL (-22)   /* bad argument / inconsistent sizes */
#define VIO_ENOMEM (-12)   /* device allocation failed */
#define VIO_EDEVICE (-5)   /* HIP runtime error */
#define VIO_ENOSYS (-38)   /* variant not supported */

/* ----------------------------------------------------------------------------------------- */
/* context = device + stream + device scratch; one per host thread.                          */
typedef struct vio_ctx vio_ctx;

int vio_ctx_create(int device, vio_ctx** out);
/* destroy every batch / tracker / front-end created on the context first: they use its stream */
void vio_ctx_destroy(vio_ctx* ctx);
/* last error message of this context (or of the last failed vio_ctx_create when ctx==NULL) */
const char* vio_ctx_last_error(const vio_ctx* ctx);
int vio_abi_version(void);
/* VIO_OK when every translation unit of this library was compiled against the same layout of its
 * internal cross-TU argument structs (a stale object after a header change is reported as VIO_EDEVICE
 * here and by vio_ctx_create instead of faulting a kernel); needs no GPU */
int vio_layout_check(void);

/* Window-BA execution route of this context's later solves / batches (the routes give the same
   results to roundoff, each with its own fixed summation order; within a route results do not depend
   on the batch):
   AUTO (default) = the cluster route for batches of up to 32 LocalBA / BA / VIBA windows (when the
   device can hold every workgroup of the batch at once), the phase kernels for larger batches; PnP
   windows always run single-kernel.
   PHASES / SINGLE_KERNEL / CLUSTER force one route for every non-PnP window (CLUSTER falls back to the
   phase kernels when the batch does not fit the device at once). */
#define VIO_BA_ROUTE_AUTO 0
#define VIO_BA_ROUTE_PHASES 1
#define VIO_BA_ROUTE_SINGLE_KERNEL 2
#define VIO_BA_ROUTE_CLUSTER 3
int vio_ctx_set_ba_route(vio_ctx* ctx, int route);

/* Device Lie maths of the BA factors, evaluated for n inputs with the same device code
   the solvers inline, for parity tests against Ceres' rotation known answers
   (thirdparty/ceres-solver/internal/ceres/rotation_test.cc:406-589).  Rotations row-major.
     VIO_LIE_SO3_EXP   in 3 (phi)        -> out 9   SO3d::Exp as the window factors evaluate it
                                                    (LieUtils.cpp:203-219; no re-projection)
     VIO_LIE_SE3_EXP   in 6 ([rho, phi]) -> out 12  SE3d::exp: R (9) | t (3) (LieUtils.cpp:305-333)
     VIO_LIE_IMU_LOG   in 9 (R)          -> out 3   InertialFactorFixedGravity::log_SO3 (Factors.cpp:1507-1519)
     VIO_LIE_SO3D_EXP  in 3              -> out 9   SO3d::Exp + the SO3d constructor's projection (IMU init)
     VIO_LIE_SO3D_LOG  in 9              -> out 3   SO3d::Log with its theta ~ pi branch (LieUtils.cpp:221-273) */
#define VIO_LIE_SO3_EXP 0
#define VIO_LIE_SE3_EXP 1
#define VIO_LIE_IMU_LOG 2
#define VIO_LIE_SO3D_EXP 3
#define VIO_LIE_SO3D_LOG 4
int vio_lie_eval(vio_ctx* ctx, int op, const double* in, int n, double* out);

/* ----------------------------------------------------------------------------------------- */
/* Bundle adjustment / PnP                                                                    */

/* rigid transform, row-major rotation, f64 (reference keeps f32 Eigen::Matrix4f and casts) */
typedef struct {
    double R[9];
    double t[3];
} vio_pose;

/* IMUPreintegration (src/processing/IMUPreintegrator.h:40-69), f32 fields as in the reference */
typedef struct {
    float delta_R[9];   /* row-major */
    float delta_V[3];
    float delta_P[3];
    float J_Rg[9], J_Vg[9], J_Va[9], J_Pg[9], J_Pa[9];
    float cov9[81];     /* covariance.block<9,9>(0,0), row-major */
    float gyro_bias[3];
    float accel_bias[3];
    float _pad[2];
    double dt_total;
} vio_preint;

/* which Optimizer entry point the problem mirrors (selects constants and fixing rules) */
enum {
    VIO_BA_LOCAL = 0, /* RunLocalBA: pose 0 constant (if observed), marginalised MPs constant,
                         chi2 threshold 5.99146 (Optimizer.cpp:726-966) */
    VIO_BA_FULL = 1,  /* RunBA(fix_first, fix_last): chi2 threshold 5.991 (Optimizer.cpp:304-486) */
    VIO_BA_VI = 2,    /* RunVIBA: + InertialFactorFixedGravity (Optimizer.cpp:493-724) */
    VIO_PNP = 3       /* SolvePnP: pose-only, 4 rounds of outlier tagging (Optimizer.cpp:83-302) */
};

/* Ceres termination types (ceres/types.h), mirrored */
enum { VIO_TERM_CONVERGENCE = 0, VIO_TERM_NO_CONVERGENCE = 1, VIO_TERM_FAILURE = 2 };

/*
 * One window = one Ceres problem.  Observation o links keyframe obs_kf[o] to landmark obs_lm[o]
 * with pixel obs_uv[2o..2o+1] (the f32 Feature::GetPixelCoord()).  Every observation given here
 * becomes one residual block (the adapter already dropped near-boundary features).
 *
 * Constant blocks: kf_const[k] != 0 → pose k is SetParameterBlockConstant; lm_const[l] != 0 →
 * point l constant.  For VIO_PNP all points are constant and lm_const marks *marginalised*
 * MapPoints (never tagged as outliers, Optimizer.cpp:219-220).  For every variant lm_marg[l]
 * marks marginalised MapPoints (exempt from outlier counting / SetBad); may be NULL.
 */
typedef struct {
    int32_t variant;          /* VIO_BA_* */
    int32_t num_kf;           /* K */
    int32_t num_lm;           /* L */
    int32_t num_obs;          /* N */
    double cols, rows;        /* ERP size (CameraParameters) */
    double huber_delta;       /* HuberLoss(δ) — 1.0 in the reference (Optimizer.cpp:28) */
    double info[4];           /* 2x2 information matrix, row-major (identity in the reference) */
    double chi2_threshold;    /* 5.99146 (LocalBA) or 5.991 (BA/VIBA/PnP) */
    const vio_pose* T_cb;     /* K entries: Frame::GetTCB() of each keyframe (raw f32->f64) */
    const vio_pose* T_wb_init;/* K entries: Frame::GetTwb() (raw f32->f64) */
    const uint8_t* kf_const;  /* K */
    const uint8_t* lm_const;  /* L */
    const uint8_t* lm_marg;   /* L, may be NULL */
    const double* lm_xyz;     /* L*3 initial positions (f32 -> f64) */
    const int32_t* obs_kf;    /* N */
    const int32_t* obs_lm;    /* N */
    const float* obs_uv;      /* 2N */
    /* VIO_BA_VI only (else NULL) */
    const vio_preint* preint; /* K entries; preint[k] links keyframe k-1 -> k (entry 0 unused) */
    const uint8_t* preint_valid; /* K; 0 → factor k-1->k missing (RunVIBA skips it) */
    const double* vel;        /* K*3 initial velocities */
    double bg[3], ba[3];      /* initial shared biases */
    double gravity[3];        /* fixed gravity in world */
    /* solver controls */
    int32_t max_iterations;   /* 50 in the reference (Optimizer.cpp:30) */
    int32_t fixed_iterations; /* != 0 → benchmark mode: run exactly max_iterations LM iterations
                                 with all convergence tests disabled */
    int32_t num_rounds;       /* VIO_PNP: outlier rounds (4); ignored otherwise */
    int32_t _pad0;
} vio_ba_problem;

typedef struct {
    int32_t success;          /* Summary::IsSolutionUsable() (and PnP inlier gate) */
    int32_t termination;      /* VIO_TERM_* of the (last) solve */
    int32_t iterations;       /* summary.iterations.size() (PnP: sum over rounds) */
    int32_t num_successful_steps;
    int32_t num_unsuccessful_steps;
    int32_t num_inliers;      /* chi2 <= threshold after the solve */
    int32_t num_outliers;
    int32_t num_bad_lm;       /* MapPoints to SetBad(): inliers==0 && outliers>=2 && !marg */
    double initial_cost;      /* summary.initial_cost (includes fixed cost) */
    double final_cost;        /* summary.final_cost  (PnP: mean inlier chi2 of last round) */
    double fixed_cost;        /* cost of residual blocks whose parameters are all constant */
    double _pad1;
} vio_ba_summary;

/* One entry of Ceres Solver::Summary::iterations (ceres/iteration_callback.h IterationSummary), pushed
   where TrustRegionMinimizer::FinalizeIterationAndCheckIfMinimizerCanContinue pushes it
   (trust_region_minimizer.cc:313-348): iteration 0 (IterationZero :195-229), every valid, invalid
   (HandleInvalidStep :453-486), accepted (HandleSuccessfulStep :806-826) or rejected (:118-129) step;
   an iteration that ends the solve on the parameter / function tolerance is not pushed (:108-114).
   The reference reads Summary::iterations.size() (src/optimization/Optimizer.cpp:481-483). */
typedef struct {
    int32_t iteration;
    int32_t step_is_valid;
    int32_t step_is_successful;
    int32_t _pad;
    double cost;                /* x or candidate cost + fixed cost */
    double cost_change;         /* x_cost - candidate_cost (0 for an invalid step) */
    double gradient_max_norm;   /* |x - Plus(x, -g)|_inf of the last linearisation */
    double step_norm;           /* |x - candidate| */
    double relative_decrease;   /* TrustRegionStepEvaluator::StepQuality */
    double trust_region_radius; /* after the step's radius update */
    double model_cost_change;   /* -(J h)^T (r + J h / 2); not an IterationSummary field (margin analysis) */
} vio_ba_iteration;

/* outputs, caller-owned; any pointer may be NULL if not wanted */
typedef struct {
    vio_pose* T_wb;           /* K: SE3(T_wb_init) * exp(delta) (constant poses: SE3(T_wb_init)) */
    double* lm_xyz;           /* L*3 final point parameters */
    double* obs_chi2;         /* N: compute_chi_square at the solution */
    uint8_t* obs_outlier;     /* N: chi2 > threshold (PnP: also !marginalised) */
    uint8_t* lm_bad;          /* L: SetBad decision */
    double* vel;              /* K*3 (VI) */
    double* bg;               /* 3 (VI) */
    double* ba;               /* 3 (VI) */
    vio_ba_summary* summary;  /* 1 */
    /* per-iteration trace (Summary::iterations): up to trace_cap entries, summary->iterations of them
       (PnP: the rounds' traces one after another); may be NULL */
    vio_ba_iteration* trace;
    int32_t trace_cap;
    int32_t _pad2;
} vio_ba_output;

/* Any window size: windows whose reduced system fits one workgroup (LocalBA / FullBA / PnP with
   K <= 16, VIBA with K <= 10) run on the windowed solver; larger ones (RunBA over hundreds of keyframes,
   RunVIBA beyond 10 keyframes: Optimizer.cpp:304-486, 493-724) on the multi-kernel global path. */
int vio_ba_solve(vio_ctx* ctx, const vio_ba_problem* prob, vio_ba_output* out);

/* n independent windows in ONE device launch (one workgroup per window); problems beyond the windowed
   path's bounds are solved one by one on the global path */
int vio_ba_solve_batched(vio_ctx* ctx, const vio_ba_problem* probs, vio_ba_output* outs, int n);

/*
 * Device-resident batched interface for benchmarking and multi-GPU sharding: upload once,
 * then vio_ba_batch_run() solves all windows from the resident copy with no host transfer.
 */
typedef struct vio_ba_batch vio_ba_batch;
/* windowed path only: VIO_ENOSYS for a window beyond its bounds (K > 16, VIBA K > 10) */
int vio_ba_batch_create(vio_ctx* ctx, const vio_ba_problem* probs, int n, vio_ba_batch** out);
int vio_ba_batch_run(vio_ba_batch* b);          /* async on the context stream */
int vio_ba_batch_sync(vio_ba_batch* b);
/* replace the IMU preintegrations of a VIO_BA_VI batch before the next run: src holds the batch's
   total keyframe count of entries, window after window in creation order (entry k of a window links
   keyframe k-1 -> k; entry 0 unused), from host (on_device = 0) or device memory (on_device = 1,
   e.g. the output of vio_imu_preintegrate_device).  The validity pattern given at creation stays
   in force.  Async on the context stream. */
int vio_ba_batch_set_preint(vio_ba_batch* b, const vio_preint* src, int count, int on_device);
int vio_ba_batch_download(vio_ba_batch* b, vio_ba_output* outs);
/* average device time (ms) of the solver kernel over the runs since the last reset */
int vio_ba_batch_kernel_ms(vio_ba_batch* b, double* avg_ms, int* count);
/* the route the batch's LocalBA / BA / VIBA windows run on (VIO_BA_ROUTE_PHASES / _SINGLE_KERNEL /
   _CLUSTER; fixed at vio_ba_batch_create), and for the cluster route the workgroups per window */
int vio_ba_batch_route(vio_ba_batch* b, int* route, int* workgroups_per_window);
void vio_ba_batch_destroy(vio_ba_batch* b);
/* diagnostics: per-phase shader-clock accounting of the solver kernel (sum over windows of the
   last run; VIO_BA_PROF_SLOTS slots, named in the Python mirror's BaBatch.PHASES) */
int vio_ba_batch_profile(vio_ba_batch* b, int enable);
#define VIO_BA_PROF_SLOTS 32
int vio_ba_batch_phase_cycles(vio_ba_batch* b, unsigned long long* out /* [VIO_BA_PROF_SLOTS] */);

/*
 * Packed per-window result records, for gathering the windows of a sharded batch over RCCL
 * (config 4: 256 windows over 8 GPUs, one ncclAllGather of the records).  A record is
 * self-describing and position-independent: {int32 K, L, N, version; int32 summary[8] (success,
 * termination, iterations, successful, unsuccessful, inliers, outliers, bad MPs); f64 summary[4]
 * (initial, final, fixed cost, 0); f64 T_wb[12K] (R row-major | t); f64 lm_xyz[3L]; f64 vel[3K];
 * f64 bias[6] (bg | ba); u8 obs_outlier[N] in the caller's observation order; u8 lm_bad[L]}, padded
 * to a multiple of 16 bytes.  Every record of a batch takes vio_ba_batch_record_bytes (the largest).
 */
#define VIO_BA_RECORD_VERSION 1
size_t vio_ba_record_bytes(int num_kf, int num_lm, int num_obs);
int vio_ba_batch_record_bytes(vio_ba_batch* b, size_t* bytes);
/* the batch's n records back to back into dst (on_device != 0: a device buffer of this context's
   device, written asynchronously on the context stream by a pack kernel; else host memory, blocking) */
int vio_ba_batch_pack(vio_ba_batch* b, void* dst, int on_device);
/* decode one record (host memory, record_bytes readable bytes) into caller-owned outputs (NULL fields
   skipped; obs_chi2 and trace are not carried: left untouched).  Records arrive from other ranks:
   VIO_EINVAL when the header is malformed or its K/L/N layout does not fit in record_bytes. */
int vio_ba_record_unpack(const void* record, size_t record_bytes, vio_ba_output* out);

/*
 * Problem assembly and write-back of the Optimizer entry points (SURVEY §8 a3 host half / a4) on a
 * flat view of the reference's Frame / Feature / MapPoint graph.  Host-only, no device work.
 *
 * The view holds the frames vector handed to RunBA / RunVIBA / RunLocalBA (window order; for
 * SolvePnP the one frame) and the MapPoints their features reference:
 *   frame f's features are [feat_begin[f], feat_begin[f+1]) in Frame::GetFeatures() order; feature
 *   g has GetPixelCoord() = feat_uv[2g..2g+1], IsValid() = feat_valid[g] (a null Feature: 0) and
 *   GetMapPoint() = feat_mp[g] (an index into the MapPoint table, -1 for none);
 *   MapPoint m has IsBad() = mp_bad[m], IsMarginalized() = mp_marg[m], GetPosition() = mp_pos[3m..];
 *   mp_key[m] orders the MapPoints as the reference's std::set<shared_ptr<MapPoint>> does (pointer
 *   order there, any unique key here, e.g. the MapPoint id); RunLocalBA also walks
 *   MapPoint::GetObservations(): entries [mp_obs_begin[m], mp_obs_begin[m+1]) with the observing
 *   frame's slot in this view (-1: expired weak_ptr or a frame outside the window) and the
 *   feature index inside that frame.
 * IsNearBoundary (Optimizer.cpp:41-46 -> Camera.cpp:134-139): margin > 0 and x < margin or
 * x > width - margin or y < margin or y > height - margin, in f32.
 */
typedef struct {
    int32_t num_frames;
    int32_t num_mappoints;
    const float* frame_Twb;      /* 16 per frame: Frame::GetTwb(), row-major 4x4 */
    const float* frame_Tcb;      /* 16 per frame: Frame::GetTCB(), row-major 4x4 */
    const int32_t* feat_begin;   /* num_frames + 1 */
    const float* feat_uv;
    const uint8_t* feat_valid;
    const int32_t* feat_mp;
    const int64_t* mp_key;
    const uint8_t* mp_bad;
    const uint8_t* mp_marg;
    const float* mp_pos;
    const int32_t* mp_obs_begin; /* num_mappoints + 1 (RunLocalBA only, else may be NULL) */
    const int32_t* mp_obs_frame;
    const int32_t* mp_obs_feat;
    int32_t width, height;       /* Camera / Frame size (CameraParameters cols, rows) */
    int32_t boundary_margin;     /* Optimizer::m_boundary_margin (20, Optimizer.cpp:33) */
    int32_t _pad;
} vio_map_view;

/* vio_ba_gather status (> 0: the reference returns its default, unsuccessful result) */
enum {
    VIO_GATHER_OK = 0,
    VIO_GATHER_FEW_FRAMES = 1,   /* frames.size() < 2 (Optimizer.cpp:307-310, 497-500, 729-732) */
    VIO_GATHER_NO_MAPPOINTS = 2, /* mappoints.empty() (:328-331, 519-522, 757-760) */
    VIO_GATHER_FEW_OBS = 3       /* SolvePnP: observations.size() < 6 (:127-130) */
};

/* The assembled problem, caller-owned arrays.  Capacities: landmarks <= num_mappoints; observations
   <= feat_begin[num_frames] (RunBA / RunVIBA / SolvePnP) or mp_obs_begin[num_mappoints] (RunLocalBA). */
typedef struct {
    int32_t status;              /* VIO_GATHER_* */
    int32_t num_lm, num_obs;
    int32_t cap_lm, cap_obs;     /* in */
    int32_t _pad;
    int32_t* lm_mp;              /* cap_lm: landmark -> MapPoint index, std::set order */
    uint8_t* lm_const;           /* cap_lm: SetParameterBlockConstant (RunLocalBA: marginalised) */
    uint8_t* lm_marg;            /* cap_lm: marginalised (exempt from SetBad / PnP outliers) */
    double* lm_xyz;              /* 3 cap_lm: GetPosition() cast to f64 */
    int32_t* obs_kf;             /* cap_obs: frame slot */
    int32_t* obs_lm;             /* cap_obs */
    float* obs_uv;               /* 2 cap_obs */
    int32_t* obs_feat;           /* cap_obs: global feature index g (AddResidualBlock order) */
    uint8_t* kf_const;           /* num_frames */
    uint8_t* kf_in_problem;      /* num_frames: the pose block has a residual (poses_in_problem, :848-852) */
    vio_pose* T_wb_init;         /* num_frames (may be NULL): GetTwb().cast<double>() */
    vio_pose* T_cb;              /* num_frames (may be NULL): GetTCB().cast<double>() */
} vio_ba_gather_out;

/* MapPoint / frame collection + residual-block filters of one entry point (variant VIO_BA_LOCAL:
   Optimizer.cpp:726-851; VIO_BA_FULL: :303-409 with fix_first / fix_last; VIO_BA_VI: :493-636
   (fix_first; the IMU factors, velocities and biases are the caller's direct copies); VIO_PNP:
   :83-130, frame 0 only, every MapPoint constant).  Fills `out` and returns VIO_OK (check
   out->status) or VIO_EINVAL. */
int vio_ba_gather(const vio_map_view* map, int variant, int fix_first, int fix_last, vio_ba_gather_out* out);

/* What the entry point writes back into the graph after the solve (caller-owned arrays; NULL
   skipped).  Frames: SetTwb(T.matrix().cast<float>()) where frame_set; VIO_BA_VI: SetVelocity for
   every frame, SetGyroBias / SetAccelBias (bias = gyro | accel) for every frame.  MapPoints:
   SetBad() where mp_set_bad, SetPosition() where mp_set.  result: BAResult / PnPResult fields. */
typedef struct {
    float* frame_Twb;            /* 16 per frame, row-major */
    uint8_t* frame_set;          /* num_frames */
    float* frame_vel;            /* 3 per frame */
    float* bias;                 /* 6 */
    float* mp_pos;               /* 3 per MapPoint */
    uint8_t* mp_set;             /* num_mappoints */
    uint8_t* mp_set_bad;         /* num_mappoints */
    int32_t success, num_inliers, num_outliers, num_poses_optimized, num_points_optimized, num_iterations;
    double initial_cost, final_cost;
} vio_ba_map_update;

/* Write-back rules (RunBA :459-474, RunVIBA :684-712, RunLocalBA :917-954, SolvePnP :272-297): `g`
   is the gather of the same view and variant, `res` the solver's output for the problem built from
   it (T_wb, lm_xyz, lm_bad, summary; vel/bg/ba for VIO_BA_VI).  A gather with status > 0 writes
   nothing and gives the reference's default result. */
int vio_ba_write_back(const vio_map_view* map, int variant, const vio_ba_gather_out* g, const vio_ba_output* res,
                      vio_ba_map_update* upd);

/* ----------------------------------------------------------------------------------------- */
/* ERP feature tracking                                                                       */

typedef struct {
    int32_t win;              /* LK window (21, FeatureTracker.cpp:33) */
    int32_t max_level;        /* 3 */
    int32_t max_iters;        /* 30 */
    float epsilon;            /* 0.01 (criteria.epsilon; squared internally) */
    float min_eig_threshold;  /* 0.01 (the reference passes epsilon here, :240) */
    int32_t _pad;
} erp_klt_params;

/* prev/curr: u8 W x H, row stride `stride` bytes, host memory.  Returns next/status/err. */
int erp_klt_track(vio_ctx* ctx, const uint8_t* prev, const uint8_t* curr, int W, int H, int stride,
                  const float* pts, int n, float* next, uint8_t* status, float* err,
                  const erp_klt_params* params);

/* goodFeaturesToTrack(img, max_corners, quality, min_dist, mask, blockSize 3, useHarris false).
   mask may be NULL.  out_xy holds up to max_corners float2, *n_out the count. */
int erp_gftt(vio_ctx* ctx, const uint8_t* img, const uint8_t* mask, int W, int H, int stride,
             int max_corners, double quality, double min_dist, float* out_xy, int* n_out);

/* rotation-only RANSAC on ERP bearings with an injected sample stream (iters*3 indices, each
   triple distinct, as FeatureTracker.cpp:280-288 draws them).  mask[n] = best hypothesis' inliers
   (all ones when no hypothesis has an inlier), *n_in = its inlier count. */
int erp_rot_ransac(vio_ctx* ctx, const float* p0, const float* p1, int n, int W, int H,
                   const int32_t* samples, int iters, float thresh_rad, uint8_t* mask, int* n_in);

/* the reference's RANSAC sample stream made deterministic: std::mt19937(seed) +
   std::uniform_int_distribution<>(0, n-1), three distinct indices per iteration
   (FeatureTracker.cpp:273-288; the reference seeds from std::random_device).  Host-only helper. */
int erp_ransac_samples(uint32_t seed, int n, int iters, int32_t* out);

/* ------------------------------------------------------------------------------------------ */
/* Device-resident frame pipeline = the numeric part of FeatureTracker::TrackFeatures
   (FeatureTracker.cpp:61-206) for one frame pair, all on the GPU with no host round trip:
     pyramids of both frames -> pyramidal LK of the previous frame's points -> status / polar /
     boundary filter (:117-126) -> rotation RANSAC on the survivors with the in-pipeline sample
     stream of erp_ransac_samples(ransac_seed, n_good, ransac_iters) (:130-134) -> GFTT
     re-detection on the current frame masked by polar ∧ boundary ∧ discs of radius
     (int)min_dist around the kept points (CreateFeatureMask :386-402, DetectNewFeatures :208-226).
   The host-side feature bookkeeping between those steps in the reference (RemoveClusteredFeatures,
   Frame::LimitFeaturesPerGrid, feature ids) is the adapter's job; the in-pipeline
   disc mask is built from every kept point. */
typedef struct erp_tracker erp_tracker;
int erp_tracker_create(vio_ctx* ctx, int W, int H, int max_points, int max_corners, erp_tracker** out);
/* copy a host frame into slot 0 (prev) or 1 (curr); erp_tracker_device_frame gives the device
   buffer of a slot (pitch *pitch bytes) for producers that write frames on the device */
int erp_tracker_upload(erp_tracker* t, int slot, const uint8_t* img, int stride);
int erp_tracker_device_frame(erp_tracker* t, int slot, uint8_t** dev_ptr, int* pitch);
/* the demo's frame path (app/main.cpp:199-204): upload a W x H u8 camera frame and resize it on the
   device with INTER_AREA (erp_resize_area) into slot's tracker resolution; integer factors only
   (VIO_ENOSYS otherwise), a frame already at tracker resolution is uploaded as is */
int erp_tracker_upload_resized(erp_tracker* t, int slot, const uint8_t* img, int W, int H, int stride);
/* swap slots 0 and 1 (the current frame becomes the previous one, m_prev_image = current) */
int erp_tracker_swap(erp_tracker* t);
typedef struct {
    int32_t ransac_iters;     /* 1000 (FeatureTracker.cpp:36) */
    float ransac_thresh_rad;  /* 2 deg (:37, 2.0f * M_PI / 180.0f) */
    uint32_t ransac_seed;     /* seed of the in-pipeline mt19937 sample stream */
    int32_t max_corners;      /* goodFeaturesToTrack maxCorners (feature_detection.max_features) */
    double quality;           /* qualityLevel (0.01) */
    double min_dist;          /* minDistance (30); disc radius (int)min_dist */
    int32_t boundary_margin;  /* camera.boundary_margin (20) */
    float polar_ratio;        /* 0.15 (Camera::CreatePolarMask / IsInPolarRegion default) */
} erp_tracker_params;
/* previous-frame points (pixel coordinates) to track */
int erp_tracker_set_points(erp_tracker* t, const float* pts, int n);
/* enqueue the whole pipeline on the context stream (asynchronous) */
int erp_tracker_run(erp_tracker* t, const erp_klt_params* klt, const erp_tracker_params* p);
int erp_tracker_sync(erp_tracker* t);
/* results of the last run: per input point next position, LK status and kept flag
   (status ∧ !polar ∧ !boundary ∧ RANSAC inlier); the new corners (≤ max_corners float2) */
int erp_tracker_download(erp_tracker* t, float* next, uint8_t* status, uint8_t* kept, float* corners,
                         int* n_corners);
/* device time (ms) of the pipeline stages of the last run (the stage values are -1 when the run did not
   record its stage events, see erp_tracker_set_stage_timing; total_ms is always measured) */
int erp_tracker_stage_ms(erp_tracker* t, double* pyr_ms, double* lk_ms, double* ransac_ms, double* gftt_ms,
                         double* total_ms);
/* on (default): runs record the per-stage events; off: only the pipeline's start and end (each event
   marker costs the stream a few microseconds) */
int erp_tracker_set_stage_timing(erp_tracker* t, int on);
/* GFTT fallbacks taken by erp_tracker_download since the tracker was created: exact_tail = runs whose greedy
   pass over the presorted local maxima could not decide (the masked-maximum tail ran after the download's
   sync), full_sort = runs whose top-K candidate prefix could not decide (every candidate sorted) */
int erp_tracker_gftt_fallbacks(erp_tracker* t, int* exact_tail, int* full_sort);
void erp_tracker_destroy(erp_tracker* t);

/* ------------------------------------------------------------------------------------------ */
/* FeatureTracker::TrackFeatures as a whole (src/processing/FeatureTracker.cpp:61-206): the device
   numeric path above plus the reference's host bookkeeping — feature ids (survivors keep theirs,
   new detections take m_next_feature_id++ in GFTT order), track counts / ages,
   RemoveClusteredFeatures (:404-497, gated by visualization.highlight_clustered_grid),
   Frame::AssignFeaturesToGrid / LimitFeaturesPerGrid (src/database/Frame.cpp:108-202, std::sort by
   track count) and CreateFeatureMask discs (:386-402).  One object per camera stream. */
typedef struct erp_frontend erp_frontend;
typedef struct {
    int32_t max_features;         /* feature_detection.max_features (1000) */
    float min_distance;           /* feature_detection.min_distance (30) */
    float quality_level;          /* feature_detection.quality_level (0.01) */
    int32_t boundary_margin;      /* camera.boundary_margin (20) */
    int32_t grid_cols, grid_rows; /* Frame grid: feature_detection.grid_cols/rows (20, 10) */
    int32_t max_features_per_grid;/* feature_detection.max_features_per_grid (10) */
    int32_t remove_clustered;     /* visualization.highlight_clustered_grid (1) */
    float clustered_std_ratio;    /* visualization.clustered_std_ratio (0.25 in the yaml) */
    uint32_t ransac_seed;         /* frame f uses erp_ransac_samples(ransac_seed + f, ...) */
} erp_frontend_params;
int erp_frontend_create(vio_ctx* ctx, int W, int H, const erp_frontend_params* p, erp_frontend** out);
/* process the next frame (u8 W x H); *n_features = features of this frame after the call */
int erp_frontend_track(erp_frontend* f, const uint8_t* img, int stride, int* n_features);
/* current frame's features in Frame order: id, pixel, track count, age (any pointer may be NULL) */
int erp_frontend_features(erp_frontend* f, int32_t* ids, float* xy, int32_t* track_count, int32_t* age, int cap);
/* GetTrackingStats (FeatureTracker.h): features after tracking, new detections of the last frame */
int erp_frontend_stats(erp_frontend* f, int* num_tracked, int* num_detected);
void erp_frontend_destroy(erp_frontend* f);

/* ------------------------------------------------------------------------------------------ */
/* IMU preintegration: the producer of vio_preint, on device.                   */

/* IMUData (src/processing/Estimator.h:32-36) */
typedef struct {
    double timestamp;         /* seconds */
    float ax, ay, az;         /* m/s^2 */
    float gx, gy, gz;         /* rad/s */
} vio_imu_data;

/* IMUPreintegrator noise densities (IMUPreintegrator.cpp:64-67 defaults 1e-4, 1e-3, 1e-6, 1e-5;
   SetNoiseParameters :131-140) */
typedef struct {
    float gyro_noise, accel_noise, gyro_bias_noise, accel_bias_noise;
} vio_imu_noise;

/*
 * IMUPreintegrator::Preintegrate (src/processing/IMUPreintegrator.cpp:143-193, with
 * IntegrateMeasurement :195-236 and UpdateCovariance :238-274) for n intervals in one launch:
 * interval i integrates the samples with t_start[i] <= timestamp < t_end[i] under the biases
 * gyro_bias[3i..], accel_bias[3i..] (the preintegrator's m_gyro_bias / m_accel_bias; NULL = 0).
 * imu[] must be sorted by non-decreasing timestamp (VIO_EINVAL otherwise).  valid[i] = 0 where
 * the reference returns nullptr (no sample in range; out[i] is then zeroed).  cov_bias_diag
 * (n*6, may be NULL) receives covariance(9..14, 9..14)'s diagonal, the random-walk block.
 * noise NULL = the reference defaults.  Blocking; out / valid / cov_bias_diag are host buffers.
 */
int vio_imu_preintegrate(vio_ctx* ctx, const vio_imu_data* imu, int n_imu, const double* t_start,
                         const double* t_end, int n, const float* gyro_bias, const float* accel_bias,
                         const vio_imu_noise* noise, vio_preint* out, uint8_t* valid, float* cov_bias_diag);
/* the same on DEVICE buffers (imu, t_start, t_end, biases, out, valid, cov_bias_diag — the last is
   required here), asynchronous on the context stream; imu must be sorted (not checked) */
int vio_imu_preintegrate_device(vio_ctx* ctx, const vio_imu_data* imu, int n_imu, const double* t_start,
                                const double* t_end, int n, const float* gyro_bias, const float* accel_bias,
                                const vio_imu_noise* noise, vio_preint* out, uint8_t* valid, float* cov_bias_diag);
/* device time (ms) of the last vio_imu_preintegrate[_device] kernel on this context (waits for it) */
int vio_imu_preintegrate_kernel_ms(vio_ctx* ctx, double* ms);

/* ------------------------------------------------------------------------------------------ */
/* IMU initialisation: Optimizer::OptimizeIMUInit (src/optimization/            */
/* Optimizer.cpp:972-1257) — stage 1 gravity direction (2) + scale, stage 2 velocities + shared */
/* biases with BiasPriorFactor (Factors.h:366-396), both over InertialGravityScaleFactor        */
/* (Factors.cpp:981-1293) with HuberLoss(sqrt(16)), DENSE_QR, default Solver::Options.          */
/* Reproduced quirks: the pose blocks are constant zero perturbations in both stages and the    */
/* factor applies SE3d::exp to them without the keyframe poses, so every factor sees identity  */
/* poses (Factors.cpp:1024-1042, Optimizer.cpp:1084-1092); the factor's square-root            */
/* information is built but never applied to the residual.  One workgroup per problem.          */

enum {
    VIO_IMU_INIT_OK = 0,
    VIO_IMU_INIT_FEW_FRAMES = 1,   /* frames.size() < 3 (:977-981) */
    VIO_IMU_INIT_NO_PREINT = 2,    /* a frame after the first lacks its preintegration (:984-989) */
    VIO_IMU_INIT_NO_FACTORS = 3    /* stage 1 kept no factor (0.001 <= dt <= 2.0, :1060-1086) */
};

typedef struct {
    int32_t num_frames;          /* keyframes, 3 .. 64 */
    int32_t max_iterations;      /* per stage: 50 (Solver::Options default) */
    const vio_pose* T_wb;        /* num_frames: GetTwb().cast<double>() (velocity initialisation) */
    const vio_preint* preint;    /* num_frames: entry i = frame i's preintegration from the last keyframe */
    const uint8_t* preint_valid; /* num_frames (entry 0 ignored) */
    double gravity_magnitude;    /* 9.81 */
    double huber_delta;          /* sqrt(16) = 4 */
    double bias_prior_weight;    /* 1.0 */
} vio_imu_init_problem;

typedef struct {
    int32_t success;             /* IMUInitResult::success */
    int32_t status;              /* VIO_IMU_INIT_* */
    int32_t iterations[2];       /* Summary::iterations.size() of stage 1 / 2 */
    int32_t termination[2];      /* VIO_TERM_* of stage 1 / 2 */
    double gravity[3];           /* R_wg (0, 0, -9.81) */
    double Rwg[9];               /* row-major */
    double gravity_dir[2];       /* the stage-1 parameters (theta_x, theta_y) */
    double scale;
    double gyro_bias[3], accel_bias[3];
    double initial_cost;         /* stage 1 Summary::initial_cost */
    double final_cost;           /* stage 2 Summary::final_cost */
    double* velocities;          /* caller-owned 3 * num_frames, may be NULL */
} vio_imu_init_result;

int vio_imu_init_solve(vio_ctx* ctx, const vio_imu_init_problem* probs, vio_imu_init_result* results, int n);

/* ------------------------------------------------------------------------------------------ */
/* Two-view triangulation: Estimator::TriangulateSinglePoint                   */
/* (src/processing/Estimator.cpp:1082-1137) for n candidates in one launch.                   */

/*
 * T_cw: n_poses world-to-camera transforms, 4x4 row-major f32 (the reference's
 * kf->GetTwc().inverse(), Estimator.cpp:1163-1164).  Candidate i triangulates bearings
 * bearings[6i..6i+2] (in camera pose_pair[2i]) and bearings[6i+3..6i+5] (in camera pose_pair[2i+1])
 * (Feature::GetBearing, unit f32).  points: 3n f32; valid[i] = TriangulateSinglePoint's return
 * (|v(3)| >= 1e-10 and a finite point); pixel_err (2n, may be NULL) = the reprojection angle errors
 * in pixels TriangulateNewMapPoints computes (:1233-1248) with `width` = GetWidth().  Blocking; host
 * buffers.  The 4x4 SVD is an f64 one-sided Jacobi on the f32-built A (reference: Eigen's f32
 * JacobiSVD; the null vector is unique up to sign, which the division cancels).
 */
int vio_triangulate(vio_ctx* ctx, const float* T_cw, int n_poses, const int32_t* pose_pair, const float* bearings,
                    int n, int width, float* points, uint8_t* valid, float* pixel_err);
/* the same on DEVICE buffers, asynchronous on the context stream (no validation of pose_pair) */
int vio_triangulate_device(vio_ctx* ctx, const float* T_cw, int n_poses, const int32_t* pose_pair,
                           const float* bearings, int n, int width, float* points, uint8_t* valid,
                           float* pixel_err);
/* device time (ms) of the last triangulation kernel on this context (waits for it) */
int vio_triangulate_kernel_ms(vio_ctx* ctx, double* ms);

/* ------------------------------------------------------------------------------------------ */
/* Dataset formats and frame preprocessing, app/main.cpp:30-119, 199-204.        */

/* LoadCameraTimestamps (app/main.cpp:30-48): one double per line.  Writes min(cap, count) values,
   *n = count (call with cap = 0 to size the buffer).  VIO_EINVAL if the file cannot be opened. */
int vio_load_camera_timestamps(const char* path, double* out, int cap, int* n);
/* LoadIMUData (app/main.cpp:50-90): header line, then "t,ax,ay,az,gx,gy,gz" rows; malformed rows
   are skipped exactly as the reference skips them.  Same sizing convention. */
int vio_load_imu_csv(const char* path, vio_imu_data* out, int cap, int* n);

/* cv::resize(img, img, Size(dW, dH), 0, 0, INTER_AREA) of a u8 grayscale frame (app/main.cpp:203),
   integer downscale factors only (W % dW == 0, H % dH == 0; else VIO_ENOSYS).  Blocking; host buffers. */
int erp_resize_area(vio_ctx* ctx, const uint8_t* src, int W, int H, int stride, uint8_t* dst, int dW, int dH,
                    int dst_stride);
/* the same for n_frames DEVICE frames (frame f at src + f*stride*H, dst + f*dst_stride*dH), async on
   the context stream */
int erp_resize_area_device(vio_ctx* ctx, const uint8_t* src, int W, int H, int stride, int n_frames, uint8_t* dst,
                           int dW, int dH, int dst_stride);
/* device time (ms) of the last resize kernel on this context (waits for it) */
int erp_resize_area_kernel_ms(vio_ctx* ctx, double* ms);


/* ------------------------------------------------------------------------------------------ */
/* Monocular initialisation: Initializer::TryMonocularInitialization           */
/* (src/processing/Initializer.cpp:47-291) — essential-matrix RANSAC (:458-621), pose recovery */
/* (:623-697, :785-835), mid-point triangulation (:699-783), validation (:889-995), scale      */
/* normalisation (:997-1048).  Config: initialization.* (config/default_config.yaml:33-41).    */

typedef struct {
    int32_t width, height;          /* m_camera_width / m_camera_height (reprojection pixels) */
    int32_t min_features;           /* initialization.min_features (100) */
    int32_t ransac_iterations;      /* initialization.ransac_iterations (200) */
    float ransac_threshold;         /* initialization.ransac_threshold (0.1) on |b2^T E b1| */
    float max_reprojection_error;   /* initialization.max_reprojection_error (5.0 px) */
} vio_mono_init_params;

/* status: where TryMonocularInitialization returned false (0 = success) */
#define VIO_INIT_OK 0
#define VIO_INIT_TOO_FEW_BEARINGS 1   /* fewer than 5 bearing pairs (:117-120) */
#define VIO_INIT_ESSENTIAL_FAILED 2   /* best RANSAC inlier count < min_features (:579-581) */
#define VIO_INIT_POSE_FAILED 3        /* no cheirality candidate with >= min_features good points (:688-690) */
#define VIO_INIT_TRIANGULATION 4      /* triangulated points < min_features (:151-154) */
#define VIO_INIT_VALIDATION 5         /* validated points < min_features, or none (:962-992) */

typedef struct {
    int32_t status;                 /* VIO_INIT_* */
    int32_t best_hypothesis;        /* first RANSAC iteration with the (strictly) largest inlier count */
    int32_t num_inliers;            /* its inlier count */
    int32_t pose_candidate;         /* chosen (R, t) candidate 0..3 (:659-663) */
    int32_t candidate_good[4];      /* TestPoseCandidate good-point counts */
    int32_t num_triangulated;       /* TriangulatePoints successes */
    int32_t num_valid;              /* ValidateInitialization valid_count */
    float mean_reproj_error;        /* ValidateInitialization mean_error (px) */
    float scale_factor;             /* NormalizeScale: 1 / median distance */
    float E[9];                     /* refined essential matrix, row-major */
    float R[9];                     /* R_c2c1 (frame 1 -> frame 2), row-major */
    float t[3];                     /* t_c2c1 after scale normalisation */
} vio_mono_init_result;

/*
 * bearings1/2: n unit bearings (Feature::GetBearing, f32 xyz) of the selected features in the
 * first / last frame of the window; samples: ransac_iterations x 8 indices (the reference draws
 * them from mt19937 seeded by std::random_device, :477-494 — inject vio_mono_init_samples).
 * Outputs (host, caller-owned): res; inlier_mask (n, may be NULL) = the best hypothesis' inliers;
 * points (3n f32, may be NULL) = the scaled mid-point triangulations in camera-1 coordinates
 * (zero where triangulation failed), before the T_BC transform of :220-224.  1 <= n <= 4096.
 * The 8x9 / nx9 null vectors and the 3x3 SVDs are f64 Jacobi on the f32-built systems (reference:
 * Eigen f32 JacobiSVD); per-point arithmetic is the reference's f32.  Blocking.
 */
int vio_mono_init_solve(vio_ctx* ctx, const float* bearings1, const float* bearings2, int n, const int32_t* samples,
                        const vio_mono_init_params* params, vio_mono_init_result* res, uint8_t* inlier_mask,
                        float* points);
/* device time (ms) of the last vio_mono_init_solve's kernels on this context (waits for them) */
int vio_mono_init_kernel_ms(vio_ctx* ctx, double* ms);
/* the reference's RANSAC sample stream with an injected seed: iters x 8 distinct indices drawn by
   std::mt19937(seed) + std::uniform_int_distribution<>(0, n-1) with duplicate rejection (:477-494) */
int vio_mono_init_samples(uint32_t seed, int n, int iters, int32_t* out);

/* Host helpers of the same path (no device work). */
/* Initializer::SelectFeaturesForInit (:351-433) on a flat view of the last frame's features:
   uv (n x 2 pixel coords), obs_count (n, Feature::GetObservationCount).  Writes the selected
   feature indices in the reference's order to out_idx (capacity n), *n_out = count (0 when fewer
   than min_features candidates have >= min_observations observations). */
int vio_init_select_features(const float* uv, const int32_t* obs_count, int n, int width, int height, int grid_cols,
                             int grid_rows, int min_observations, int min_features, int32_t* out_idx, int* n_out);
/* Initializer::ComputeParallax (:293-349): median pixel displacement of features matched by id
   (first match in frame 2 for each frame-1 feature); 0 when nothing matches. */
int vio_init_parallax(const int32_t* ids1, const float* uv1, int n1, const int32_t* ids2, const float* uv2, int n2,
                      float* parallax);
/* Frame poses of :184-204 from T_BC (4x4 row-major, camera-to-body) and the result's R, t:
   T_wb1 = I, T_wb2 = T_BC * T_c1c2^-1 * T_BC^-1 (f32); also maps points (3n, camera-1 frame) to
   the world frame in place (p <- R_BC p + t_BC, :217-224) when points != NULL. */
int vio_init_compose(const float* T_BC, const float* R, const float* t, float* T_wb1, float* T_wb2, float* points,
                     int n);


/* ------------------------------------------------------------------------------------------ */
/* Estimator sliding-window bookkeeping on a host-side keyframe / MapPoint graph:  */
/* Estimator::CreateKeyframe's observation update and window slide (src/processing/Estimator.cpp: */
/* 671-754: reference-keyframe transfer, marginalisation, SetBad, RemoveObservation),             */
/* LinkMapPointsFromPreviousFrame (:806-843) and TriangulateNewMapPoints (:1141-1318, the          */
/* triangulation itself on device through vio_triangulate).  MapPoints are handles 0, 1, ... in   */
/* creation order; frames are identified by Frame::GetFrameId().  Not thread-safe.                */

typedef struct vio_window vio_window;

/* a keyframe handed to vio_window_add_keyframe (copied; the caller keeps its buffers) */
typedef struct {
    int32_t frame_id;
    int32_t num_features;
    int32_t width;               /* Frame::GetWidth (pixel error scale of the triangulation check) */
    int32_t _pad;
    const float* T_wb;           /* 16, row-major: Frame::GetTwb() */
    const float* T_bc;           /* 16, row-major: Frame::GetTBC() (camera-to-body) */
    const int32_t* feature_id;   /* n: Feature::GetFeatureId() */
    const float* uv;             /* 2n: GetPixelCoord() (carried for the BA map view) */
    const float* bearing;        /* 3n: GetBearing() */
    const uint8_t* valid;        /* n: IsValid() */
    const int32_t* mappoint;     /* n: GetMapPoint() handle (-1: none), e.g. from vio_window_link_mappoints */
    /* Feature::GetObservations() of each feature (its track): CSR, entries (frame id, feature index);
       may be NULL (no track history) */
    const int32_t* track_begin;  /* n + 1 */
    const int32_t* track_frame;
    const int32_t* track_feat;
} vio_window_frame;

typedef struct {
    int32_t obs_added;           /* observations the new keyframe added (:679-690) */
    int32_t transferred;         /* reference-keyframe transfers (marginalised MapPoints, :720-725) */
    int32_t deleted;             /* referenced MapPoints no other keyframe observes, set bad (:726-729);
                                    MapPoints left without observations (:747-749) also turn bad */
    int32_t removed_frame;       /* frame id of the keyframe slid out (-1: none) */
    int32_t num_keyframes;       /* window size after the call */
    int32_t _pad;
} vio_window_kf_stats;

typedef struct {
    float pos[3];
    int32_t bad, marginalized, triangulated;
    int32_t reference_frame;     /* reference keyframe id, -1 none */
    int32_t num_observations;
} vio_window_mappoint_info;

int vio_window_create(int max_keyframes, vio_window** out);   /* max_keyframes: 10 (:693) */
void vio_window_destroy(vio_window* win);
/* new MapPoint at pos (e.g. Initializer::CreateMapPoints); reference_frame -1 for none */
int vio_window_add_mappoint(vio_window* win, const float* pos, int32_t reference_frame, int32_t* handle);
/* MapPoint::AddObservation(frame, feat) + Frame::SetMapPoint(feat, mp) for a keyframe of the store */
int vio_window_add_observation(vio_window* win, int32_t mp, int32_t frame_id, int32_t feat);
/* LinkMapPointsFromPreviousFrame: curr_mp[i] = the previous frame's (valid, last-by-id) feature's
   MapPoint if it exists and is not bad, else -1 */
int vio_window_link_mappoints(const vio_window* win, const int32_t* prev_id, const uint8_t* prev_valid,
                              const int32_t* prev_mp, int n_prev, const int32_t* curr_id, int n_curr, int32_t* curr_mp);
/* CreateKeyframe: append the keyframe, add its MapPoint observations, slide the window */
int vio_window_add_keyframe(vio_window* win, const vio_window_frame* frame, vio_window_kf_stats* stats);
/* TriangulateNewMapPoints(kf1, kf2) in two host halves around the device triangulation:
   candidates: matched (kf1 index, kf2 index) pairs in kf2 order, their bearings (6 per pair) and the
   two world-to-camera transforms GetTwc().inverse() (T_cw, 32 floats) -> vio_triangulate;
   commit: creates a MapPoint per valid triangulation (reference kf1, observations kf1, kf2 and the
   in-window keyframes of kf2's feature track) and returns the handles in new_mp (-1 where invalid).
   vio_window_triangulate does both with the device in between; *n_new = new MapPoints. */
int vio_window_triangulation_candidates(const vio_window* win, int32_t kf1_id, int32_t kf2_id, int32_t* pairs,
                                        float* bearings, float* T_cw, int cap, int* n);
int vio_window_commit_triangulation(vio_window* win, int32_t kf1_id, int32_t kf2_id, const int32_t* pairs,
                                    const float* points, const uint8_t* valid, int n, int32_t* new_mp, int* n_new);
int vio_window_triangulate(vio_window* win, vio_ctx* ctx, int32_t kf1_id, int32_t kf2_id, int* n_new);
/* queries */
int vio_window_keyframes(const vio_window* win, int32_t* frame_ids, int cap, int* n);   /* oldest first */
int vio_window_num_mappoints(const vio_window* win);
int vio_window_mappoint(const vio_window* win, int32_t mp, vio_window_mappoint_info* info);
/* MapPoint::GetObservations() in order: (frame id, feature index) pairs */
int vio_window_mappoint_observations(const vio_window* win, int32_t mp, int32_t* frame_ids, int32_t* feats, int cap,
                                     int* n);
int vio_window_frame_mappoints(const vio_window* win, int32_t frame_id, int32_t* mp, int cap, int* n);
/* BA over the window: a vio_map_view of the window's keyframes (oldest first) and every MapPoint
   (arrays owned by the window, valid until its next mutating call), for vio_ba_gather /
   vio_ba_write_back; then the write-back applied to the window (frame poses, MapPoint positions,
   SetBad) */
int vio_window_map_view(vio_window* win, int height, int boundary_margin, vio_map_view* view);
int vio_window_apply_update(vio_window* win, const vio_ba_map_update* upd);

#ifdef __cplusplus
}
#endif
#endif /* VIO360_H_ */
