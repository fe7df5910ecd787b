/*
 * acinoset_hip.h — C ABI of the MI355X-native AcinoSet SBA/FTE core
 * (libacinoset_hip.so, HIP kernels for gfx950).
 *
 * The reference has no FFI layer: its seams are Python call signatures. Every entry
 * point below replaces the numeric body of one of those seams (cited per function);
 * the Python drop-ins in acinoset_amd/lib and acinoset_amd/core bind them via ctypes
 * (INTEGRATION.md shows the binding a reference maintainer would add).
 *
 * Conventions
 *  - All functions return an int status: ACS_OK (0) or a negative ACS_E_* code; the
 *    message is in acs_last_error(ctx).
 *  - Array arguments are HOST pointers (copied into context-owned device buffers and
 *    back) unless ACS_DEVICE_PTRS is set in `flags`, in which case every array pointer
 *    of that call is a device pointer and the call is asynchronous on the context
 *    stream (results valid after acs_ctx_sync or a later synchronous call).
 *  - float64 everywhere (the reference is float64 throughout: src/lib/utils.py:68-71).
 *  - Camera block: ACS_CAM_STRIDE doubles per camera:
 *      [fx, fy, cx, cy, k1, k2, k3, k4, R00..R22 (row-major), t0, t1, t2]
 *    = K[0,0], K[1,1], K[0,2], K[1,2] of the scene JSON 'k', 'd' (4), 'r' (3x3), 't' (3)
 *    (src/lib/utils.py:55-74). Skew K[0,1] is ignored, as by cv::fisheye (alpha = 0).
 *  - One context = one HIP device + one stream; calls on a context are not thread-safe.
 */
#ifndef ACINOSET_HIP_H
#define ACINOSET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACS_ABI_VERSION 5
#define ACS_CAM_STRIDE 20

/* status codes */
#define ACS_OK 0
#define ACS_E_INVALID -1   /* bad argument / shape */
#define ACS_E_HIP -2       /* HIP runtime error */
#define ACS_E_NOMEM -3     /* device allocation failed */
#define ACS_E_NODEV -4     /* no usable gfx950 device */

/* flags */
#define ACS_DEVICE_PTRS 1u  /* array arguments are device pointers; call is async */

/* per-problem convergence status (acs_report.status_counts index / oracle/sba.py) */
/* acs_ekf_run / acs_sba_ekf_pipeline measurement-model mode (their ref_numerics argument) */
#define ACS_EKF_ANALYTIC_H 2

#define ACS_STATUS_RUNNING 0
#define ACS_STATUS_GTOL 1
#define ACS_STATUS_FTOL 2
#define ACS_STATUS_XTOL 3
#define ACS_STATUS_STALLED 4
#define ACS_STATUS_MAXITER 5
#define ACS_STATUS_NOOBS 6
#define ACS_N_STATUS 7

/* LM steps whose model decrease -g.dx - dx.H.dx/2 is <= ACS_COST_RES * cost are below the
 * resolution of a float64 cost sum: the problem stops as converged (ACS_STATUS_FTOL)
 * instead of letting rounding accept or reject the step (points-only SBA).              */
#define ACS_COST_RES 1e-14

typedef struct acs_ctx acs_ctx;

typedef struct {
  int32_t max_iters;  /* LM iterations (accepted + rejected) per problem; default 100 */
  int32_t reserved;
  double f_scale;     /* Cauchy soft-threshold in px; reference default 50 (src/lib/sba.py:181) */
  double ftol;        /* relative cost decrease; reference passes 1e-15 (src/lib/sba.py:189) */
  double xtol;        /* relative step; default 1e-9 (scipy default 1e-8) */
  double gtol;        /* max |gradient|; default 1e-10 */
} acs_sba_opts;

typedef struct {
  int64_t n_problems;                   /* points (SBA) or 1 (FTE) */
  int64_t status_counts[ACS_N_STATUS];  /* problems ending in each ACS_STATUS_* */
  int64_t iters_max;                    /* max LM iterations over problems */
  int64_t iters_sum;                    /* total LM iterations */
  int64_t nfev_sum;                     /* total cost evaluations */
  double cost_before;                   /* sum of robust cost at x0 */
  double cost_after;                    /* sum of robust cost at the solution */
} acs_report;

/* ---- context -------------------------------------------------------------------- */
int acs_ctx_create(int device, acs_ctx** out);
int acs_ctx_destroy(acs_ctx* ctx);
const char* acs_last_error(const acs_ctx* ctx);
int acs_ctx_set_stream(acs_ctx* ctx, void* hip_stream);  /* NULL = context's own stream */
int acs_ctx_sync(acs_ctx* ctx);
int acs_abi_version(void);
int acs_device_count(int* n);
/* Device and pinned-host allocations + frees the library has made in this process (a
 * counter; no GPU needed): a timed region that reuses its buffers leaves it unchanged. */
int64_t acs_alloc_events(void);
void acs_sba_default_opts(acs_sba_opts* o);

/* ---- a1: fisheye projection (src/lib/calib.py:132-136, src/core/fte.py:80-96) -------
 * uv[i] = project(cams[cam_idx[i]], pts[i]); cam_idx may be NULL (all camera 0).
 * fte_form != 0 uses the FTE restatement r = sqrt(a^2 + b^2 + 1e-12) (fte.py:88)
 * instead of OpenCV's r > 1e-8 guard.                                                 */
int acs_project_fisheye(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* pts,
                        const int32_t* cam_idx, int64_t n, int32_t fte_form, double* uv_out,
                        uint32_t flags);

/* ---- a2: SBA residual vector (cost_func_points_only, src/lib/sba.py:149-153) -------
 * resid[2i+d] = project(cams[cam_idx[i]], pts[pt_idx[i]])[d] - uv[2i+d]              */
int acs_sba_residuals(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                      const int32_t* pt_idx, const int32_t* cam_idx, int64_t n_obs,
                      const double* pts, int64_t n_pts, double* resid_out, uint32_t flags);

/* ---- a3/a4: points-only SBA (bundle_adjust_points_only, src/lib/sba.py:181-195) -----
 * Observation list as the reference passes it (points_2d, point_3d_indices,
 * camera_indices; any order, duplicates allowed). pts (n_pts x 3) is the initial
 * estimate on input and the solution on output. resid_before / resid_after (2*n_obs,
 * may be NULL) are the reference's residuals['before'/'after']. report may be NULL.  */
int acs_sba_points(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                   const int32_t* pt_idx, const int32_t* cam_idx, int64_t n_obs, double* pts,
                   int64_t n_pts, const acs_sba_opts* opts, double* resid_before,
                   double* resid_after, acs_report* report, uint32_t flags);

/* ---- dense observation-tensor SBA (the core.sba layout, src/core/sba.py:41-43) ------
 * Point p = one (frame, marker); uv is (n_pts, n_cams, 2), mask (n_pts, n_cams) u8
 * (1 = valid observation). Same solver as acs_sba_points.                             */
int acs_sba_points_dense(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                         const uint8_t* mask, int64_t n_pts, double* pts,
                         const acs_sba_opts* opts, acs_report* report, uint32_t flags);
/* Same solve with separate initial (pts_in) and solution (pts_out) buffers, so a repeated
 * solve from one initialisation needs no reset copy (pts_in == pts_out is allowed).    */
int acs_sba_points_dense_io(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                            const uint8_t* mask, int64_t n_pts, const double* pts_in, double* pts_out,
                            const acs_sba_opts* opts, acs_report* report, uint32_t flags);

/* ---- a9: redescending loss (src/lib/misc.py:329-343), elementwise ------------------ */
int acs_redescending_loss(acs_ctx* ctx, const double* err, int64_t n, double a, double b, double c,
                          double* out, double* dout /* d loss/d err, may be NULL */, uint32_t flags);

/* ---- a7: forward kinematics (get_3d_marker_coords, src/lib/misc.py:144-326) ----------
 * Skeleton tables come from acinoset_amd.kinematics.build_table (int/real blobs).
 * x, dx, ddx: (n, P); tau: (n,) or NULL; intermode 0 pos / 1 vel / 2 acc;
 * out: (n, L + 2*directions, 3); jac (n, L, 3, P) may be NULL.                        */
int acs_fk(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
           int64_t n_reals, const double* x, const double* dx, const double* ddx, const double* tau,
           int64_t n, int32_t intermode, int32_t directions, double* out, double* jac,
           uint32_t flags);

/* ---- a10-a13: FTE trajectory solve (src/core/fte.py:176-555) ------------------------
 * Unknowns: X ((n_frames + 2) x P, row f = frame f - 2; rows 0, 1 are the virtual frames
 * carrying the reference's free dx[1], ddx[1]) and tau, only when shutter_delay:
 * sd_mode 0 = 'const' (fte.py:236): tau (n_cams), tau[0] pinned to 0; sd_mode 1 =
 * 'variable' (fte.py:238): tau (n_frames x n_cams, frame major), tau[n][0] pinned to 0;
 * |tau| <= Ts (fte.py:304-318; a delay on the bound whose descent direction points out is
 * held for that step). meas (n_frames, n_cams, L, 2) pixels,
 * w (n_frames, n_cams, L) = 1/R where likelihood > thresh else 0 (fte.py:210-215),
 * qinv (P) = 1/Q_p = 1/_Q[p]^2 (fte.py:113-144, 217-218). intermode 0 pos / 1 vel / 2 acc
 * (shutter_delay requires vel/acc, fte.py:44-48). X and tau are in/out.                 */
typedef struct {
  int32_t max_iters;  /* LM iterations; default 200 */
  int32_t window;     /* reserved (0) */
  double ftol;        /* relative cost decrease (|F|); default 1e-12 */
  double xtol;        /* relative step; default 1e-12 */
  double gtol;        /* max |gradient|; default 1e-8 */
  double lambda0;     /* initial LM damping; default 1e-3 */
  double redesc_a, redesc_b, redesc_c;  /* redescending loss knots; 3, 10, 20 (fte.py:53-55) */
} acs_fte_opts;

typedef struct {
  int32_t status;      /* ACS_STATUS_* */
  int32_t iters;       /* LM iterations (accepted + rejected) */
  int32_t n_accepted;
  int32_t n_bad_pivots;
  double cost_before, cost_after, cost_meas, cost_model;
  double grad_max, lambda_final;
} acs_fte_report;

void acs_fte_default_opts(acs_fte_opts* o);
int acs_fte_solve(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                  int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                  const double* w, int32_t n_frames, int32_t shutter_delay, double Ts,
                  const double* qinv, int32_t sd_mode, int32_t intermode, double* X, double* tau,
                  const acs_fte_opts* opts, acs_fte_report* report, uint32_t flags);
/* objective (cost3 = [total, measurement, model]), gradient (nv = (n_frames+2)*P + the
 * number of delays: C const / n_frames*C variable, if shutter_delay) and the dense undamped GN normal matrix (nv x nv, may be NULL) at
 * (X, tau): the linearisation acs_fte_solve uses, exported for parity tests. Host ptrs. */
int acs_fte_eval(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                 int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                 const double* w, int32_t n_frames, int32_t shutter_delay, double Ts,
                 const double* qinv, int32_t sd_mode, int32_t intermode, const double* X,
                 const double* tau, double* cost3, double* grad, double* H, uint32_t flags);
/* Test hook: the damped 3-frame super-blocks D_i (n_blk x BP x BP, BP = 3P padded to 16) of
 * acs_fte_solve's block-tridiagonal system at (X, tau) with damping lam, after `levels`
 * cyclic-reduction levels with every pending Schur term applied (0: as assembled; L > 0:
 * blocks 2^L m hold the D the next level factors). dims = {n_blk, BP, levels run}. Constant
 * or no shutter delay; host pointers, or ACS_DEVICE_PTRS for every array. */
int acs_fte_debug_blocks(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                         int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                         const double* w, int32_t n_frames, int32_t shutter_delay, double Ts,
                         const double* qinv, int32_t sd_mode, int32_t intermode, const double* X,
                         const double* tau, double lam, int32_t levels, double* D_out, int64_t* dims,
                         uint32_t flags);

/* ---- §8(e): frame-window distributed FTE (configs[3]) --------------------------------
 * One handle per rank (rank of world); every rank gets the full-size inputs of
 * acs_fte_solve. The super-blocks of 3 frames are split into `world` chains that share their
 * end blocks; a term belongs to the chain holding its lowest row. X is kept only on the
 * rank's own chain (its rows and both shared end blocks).
 * ONE all-reduce (sum) per LM step, of one DEVICE payload of payload_sizes[0] doubles: the
 * chain ends' reduced system (~ (world+1) (2 BP^2 + BP GR) doubles) followed by the pending
 * step's trial cost and step / state norms (4 doubles):
 *   init(P0) -> all-reduce(P0) -> round(P0, P1) -> all-reduce(P1) -> round(P1, P0) -> ...
 * round(in, out), on the summed `in`: every rank takes the same accept / reject decision on
 * the pending step (its cost is in `in`), solves the reduced system of `in`, back-substitutes
 * and steps its own chain, and writes into `out` the new step's trial cost and the reduced
 * system at the trial state, formed speculatively with the damping an acceptance gives
 * (linearised there already for the trial cost). After a rejection the round writes the
 * reduced system at the unchanged state with the new damping instead, and no step: a
 * rejection costs one extra round. Decisions are taken on the device; a round never waits
 * for the host. poll(h, r, &status) waits for round r (0-based) only and returns the LM
 * status after it (0 = running), so a host can queue round r + 1 first (a round after the
 * stop changes nothing). Then gather(p2) -> all-reduce(p2) -> scatter(p2) (the solution
 * rows, n_blocks x BP doubles = payload_sizes[1], once per solve) before result(). Every
 * rank runs the same reduced solve and takes the same decisions; the result equals
 * acs_fte_solve up to summation order.
 * shutter_delay with sd_mode 1 ('variable'): each frame's delays are interior unknowns of
 * the rank that owns the frame, eliminated in its rows and stepped by that rank; they are
 * gathered with the solution rows by p2, and result() returns tau as (n_frames, n_cams).  */
typedef struct acs_fte_dist acs_fte_dist;
int acs_fte_dist_create(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                        int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                        const double* w, int32_t n_frames, int32_t shutter_delay, double Ts,
                        const double* qinv, int32_t sd_mode, int32_t intermode, const double* X,
                        const double* tau, const acs_fte_opts* opts, int32_t rank, int32_t world,
                        acs_fte_dist** out, int64_t* payload_sizes, uint32_t flags);
int acs_fte_dist_init(acs_fte_dist* h, double* payload);
int acs_fte_dist_round(acs_fte_dist* h, const double* in, double* out);
int acs_fte_dist_poll(acs_fte_dist* h, int64_t round, int32_t* status);
int acs_fte_dist_gather(acs_fte_dist* h, double* p2);
int acs_fte_dist_scatter(acs_fte_dist* h, const double* p2);
int acs_fte_dist_result(acs_fte_dist* h, double* X, double* tau, acs_fte_report* report, uint32_t flags);
int acs_fte_dist_destroy(acs_fte_dist* h);
/* A new solve on the same handle from X ((n_frames + 2) x P) and tau (NULL = zeros), host
 * pointers or ACS_DEVICE_PTRS: the LM restarts as after acs_fte_dist_create (then
 * acs_fte_dist_init), with no allocation (the arena, payload sizes and captured round graphs
 * are kept), so a timed multi-GPU solve reuses one handle per rank. */
int acs_fte_dist_reset(acs_fte_dist* h, const double* X, const double* tau, uint32_t flags);

/* ---- next: fisheye triangulation -------------------------------------
 * acs_triangulate_pairs: triangulate_points_fisheye (src/lib/calib.py:120-129) for n
 * (view a, view b) pairs; uv_a/uv_b (n, 2) pixels, cam_a/cam_b (n) camera ids, out (n, 3).
 * acs_triangulate_dense: get_pairwise_3d_points_from_df (src/lib/utils.py:319-349) on the
 * dense (n_pts, n_cams) observation tensor: mean over adjacent pairs (c, c+1 mod C) seen
 * by both cameras; n_pairs_out (may be NULL) = number of pairs (0 -> NaN point).      */
int acs_triangulate_pairs(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv_a,
                          const double* uv_b, const int32_t* cam_a, const int32_t* cam_b, int64_t n,
                          double* xyz_out, uint32_t flags);
int acs_triangulate_dense(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                          const uint8_t* mask, int64_t n_pts, double* xyz_out, int32_t* n_pairs_out,
                          uint32_t flags);

/* ---- §8(a) a6: bundle adjustment of points AND extrinsics ---------------------------
 * bundle_adjust_points_and_extrinsics (src/lib/sba.py:158-178): least_squares(trf,
 * loss='cauchy', f_scale=1) over cost_func_points_extrinsics (:142-146), x = [rvecs, tvecs,
 * points]. Schur-complement LM on the GPU; cams (n_cams <= 16 records) and pts are in/out
 * (rotation and translation of every camera refined, intrinsics kept). Observation list
 * form as acs_sba_points; a point may have at most 64 observations.                   */
typedef struct {
  int32_t max_iters;  /* LM iterations; default 500 */
  int32_t reserved;
  double f_scale;     /* Cauchy scale; default 1 (scipy default used at sba.py:168) */
  double ftol, xtol, gtol;  /* defaults 1e-12, 1e-12, 1e-8 */
  double lambda0;     /* default 1e-3 */
} acs_sba_ext_opts;

typedef struct {
  int32_t status, iters, n_accepted, n_bad_pivots;
  double cost_before, cost_after, grad_max, lambda_final;
} acs_sba_ext_report;

void acs_sba_ext_default_opts(acs_sba_ext_opts* o);
int acs_sba_extrinsics(acs_ctx* ctx, double* cams, int32_t n_cams, const double* uv,
                       const int32_t* pt_idx, const int32_t* cam_idx, int64_t n_obs, double* pts,
                       int64_t n_pts, const acs_sba_ext_opts* opts, double* resid_before,
                       double* resid_after, acs_sba_ext_report* report, uint32_t flags);

/* ---- §8(e): points + extrinsics SBA over ranks -------------------------------------
 * Each rank passes its own points and their observations (point indices local to the
 * rank); cameras are replicated. ONE all-reduce per LM step:
 *   init(P) -> all-reduce(P, sum); then for k = 0, 1, ...:
 *     round(P, P') -> all-reduce(P', sum); poll(k - 1, &status) until status != 0
 * P = [p1 | p3] (payload_sizes[0] doubles): p1 = the reduced camera system
 * [S (6C x 6C) | b | diag U | g_c] + one |g| slot per rank, p3 = (cost, |dX|^2, |X|^2) of the
 * rank's points at the pending trial. A round decides on the pending trial from p3 (the
 * rule of acs_sba_extrinsics), steps from p1, and forms the next p1 at the new trial state
 * with the damping an acceptance sets (a rejected trial costs one extra round that
 * re-forms the system). poll() waits only for that round (pinned status ring of 4).
 * Device buffers. result() returns the (replicated) cameras and this rank's points.    */
typedef struct acs_sba_ext_dist acs_sba_ext_dist;
int acs_sba_ext_dist_create(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                            const int32_t* pt_idx, const int32_t* cam_idx, int64_t n_obs,
                            const double* pts, int64_t n_pts, const acs_sba_ext_opts* opts,
                            int32_t rank, int32_t world, acs_sba_ext_dist** out,
                            int64_t* payload_sizes, uint32_t flags);
int acs_sba_ext_dist_init(acs_sba_ext_dist* h, double* payload);
int acs_sba_ext_dist_round(acs_sba_ext_dist* h, const double* in, double* out);
int acs_sba_ext_dist_poll(acs_sba_ext_dist* h, int64_t round, int32_t* status);
int acs_sba_ext_dist_result(acs_sba_ext_dist* h, double* cams, double* pts, acs_sba_ext_report* report,
                            uint32_t flags);
int acs_sba_ext_dist_destroy(acs_sba_ext_dist* h);

/* ---- §8(f)-2: EKF + RTS smoother (core.ekf, src/core/ekf.py:26-347) -----------------
 * n_seq independent sequences of n_frames frames (one workgroup each). State n = 3P:
 * [x, dx, ddx]. meas (n_seq, n_frames, n_cams, L, 2) pixels (NaN = missing), likelihood
 * (n_seq, n_frames, n_cams, L); R = diag(s^2) with s = r_std_base[cam] (the reference's
 * 2 cov_c / min cov, :244-248) or max_pixel_err below `thresh`. Q, P0: n x n; s0: (n_seq, n).
 * ref_numerics (the measurement-model mode): 1 reproduces the reference's float32
 * prediction cast and float32 Jacobian perturbation (:79, :81-96; eps = the forward-
 * difference step, 1e-3); 0 is the same forward-difference H in float64;
 * ACS_EKF_ANALYTIC_H (2) replaces the P+1 forward-difference poses by the analytic H
 * (SURVEY §8(f)2): one FK with its Jacobian d pos / d x, times the projection's 2 x 3
 * Jacobian, in float64 (eps unused).
 * Outputs (n_seq, n_frames, n) x_pred (may be NULL), x_est, x_smooth; (.., n, n) P_est,
 * P_smooth (may be NULL); outliers (n_seq) = the reference's 3-sigma count (may be NULL). */
int acs_ekf_run(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                const double* likelihood, int32_t n_seq, int32_t n_frames, double fps, double thresh,
                double max_pixel_err, const double* r_std_base, const double* Q, const double* P0,
                const double* s0, int32_t ref_numerics, double eps, double* x_pred, double* x_est,
                double* x_smooth, double* P_est, double* P_smooth, int64_t* outliers, uint32_t flags);
/* Singular solves (I + A P_xx in an update, P_pred in a gain) of the last EKF enqueue on this
 * context (acs_ekf_run or acs_sba_ekf_pipeline); waits for the context stream. A call that
 * synchronises anyway (host arrays, or an outlier report) already fails on them; a
 * device-pointer call without outliers does not check, and this reads the count afterwards. */
int acs_ekf_singular_count(acs_ctx* ctx, int32_t* count);

/* ---- configs[4]: SBA + EKF fused on one observation tensor ------------------------------
 * core.sba (src/core/sba.py:27-70) and core.ekf (src/core/ekf.py:26-298) of the same
 * DLC observations as one device-resident enqueue: pairwise triangulation and points-only
 * SBA of every (sequence, frame, marker) with likelihood > thresh (src/core/sba.py:41;
 * points no adjacent camera pair saw are left out, as the reference's inner merge does,
 * src/lib/sba.py:299), then per sequence the initial state of src/core/ekf.py:121-157 (nose /
 * lure line fits; init->from_sba = 1: on the SBA points, 0: on the triangulated points as
 * core.ekf does) and the EKF + RTS smoother of acs_ekf_run on the EKF model's markers.
 * meas (n_seq, n_frames, n_cams, n_markers, 2), likelihood (n_seq, n_frames, n_cams,
 * n_markers); ekf_markers (L of the skeleton table): observation marker index of every EKF
 * model marker. skel_ints / skel_reals / ekf_markers / sba_opts / init are HOST descriptors
 * whatever `flags` says; the arrays follow `flags`.
 * Outputs: pts_out (n_seq, n_frames, n_markers, 3) SBA points (NaN where not triangulated),
 * x_est, x_smooth (n_seq, n_frames, 3P); outliers (n_seq, may be NULL); sba_report (may be
 * NULL; waits for the SBA). Without ACS_DEVICE_PTRS (or with outliers) the call waits and
 * fails if a sequence's nose was seen in fewer than two frames.                        */
typedef struct {
  int32_t nose;      /* observation marker index of the nose */
  int32_t lure;      /* ... of the lure, -1 if the model has none */
  int32_t x0, y0, psi0;  /* pose parameter indices of x_0, y_0, psi_0 */
  int32_t xl, yl;    /* ... of x_l, y_l (-1: no lure states) */
  int32_t from_sba;  /* 1: line fits on the SBA points, 0: on the triangulated points */
} acs_ekf_init_spec;
int acs_sba_ekf_pipeline(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                         int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                         const double* likelihood, int32_t n_seq, int32_t n_frames, int32_t n_markers,
                         const int32_t* ekf_markers, double fps, double thresh, double max_pixel_err,
                         const double* r_std_base, const double* Q, const double* P0, const acs_sba_opts* sba_opts,
                         const acs_ekf_init_spec* init, int32_t ref_numerics, double eps, double* pts_out,
                         double* x_est, double* x_smooth, int64_t* outliers, acs_report* sba_report,
                         uint32_t flags);

#ifdef __cplusplus
}
#endif
#endif /* ACINOSET_HIP_H */
