// common.hpp — context, device workspace, error plumbing and the fisheye camera model
// shared by every translation unit of libacinoset_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "acinoset_hip.h"

// ------------------------------------------------------------------------------------
// Context
// ------------------------------------------------------------------------------------
enum WsSlot {
  WS_CAMS = 0, WS_UV, WS_MASK, WS_CAMID, WS_PTS, WS_PTIDX, WS_CAMIDX, WS_OUT0, WS_OUT1,
  WS_PERPT_F0, WS_PERPT_F1, WS_PERPT_I, WS_REPORT, WS_SORT0, WS_SORT1, WS_SORT2, WS_SORT3,
  WS_TMP0, WS_TMP1, WS_TMP2, WS_TMP3, WS_TMP4, WS_TMP5, WS_TMP6, WS_TMP7,
  WS_FTE0, WS_FTE1, WS_FTE2, WS_FTE3, WS_FTE4, WS_FTE5, WS_FTE6, WS_FTE7, WS_FTE8, WS_FTE9,
  WS_FTE10, WS_FTE11, WS_FTE12, WS_FTE13, WS_FTE14, WS_FTE15,
  WS_PIPE0, WS_PIPE1, WS_PIPE2, WS_PIPE3, WS_PIPE4, WS_PIPE5, WS_PIPE6, WS_PIPE7,
  WS_NSLOTS
};
struct acs_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string err;
  void* ws[WS_NSLOTS] = {};
  size_t ws_bytes[WS_NSLOTS] = {};
  int n_cu = 256;
  // pinned (coherent) host slots the kernels write device-state snapshots into (the FTE
  // solve reads the LM status of iteration n while iteration n + 1 runs)
  void* pinned = nullptr;
  size_t pinned_bytes = 0;
  // device counter of singular solves of the last EKF enqueue (acs_ekf_run / the pipeline);
  // its own allocation, so that a device-pointer call can be checked after the fact
  // (acs_ekf_singular_count) whatever the workspace slots did since
  int* ekf_bad = nullptr;
};

// Every device / pinned-host allocation and free the library makes goes through these, and
// counts one event in a process-wide counter (acs_alloc_events): a timed region that reuses its
// buffers shows no change.
hipError_t acs_dev_malloc(void** p, size_t bytes);
hipError_t acs_dev_free(void* p);
hipError_t acs_host_malloc(void** p, size_t bytes, unsigned flags);
hipError_t acs_host_free(void* p);

// Coherent pinned host buffer of at least `bytes` (grow-only).
// Returns nullptr (and sets the error) on failure.
void* acs_pinned(acs_ctx* ctx, size_t bytes);

int acs_fail(acs_ctx* ctx, int code, const char* fmt, ...);

// Makes `device` current for the lifetime of the guard and restores the caller's current
// device afterwards. Every exported entry point that allocates or launches holds one, so two
// contexts on different devices (or a call from another host thread) allocate workspace and
// launch on the context's own device, and the caller's (e.g. torch's) current device is left
// as it was.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int device) {
    if (device < 0) return;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != device) (void)hipSetDevice(device);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};
#define ACS_DEVICE_GUARD(ctx) DeviceGuard _acs_dev_guard((ctx) ? (ctx)->device : -1)

#define ACS_HIP(ctx, call)                                                                 \
  do {                                                                                     \
    hipError_t _e = (call);                                                                \
    if (_e != hipSuccess)                                                                  \
      return acs_fail((ctx), ACS_E_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), \
                      __FILE__, __LINE__);                                                 \
  } while (0)

#define ACS_CHECK(ctx, cond, ...)                                                          \
  do {                                                                                     \
    if (!(cond)) return acs_fail((ctx), ACS_E_INVALID, __VA_ARGS__);                       \
  } while (0)

// Grow-only device workspace slot. Returns nullptr (and sets the error) on failure.
void* acs_ws(acs_ctx* ctx, int slot, size_t bytes);

// Host<->device staging: with ACS_DEVICE_PTRS the pointer is used as is.
int acs_stage_in(acs_ctx* ctx, int slot, const void* src, size_t bytes, uint32_t flags, void** dev);
int acs_stage_out(acs_ctx* ctx, void* dst, const void* dev, size_t bytes, uint32_t flags);
// Output buffer: the caller's device pointer, or a workspace slot to copy back later.
void* acs_out_buf(acs_ctx* ctx, int slot, void* dst, size_t bytes, uint32_t flags);

static inline int acs_grid(int64_t n, int block) { return (int)((n + block - 1) / block); }

// Observation list (any order) -> per-point slot tensor (n_pts, K): uv_pad, mask, camid,
// deterministic (stable radix sort by point id). Defined in sba.hip. *K_out = max obs/pt.
int acs_obs_to_slots(acs_ctx* ctx, const double* duv, const int32_t* dpi, const int32_t* dci, int64_t n_obs,
                     int64_t n_pts, int n_cams, double2** uv_pad, uint8_t** mask, uint8_t** camid, int* K_out);

// ---- device-buffer stages shared by the entry points and the fused pipeline -------------
// Dense points-only SBA (sba.hip): the fused LM over (n_pts, C) observation slots; with a
// report, waits for it (else asynchronous on the context stream).
int acs_sba_dense_enqueue(acs_ctx* ctx, const double* dcams, int C, const double2* duv, const uint8_t* dmask,
                          int64_t n_pts, const double* dpts_in, double* dpts_out, const acs_sba_opts* opts,
                          acs_report* report);
// Pairwise fisheye triangulation of the dense slots (tri.hip): mean over adjacent pairs.
int acs_tri_dense_enqueue(acs_ctx* ctx, const double* dcams, int C, const double* duv, const uint8_t* dmask,
                          int64_t n_pts, double* dout, int32_t* dcnt);
// EKF + RTS smoother (ekf.hip) on device buffers.
struct EkfIo {
  const int* I = nullptr;
  const double *R = nullptr, *cams = nullptr, *meas = nullptr, *lik = nullptr, *rstd = nullptr, *Q = nullptr,
               *P0 = nullptr, *s0 = nullptr;
  double *x_pred = nullptr, *x_est = nullptr, *x_smooth = nullptr, *P_est = nullptr, *P_smooth = nullptr;
  long long* outliers = nullptr;  // set by acs_ekf_enqueue (device, one per sequence)
  int* bad = nullptr;             // set by acs_ekf_enqueue (device): singular update / gain solves
};
int acs_ekf_enqueue(acs_ctx* ctx, int n_ints, int n_reals, const int* hdr, int n_cams, int n_seq, int n_frames,
                    double fps, double thresh, double max_pixel_err, double eps, int ref_numerics, EkfIo& io);

#include "fastmath.hpp"

// ------------------------------------------------------------------------------------
// Fisheye camera model (cv::fisheye::projectPoints with alpha = 0; src/lib/calib.py:132,
// restated by the reference itself in src/core/fte.py:80-96). Camera record layout:
// [fx fy cx cy k1 k2 k3 k4 R00..R22 t0 t1 t2] (ACS_CAM_STRIDE = 20 doubles).
// ------------------------------------------------------------------------------------
struct ProjOut {
  double u, v;
  double J[6];   // d(u,v)/dX (world point), row-major 2x3
  double JY[6];  // d(u,v)/dY (camera-frame point Y = R X + t)
  double Y[3];
};

template <bool JAC, bool FTE_FORM = false>
__device__ __forceinline__ void fisheye_project(const double* __restrict__ c, double X0, double X1,
                                                double X2, ProjOut& o) {
  const double Y0 = fma(c[8], X0, fma(c[9], X1, fma(c[10], X2, c[17])));
  const double Y1 = fma(c[11], X0, fma(c[12], X1, fma(c[13], X2, c[18])));
  const double Y2 = fma(c[14], X0, fma(c[15], X1, fma(c[16], X2, c[19])));
  const double iz = rcp_nr(Y2);
  const double a = Y0 * iz;
  const double b = Y1 * iz;
  const double r2 = a * a + b * b;
  const double k1 = c[4], k2 = c[5], k3 = c[6], k4 = c[7];
  // r and 1/r from one reciprocal square root; OpenCV's guard r > 1e-8 (the FTE form's
  // r = sqrt(r2 + 1e-12) needs none)
  const bool big = FTE_FORM ? true : (r2 > 1e-16);
  const double rr = FTE_FORM ? r2 + 1e-12 : (big ? r2 : 1.0);
  const double ir = rsq_nr(rr);
  const double r = big ? rr * ir : 0.0;
  const double th = atan_pos(r);
  const double th2 = th * th;
  const double poly = 1.0 + th2 * (k1 + th2 * (k2 + th2 * (k3 + th2 * k4)));
  const double thd = th * poly;
  const double s = big ? thd * ir : 1.0;
  o.u = c[0] * (a * s) + c[2];
  o.v = c[1] * (b * s) + c[3];
  if (JAC) {
    // s'(r)/r = (thd'(th) r / (1 + r^2) - thd) / r^3   (0 below OpenCV's guard)
    const double dthd = 1.0 + th2 * (3.0 * k1 + th2 * (5.0 * k2 + th2 * (7.0 * k3 + th2 * 9.0 * k4)));
    double spr;
    if (FTE_FORM) {
      // r = sqrt(a^2+b^2+eps): dr/da = a/r, same formula with this r
      spr = (dthd * r * rcp_nr(1.0 + r * r) - thd) * (ir * ir * ir);
    } else {
      // zero below the guard by a multiply, not a branch (there the factor is exactly 0:
      // r = 0, thd = 0, ir = 1); the 0/1 factor is opaque to the compiler so that it does
      // not turn the product back into a branch around the reciprocal
      double keep = big ? 1.0 : 0.0;
      asm volatile("" : "+v"(keep));
      spr = (dthd * r * rcp_nr(1.0 + r2) - thd) * (ir * ir * ir) * keep;
    }
    const double duda = c[0] * (s + a * a * spr);
    const double dudb = c[0] * (a * b * spr);
    const double dvda = c[1] * (a * b * spr);
    const double dvdb = c[1] * (s + b * b * spr);
    // d(u,v)/dY = J_uv_ab * [[iz, 0, -a iz], [0, iz, -b iz]]
    const double u0 = duda * iz, u1 = dudb * iz, u2 = -(duda * a + dudb * b) * iz;
    const double v0 = dvda * iz, v1 = dvdb * iz, v2 = -(dvda * a + dvdb * b) * iz;
    o.JY[0] = u0;
    o.JY[1] = u1;
    o.JY[2] = u2;
    o.JY[3] = v0;
    o.JY[4] = v1;
    o.JY[5] = v2;
    o.Y[0] = Y0;
    o.Y[1] = Y1;
    o.Y[2] = Y2;
    // times R
    o.J[0] = u0 * c[8] + u1 * c[11] + u2 * c[14];
    o.J[1] = u0 * c[9] + u1 * c[12] + u2 * c[15];
    o.J[2] = u0 * c[10] + u1 * c[13] + u2 * c[16];
    o.J[3] = v0 * c[8] + v1 * c[11] + v2 * c[14];
    o.J[4] = v0 * c[9] + v1 * c[12] + v2 * c[15];
    o.J[5] = v0 * c[10] + v1 * c[13] + v2 * c[16];
  }
}

// u, v and d(u, v)/dX of the same model (OpenCV's r > 1e-8 guard) for the points-only SBA
// LM (k_sba_lm), with the camera-frame Jacobian folded into R's rows: with A = R_0 - a R_2 and
// B = R_1 - b R_2 (shared by both image rows), J_u = iz (du/da A + du/db B) and J_v likewise:
// 22 f64 operations instead of the 28 of forming d(u,v)/dY and multiplying by R
// (fisheye_project, which also returns JY and Y for the extrinsics SBA).
__device__ __forceinline__ void fisheye_uvj(const double* __restrict__ c, double X0, double X1, double X2, double& u,
                                            double& v, double* J) {
  const double Y0 = fma(c[8], X0, fma(c[9], X1, fma(c[10], X2, c[17])));
  const double Y1 = fma(c[11], X0, fma(c[12], X1, fma(c[13], X2, c[18])));
  const double Y2 = fma(c[14], X0, fma(c[15], X1, fma(c[16], X2, c[19])));
  const double iz = rcp_nr(Y2);
  const double a = Y0 * iz;
  const double b = Y1 * iz;
  const double r2 = a * a + b * b;
  const double k1 = c[4], k2 = c[5], k3 = c[6], k4 = c[7];
  const bool big = r2 > 1e-16;
  const double rr = big ? r2 : 1.0;
  const double ir = rsq_nr(rr);
  const double r = big ? rr * ir : 0.0;
  const double th = atan_pos(r);
  const double th2 = th * th;
  const double poly = 1.0 + th2 * (k1 + th2 * (k2 + th2 * (k3 + th2 * k4)));
  const double thd = th * poly;
  const double s = big ? thd * ir : 1.0;
  u = c[0] * (a * s) + c[2];
  v = c[1] * (b * s) + c[3];
  const double dthd = 1.0 + th2 * (3.0 * k1 + th2 * (5.0 * k2 + th2 * (7.0 * k3 + th2 * 9.0 * k4)));
  double keep = big ? 1.0 : 0.0;  // opaque 0 / 1 factor, as in fisheye_project
  asm volatile("" : "+v"(keep));
  const double spr = (dthd * r * rcp_nr(1.0 + r2) - thd) * (ir * ir * ir) * keep;
  const double ab = a * b * spr;
  const double fu = c[0] * iz, fv = c[1] * iz;
  const double ua = fu * (s + a * a * spr), ub = fu * ab;  // iz du/da, iz du/db
  const double va = fv * ab, vb = fv * (s + b * b * spr);  // iz dv/da, iz dv/db
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const double A = fma(-a, c[14 + j], c[8 + j]), B = fma(-b, c[14 + j], c[11 + j]);
    J[j] = fma(ua, A, ub * B);
    J[3 + j] = fma(va, A, vb * B);
  }
}

// ------------------------------------------------------------------------------------
// Redescending loss (src/lib/misc.py:329-343): value, d/de and d2/de2.
// ------------------------------------------------------------------------------------
struct LossOut {
  double f, d1, d2;
};

__device__ __forceinline__ LossOut redescending(double err, double a, double b, double c) {
  const double E = fabs(err);
  const double sa = rcp_nr(1.0 + exp(-(E - a)));
  const double sb = rcp_nr(1.0 + exp(-(E - b)));
  const double sc = rcp_nr(1.0 + exp(-(E - c)));
  const double da = sa * (1.0 - sa), db = sb * (1.0 - sb), dc = sc * (1.0 - sc);
  const double dda = da * (1.0 - 2.0 * sa), ddb = db * (1.0 - 2.0 * sb), ddc = dc * (1.0 - 2.0 * sc);
  const double lin = a * E - 0.5 * a * a;
  const double K3 = a * b - 0.5 * a * a;
  const double cb = c - b;
  const double icb = rcp_nr(cb);
  const double w = (c - E) * icb;
  const double q = K3 + (0.5 * a * cb) * (1.0 - w * w);
  const double q1 = a * (c - E) * icb;
  const double q2 = -a * icb;
  const double K4 = K3 + 0.5 * a * cb;
  LossOut o;
  o.f = (1.0 - sa) * 0.5 * E * E + (sa - sb) * lin + (sb - sc) * q + sc * K4;
  const double dE = -0.5 * da * E * E + (1.0 - sa) * E + (da - db) * lin + (sa - sb) * a +
                    (db - dc) * q + (sb - sc) * q1 + dc * K4;
  const double ddE = -0.5 * dda * E * E - 2.0 * da * E + (1.0 - sa) + (dda - ddb) * lin +
                     2.0 * (da - db) * a + (ddb - ddc) * q + 2.0 * (db - dc) * q1 + (sb - sc) * q2 +
                     ddc * K4;
  const double sg = err > 0.0 ? 1.0 : (err < 0.0 ? -1.0 : 0.0);
  o.d1 = dE * sg;
  o.d2 = ddE;
  return o;
}

// Sum inside an aligned group of G lanes; every lane ends with the bit-identical total
// (each step adds a lane's value to its partner's, and IEEE addition is commutative).
// Within a 16-lane row the partners come from DPP lane permutes (quad xor 1, quad xor 2,
// half-row mirror, row mirror) on the VALU; wider groups finish with LDS-routed shuffles.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

template <int G>
__device__ __forceinline__ double group_sum(double v) {
  if (G >= 2) v += dpp_f64<0xB1>(v);   // quad_perm [1,0,3,2]
  if (G >= 4) v += dpp_f64<0x4E>(v);   // quad_perm [2,3,0,1]
  if (G >= 8) v += dpp_f64<0x141>(v);  // row_half_mirror: quad 0 <-> quad 1 (quads uniform)
  if (G >= 16) v += dpp_f64<0x140>(v); // row_mirror: half 0 <-> half 1
  if (G >= 32) v += __shfl_xor(v, 16, G);
  if (G >= 64) v += __shfl_xor(v, 32, G);
  return v;
}
