// ctx.hip — context lifecycle, workspace, staging, and the small elementwise entry
// points (projection a1, residual vector a2, redescending loss a9).
#include <atomic>

#include "common.hpp"

static std::atomic<long long> g_alloc_events{0};

hipError_t acs_dev_malloc(void** p, size_t bytes) {
  g_alloc_events.fetch_add(1, std::memory_order_relaxed);
  return hipMalloc(p, bytes);
}
hipError_t acs_dev_free(void* p) {
  if (!p) return hipSuccess;
  g_alloc_events.fetch_add(1, std::memory_order_relaxed);
  return hipFree(p);
}
hipError_t acs_host_malloc(void** p, size_t bytes, unsigned flags) {
  g_alloc_events.fetch_add(1, std::memory_order_relaxed);
  return hipHostMalloc(p, bytes, flags);
}
hipError_t acs_host_free(void* p) {
  if (!p) return hipSuccess;
  g_alloc_events.fetch_add(1, std::memory_order_relaxed);
  return hipHostFree(p);
}

int acs_fail(acs_ctx* ctx, int code, const char* fmt, ...) {
  if (ctx) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    ctx->err = buf;
  }
  return code;
}

void* acs_ws(acs_ctx* ctx, int slot, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (ctx->ws_bytes[slot] >= bytes) return ctx->ws[slot];
  if (ctx->ws[slot]) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)acs_dev_free(ctx->ws[slot]);
    ctx->ws[slot] = nullptr;
    ctx->ws_bytes[slot] = 0;
  }
  size_t n = bytes + bytes / 4;  // grow with slack
  n = (n + 255) & ~size_t(255);
  if (acs_dev_malloc(&ctx->ws[slot], n) != hipSuccess) {
    ctx->ws[slot] = nullptr;
    acs_fail(ctx, ACS_E_NOMEM, "hipMalloc(%zu) failed for workspace slot %d", n, slot);
    return nullptr;
  }
  ctx->ws_bytes[slot] = n;
  return ctx->ws[slot];
}

void* acs_pinned(acs_ctx* ctx, size_t bytes) {
  if (ctx->pinned_bytes >= bytes) return ctx->pinned;
  if (ctx->pinned) {
    (void)hipStreamSynchronize(ctx->stream);
    (void)acs_host_free(ctx->pinned);
    ctx->pinned = nullptr;
    ctx->pinned_bytes = 0;
  }
  const size_t n = (bytes + 255) & ~size_t(255);
  // coherent (fine-grained): kernels write their state snapshots straight into it
  if (acs_host_malloc(&ctx->pinned, n, hipHostMallocCoherent) != hipSuccess) {
    ctx->pinned = nullptr;
    acs_fail(ctx, ACS_E_NOMEM, "hipHostMalloc(%zu) failed", n);
    return nullptr;
  }
  ctx->pinned_bytes = n;
  return ctx->pinned;
}

int acs_stage_in(acs_ctx* ctx, int slot, const void* src, size_t bytes, uint32_t flags, void** dev) {
  if (flags & ACS_DEVICE_PTRS) {
    *dev = const_cast<void*>(src);
    return ACS_OK;
  }
  void* d = acs_ws(ctx, slot, bytes);
  if (!d) return ACS_E_NOMEM;
  if (bytes) ACS_HIP(ctx, hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  *dev = d;
  return ACS_OK;
}

int acs_stage_out(acs_ctx* ctx, void* dst, const void* dev, size_t bytes, uint32_t flags) {
  if ((flags & ACS_DEVICE_PTRS) || dst == nullptr || bytes == 0) return ACS_OK;
  ACS_HIP(ctx, hipMemcpyAsync(dst, dev, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return ACS_OK;
}

void* acs_out_buf(acs_ctx* ctx, int slot, void* dst, size_t bytes, uint32_t flags) {
  if (flags & ACS_DEVICE_PTRS) return dst;
  return acs_ws(ctx, slot, bytes);
}

extern "C" {

int acs_abi_version(void) { return ACS_ABI_VERSION; }

int64_t acs_alloc_events(void) { return g_alloc_events.load(std::memory_order_relaxed); }

int acs_device_count(int* n) {
  int c = 0;
  if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
  *n = c;
  return ACS_OK;
}

void acs_sba_default_opts(acs_sba_opts* o) {
  o->max_iters = 100;
  o->reserved = 0;
  o->f_scale = 50.0;
  o->ftol = 1e-15;
  o->xtol = 1e-9;
  o->gtol = 1e-10;
}

int acs_ctx_create(int device, acs_ctx** out) {
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return ACS_E_NODEV;
  if (device < 0 || device >= n) return ACS_E_NODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return ACS_E_NODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return ACS_E_NODEV;
  DeviceGuard guard(device);  // the stream belongs to `device`; the caller's device is restored
  acs_ctx* c = new acs_ctx();
  c->device = device;
  c->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return ACS_E_HIP;
  }
  c->stream = c->own_stream;
  *out = c;
  return ACS_OK;
}

int acs_ctx_destroy(acs_ctx* ctx) {
  if (!ctx) return ACS_OK;
  ACS_DEVICE_GUARD(ctx);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  for (int i = 0; i < WS_NSLOTS; ++i)
    if (ctx->ws[i]) (void)acs_dev_free(ctx->ws[i]);
  if (ctx->pinned) (void)acs_host_free(ctx->pinned);
  if (ctx->ekf_bad) (void)acs_dev_free(ctx->ekf_bad);
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  delete ctx;
  return ACS_OK;
}

const char* acs_last_error(const acs_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int acs_ctx_set_stream(acs_ctx* ctx, void* s) {
  ctx->stream = s ? (hipStream_t)s : ctx->own_stream;
  return ACS_OK;
}

int acs_ctx_sync(acs_ctx* ctx) {
  ACS_DEVICE_GUARD(ctx);
  ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

}  // extern "C"

// ------------------------------------------------------------------------------------
// a1: projection, a2: residual vector, a9: loss
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_project(const double* __restrict__ cams, int n_cams,
                                                 const double* __restrict__ pts,
                                                 const int32_t* __restrict__ cam_idx, int64_t n,
                                                 int fte_form, double* __restrict__ uv) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int c = cam_idx ? cam_idx[i] : 0;
  if (c < 0 || c >= n_cams) {
    uv[2 * i] = uv[2 * i + 1] = __builtin_nan("");
    return;
  }
  ProjOut o;
  if (fte_form)
    fisheye_project<false, true>(cams + c * ACS_CAM_STRIDE, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], o);
  else
    fisheye_project<false, false>(cams + c * ACS_CAM_STRIDE, pts[3 * i], pts[3 * i + 1], pts[3 * i + 2], o);
  uv[2 * i] = o.u;
  uv[2 * i + 1] = o.v;
}

__global__ __launch_bounds__(256) void k_residuals(const double* __restrict__ cams, int n_cams,
                                                   const double* __restrict__ uvobs,
                                                   const int32_t* __restrict__ pt_idx,
                                                   const int32_t* __restrict__ cam_idx, int64_t n_obs,
                                                   const double* __restrict__ pts, int64_t n_pts,
                                                   double* __restrict__ res) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_obs) return;
  int c = cam_idx[i];
  int64_t p = pt_idx[i];
  if (c < 0 || c >= n_cams || p < 0 || p >= n_pts) {
    res[2 * i] = res[2 * i + 1] = __builtin_nan("");
    return;
  }
  ProjOut o;
  fisheye_project<false>(cams + c * ACS_CAM_STRIDE, pts[3 * p], pts[3 * p + 1], pts[3 * p + 2], o);
  res[2 * i] = o.u - uvobs[2 * i];
  res[2 * i + 1] = o.v - uvobs[2 * i + 1];
}

__global__ __launch_bounds__(256) void k_loss(const double* __restrict__ e, int64_t n, double a, double b,
                                              double c, double* __restrict__ out, double* __restrict__ dout) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  LossOut l = redescending(e[i], a, b, c);
  out[i] = l.f;
  if (dout) dout[i] = l.d1;
}

extern "C" {

int acs_project_fisheye(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* pts,
                        const int32_t* cam_idx, int64_t n, int32_t fte_form, double* uv_out,
                        uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n >= 0 && n_cams > 0, "acs_project_fisheye: n=%lld n_cams=%d", (long long)n, n_cams);
  if (n == 0) return ACS_OK;
  void *dc, *dp, *di = nullptr;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dc))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTS, pts, sizeof(double) * 3 * n, flags, &dp))) return rc;
  if (cam_idx && (rc = acs_stage_in(ctx, WS_CAMIDX, cam_idx, sizeof(int32_t) * n, flags, &di))) return rc;
  double* duv = (double*)acs_out_buf(ctx, WS_OUT0, uv_out, sizeof(double) * 2 * n, flags);
  if (!duv) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_project, dim3(acs_grid(n, 256)), dim3(256), 0, ctx->stream, (const double*)dc, n_cams,
                     (const double*)dp, (const int32_t*)di, n, fte_form, duv);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_stage_out(ctx, uv_out, duv, sizeof(double) * 2 * n, flags))) return rc;
  if (!(flags & ACS_DEVICE_PTRS)) ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

int acs_sba_residuals(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                      const int32_t* pt_idx, const int32_t* cam_idx, int64_t n_obs, const double* pts,
                      int64_t n_pts, double* resid_out, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n_obs >= 0 && n_pts >= 0 && n_cams > 0, "acs_sba_residuals: bad sizes");
  if (n_obs == 0) return ACS_OK;
  void *dc, *duv, *dpi, *dci, *dp;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dc))) return rc;
  if ((rc = acs_stage_in(ctx, WS_UV, uv, sizeof(double) * 2 * n_obs, flags, &duv))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTIDX, pt_idx, sizeof(int32_t) * n_obs, flags, &dpi))) return rc;
  if ((rc = acs_stage_in(ctx, WS_CAMIDX, cam_idx, sizeof(int32_t) * n_obs, flags, &dci))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTS, pts, sizeof(double) * 3 * n_pts, flags, &dp))) return rc;
  double* dr = (double*)acs_out_buf(ctx, WS_OUT0, resid_out, sizeof(double) * 2 * n_obs, flags);
  if (!dr) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_residuals, dim3(acs_grid(n_obs, 256)), dim3(256), 0, ctx->stream, (const double*)dc,
                     n_cams, (const double*)duv, (const int32_t*)dpi, (const int32_t*)dci, n_obs,
                     (const double*)dp, n_pts, dr);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_stage_out(ctx, resid_out, dr, sizeof(double) * 2 * n_obs, flags))) return rc;
  if (!(flags & ACS_DEVICE_PTRS)) ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

int acs_redescending_loss(acs_ctx* ctx, const double* err, int64_t n, double a, double b, double c,
                          double* out, double* dout, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n >= 0 && c > b, "acs_redescending_loss: bad args");
  if (n == 0) return ACS_OK;
  void* de;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_TMP0, err, sizeof(double) * n, flags, &de))) return rc;
  double* dout0 = (double*)acs_out_buf(ctx, WS_OUT0, out, sizeof(double) * n, flags);
  double* dout1 = dout ? (double*)acs_out_buf(ctx, WS_OUT1, dout, sizeof(double) * n, flags) : nullptr;
  if (!dout0 || (dout && !dout1)) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_loss, dim3(acs_grid(n, 256)), dim3(256), 0, ctx->stream, (const double*)de, n, a, b, c,
                     dout0, dout1);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_stage_out(ctx, out, dout0, sizeof(double) * n, flags))) return rc;
  if (dout && (rc = acs_stage_out(ctx, dout, dout1, sizeof(double) * n, flags))) return rc;
  if (!(flags & ACS_DEVICE_PTRS)) ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

}  // extern "C"
