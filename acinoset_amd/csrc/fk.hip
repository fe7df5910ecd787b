// fk.hip — batched forward kinematics entry point (get_3d_marker_coords,
// src/lib/misc.py:144-326, and get_all_marker_coords_from_states :126-141).
// One 64-lane workgroup per frame evaluates the skeleton table in LDS (fk.hpp).
#include "fk.hpp"

__global__ __launch_bounds__(64) void k_fk(const int* __restrict__ I, const double* __restrict__ Rl,
                                           const double* __restrict__ x, const double* __restrict__ dx,
                                           const double* __restrict__ ddx, const double* __restrict__ tau,
                                           int64_t n, int intermode, int directions, double* __restrict__ out,
                                           double* __restrict__ jac) {
  __shared__ FkShared sh;
  const SkelView s = skel_view(I, Rl);
  const int64_t f = blockIdx.x;
  if (f >= n) return;
  const int tid = threadIdx.x;
  fk_frame(s, x + f * s.P, sh, tid, blockDim.x);
  __syncthreads();
  // shutter-delay shift of the head (src/lib/misc.py:190-192)
  double sh0 = 0.0, sh1 = 0.0, sh2 = 0.0;
  if (tau && intermode >= 1) {
    const double t = tau[f];
    for (int q = 0; q < s.P; ++q) {
      if (s.pk[4 * q] != PK_TRANS) continue;
      const int ax = s.pk[4 * q + 1];
      double v = dx[f * s.P + q] * t;
      if (intermode >= 2) v += ddx[f * s.P + q] * (t * t);
      if (ax == 0) sh0 = v;
      if (ax == 1) sh1 = v;
      if (ax == 2) sh2 = v;
    }
  }
  const int Lo = s.L + (directions ? 2 : 0);
  for (int l = tid; l < Lo; l += blockDim.x) {
    double p[3];
    if (l < s.L) {
      const int node = s.outn[l];
      const bool world = s.nodes[4 * node + 3] != 0;
      p[0] = sh.pos[node][0] + (world ? 0.0 : sh0);
      p[1] = sh.pos[node][1] + (world ? 0.0 : sh1);
      p[2] = sh.pos[node][2] + (world ? 0.0 : sh2);
    } else {
      const double* h = sh.pos[s.head];
      p[0] = h[0] + sh0;
      p[1] = h[1] + sh1;
      p[2] = h[2] + sh2;
      if (l == s.L + 1) {  // gaze target: p_head + R0_I @ [3, 0, 0]
        p[0] += 3.0 * sh.M[0][0];
        p[1] += 3.0 * sh.M[0][3];
        p[2] += 3.0 * sh.M[0][6];
      }
    }
    double* o = out + (f * Lo + l) * 3;
    o[0] = p[0];
    o[1] = p[1];
    o[2] = p[2];
  }
  if (jac) {
    for (int e = tid; e < s.L * s.P; e += blockDim.x) {
      const int l = e / s.P, q = e % s.P;
      double d[3];
      fk_dpos(s, sh, s.outn[l], q, d);
      double* o = jac + ((f * s.L + l) * 3) * s.P + q;
      o[0] = d[0];
      o[s.P] = d[1];
      o[2 * s.P] = d[2];
    }
  }
}

extern "C" int acs_fk(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                      int64_t n_reals, const double* x, const double* dx, const double* ddx, const double* tau,
                      int64_t n, int32_t intermode, int32_t directions, double* out, double* jac, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n >= 0 && n_ints >= FK_HDR && skel_ints, "acs_fk: bad arguments");
  // table sizes are read on the host from the (host) header when possible
  int hdr[FK_HDR];
  if (flags & ACS_DEVICE_PTRS)
    ACS_HIP(ctx, hipMemcpy(hdr, skel_ints, sizeof(hdr), hipMemcpyDeviceToHost));
  else
    std::memcpy(hdr, skel_ints, sizeof(hdr));
  const int J = hdr[0], K = hdr[1], P = hdr[2], L = hdr[3];
  ACS_CHECK(ctx, J > 0 && J <= FK_MAXJ && K > 0 && K <= FK_MAXN && P > 0 && P <= FK_MAXP && L > 0 && L <= K,
            "acs_fk: skeleton table out of range (J=%d K=%d P=%d L=%d)", J, K, P, L);
  ACS_CHECK(ctx, n_ints == FK_HDR + 9 * J + 4 * K + L + 4 * P + K * P && n_reals == 3 * K,
            "acs_fk: skeleton blob sizes inconsistent");
  ACS_CHECK(ctx, intermode == 0 || ((intermode == 1 || intermode == 2) && dx && tau && (intermode == 1 || ddx)),
            "acs_fk: intermode %d needs dx/ddx/tau", intermode);
  if (n == 0) return ACS_OK;
  void *dI, *dR, *dxx, *ddx1 = nullptr, *dddx = nullptr, *dtau = nullptr;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_TMP0, skel_ints, sizeof(int32_t) * n_ints, flags, &dI))) return rc;
  if ((rc = acs_stage_in(ctx, WS_TMP1, skel_reals, sizeof(double) * n_reals, flags, &dR))) return rc;
  if ((rc = acs_stage_in(ctx, WS_TMP2, x, sizeof(double) * n * P, flags, &dxx))) return rc;
  if (dx && (rc = acs_stage_in(ctx, WS_TMP3, dx, sizeof(double) * n * P, flags, &ddx1))) return rc;
  if (ddx && (rc = acs_stage_in(ctx, WS_TMP4, ddx, sizeof(double) * n * P, flags, &dddx))) return rc;
  if (tau && (rc = acs_stage_in(ctx, WS_TMP5, tau, sizeof(double) * n, flags, &dtau))) return rc;
  const int Lo = L + (directions ? 2 : 0);
  double* dout = (double*)acs_out_buf(ctx, WS_OUT0, out, sizeof(double) * n * Lo * 3, flags);
  double* djac = jac ? (double*)acs_out_buf(ctx, WS_OUT1, jac, sizeof(double) * n * L * 3 * P, flags) : nullptr;
  if (!dout || (jac && !djac)) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_fk, dim3((unsigned)n), dim3(64), 0, ctx->stream, (const int*)dI, (const double*)dR,
                     (const double*)dxx, (const double*)ddx1, (const double*)dddx, (const double*)dtau, n, intermode,
                     directions, dout, djac);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_stage_out(ctx, out, dout, sizeof(double) * n * Lo * 3, flags))) return rc;
  if (jac && (rc = acs_stage_out(ctx, jac, djac, sizeof(double) * n * L * 3 * P, flags))) return rc;
  if (!(flags & ACS_DEVICE_PTRS)) ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}
