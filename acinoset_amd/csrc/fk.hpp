// fk.hpp — table-driven forward kinematics + analytic FK Jacobian, evaluated
// cooperatively by the lanes of one workgroup for one frame, all state in LDS.
//
// Restates get_3d_marker_coords (src/lib/misc.py:144-326): joint frames
// M_j = R_j_I = RI_j^T with RI_j = R_a(t_a) R_b(t_b) ... RI_parent (rot_x/y/z of
// misc.py:381-420 are passive rotations, so each factor's transpose is an active
// rotation A); nodes p_k = p_base + M_frame @ offset.
// Jacobian: for a rotation parameter alpha of joint j, d p_k / d alpha =
// omega_alpha x (p_k - p_origin(j)) where omega_alpha = M_parent(j) A_{n-1}..A_{r+1} e_axis
// is the world-frame rotation axis; translations give e_axis; the neck length l_1
// gives M_frame e_x. Table layout: acinoset_amd/kinematics.py::build_table.
#pragma once
#include "common.hpp"

#define FK_MAXP 32
#define FK_MAXJ 16
#define FK_MAXN 32
#define FK_HDR 8

enum { PK_TRANS = 0, PK_ROT = 1, PK_LEN = 2, PK_WORLD = 3 };

struct SkelView {
  int J, K, P, L, head;
  const int* joints;   // J*8: parent, nrot, ax0..2, p0..2
  const int* jorigin;  // J
  const int* nodes;    // K*4: base, frame, offset_param, is_world
  const int* outn;     // L
  const int* pk;       // P*4: kind, a, b, c
  const int* deriv;    // K*P
  const double* off;   // K*3
};

__device__ __forceinline__ SkelView skel_view(const int* I, const double* R) {
  SkelView s;
  s.J = I[0];
  s.K = I[1];
  s.P = I[2];
  s.L = I[3];
  s.head = I[4];
  const int* q = I + FK_HDR;
  s.joints = q;
  q += 8 * s.J;
  s.jorigin = q;
  q += s.J;
  s.nodes = q;
  q += 4 * s.K;
  s.outn = q;
  q += s.L;
  s.pk = q;
  q += 4 * s.P;
  s.deriv = q;
  s.off = R;
  return s;
}

// Largest skeleton table (ints): header, joints + origins, nodes, outputs, parameter
// kinds, node-parameter dependence.
#define FK_MAX_INTS (FK_HDR + 9 * FK_MAXJ + 4 * FK_MAXN + FK_MAXN + 4 * FK_MAXP + FK_MAXN * FK_MAXP)

// Stage the skeleton table (global) in LDS: the FK and its Jacobian walk it with dependent
// loads, which must not be HBM round trips. Ends with a barrier.
__device__ __forceinline__ SkelView skel_stage(const int* __restrict__ I, const double* __restrict__ R, int* sI,
                                               double* sR, int tid, int nth) {
  const int J = I[0], K = I[1], P = I[2], L = I[3];
  const int ni = FK_HDR + 9 * J + 4 * K + L + 4 * P + K * P, nr = 3 * K;
  for (int e = tid; e < ni; e += nth) sI[e] = I[e];
  for (int e = tid; e < nr; e += nth) sR[e] = R[e];
  __syncthreads();
  return skel_view(sI, sR);
}

// The copy of skel_stage with the table's sizes known to the caller (no dependent header load
// first, and the caller's other loads in flight with it); the caller synchronises, then takes
// skel_view of the LDS copy.
__device__ __forceinline__ void skel_copy(const int* __restrict__ I, const double* __restrict__ R, int* sI,
                                          double* sR, int ni, int nr, int tid, int nth) {
  for (int e = tid; e < ni; e += nth) sI[e] = I[e];
  for (int e = tid; e < nr; e += nth) sR[e] = R[e];
}

struct FkShared {
  double sn[FK_MAXP], cs[FK_MAXP], xp[FK_MAXP];
  double root[3], world[3];  // head-root translation (x_0, y_0, z_0) and world (lure) position
  double G[FK_MAXJ][9];
  double M[FK_MAXJ][9];
  double pos[FK_MAXN][3];
  double om[FK_MAXP][3];
};

// y = A_axis(angle) @ x for the active rotation A = rot_axis(angle)^T
__device__ __forceinline__ void act_rot_vec(int axis, double s, double c, const double* x, double* y) {
  if (axis == 0) {  // rot_x^T = [[1,0,0],[0,c,-s],[0,s,c]]
    y[0] = x[0];
    y[1] = c * x[1] - s * x[2];
    y[2] = s * x[1] + c * x[2];
  } else if (axis == 1) {  // rot_y^T = [[c,0,s],[0,1,0],[-s,0,c]]
    y[0] = c * x[0] + s * x[2];
    y[1] = x[1];
    y[2] = -s * x[0] + c * x[2];
  } else {  // rot_z^T = [[c,-s,0],[s,c,0],[0,0,1]]
    y[0] = c * x[0] - s * x[1];
    y[1] = s * x[0] + c * x[1];
    y[2] = x[2];
  }
}

__device__ __forceinline__ void mat3_mul(const double* A, const double* B, double* C) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

// Evaluate one frame. `x` may live in global or shared memory. Caller must
// __syncthreads() before reading sh (positions / M / om). Positions exclude any
// shutter-delay shift (callers add it). F32_TRIG: cos / sin in float32 of the float32
// angle (the reference EKF's numerics, src/core/ekf.py:79 + misc.py:381-420).
// FK_MARK(slot): phase marks of thread 0 of block 0 (a profiling build defines it)
#ifndef FK_MARK
#define FK_MARK(slot)
#define FK_MARK_T0
#endif
template <bool F32_TRIG = false>
__device__ void fk_frame(const SkelView& s, const double* x, FkShared& sh, int tid, int nth) {
  FK_MARK_T0
  for (int p = tid; p < s.P; p += nth) {
    double v = x[p];
    sh.xp[p] = v;
    if (F32_TRIG) {
      float sf, cf;
      sincosf((float)v, &sf, &cf);
      sh.sn[p] = sf;
      sh.cs[p] = cf;
    } else {
      sincos(v, &sh.sn[p], &sh.cs[p]);
    }
  }
  FK_MARK(24);
  __syncthreads();
  FK_MARK(25);
  // translation parameters, summed once per frame instead of once per node chain, from the
  // LDS copy (a loop of global loads here was a chain of cache round trips) by the last two
  // threads; the joint loop below runs over 3*J (joint, column) items, so these two are
  // idle there only when nth >= 3*J + 2 (with fewer threads they take joint items too, after
  // their sums, which is still correct)
  if (tid >= nth - 2) {
    const int kind = tid == nth - 2 ? PK_TRANS : PK_WORLD;
    double t[3] = {0.0, 0.0, 0.0};
    for (int q = 0; q < s.P; ++q)
      if (s.pk[4 * q] == kind) {
        const int a = s.pk[4 * q + 1];
        const double v = sh.xp[q];
        t[0] += a == 0 ? v : 0.0;
        t[1] += a == 1 ? v : 0.0;
        t[2] += a == 2 ? v : 0.0;
      }
    double* dst = kind == PK_TRANS ? sh.root : sh.world;
    dst[0] = t[0];
    dst[1] = t[1];
    dst[2] = t[2];
  }
  // G = A_{n-1} ... A_0 (apply A_0 first), one thread per (joint, column): the column
  // starts as a unit vector and takes the joint's <= 3 rotations; the joint's table entries
  // and their sines / cosines are loaded together, and the axis is selected, not branched on
  // (the three candidate results are act_rot_vec's expressions, so the same bits)
  for (int jc = tid; jc < 3 * s.J; jc += nth) {
    const int j = jc / 3, col = jc - 3 * j;
    const int* jt = s.joints + 8 * j;
    const int nrot = jt[1];
    int ax[3], pr[3];
    double sr[3], cr[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      ax[r] = jt[2 + r];
      pr[r] = r < nrot ? jt[5 + r] : 0;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      sr[r] = sh.sn[pr[r]];
      cr[r] = sh.cs[pr[r]];
    }
    double v0 = col == 0 ? 1.0 : 0.0, v1 = col == 1 ? 1.0 : 0.0, v2 = col == 2 ? 1.0 : 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      if (r >= nrot) break;
      const double sv = sr[r], c = cr[r];
      const double x0 = v0, x1 = v1, x2 = v2;
      const int a = ax[r];
      // axis 0: (x0, c x1 - s x2, s x1 + c x2); 1: (c x0 + s x2, x1, -s x0 + c x2);
      // 2: (c x0 - s x1, s x0 + c x1, x2)
      v0 = a == 0 ? x0 : (a == 1 ? c * x0 + sv * x2 : c * x0 - sv * x1);
      v1 = a == 0 ? c * x1 - sv * x2 : (a == 1 ? x1 : sv * x0 + c * x1);
      v2 = a == 0 ? sv * x1 + c * x2 : (a == 1 ? -sv * x0 + c * x2 : x2);
    }
    sh.G[j][col] = v0;
    sh.G[j][3 + col] = v1;
    sh.G[j][6 + col] = v2;
  }
  FK_MARK(26);
  __syncthreads();
  constexpr int FK_D = 8;  // unrolled chain depth of the node positions below
  for (int j = tid; j < s.J; j += nth) {
    double Mm[9], T[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) Mm[i] = sh.G[j][i];
    int k = s.joints[8 * j];
    while (k >= 0) {  // M_j = G_root ... G_parent G_j
      mat3_mul(sh.G[k], Mm, T);
#pragma unroll
      for (int i = 0; i < 9; ++i) Mm[i] = T[i];
      k = s.joints[8 * k];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) sh.M[j][i] = Mm[i];
  }
  FK_MARK(27);
  __syncthreads();
  const int* pk = s.pk;
  // node positions: the chain of (node, frame, offset parameter) up to the root first
  // (int loads only), then every term's M and offset loads at once; terms are added in walk
  // order with the root / world translation last, as a walk up would
  for (int k = tid; k < s.K; k += nth) {
    double p0 = 0.0, p1 = 0.0, p2 = 0.0;
    int cn[FK_D], cf[FK_D], co[FK_D];
    bool add[FK_D];
    int node = k, endb = 0;
    bool live = true;
#pragma unroll
    for (int a = 0; a < FK_D; ++a) {
      const int* nd = s.nodes + 4 * (live ? node : 0);
      const int b = nd[0];
      cn[a] = node;
      cf[a] = nd[1];
      co[a] = nd[2];
      add[a] = live && b >= 0;
      if (live && b < 0) {
        endb = b;
        live = false;
      }
      if (add[a]) node = b;
    }
    auto term = [&](int nn, int fr, int op) {
      const double* Mf = sh.M[fr];
      double o0 = s.off[3 * nn], o1 = s.off[3 * nn + 1], o2 = s.off[3 * nn + 2];
      if (op >= 0) o0 = sh.xp[op];
      p0 += Mf[0] * o0 + Mf[1] * o1 + Mf[2] * o2;
      p1 += Mf[3] * o0 + Mf[4] * o1 + Mf[5] * o2;
      p2 += Mf[6] * o0 + Mf[7] * o1 + Mf[8] * o2;
    };
#pragma unroll
    for (int a = 0; a < FK_D; ++a)
      if (add[a]) term(cn[a], cf[a], co[a]);
    while (live) {  // chains deeper than FK_D
      const int* nd = s.nodes + 4 * node;
      const int b = nd[0];
      if (b < 0) {
        endb = b;
        break;
      }
      term(node, nd[1], nd[2]);
      node = b;
    }
    if (endb == -2) {  // world node (lure): params of PK_WORLD kind
      p0 += sh.world[0];
      p1 += sh.world[1];
      p2 += sh.world[2];
    } else {  // head root: (x_0, y_0, z_0)
      p0 += sh.root[0];
      p1 += sh.root[1];
      p2 += sh.root[2];
    }
    sh.pos[k][0] = p0;
    sh.pos[k][1] = p1;
    sh.pos[k][2] = p2;
  }
  FK_MARK(28);
  for (int q = tid; q < s.P; q += nth) {
    if (pk[4 * q] != PK_ROT) {
      sh.om[q][0] = sh.om[q][1] = sh.om[q][2] = 0.0;
      continue;
    }
    const int j = pk[4 * q + 1], r = pk[4 * q + 2];
    const int* jt = s.joints + 8 * j;
    const int nrot = jt[1];
    const int ax = jt[2 + r];
    double v[3] = {ax == 0 ? 1.0 : 0.0, ax == 1 ? 1.0 : 0.0, ax == 2 ? 1.0 : 0.0};
    for (int rr = r + 1; rr < nrot; ++rr) {
      double w[3];
      const int p = jt[5 + rr];
      act_rot_vec(jt[2 + rr], sh.sn[p], sh.cs[p], v, w);
      v[0] = w[0];
      v[1] = w[1];
      v[2] = w[2];
    }
    const int par = jt[0];
    if (par >= 0) {
      const double* Mp = sh.M[par];
      sh.om[q][0] = Mp[0] * v[0] + Mp[1] * v[1] + Mp[2] * v[2];
      sh.om[q][1] = Mp[3] * v[0] + Mp[4] * v[1] + Mp[5] * v[2];
      sh.om[q][2] = Mp[6] * v[0] + Mp[7] * v[1] + Mp[8] * v[2];
    } else {
      sh.om[q][0] = v[0];
      sh.om[q][1] = v[1];
      sh.om[q][2] = v[2];
    }
  }
}

// d pos[node] / d x[q] (3-vector). Valid after fk_frame + __syncthreads().
__device__ __forceinline__ void fk_dpos(const SkelView& s, const FkShared& sh, int node, int q, double* d) {
  d[0] = d[1] = d[2] = 0.0;
  if (!s.deriv[node * s.P + q]) return;
  const int* pk = s.pk + 4 * q;
  switch (pk[0]) {
    case PK_TRANS:
    case PK_WORLD:  // unit vector along axis pk[1] (selects, no indexed private store)
      d[0] = pk[1] == 0 ? 1.0 : 0.0;
      d[1] = pk[1] == 1 ? 1.0 : 0.0;
      d[2] = pk[1] == 2 ? 1.0 : 0.0;
      break;
    case PK_LEN: {
      const int owner = pk[1];
      const double* Mf = sh.M[s.nodes[4 * owner + 1]];
      d[0] = Mf[0];
      d[1] = Mf[3];
      d[2] = Mf[6];
      break;
    }
    case PK_ROT: {
      const int o = s.jorigin[pk[1]];
      const double r0 = sh.pos[node][0] - sh.pos[o][0];
      const double r1 = sh.pos[node][1] - sh.pos[o][1];
      const double r2 = sh.pos[node][2] - sh.pos[o][2];
      const double* w = sh.om[q];
      d[0] = w[1] * r2 - w[2] * r1;
      d[1] = w[2] * r0 - w[0] * r2;
      d[2] = w[0] * r1 - w[1] * r0;
      break;
    }
  }
}

// Per-parameter data of fk_dpos resolved once per frame (after fk_frame + a barrier), so
// that a derivative needs no chain of dependent table lookups: typ 0 = constant vector
// `vec` (translations: unit axis; neck length: M_frame e_x), 1 = rotation, d = om x (pos -
// org). Same arithmetic as fk_dpos, so the same bits.
struct FkDeriv {
  int typ[FK_MAXP];
  double vec[FK_MAXP][3];
  double org[FK_MAXP][3];
};

__device__ __forceinline__ void fk_deriv_prep(const SkelView& s, const FkShared& sh, FkDeriv& dv, int q) {
  const int* pk = s.pk + 4 * q;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0;
  int typ = 0;
  switch (pk[0]) {
    case PK_TRANS:
    case PK_WORLD:
      v0 = pk[1] == 0 ? 1.0 : 0.0;
      v1 = pk[1] == 1 ? 1.0 : 0.0;
      v2 = pk[1] == 2 ? 1.0 : 0.0;
      break;
    case PK_LEN: {
      const double* Mf = sh.M[s.nodes[4 * pk[1] + 1]];
      v0 = Mf[0];
      v1 = Mf[3];
      v2 = Mf[6];
      break;
    }
    case PK_ROT: {
      typ = 1;
      const int o = s.jorigin[pk[1]];
      dv.org[q][0] = sh.pos[o][0];
      dv.org[q][1] = sh.pos[o][1];
      dv.org[q][2] = sh.pos[o][2];
      v0 = sh.om[q][0];
      v1 = sh.om[q][1];
      v2 = sh.om[q][2];
      break;
    }
  }
  dv.typ[q] = typ;
  dv.vec[q][0] = v0;
  dv.vec[q][1] = v1;
  dv.vec[q][2] = v2;
}

// fk_dpos from the resolved table (valid after fk_deriv_prep of every q + a barrier)
__device__ __forceinline__ void fk_dpos_fast(const SkelView& s, const FkShared& sh, const FkDeriv& dv, int node, int q,
                                             double* d) {
  const bool on = s.deriv[node * s.P + q] != 0;
  const double w0 = dv.vec[q][0], w1 = dv.vec[q][1], w2 = dv.vec[q][2];
  if (dv.typ[q] == 1) {
    const double r0 = sh.pos[node][0] - dv.org[q][0];
    const double r1 = sh.pos[node][1] - dv.org[q][1];
    const double r2 = sh.pos[node][2] - dv.org[q][2];
    d[0] = on ? w1 * r2 - w2 * r1 : 0.0;
    d[1] = on ? w2 * r0 - w0 * r2 : 0.0;
    d[2] = on ? w0 * r1 - w1 * r0 : 0.0;
  } else {
    d[0] = on ? w0 : 0.0;
    d[1] = on ? w1 : 0.0;
    d[2] = on ? w2 : 0.0;
  }
}
