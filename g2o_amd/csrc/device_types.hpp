// Device-side vertex/edge math for the three edge families on the BlockSolver path.
//
//   EdgeSE3ProjectXYZ  types/sba/types_six_dof_expmap.h:201-229, .cpp:395-455
//   EdgeSE3 (QUAT)     types/slam3d/edge_se3.cpp:77-103, isometry3d_gradients.h:194-260
//   EdgeSE2            types/slam2d/edge_se2.h:46-52, edge_se2.cpp:77-103
//   EdgeSE2PointXY     types/slam2d/edge_se2_pointxy.h:41-75, edge_se2_pointxy.cpp:63-87
//   oplus              types_six_dof_expmap.h:97-100 (SE3Quat::exp * T, se3quat.h:217-257),
//                      types_sba.h:149-153, vertex_se3.h:105-113, vertex_se2.h:51-58
//
// State layouts in HBM (fp64):
//   SE3Quat camera  [8]  tx ty tz qx qy qz qw pad     (one 64-B line per camera)
//   XYZ point       [3]
//   Isometry3 pose  [12] R (row-major 3x3) tx ty tz
//   SE2 pose        [3]  x y theta
//   XY point        [2]
// Jacobians are produced row-major (D x dim) in registers; nothing is stored.
#pragma once
#include <hip/hip_runtime.h>

namespace g2ohip {
namespace dev {

#define DI __device__ __forceinline__

DI void quat_to_R(double qx, double qy, double qz, double qw, double* R) {  // row-major
  const double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
  const double twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const double txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
  R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

// quaternion (x,y,z,w) from a rotation matrix (row-major), Eigen's branch structure
DI void R_to_quat(const double* R, double* q) {
  double t = R[0] + R[4] + R[8];
  if (t > 0) {
    t = sqrt(t + 1.0);
    q[3] = 0.5 * t;
    t = 0.5 / t;
    q[0] = (R[7] - R[5]) * t;
    q[1] = (R[2] - R[6]) * t;
    q[2] = (R[3] - R[1]) * t;
  } else {
    int i = 0;
    if (R[4] > R[0]) i = 1;
    if (R[8] > R[i * 4]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrt(R[i * 4] - R[j * 4] - R[k * 4] + 1.0);
    double c[3];
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q[3] = (R[k * 3 + j] - R[j * 3 + k]) * t;
    c[j] = (R[j * 3 + i] + R[i * 3 + j]) * t;
    c[k] = (R[k * 3 + i] + R[i * 3 + k]) * t;
    q[0] = c[0]; q[1] = c[1]; q[2] = c[2];
  }
}

DI void qrot(const double* q, const double* v, double* out) {  // q = (x,y,z,w)
  double uv0 = q[1] * v[2] - q[2] * v[1];
  double uv1 = q[2] * v[0] - q[0] * v[2];
  double uv2 = q[0] * v[1] - q[1] * v[0];
  uv0 += uv0; uv1 += uv1; uv2 += uv2;
  out[0] = v[0] + q[3] * uv0 + (q[1] * uv2 - q[2] * uv1);
  out[1] = v[1] + q[3] * uv1 + (q[2] * uv0 - q[0] * uv2);
  out[2] = v[2] + q[3] * uv2 + (q[0] * uv1 - q[1] * uv0);
}

DI void qmul(const double* a, const double* b, double* o) {  // (x,y,z,w)
  o[3] = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  o[0] = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  o[1] = a[3] * b[1] + a[1] * b[3] + a[2] * b[0] - a[0] * b[2];
  o[2] = a[3] * b[2] + a[2] * b[3] + a[0] * b[1] - a[1] * b[0];
}

DI void qnormalize_pos(double* q) {  // SE3Quat::normalizeRotation
  if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  q[0] /= n; q[1] /= n; q[2] /= n; q[3] /= n;
}

DI void mat3mul(const double* A, const double* B, double* C) {  // row-major
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
}

// ---------------------------------------------------------------- SE3Quat exp (se3quat.h:217-257)
DI void se3_exp(const double* u, double* q, double* t) {
  const double w0 = u[0], w1 = u[1], w2 = u[2];
  const double theta = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  // Omega = skew(omega) row-major
  const double Om[9] = {0, -w2, w1, w2, 0, -w0, -w1, w0, 0};
  double Om2[9];
  mat3mul(Om, Om, Om2);
  double a, b, c, d;  // R = I + a Om + b Om2 ; V = I + c Om + d Om2
  if (theta < 0.00001) {
    a = 1.0; b = 0.5; c = 0.5; d = 1.0 / 6.0;
  } else {
    const double s = sin(theta), co = cos(theta);
    a = s / theta;
    b = (1 - co) / (theta * theta);
    c = (1 - co) / (theta * theta);
    d = (theta - s) / (theta * theta * theta);
  }
  double R[9], V[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const double I = (k % 4 == 0) ? 1.0 : 0.0;
    R[k] = I + a * Om[k] + b * Om2[k];
    V[k] = I + c * Om[k] + d * Om2[k];
  }
  R_to_quat(R, q);
  t[0] = V[0] * u[3] + V[1] * u[4] + V[2] * u[5];
  t[1] = V[3] * u[3] + V[4] * u[4] + V[5] * u[5];
  t[2] = V[6] * u[3] + V[7] * u[4] + V[8] * u[5];
  qnormalize_pos(q);
}

// ---------------------------------------------------------------- Isometry helpers
DI void iso_inv(const double* X, double* Y) {  // X = [R(9) t(3)]
  Y[0] = X[0]; Y[1] = X[3]; Y[2] = X[6];
  Y[3] = X[1]; Y[4] = X[4]; Y[5] = X[7];
  Y[6] = X[2]; Y[7] = X[5]; Y[8] = X[8];
  Y[9] = -(Y[0] * X[9] + Y[1] * X[10] + Y[2] * X[11]);
  Y[10] = -(Y[3] * X[9] + Y[4] * X[10] + Y[5] * X[11]);
  Y[11] = -(Y[6] * X[9] + Y[7] * X[10] + Y[8] * X[11]);
}
DI void iso_mul(const double* A, const double* B, double* C) {
  mat3mul(A, B, C);
#pragma unroll
  for (int i = 0; i < 3; ++i) C[9 + i] = A[i * 3] * B[9] + A[i * 3 + 1] * B[10] + A[i * 3 + 2] * B[11] + A[9 + i];
}
// toCompactQuaternion (isometry3d_mappings.cpp:80-85): normalized, w >= 0
DI void compact_quat(const double* R, double* v) {
  double q[4];
  R_to_quat(R, q);
  const double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  double s = 1.0 / n;
  if (q[3] < 0) s = -s;
  v[0] = q[0] / n * (q[3] < 0 ? -1.0 : 1.0);
  v[1] = q[1] / n * (q[3] < 0 ? -1.0 : 1.0);
  v[2] = q[2] / n * (q[3] < 0 ? -1.0 : 1.0);
  (void)s;
}

// dq/dR for the (x,y,z) of the w>=0 quaternion, column-major entries of R (dquat2mat.cpp:63-86).
// Rr is row-major; out[3][9].
DI void dq_dR(const double* Rr, double* out) {
  const double r00 = Rr[0], r01 = Rr[1], r02 = Rr[2];
  const double r10 = Rr[3], r11 = Rr[4], r12 = Rr[5];
  const double r20 = Rr[6], r21 = Rr[7], r22 = Rr[8];
  enum { I00 = 0, I10 = 1, I20 = 2, I01 = 3, I11 = 4, I21 = 5, I02 = 6, I12 = 7, I22 = 8 };
#pragma unroll
  for (int i = 0; i < 27; ++i) out[i] = 0.0;
  const double tr = r00 + r11 + r22;
  double qw;
  if (tr > 0) {
    const double S = sqrt(tr + 1.0) * 2;
    qw = 0.25 * S;
    const double iw = 1.0 / qw, iw3 = iw * iw * iw;
    const double a0 = r21 - r12, a1 = r02 - r20, a2 = r10 - r01;
    const double d0 = -0.03125 * a0 * iw3, d1 = -0.03125 * a1 * iw3, d2 = -0.03125 * a2 * iw3;
    out[I00] = d0; out[I11] = d0; out[I22] = d0;
    out[9 + I00] = d1; out[9 + I11] = d1; out[9 + I22] = d1;
    out[18 + I00] = d2; out[18 + I11] = d2; out[18 + I22] = d2;
    out[I21] = 0.25 * iw; out[I12] = -0.25 * iw;
    out[9 + I02] = 0.25 * iw; out[9 + I20] = -0.25 * iw;
    out[18 + I10] = 0.25 * iw; out[18 + I01] = -0.25 * iw;
  } else if ((r00 > r11) & (r00 > r22)) {
    const double S = sqrt(1.0 + r00 - r11 - r22) * 2;
    qw = (r21 - r12) / S;
    const double ix = 1.0 / (0.25 * S), ix3 = ix * ix * ix;
    const double sg[3] = {1.0, -1.0, -1.0};
    const int dg[3] = {I00, I11, I22};
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      out[dg[m]] = sg[m] * 0.125 * ix;
      out[9 + dg[m]] = -0.03125 * (r01 + r10) * sg[m] * ix3;
      out[18 + dg[m]] = -0.03125 * (r02 + r20) * sg[m] * ix3;
    }
    out[9 + I01] = 0.25 * ix; out[9 + I10] = 0.25 * ix;
    out[18 + I02] = 0.25 * ix; out[18 + I20] = 0.25 * ix;
  } else if (r11 > r22) {
    const double S = sqrt(1.0 + r11 - r00 - r22) * 2;
    qw = (r02 - r20) / S;
    const double iy = 1.0 / (0.25 * S), iy3 = iy * iy * iy;
    const double sg[3] = {-1.0, 1.0, -1.0};
    const int dg[3] = {I00, I11, I22};
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      out[9 + dg[m]] = sg[m] * 0.125 * iy;
      out[dg[m]] = -0.03125 * (r01 + r10) * sg[m] * iy3;
      out[18 + dg[m]] = -0.03125 * (r12 + r21) * sg[m] * iy3;
    }
    out[I01] = 0.25 * iy; out[I10] = 0.25 * iy;
    out[18 + I12] = 0.25 * iy; out[18 + I21] = 0.25 * iy;
  } else {
    const double S = sqrt(1.0 + r22 - r00 - r11) * 2;
    qw = (r10 - r01) / S;
    const double iz = 1.0 / (0.25 * S), iz3 = iz * iz * iz;
    const double sg[3] = {-1.0, -1.0, 1.0};
    const int dg[3] = {I00, I11, I22};
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      out[18 + dg[m]] = sg[m] * 0.125 * iz;
      out[dg[m]] = -0.03125 * (r02 + r20) * sg[m] * iz3;
      out[9 + dg[m]] = -0.03125 * (r12 + r21) * sg[m] * iz3;
    }
    out[I02] = 0.25 * iz; out[I20] = 0.25 * iz;
    out[9 + I12] = 0.25 * iz; out[9 + I21] = 0.25 * iz;
  }
  if (qw <= 0) {
#pragma unroll
    for (int i = 0; i < 27; ++i) out[i] = -out[i];
  }
}

DI double normalize_theta(double theta) {  // stuff/misc.h:114-127
  const double pi = 3.14159265358979323846;
  if (theta >= -pi && theta < pi) return theta;
  const double m = floor(theta / (2 * pi));
  theta = theta - m * 2 * pi;
  if (theta >= pi) theta -= 2 * pi;
  if (theta < -pi) theta += 2 * pi;
  return theta;
}

// ================================================================ edge families
// Each family: D (error dim), DI_/DJ (vertex dims), meas/info loads, error, Jacobians.

struct EdgeData {
  const int* v0;            // local index of vertex 0 (in its type's state array)
  const int* v1;
  const double* meas;       // per-edge measurement payload (family-specific stride; host-J: e | Ji | Jj)
  const double* info;       // packed upper information (family-specific stride)
  const double* params;     // BA intrinsics [4] or nullptr
  const double* s0;         // state array of vertex-0 type
  const double* s1;         // state array of vertex-1 type
  int rk;                   // robust kernel of the edge set (G2OHIP_RK_*), 0 none
  double rk_delta;          // RobustKernel::delta
  int ue = 0;               // uniform records: bit 0 one information record for every edge, bit 1 one intrinsics record
};
// an edge's packed information / intrinsics record (a single shared record when the edge group's are all equal)
DI const double* info_rec(const EdgeData& d, int e, int stride) {
  return d.info + ((d.ue & 1) ? 0 : (size_t)e * stride);
}
DI const double* param_rec(const EdgeData& d, int e, int stride) {
  return d.params + ((d.ue & 2) ? 0 : (size_t)e * stride);
}

// RobustKernel*::robustify (robust_kernel_impl.cpp:65-200): rho[0] = rho(e2), rho[1] = rho'(e2) (rho'' is not
// used on this path: base_edge.h:117-123 builds the weighted information from rho' only)
DI void robustify(int kind, double delta, double e2, double& r0, double& r1) {
  switch (kind) {
    case 1: {  // Huber
      const double dsqr = delta * delta;
      if (e2 <= dsqr) { r0 = e2; r1 = 1.0; }
      else { const double sq = sqrt(e2); r0 = 2 * sq * delta - dsqr; r1 = delta / sq; }
      break;
    }
    case 2: {  // PseudoHuber
      const double dsqr = delta * delta, aux1 = (1. / dsqr) * e2 + 1.0, aux2 = sqrt(aux1);
      r0 = 2 * dsqr * (aux2 - 1);
      r1 = 1. / aux2;
      break;
    }
    case 3: {  // Cauchy
      const double dsqr = delta * delta, aux = (1. / dsqr) * e2 + 1.0;
      r0 = dsqr * log(aux);
      r1 = 1. / aux;
      break;
    }
    case 4: {  // GemanMcClure
      const double aux = delta / (delta + e2);
      r0 = e2 * aux;
      r1 = aux * aux;
      break;
    }
    case 5: {  // Welsch
      const double dsqr = delta * delta, aux2 = exp(-(e2 / dsqr));
      r0 = dsqr * (1. - aux2);
      r1 = aux2;
      break;
    }
    case 6: {  // Fair
      const double aux = sqrt(e2) / delta;
      r0 = 2. * delta * delta * (aux - log(1. + aux));
      r1 = 1. / (1. + aux);
      break;
    }
    case 7: {  // Tukey
      const double e = sqrt(e2), delta2 = delta * delta;
      if (e <= delta) {
        const double aux = 1. - e2 / delta2;
        r0 = delta2 * (1. - aux * aux * aux) / 3.;
        r1 = aux * aux;
      } else {
        r0 = delta2 / 3.;
        r1 = 0;
      }
      break;
    }
    case 8: {  // Saturated
      const double dsqr = delta * delta;
      if (e2 <= dsqr) { r0 = e2; r1 = 1.; }
      else { r0 = dsqr; r1 = 0.; }
      break;
    }
    case 9: {  // DCS (delta = phi)
      double scale = (2.0 * delta) / (delta + e2);
      if (scale >= 1.0) scale = 1.0;
      r0 = scale * e2 * scale;
      r1 = scale * scale;
      break;
    }
    default: r0 = e2; r1 = 1.0; break;
  }
}

DI int up_idx(int r, int c) { return c * (c + 1) / 2 + r; }  // packed upper, r <= c

template <int D>
DI void load_info(const double* p, double* Om) {  // packed upper -> full row-major
  int k = 0;
#pragma unroll
  for (int c = 0; c < D; ++c)
#pragma unroll
    for (int r = 0; r <= c; ++r) {
      const double v = p[k++];
      Om[r * D + c] = v;
      Om[c * D + r] = v;
    }
}

// ---- EdgeSE3ProjectXYZ: v0 = point (3), v1 = camera SE3Quat (6) ----
struct FamilyBA {
  static constexpr int D = 2, DA = 3, DB = 6, MEAS = 2, INFO = 3;
  static constexpr int SA = 8 /*unused*/, S0 = 3, S1 = 8;  // state strides
  DI static void error(const EdgeData& d, int e, double* err) {
    const double* c = d.s1 + (size_t)d.v1[e] * 8;
    const double* p = d.s0 + (size_t)d.v0[e] * 3;
    double pc[3];
    const double q[4] = {c[3], c[4], c[5], c[6]};
    const double pv[3] = {p[0], p[1], p[2]};
    qrot(q, pv, pc);
    pc[0] += c[0]; pc[1] += c[1]; pc[2] += c[2];
    const double* K = param_rec(d, e, 4);
    err[0] = d.meas[(size_t)e * 2 + 0] - (pc[0] / pc[2] * K[0] + K[2]);
    err[1] = d.meas[(size_t)e * 2 + 1] - (pc[1] / pc[2] * K[1] + K[3]);
  }
  DI static void linearize(const EdgeData& d, int e, double* err, double* A, double* B) {
    double pc[3];
    linearize(d, e, err, A, B, pc);
  }
  // ... and the point in the camera frame (x, y, z): the camera Jacobian is B = diag(fx, fy) Bt(x/z, y/z, 1/z)
  DI static void linearize(const EdgeData& d, int e, double* err, double* A, double* B, double* pc) {
    linearize_at(d, e, d.v0[e], d.v1[e], err, A, B, pc);
  }
  // the same with the edge's vertex indices given (a caller that prefetched them: no dependent index load); NT: the
  // measurement (streamed once per pass) is read nontemporally, so it does not push the reused landmark lines out of L2
  template <bool NT = false>
  DI static void linearize_at(const EdgeData& d, int e, int v0, int v1, double* err, double* A, double* B, double* pc) {
    const double* c = d.s1 + (size_t)v1 * 8;
    const double* p = d.s0 + (size_t)v0 * 3;
    const double q[4] = {c[3], c[4], c[5], c[6]};
    const double pv[3] = {p[0], p[1], p[2]};
    qrot(q, pv, pc);
    pc[0] += c[0]; pc[1] += c[1]; pc[2] += c[2];
    const double* K = param_rec(d, e, 4);
    const double fx = K[0], fy = K[1];
    const double x = pc[0], y = pc[1], z = pc[2], z2 = z * z;
    const double m0 = NT ? __builtin_nontemporal_load(d.meas + (size_t)e * 2) : d.meas[(size_t)e * 2 + 0];
    const double m1 = NT ? __builtin_nontemporal_load(d.meas + (size_t)e * 2 + 1) : d.meas[(size_t)e * 2 + 1];
    err[0] = m0 - (x / z * fx + K[2]);
    err[1] = m1 - (y / z * fy + K[3]);
    double R[9];
    quat_to_R(q[0], q[1], q[2], q[3], R);
    const double iz = -1. / z;
    const double t00 = iz * fx, t02 = iz * (-x / z * fx);
    const double t11 = iz * fy, t12 = iz * (-y / z * fy);
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) {
      A[cc] = t00 * R[cc] + t02 * R[6 + cc];
      A[3 + cc] = t11 * R[3 + cc] + t12 * R[6 + cc];
    }
    B[0] = x * y / z2 * fx;
    B[1] = -(1 + (x * x / z2)) * fx;
    B[2] = y / z * fx;
    B[3] = -1. / z * fx;
    B[4] = 0;
    B[5] = x / z2 * fx;
    B[6] = (1 + y * y / z2) * fy;
    B[7] = -x * y / z2 * fy;
    B[8] = -x / z * fy;
    B[9] = 0;
    B[10] = -1. / z * fy;
    B[11] = y / z2 * fy;
  }
};

// ---- EdgeSE3 (Isometry3): meas payload = Zinv [12], info packed upper 21 ----
struct FamilySE3 {
  static constexpr int D = 6, DA = 6, DB = 6, MEAS = 12, INFO = 21;
  DI static void error(const EdgeData& d, int e, double* err) {
    const double* Xi = d.s0 + (size_t)d.v0[e] * 12;
    const double* Xj = d.s1 + (size_t)d.v1[e] * 12;
    const double* Zi = d.meas + (size_t)e * 12;
    double Xii[12], T[12], E[12], a[12], b[12], z[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) { a[k] = Xi[k]; b[k] = Xj[k]; z[k] = Zi[k]; }
    iso_inv(a, Xii);
    iso_mul(z, Xii, T);
    iso_mul(T, b, E);
    err[0] = E[9]; err[1] = E[10]; err[2] = E[11];
    compact_quat(E, err + 3);
  }
  DI static void linearize(const EdgeData& d, int e, double* err, double* Ji, double* Jj) {
    const double* Xi = d.s0 + (size_t)d.v0[e] * 12;
    const double* Xj = d.s1 + (size_t)d.v1[e] * 12;
    const double* Zi = d.meas + (size_t)e * 12;
    double a[12], b[12], A[12], Xii[12], Bm[12], E[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) { a[k] = Xi[k]; b[k] = Xj[k]; A[k] = Zi[k]; }
    {  // error exactly as computeError (association (Zinv*Xi^-1)*Xj)
      double T[12], Ee[12];
      iso_inv(a, Xii);
      iso_mul(A, Xii, T);
      iso_mul(T, b, Ee);
      err[0] = Ee[9]; err[1] = Ee[10]; err[2] = Ee[11];
      compact_quat(Ee, err + 3);
    }
    iso_mul(Xii, b, Bm);  // B = Xi^-1 Xj
    iso_mul(A, Bm, E);    // E = A B
    const double* Re = E;
    const double* Ra = A;
    const double* Rb = Bm;
    double dq[27];
    dq_dR(Re, dq);
#pragma unroll
    for (int k = 0; k < 36; ++k) { Ji[k] = 0; Jj[k] = 0; }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        Ji[r * 6 + c] = -Ra[r * 3 + c];
        Jj[r * 6 + c] = Re[r * 3 + c];
      }
    {  // dte/dqi = Ra * skewT(tb)
      const double X = 2 * Bm[9], Y = 2 * Bm[10], Z = 2 * Bm[11];
      const double S[9] = {0, -Z, Y, Z, 0, -X, -Y, X, 0};
      double M[9];
      mat3mul(Ra, S, M);
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) Ji[r * 6 + 3 + c] = M[r * 3 + c];
    }
    // dre/dqi = dq * [vec(Ra*Sxt) vec(Ra*Syt) vec(Ra*Szt)], skewT of Rb
    {
      const double r11 = 2 * Rb[0], r12 = 2 * Rb[1], r13 = 2 * Rb[2];
      const double r21 = 2 * Rb[3], r22 = 2 * Rb[4], r23 = 2 * Rb[5];
      const double r31 = 2 * Rb[6], r32 = 2 * Rb[7], r33 = 2 * Rb[8];
      const double Sx[9] = {0, 0, 0, r31, r32, r33, -r21, -r22, -r23};
      const double Sy[9] = {-r31, -r32, -r33, 0, 0, 0, r11, r12, r13};
      const double Sz[9] = {r21, r22, r23, -r11, -r12, -r13, 0, 0, 0};
      double Mx[9], My[9], Mz[9];
      mat3mul(Ra, Sx, Mx);
      mat3mul(Ra, Sy, My);
      mat3mul(Ra, Sz, Mz);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        double s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {  // k: column-major index of the 3x3 -> (k%3, k/3)
          const int rr = k % 3, cc = k / 3;
          s0 += dq[r * 9 + k] * Mx[rr * 3 + cc];
          s1 += dq[r * 9 + k] * My[rr * 3 + cc];
          s2 += dq[r * 9 + k] * Mz[rr * 3 + cc];
        }
        Ji[(3 + r) * 6 + 3] = s0; Ji[(3 + r) * 6 + 4] = s1; Ji[(3 + r) * 6 + 5] = s2;
      }
    }
    // dre/dqj = dq * [vec(Re*Sx) ...] with skew(I) (non-transposed form, entries 2)
    {
      const double Sx[9] = {0, 0, 0, 0, 0, -2, 0, 2, 0};
      const double Sy[9] = {0, 0, 2, 0, 0, 0, -2, 0, 0};
      const double Sz[9] = {0, -2, 0, 2, 0, 0, 0, 0, 0};
      double Mx[9], My[9], Mz[9];
      mat3mul(Re, Sx, Mx);
      mat3mul(Re, Sy, My);
      mat3mul(Re, Sz, Mz);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        double s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          const int rr = k % 3, cc = k / 3;
          s0 += dq[r * 9 + k] * Mx[rr * 3 + cc];
          s1 += dq[r * 9 + k] * My[rr * 3 + cc];
          s2 += dq[r * 9 + k] * Mz[rr * 3 + cc];
        }
        Jj[(3 + r) * 6 + 3] = s0; Jj[(3 + r) * 6 + 4] = s1; Jj[(3 + r) * 6 + 5] = s2;
      }
    }
  }
};

// ---- EdgeSE2: meas payload = inverse measurement (x y theta), info packed 6 ----
struct FamilySE2 {
  static constexpr int D = 3, DA = 3, DB = 3, MEAS = 3, INFO = 6;
  DI static void compose(const double* a, const double* b, double* o) {
    const double c = cos(a[2]), s = sin(a[2]);
    o[0] = a[0] + (c * b[0] - s * b[1]);
    o[1] = a[1] + (s * b[0] + c * b[1]);
    o[2] = normalize_theta(a[2] + b[2]);
  }
  DI static void inverse(const double* a, double* o) {
    o[2] = normalize_theta(-a[2]);
    const double c = cos(o[2]), s = sin(o[2]);
    o[0] = c * (-a[0]) - s * (-a[1]);
    o[1] = s * (-a[0]) + c * (-a[1]);
  }
  DI static void error(const EdgeData& d, int e, double* err) {
    const double* xi = d.s0 + (size_t)d.v0[e] * 3;
    const double* xj = d.s1 + (size_t)d.v1[e] * 3;
    const double* mi = d.meas + (size_t)e * 3;
    double a[3] = {xi[0], xi[1], xi[2]}, b[3] = {xj[0], xj[1], xj[2]}, m[3] = {mi[0], mi[1], mi[2]};
    double ai[3], t[3];
    inverse(a, ai);
    compose(ai, b, t);
    compose(m, t, err);
  }
  DI static void linearize(const EdgeData& d, int e, double* err, double* Ji, double* Jj) {
    error(d, e, err);
    const double* xi = d.s0 + (size_t)d.v0[e] * 3;
    const double* xj = d.s1 + (size_t)d.v1[e] * 3;
    const double* mi = d.meas + (size_t)e * 3;
    const double thetai = xi[2];
    const double dtx = xj[0] - xi[0], dty = xj[1] - xi[1];
    const double si = sin(thetai), ci = cos(thetai);
    const double A[9] = {-ci, -si, -si * dtx + ci * dty, si, -ci, -ci * dtx - si * dty, 0, 0, -1};
    const double B[9] = {ci, si, 0, -si, ci, 0, 0, 0, 1};
    const double rc = cos(mi[2]), rs = sin(mi[2]);
    const double Z[9] = {rc, -rs, 0, rs, rc, 0, 0, 0, 1};
    mat3mul(Z, A, Ji);
    mat3mul(Z, B, Jj);
  }
};

// ---- EdgeSE2PointXY (BlockSolver_3_2 landmark edge): v0 = SE2 pose (3), v1 = XY point (2); meas x y, info packed 3.
// error = v0^-1 * l - z (edge_se2_pointxy.h:44-49, SE2::inverse se2.h:82-87, SE2 * Vector2 = t + R v se2.h:77-80),
// Jacobians edge_se2_pointxy.cpp:63-87 ----
struct FamilySE2XY {
  static constexpr int D = 2, DA = 3, DB = 2, MEAS = 2, INFO = 3;
  DI static void error(const EdgeData& d, int e, double* err) {
    const double* xi = d.s0 + (size_t)d.v0[e] * 3;
    const double* l = d.s1 + (size_t)d.v1[e] * 2;
    const double* m = d.meas + (size_t)e * 2;
    const double a[3] = {xi[0], xi[1], xi[2]};
    double ai[3];
    FamilySE2::inverse(a, ai);
    const double c = cos(ai[2]), s = sin(ai[2]), l0 = l[0], l1 = l[1];
    err[0] = (ai[0] + (c * l0 - s * l1)) - m[0];
    err[1] = (ai[1] + (s * l0 + c * l1)) - m[1];
  }
  DI static void linearize(const EdgeData& d, int e, double* err, double* Ji, double* Jj) {
    error(d, e, err);
    const double* xi = d.s0 + (size_t)d.v0[e] * 3;
    const double* l = d.s1 + (size_t)d.v1[e] * 2;
    const double x1 = xi[0], y1 = xi[1], x2 = l[0], y2 = l[1];
    const double c = cos(xi[2]), s = sin(xi[2]);
    Ji[0] = -c;
    Ji[1] = -s;
    Ji[2] = c * y2 - c * y1 - s * x2 + s * x1;
    Ji[3] = s;
    Ji[4] = -c;
    Ji[5] = -s * y2 + s * y1 - c * x2 + c * x1;
    Jj[0] = c;
    Jj[1] = s;
    Jj[2] = -s;
    Jj[3] = c;
  }
};

// ---- host-Jacobian edges (an edge type the device does not know): the host's linearizeOplus
// (base_binary_edge.hpp:198-266 numeric, or the type's own analytic one) supplies, per edge, the error and
// both Jacobians row-major in the meas payload: [e (D) | Ji (D x DA) | Jj (D x DB)] ----
template <int D_, int DA_, int DB_>
struct FamilyHostJ {
  static constexpr int D = D_, DA = DA_, DB = DB_, INFO = D * (D + 1) / 2, P = D + D * DA + D * DB;
  DI static void error(const EdgeData& d, int e, double* err) {
    const double* p = d.meas + (size_t)e * P;
#pragma unroll
    for (int i = 0; i < D; ++i) err[i] = p[i];
  }
  DI static void linearize(const EdgeData& d, int e, double* err, double* A, double* B) {
    const double* p = d.meas + (size_t)e * P;
#pragma unroll
    for (int i = 0; i < D; ++i) err[i] = p[i];
#pragma unroll
    for (int i = 0; i < D * DA; ++i) A[i] = p[D + i];
#pragma unroll
    for (int i = 0; i < D * DB; ++i) B[i] = p[D + D * DA + i];
  }
};

}  // namespace dev
}  // namespace g2ohip
