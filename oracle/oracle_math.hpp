// ORACLE — test infrastructure only. Never linked into the product (g2o_amd/).
//
// Plain C++ restatement (no Eigen) of the vertex/edge math on the reference's
// BlockSolver hot path.  Eigen is a third-party dependency absent from
// /root/reference (unpinned upstream: cmake_modules/FindEigen3.cmake:18-20);
// the few Eigen algorithms the reference relies on are restated from Eigen's
// published Geometry module (Quaternion from rotation matrix, quaternion
// product, quaternion*vector, toRotationMatrix, 3x3 cofactor inverse).
//
// Every function cites the reference file:line it follows
// (paths relative to /root/reference).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstring>

namespace oracle {

struct V3 { double x, y, z; };
struct M3 { double m[3][3]; };  // m[row][col]
struct Quat { double w, x, y, z; };

inline V3 v3(double a, double b, double c) { return V3{a, b, c}; }
inline V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V3 sub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V3 scale(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
inline V3 cross(V3 a, V3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

inline M3 mzero() { M3 r; std::memset(&r, 0, sizeof r); return r; }
inline M3 meye() { M3 r = mzero(); r.m[0][0] = r.m[1][1] = r.m[2][2] = 1.0; return r; }
inline M3 mmul(const M3& a, const M3& b) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
  return r;
}
inline M3 mT(const M3& a) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[j][i];
  return r;
}
inline V3 mv(const M3& a, V3 v) {
  return {a.m[0][0] * v.x + a.m[0][1] * v.y + a.m[0][2] * v.z, a.m[1][0] * v.x + a.m[1][1] * v.y + a.m[1][2] * v.z,
          a.m[2][0] * v.x + a.m[2][1] * v.y + a.m[2][2] * v.z};
}
inline M3 madd(const M3& a, const M3& b, double sb = 1.0) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j] + sb * b.m[i][j];
  return r;
}
inline M3 mscale(const M3& a, double s) {
  M3 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j] * s;
  return r;
}
// se3quat.h skew(): [0 -z y; z 0 -x; -y x 0]
inline M3 skew(V3 v) {
  M3 r = mzero();
  r.m[0][1] = -v.z; r.m[0][2] = v.y;
  r.m[1][0] = v.z;  r.m[1][2] = -v.x;
  r.m[2][0] = -v.y; r.m[2][1] = v.x;
  return r;
}

// ---- Eigen quaternion algorithms (published Eigen/Geometry, restated) ----
inline Quat qmul(const Quat& a, const Quat& b) {
  return {a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
          a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
inline Quat qconj(const Quat& q) { return {q.w, -q.x, -q.y, -q.z}; }
inline V3 qrot(const Quat& q, V3 v) {  // Eigen _transformVector
  V3 u{q.x, q.y, q.z};
  V3 uv = cross(u, v);
  uv = add(uv, uv);
  return add(add(v, scale(uv, q.w)), cross(u, uv));
}
inline M3 qToR(const Quat& q) {  // Eigen QuaternionBase::toRotationMatrix
  const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
  const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  M3 r;
  r.m[0][0] = 1 - (tyy + tzz); r.m[0][1] = txy - twz; r.m[0][2] = txz + twy;
  r.m[1][0] = txy + twz; r.m[1][1] = 1 - (txx + tzz); r.m[1][2] = tyz - twx;
  r.m[2][0] = txz - twy; r.m[2][1] = tyz + twx; r.m[2][2] = 1 - (txx + tyy);
  return r;
}
inline Quat qFromR(const M3& R) {  // Eigen quaternionbase_assign_impl<Matrix3>
  Quat q;
  double t = R.m[0][0] + R.m[1][1] + R.m[2][2];
  if (t > 0) {
    t = std::sqrt(t + 1.0);
    q.w = 0.5 * t;
    t = 0.5 / t;
    q.x = (R.m[2][1] - R.m[1][2]) * t;
    q.y = (R.m[0][2] - R.m[2][0]) * t;
    q.z = (R.m[1][0] - R.m[0][1]) * t;
  } else {
    int i = 0;
    if (R.m[1][1] > R.m[0][0]) i = 1;
    if (R.m[2][2] > R.m[i][i]) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(R.m[i][i] - R.m[j][j] - R.m[k][k] + 1.0);
    double c[3];
    c[i] = 0.5 * t;
    t = 0.5 / t;
    q.w = (R.m[k][j] - R.m[j][k]) * t;
    c[j] = (R.m[j][i] + R.m[i][j]) * t;
    c[k] = (R.m[k][i] + R.m[i][k]) * t;
    q.x = c[0]; q.y = c[1]; q.z = c[2];
  }
  return q;
}
inline Quat qnormalized(const Quat& q) {
  double n = std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
  return {q.w / n, q.x / n, q.y / n, q.z / n};
}

// ---- SE3Quat (types/slam3d/se3quat.h) ----
struct SE3Quat {
  Quat r{1, 0, 0, 0};
  V3 t{0, 0, 0};
  // se3quat.h:300-305 normalizeRotation
  void normalizeRotation() {
    if (r.w < 0) { r.w = -r.w; r.x = -r.x; r.y = -r.y; r.z = -r.z; }
    r = qnormalized(r);
  }
};
// se3quat.h:96-102 operator*
inline SE3Quat se3mul(const SE3Quat& a, const SE3Quat& b) {
  SE3Quat res = a;
  res.t = add(res.t, qrot(a.r, b.t));
  res.r = qmul(a.r, b.r);
  res.normalizeRotation();
  return res;
}
// se3quat.h:115-120 inverse
inline SE3Quat se3inv(const SE3Quat& a) {
  SE3Quat ret;
  ret.r = qconj(a.r);
  ret.t = qrot(ret.r, scale(a.t, -1.0));
  return ret;
}
// se3quat.h:211-214 map
inline V3 se3map(const SE3Quat& a, V3 p) { return add(qrot(a.r, p), a.t); }
// se3quat.h:217-257 exp (update = [omega; upsilon])
inline SE3Quat se3exp(const double* u) {
  V3 omega{u[0], u[1], u[2]}, upsilon{u[3], u[4], u[5]};
  double theta = std::sqrt(dot(omega, omega));
  M3 Om = skew(omega);
  M3 Om2 = mmul(Om, Om);
  M3 R, V;
  if (theta < 0.00001) {
    R = madd(madd(meye(), Om), Om2, 0.5);
    V = madd(madd(meye(), Om, 0.5), Om2, 1.0 / 6.0);
  } else {
    R = madd(madd(meye(), Om, std::sin(theta) / theta), Om2, (1 - std::cos(theta)) / (theta * theta));
    V = madd(madd(meye(), Om, (1 - std::cos(theta)) / (theta * theta)), Om2,
             (theta - std::sin(theta)) / std::pow(theta, 3));
  }
  SE3Quat res;
  res.r = qFromR(R);
  res.t = mv(V, upsilon);
  res.normalizeRotation();  // SE3Quat(const Quaternion&, const Vector3&) normalizes (se3quat.h:57-59)
  return res;
}

// se3quat.h:173-209 log (se3_ops.hpp:27-47 skew / deltaR): [omega; upsilon]
inline void se3log(const SE3Quat& a, double* res) {
  const M3 R = qToR(a.r);
  const double d = 0.5 * (R.m[0][0] + R.m[1][1] + R.m[2][2] - 1);
  const V3 dR{R.m[2][1] - R.m[1][2], R.m[0][2] - R.m[2][0], R.m[1][0] - R.m[0][1]};
  V3 omega;
  M3 Vinv;
  if (d > 0.99999) {
    omega = scale(dR, 0.5);
    const M3 Om = skew(omega);
    Vinv = madd(madd(meye(), Om, -0.5), mmul(Om, Om), 1. / 12.);
  } else {
    const double theta = std::acos(d);
    omega = scale(dR, theta / (2 * std::sqrt(1 - d * d)));
    const M3 Om = skew(omega);
    Vinv = madd(madd(meye(), Om, -0.5), mmul(Om, Om), (1 - theta / (2 * std::tan(theta / 2))) / (theta * theta));
  }
  const V3 ups = mv(Vinv, a.t);
  res[0] = omega.x; res[1] = omega.y; res[2] = omega.z;
  res[3] = ups.x; res[4] = ups.y; res[5] = ups.z;
}

// ---- Isometry3 (Eigen::Isometry3d as used by types/slam3d) ----
struct Iso3 {
  M3 R = meye();
  V3 t{0, 0, 0};
};
inline Iso3 isomul(const Iso3& a, const Iso3& b) {
  Iso3 r;
  r.R = mmul(a.R, b.R);
  r.t = add(mv(a.R, b.t), a.t);
  return r;
}
inline Iso3 isoinv(const Iso3& a) {  // Eigen Transform::inverse(Isometry)
  Iso3 r;
  r.R = mT(a.R);
  r.t = scale(mv(r.R, a.t), -1.0);
  return r;
}
// isometry3d_mappings.cpp:126-131 fromVectorQT: v = (x y z qx qy qz qw)
inline Iso3 fromVectorQT(const double* v) {
  Iso3 r;
  r.R = qToR(Quat{v[6], v[3], v[4], v[5]});
  r.t = {v[0], v[1], v[2]};
  return r;
}
// isometry3d_mappings.cpp:98-104 toVectorQT
inline void toVectorQT(const Iso3& a, double* v) {
  Quat q = qnormalized(qFromR(a.R));
  v[0] = a.t.x; v[1] = a.t.y; v[2] = a.t.z;
  v[3] = q.x; v[4] = q.y; v[5] = q.z; v[6] = q.w;
}
// isometry3d_mappings.cpp:80-85 toCompactQuaternion (+ normalize :37-43)
inline V3 toCompactQuaternion(const M3& R) {
  Quat q = qnormalized(qFromR(R));
  if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
  return {q.x, q.y, q.z};
}
// isometry3d_mappings.cpp:87-94 fromCompactQuaternion
inline M3 fromCompactQuaternion(V3 v) {
  double w = 1 - dot(v, v);
  if (w < 0) return meye();
  w = std::sqrt(w);
  return qToR(Quat{w, v.x, v.y, v.z});
}
// isometry3d_mappings.cpp:89-94 toVectorMQT
inline void toVectorMQT(const Iso3& a, double* v) {
  V3 q = toCompactQuaternion(a.R);
  v[0] = a.t.x; v[1] = a.t.y; v[2] = a.t.z; v[3] = q.x; v[4] = q.y; v[5] = q.z;
}
// isometry3d_mappings.cpp:106-111 fromVectorMQT
inline Iso3 fromVectorMQT(const double* v) {
  Iso3 r;
  r.R = fromCompactQuaternion(V3{v[3], v[4], v[5]});
  r.t = {v[0], v[1], v[2]};
  return r;
}
// isometry3d_mappings.h:81-86 approximateNearestOrthogonalMatrix
inline void approximateNearestOrthogonalMatrix(M3& R) {
  M3 E = mmul(mT(R), R);
  for (int i = 0; i < 3; ++i) E.m[i][i] -= 1;
  R = madd(R, mmul(R, E), -0.5);
}

// isometry3d_mappings.cpp:48-58 toEuler (roll, pitch, yaw) from the quaternion of R
inline V3 toEuler(const M3& R) {
  const Quat q = qFromR(R);
  const double q0 = q.w, q1 = q.x, q2 = q.y, q3 = q.z;
  return {std::atan2(2 * (q0 * q1 + q2 * q3), 1 - 2 * (q1 * q1 + q2 * q2)), std::asin(2 * (q0 * q2 - q3 * q1)),
          std::atan2(2 * (q0 * q3 + q1 * q2), 1 - 2 * (q2 * q2 + q3 * q3))};
}
// isometry3d_mappings.cpp:60-76 fromEuler: the quaternion of roll / pitch / yaw half angles, then toRotationMatrix
inline M3 fromEuler(V3 v) {
  const double sy = std::sin(v.z * 0.5), cy = std::cos(v.z * 0.5);
  const double sp = std::sin(v.y * 0.5), cp = std::cos(v.y * 0.5);
  const double sr = std::sin(v.x * 0.5), cr = std::cos(v.x * 0.5);
  return qToR(Quat{cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                   cr * cp * sy - sr * sp * cy});
}
// isometry3d_mappings.cpp:102-107 toVectorET, :125-130 fromVectorET: (x y z roll pitch yaw)
inline void toVectorET(const Iso3& a, double* v) {
  const V3 e = toEuler(a.R);
  v[0] = a.t.x; v[1] = a.t.y; v[2] = a.t.z; v[3] = e.x; v[4] = e.y; v[5] = e.z;
}
inline Iso3 fromVectorET(const double* v) {
  Iso3 r;
  r.R = fromEuler(V3{v[3], v[4], v[5]});
  r.t = {v[0], v[1], v[2]};
  return r;
}
inline double det3(const M3& a) {
  return a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) -
         a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]) +
         a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
}
// isometry3d_mappings.h:64-73 nearestOrthogonalMatrix: R = U' V^T from the SVD R = U S V^T (Eigen JacobiSVD, an
// unvendored dependency: restated as a one-sided Jacobi SVD with singular values sorted decreasing, as Eigen returns
// them), with U's first column divided by det(U V^T). Not on the solver path (VertexSE3::oplusImpl uses the approximate
// form below); restated to pin the reference's own orthogonal_matrix.cpp test.
inline void nearestOrthogonalMatrix(M3& R) {
  M3 A = R, V = meye();
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0;
    for (int p = 0; p < 2; ++p)
      for (int q = p + 1; q < 3; ++q) {
        double a = 0, b = 0, g = 0;
        for (int i = 0; i < 3; ++i) {
          a += A.m[i][p] * A.m[i][p];
          b += A.m[i][q] * A.m[i][q];
          g += A.m[i][p] * A.m[i][q];
        }
        if (std::fabs(g) <= 1e-300) continue;
        off = std::max(off, std::fabs(g) / std::sqrt(a * b));
        const double zeta = (b - a) / (2 * g);
        const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
        const double c = 1 / std::sqrt(1 + t * t), s = c * t;
        for (int i = 0; i < 3; ++i) {
          const double x = A.m[i][p], y = A.m[i][q];
          A.m[i][p] = c * x - s * y;
          A.m[i][q] = s * x + c * y;
          const double vx = V.m[i][p], vy = V.m[i][q];
          V.m[i][p] = c * vx - s * vy;
          V.m[i][q] = s * vx + c * vy;
        }
      }
    if (off < 1e-15) break;
  }
  double sg[3];
  int ord[3] = {0, 1, 2};
  for (int k = 0; k < 3; ++k) sg[k] = std::sqrt(A.m[0][k] * A.m[0][k] + A.m[1][k] * A.m[1][k] + A.m[2][k] * A.m[2][k]);
  std::sort(ord, ord + 3, [&](int a, int b) { return sg[a] > sg[b]; });
  M3 U, Vs;
  for (int k = 0; k < 3; ++k)
    for (int i = 0; i < 3; ++i) {
      U.m[i][k] = A.m[i][ord[k]] / sg[ord[k]];
      Vs.m[i][k] = V.m[i][ord[k]];
    }
  const double det = det3(mmul(U, mT(Vs)));
  for (int i = 0; i < 3; ++i) U.m[i][0] /= det;
  R = mmul(U, mT(Vs));
}
// ---- dq/dR (dquat2mat.cpp:63-86) -------------------------------------------
// Derivative of the (x,y,z) part of the quaternion extracted from R (with the
// w>=0 sign convention) w.r.t. the 9 entries of R in column-major order
// (r00 r10 r20 r01 r11 r21 r02 r12 r22).  The reference ships maxima-generated
// code (dquat2mat_maxima_generated.cpp); here the same four branches of
// _q2m are differentiated by hand.  out[row*9 + col].
inline void compute_dq_dR(double* out, const M3& R) {
  const double r00 = R.m[0][0], r10 = R.m[1][0], r20 = R.m[2][0];
  const double r01 = R.m[0][1], r11 = R.m[1][1], r21 = R.m[2][1];
  const double r02 = R.m[0][2], r12 = R.m[1][2], r22 = R.m[2][2];
  enum { I00 = 0, I10 = 1, I20 = 2, I01 = 3, I11 = 4, I21 = 5, I02 = 6, I12 = 7, I22 = 8 };
  for (int i = 0; i < 27; ++i) out[i] = 0.0;
  double tr = r00 + r11 + r22;
  double qw;
  if (tr > 0) {
    // qw = 0.5 sqrt(1+tr); q = (r21-r12, r02-r20, r10-r01) / (4 qw)
    const double S = std::sqrt(tr + 1.0) * 2;
    qw = 0.25 * S;
    const double w = qw, iw3 = 1.0 / (w * w * w);
    const double a[3] = {r21 - r12, r02 - r20, r10 - r01};
    for (int k = 0; k < 3; ++k) {
      const double d = -0.03125 * a[k] * iw3;  // d/d(diag) through qw
      out[k * 9 + I00] = d; out[k * 9 + I11] = d; out[k * 9 + I22] = d;
    }
    out[0 * 9 + I21] = 0.25 / w; out[0 * 9 + I12] = -0.25 / w;
    out[1 * 9 + I02] = 0.25 / w; out[1 * 9 + I20] = -0.25 / w;
    out[2 * 9 + I10] = 0.25 / w; out[2 * 9 + I01] = -0.25 / w;
  } else if ((r00 > r11) & (r00 > r22)) {
    // qx = 0.5 sqrt(1+r00-r11-r22); qy = (r01+r10)/(4qx); qz = (r02+r20)/(4qx); qw = (r21-r12)/(4qx)
    const double S = std::sqrt(1.0 + r00 - r11 - r22) * 2;
    qw = (r21 - r12) / S;
    const double x = 0.25 * S, ix = 1.0 / x, ix3 = ix * ix * ix;
    const double sg[3] = {1.0, -1.0, -1.0};  // d(qx)/d(r00,r11,r22) = sg/(8 qx)
    const int dg[3] = {I00, I11, I22};
    for (int m = 0; m < 3; ++m) {
      out[0 * 9 + dg[m]] = sg[m] * 0.125 * ix;
      out[1 * 9 + dg[m]] = -0.03125 * (r01 + r10) * sg[m] * ix3;
      out[2 * 9 + dg[m]] = -0.03125 * (r02 + r20) * sg[m] * ix3;
    }
    out[1 * 9 + I01] = 0.25 * ix; out[1 * 9 + I10] = 0.25 * ix;
    out[2 * 9 + I02] = 0.25 * ix; out[2 * 9 + I20] = 0.25 * ix;
  } else if (r11 > r22) {
    // qy = 0.5 sqrt(1+r11-r00-r22); qx = (r01+r10)/(4qy); qz = (r12+r21)/(4qy); qw = (r02-r20)/(4qy)
    const double S = std::sqrt(1.0 + r11 - r00 - r22) * 2;
    qw = (r02 - r20) / S;
    const double y = 0.25 * S, iy = 1.0 / y, iy3 = iy * iy * iy;
    const double sg[3] = {-1.0, 1.0, -1.0};
    const int dg[3] = {I00, I11, I22};
    for (int m = 0; m < 3; ++m) {
      out[1 * 9 + dg[m]] = sg[m] * 0.125 * iy;
      out[0 * 9 + dg[m]] = -0.03125 * (r01 + r10) * sg[m] * iy3;
      out[2 * 9 + dg[m]] = -0.03125 * (r12 + r21) * sg[m] * iy3;
    }
    out[0 * 9 + I01] = 0.25 * iy; out[0 * 9 + I10] = 0.25 * iy;
    out[2 * 9 + I12] = 0.25 * iy; out[2 * 9 + I21] = 0.25 * iy;
  } else {
    // qz = 0.5 sqrt(1+r22-r00-r11); qx = (r02+r20)/(4qz); qy = (r12+r21)/(4qz); qw = (r10-r01)/(4qz)
    const double S = std::sqrt(1.0 + r22 - r00 - r11) * 2;
    qw = (r10 - r01) / S;
    const double z = 0.25 * S, iz = 1.0 / z, iz3 = iz * iz * iz;
    const double sg[3] = {-1.0, -1.0, 1.0};
    const int dg[3] = {I00, I11, I22};
    for (int m = 0; m < 3; ++m) {
      out[2 * 9 + dg[m]] = sg[m] * 0.125 * iz;
      out[0 * 9 + dg[m]] = -0.03125 * (r02 + r20) * sg[m] * iz3;
      out[1 * 9 + dg[m]] = -0.03125 * (r12 + r21) * sg[m] * iz3;
    }
    out[0 * 9 + I02] = 0.25 * iz; out[0 * 9 + I20] = 0.25 * iz;
    out[1 * 9 + I12] = 0.25 * iz; out[1 * 9 + I21] = 0.25 * iz;
  }
  if (qw <= 0)
    for (int i = 0; i < 27; ++i) out[i] = -out[i];
}

// ---- SE2 (types/slam2d/se2.h) ----
// stuff/misc.h:114-127 normalize_theta
inline double normalize_theta(double theta) {
  const double pi = 3.14159265358979323846;
  if (theta >= -pi && theta < pi) return theta;
  double multiplier = std::floor(theta / (2 * pi));
  theta = theta - multiplier * 2 * pi;
  if (theta >= pi) theta -= 2 * pi;
  if (theta < -pi) theta += 2 * pi;
  return theta;
}
struct SE2 { double x = 0, y = 0, th = 0; };
inline SE2 se2mul(const SE2& a, const SE2& b) {  // se2.h:64-76
  SE2 r;
  const double c = std::cos(a.th), s = std::sin(a.th);
  r.x = a.x + (c * b.x - s * b.y);
  r.y = a.y + (s * b.x + c * b.y);
  r.th = normalize_theta(a.th + b.th);
  return r;
}
inline SE2 se2inv(const SE2& a) {  // se2.h:84-94
  SE2 r;
  r.th = normalize_theta(-a.th);
  const double c = std::cos(r.th), s = std::sin(r.th);
  const double tx = -a.x, ty = -a.y;
  r.x = c * tx - s * ty;
  r.y = s * tx + c * ty;
  return r;
}

// se2.h:45-47 SE2(const Isometry2&): translation, and Rotation2D's angle of the linear part (Eigen
// Rotation2D::fromRotationMatrix: atan2(R(1,0), R(0,0)))
inline SE2 se2FromIso(const double* R2 /* col-major 2x2 */, const double* t) {
  SE2 r;
  r.x = t[0];
  r.y = t[1];
  r.th = std::atan2(R2[1], R2[0]);
  return r;
}

// 3x3 inverse by cofactors (Eigen compute_inverse_size3_helper, restated).
inline void inverse3(const double* A /*col-major*/, double* out /*col-major*/) {
  auto a = [&](int r, int c) { return A[c * 3 + r]; };
  const double c00 = a(1, 1) * a(2, 2) - a(1, 2) * a(2, 1);
  const double c10 = a(0, 2) * a(2, 1) - a(0, 1) * a(2, 2);
  const double c20 = a(0, 1) * a(1, 2) - a(0, 2) * a(1, 1);
  const double det = c00 * a(0, 0) + c10 * a(1, 0) + c20 * a(2, 0);
  const double inv = 1.0 / det;
  // result row0 = cofactors col0 * invdet
  double r[3][3];
  r[0][0] = c00 * inv; r[0][1] = c10 * inv; r[0][2] = c20 * inv;
  r[1][0] = (a(1, 2) * a(2, 0) - a(1, 0) * a(2, 2)) * inv;
  r[1][1] = (a(0, 0) * a(2, 2) - a(0, 2) * a(2, 0)) * inv;
  r[1][2] = (a(0, 2) * a(1, 0) - a(0, 0) * a(1, 2)) * inv;
  r[2][0] = (a(1, 0) * a(2, 1) - a(1, 1) * a(2, 0)) * inv;
  r[2][1] = (a(0, 1) * a(2, 0) - a(0, 0) * a(2, 1)) * inv;
  r[2][2] = (a(0, 0) * a(1, 1) - a(0, 1) * a(1, 0)) * inv;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) out[j * 3 + i] = r[i][j];
}

}  // namespace oracle
