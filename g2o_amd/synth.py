"""Synthetic problem generators for the BASELINE configs.

All generators are seeded with a counter-based RNG (numpy Philox), so the
oracle, the CPU baseline and the HIP backend see byte-identical inputs.  They
return a :class:`Problem` holding plain arrays in the C-ABI layout of
``include/g2o_hip.h`` (the same layout ``oracle/oracle.h`` accepts).

Recipes:
  * ``sphere``  - ``g2o/examples/sphere/create_sphere.cpp:40-231`` (SE3 pose graph,
    EDGE_SE3:QUAT), optionally with the extra lap f-2 loop closures of config C3.
  * ``se2_grid`` - SE2 lattice random walk with odometry plus up to 3 spatially
    local loop closures per pose (config C2).
  * ``slam2d``  - 2D landmark SLAM for BlockSolver_3_2 (VERTEX_SE2 poses, VERTEX_XY landmarks, EDGE_SE2
    odometry, EDGE_SE2_XY range-limited point observations), the shape of g2o/examples/tutorial_slam2d.
  * ``ba``      - BAL-style bundle adjustment after ``g2o/examples/ba/ba_demo.cpp:86-300``
    (VERTEX_SE3:EXPMAP cameras, VERTEX_XYZ points, EDGE_SE3_PROJECT_XYZ:EXPMAP),
    each point observed by exactly k cameras of a window of W consecutive ones.
"""
from __future__ import annotations

import dataclasses
import math
from typing import List

import numpy as np

SEED = 20261015

# vertex / edge type codes (include/g2o_hip.h)
V_SE3_EXPMAP, V_XYZ, V_SE3_QUAT, V_SE2, V_XY = 1, 2, 3, 4, 5
E_SE3_PROJECT_XYZ, E_SE3_QUAT, E_SE2, E_SE2_XY = 1, 2, 3, 5
EST_DIM = {V_SE3_EXPMAP: 7, V_XYZ: 3, V_SE3_QUAT: 7, V_SE2: 3, V_XY: 2}
MEAS_DIM = {E_SE3_PROJECT_XYZ: 2, E_SE3_QUAT: 7, E_SE2: 3, E_SE2_XY: 2}
ERR_DIM = {E_SE3_PROJECT_XYZ: 2, E_SE3_QUAT: 6, E_SE2: 3, E_SE2_XY: 2}


@dataclasses.dataclass
class VertexSet:
    vtype: int
    ids: np.ndarray          # int32 [n]
    est: np.ndarray          # float64 [n, EST_DIM]
    fixed: np.ndarray        # int32 [n]
    marginalized: np.ndarray  # int32 [n]


@dataclasses.dataclass
class EdgeSet:
    etype: int
    v0: np.ndarray      # int32 [n] vertex ids
    v1: np.ndarray      # int32 [n]
    meas: np.ndarray    # float64 [n, MEAS_DIM]
    info: np.ndarray    # float64 [n, D, D]
    params: np.ndarray | None = None  # float64 [n, 4] (fx fy cx cy) for projection edges


@dataclasses.dataclass
class Problem:
    name: str
    vertices: List[VertexSet]
    edges: List[EdgeSet]
    pose_dim: int
    landmark_dim: int  # 0 when there is no Schur complement

    @property
    def num_vertices(self) -> int:
        return sum(len(v.ids) for v in self.vertices)

    @property
    def num_edges(self) -> int:
        return sum(len(e.v0) for e in self.edges)


def _rng(seed: int, stream: int) -> np.random.Generator:
    return np.random.Generator(np.random.Philox(key=seed + (stream << 32)))


# ---------------------------------------------------------------- rotations
def _axis_angle(axis: np.ndarray, angle: np.ndarray) -> np.ndarray:
    """Rotation matrices for unit axes [n,3] and angles [n] (Rodrigues)."""
    angle = np.asarray(angle, dtype=np.float64)
    k = axis / np.linalg.norm(axis, axis=-1, keepdims=True)
    K = np.zeros(k.shape[:-1] + (3, 3))
    K[..., 0, 1], K[..., 0, 2] = -k[..., 2], k[..., 1]
    K[..., 1, 0], K[..., 1, 2] = k[..., 2], -k[..., 0]
    K[..., 2, 0], K[..., 2, 1] = -k[..., 1], k[..., 0]
    s, c = np.sin(angle)[..., None, None], np.cos(angle)[..., None, None]
    eye = np.broadcast_to(np.eye(3), K.shape)
    return eye + s * K + (1 - c) * (K @ K)


def rot_to_quat(R: np.ndarray) -> np.ndarray:
    """Rotation matrices [n,3,3] -> quaternions [n,4] as (x, y, z, w), w >= 0."""
    R = np.asarray(R)
    n = R.shape[0]
    q = np.zeros((n, 4))
    tr = R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]
    m0 = tr > 0
    t = np.sqrt(np.maximum(tr[m0] + 1.0, 0.0))
    w = 0.5 * t
    f = 0.5 / t
    q[m0, 0] = (R[m0, 2, 1] - R[m0, 1, 2]) * f
    q[m0, 1] = (R[m0, 0, 2] - R[m0, 2, 0]) * f
    q[m0, 2] = (R[m0, 1, 0] - R[m0, 0, 1]) * f
    q[m0, 3] = w
    for idx in np.nonzero(~m0)[0]:
        M = R[idx]
        i = 0
        if M[1, 1] > M[0, 0]:
            i = 1
        if M[2, 2] > M[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        tt = math.sqrt(M[i, i] - M[j, j] - M[k, k] + 1.0)
        c = [0.0, 0.0, 0.0]
        c[i] = 0.5 * tt
        tt = 0.5 / tt
        ww = (M[k, j] - M[j, k]) * tt
        c[j] = (M[j, i] + M[i, j]) * tt
        c[k] = (M[k, i] + M[i, k]) * tt
        q[idx] = [c[0], c[1], c[2], ww]
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    q[q[:, 3] < 0] *= -1
    return q


def quat_to_rot(q: np.ndarray) -> np.ndarray:
    """(x, y, z, w) [n,4] -> [n,3,3] (Eigen toRotationMatrix formula)."""
    x, y, z, w = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    R = np.empty((q.shape[0], 3, 3))
    R[:, 0, 0] = 1 - (ty * y + tz * z)
    R[:, 0, 1] = tx * y - tz * w
    R[:, 0, 2] = tx * z + ty * w
    R[:, 1, 0] = tx * y + tz * w
    R[:, 1, 1] = 1 - (tx * x + tz * z)
    R[:, 1, 2] = ty * z - tx * w
    R[:, 2, 0] = tx * z - ty * w
    R[:, 2, 1] = ty * z + tx * w
    R[:, 2, 2] = 1 - (tx * x + ty * y)
    return R


def _iso_vec(R: np.ndarray, t: np.ndarray) -> np.ndarray:
    q = rot_to_quat(R)
    return np.concatenate([t, q], axis=1)


# ---------------------------------------------------------------- SE3 sphere
def sphere(nodes_per_level: int = 50, laps: int = 50, radius: float = 100.0, extra_lap2: bool = False,
           noise_t=(0.01, 0.01, 0.01), noise_q=(0.005, 0.005, 0.005), seed: int = SEED) -> Problem:
    """create_sphere.cpp:40-231; ``extra_lap2`` adds lap f-2 offset-0 closures (config C3)."""
    npl = nodes_per_level
    N = npl * laps
    ids = np.arange(N)
    f = ids // npl
    n = ids % npl
    idp1 = ids + 1  # create_sphere uses the post-incremented id in roty (:104-106)
    rz = _axis_angle(np.tile([0.0, 0.0, 1.0], (N, 1)), -math.pi + 2 * n * math.pi / npl)
    ry = _axis_angle(np.tile([0.0, 1.0, 0.0], (N, 1)), -0.5 * math.pi + idp1 * math.pi / (laps * npl))
    Rt = rz @ ry
    tt = Rt @ np.array([radius, 0.0, 0.0])
    e_from: list = [np.arange(0, N - 1)]
    e_to: list = [np.arange(1, N)]
    for ff in range(1, laps):
        nn = np.arange(npl)
        for off in (-1, 0, 1):
            if ff == laps - 1 and off == 1:
                continue
            e_from.append((ff - 1) * npl + nn)
            e_to.append(ff * npl + nn + off)
    if extra_lap2:
        for ff in range(2, laps):
            nn = np.arange(npl)
            e_from.append((ff - 2) * npl + nn)
            e_to.append(ff * npl + nn)
    a = np.concatenate(e_from)
    b = np.concatenate(e_to)
    # ground-truth relative transforms prev^-1 * cur
    Rrel = np.transpose(Rt[a], (0, 2, 1)) @ Rt[b]
    trel = np.einsum("nji,nj->ni", Rt[a], tt[b] - tt[a])
    # noise (create_sphere.cpp:161-182)
    rng = _rng(seed, 1)
    m = len(a)
    qn = rng.standard_normal((m, 3)) * np.asarray(noise_q)
    qw = 1.0 - np.linalg.norm(qn, axis=1)
    qw = np.maximum(qw, 0.0)
    qnoise = np.concatenate([qn, qw[:, None]], axis=1)
    qnoise /= np.linalg.norm(qnoise, axis=1, keepdims=True)
    gtq = rot_to_quat(Rrel)
    # gtQuat * noise
    x1, y1, z1, w1 = gtq.T
    x2, y2, z2, w2 = qnoise.T
    qm = np.stack([w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                   w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2,
                   w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2,
                   w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2], axis=1)
    qm /= np.linalg.norm(qm, axis=1, keepdims=True)
    qm[qm[:, 3] < 0] *= -1
    tm = trel + rng.standard_normal((m, 3)) * np.asarray(noise_t)
    meas = np.concatenate([tm, qm], axis=1)
    info = np.zeros((6, 6))
    info[0:3, 0:3] = np.diag(1.0 / np.square(noise_t))
    info[3:6, 3:6] = np.diag(1.0 / np.square(noise_q))
    # initial estimate: chain the (noisy) odometry from vertex 0 (:184-191)
    Rm = quat_to_rot(qm[: N - 1])
    Rc = np.empty((N, 3, 3))
    tc = np.empty((N, 3))
    Rc[0], tc[0] = Rt[0], tt[0]
    for i in range(1, N):
        Rc[i] = Rc[i - 1] @ Rm[i - 1]
        tc[i] = Rc[i - 1] @ tm[i - 1] + tc[i - 1]
    est = _iso_vec(Rc, tc)
    fixed = np.zeros(N, np.int32)
    fixed[0] = 1
    verts = VertexSet(V_SE3_QUAT, ids.astype(np.int32), est, fixed, np.zeros(N, np.int32))
    edges = EdgeSet(E_SE3_QUAT, a.astype(np.int32), b.astype(np.int32), meas, np.broadcast_to(info, (m, 6, 6)).copy())
    name = f"sphere{npl}x{laps}" + ("_lap2" if extra_lap2 else "")
    return Problem(name, [verts], [edges], 6, 0)


# ---------------------------------------------------------------- SE2 grid
def _se2_compose(a, b):
    c, s = np.cos(a[..., 2]), np.sin(a[..., 2])
    x = a[..., 0] + c * b[..., 0] - s * b[..., 1]
    y = a[..., 1] + s * b[..., 0] + c * b[..., 1]
    th = np.mod(a[..., 2] + b[..., 2] + np.pi, 2 * np.pi) - np.pi
    return np.stack([x, y, th], axis=-1)


def _se2_between(a, b):
    c, s = np.cos(a[..., 2]), np.sin(a[..., 2])
    dx, dy = b[..., 0] - a[..., 0], b[..., 1] - a[..., 1]
    th = np.mod(b[..., 2] - a[..., 2] + np.pi, 2 * np.pi) - np.pi
    return np.stack([c * dx + s * dy, -s * dx + c * dy, th], axis=-1)


def se2_grid(num_poses: int = 1000, loops_per_pose: int = 3, radius: float = 2.0,
             noise=(0.05, 0.05, 0.02), seed: int = SEED) -> Problem:
    """SE2 lattice random walk (config C2): odometry + up to ``loops_per_pose``
    closures to the most recent earlier poses within ``radius`` (excluding i-1)."""
    rng = _rng(seed, 2)
    N = num_poses
    turns = rng.choice([-1, 0, 0, 1], size=N)
    heading = np.zeros(N, np.int64)
    pos = np.zeros((N, 2), np.int64)
    dirs = np.array([[1, 0], [0, 1], [-1, 0], [0, -1]])
    for i in range(1, N):
        heading[i] = (heading[i - 1] + turns[i]) % 4
        pos[i] = pos[i - 1] + dirs[heading[i]]
    th = heading * (np.pi / 2)
    th = np.mod(th + np.pi, 2 * np.pi) - np.pi
    gt = np.stack([pos[:, 0].astype(float), pos[:, 1].astype(float), th], axis=1)
    a_list = [np.arange(N - 1)]
    b_list = [np.arange(1, N)]
    cells: dict = {}
    r = int(math.ceil(radius))
    la, lb = [], []
    for i in range(N):
        px, py = int(pos[i, 0]), int(pos[i, 1])
        cand = []
        for dx in range(-r, r + 1):
            for dy in range(-r, r + 1):
                if dx * dx + dy * dy > radius * radius:
                    continue
                for j in cells.get((px + dx, py + dy), ()):
                    if j < i - 1:
                        cand.append(j)
        if cand:
            cand = sorted(set(cand))[-loops_per_pose:]
            for j in cand:
                la.append(j)
                lb.append(i)
        cells.setdefault((px, py), []).append(i)
        lst = cells[(px, py)]
        if len(lst) > 8:
            del lst[0]
    a_list.append(np.asarray(la, np.int64))
    b_list.append(np.asarray(lb, np.int64))
    a = np.concatenate(a_list)
    b = np.concatenate(b_list)
    rel = _se2_between(gt[a], gt[b])
    m = len(a)
    nz = rng.standard_normal((m, 3)) * np.asarray(noise)
    meas = rel + nz
    meas[:, 2] = np.mod(meas[:, 2] + np.pi, 2 * np.pi) - np.pi
    info = np.diag(1.0 / np.square(noise))
    est = np.empty((N, 3))
    est[0] = gt[0]
    for i in range(1, N):
        est[i] = _se2_compose(est[i - 1], meas[i - 1])
    fixed = np.zeros(N, np.int32)
    fixed[0] = 1
    verts = VertexSet(V_SE2, np.arange(N, dtype=np.int32), est, fixed, np.zeros(N, np.int32))
    edges = EdgeSet(E_SE2, a.astype(np.int32), b.astype(np.int32), meas, np.broadcast_to(info, (m, 3, 3)).copy())
    return Problem(f"se2grid{N}", [verts], [edges], 3, 0)


# ---------------------------------------------------------------- 2D landmark SLAM (BlockSolver_3_2)
def slam2d(num_poses: int = 1000, landmarks_per_cell: float = 1.0, sensor_range: float = 2.5,
           max_obs_per_pose: int = 8, odo_noise=(0.05, 0.05, 0.01), point_noise=(0.05, 0.05),
           seed: int = SEED) -> Problem:
    """SE2 lattice random walk (as ``se2_grid``) with XY landmarks scattered over the visited area
    (``landmarks_per_cell`` per unit cell); every pose observes up to ``max_obs_per_pose`` nearest landmarks
    within ``sensor_range`` (EdgeSE2PointXY: z = x_i^-1 * l + noise), consecutive poses are joined by EdgeSE2
    odometry. Landmarks nobody observes are dropped; pose 0 is fixed; landmarks are marginalised (Schur).
    Initial estimates: chained noisy odometry for the poses, each landmark from its first observation."""
    rng = _rng(seed, 4)
    N = num_poses
    turns = rng.choice([-1, 0, 0, 1], size=N)
    heading = np.zeros(N, np.int64)
    pos = np.zeros((N, 2), np.int64)
    dirs = np.array([[1, 0], [0, 1], [-1, 0], [0, -1]])
    for i in range(1, N):
        heading[i] = (heading[i - 1] + turns[i]) % 4
        pos[i] = pos[i - 1] + dirs[heading[i]]
    th = np.mod(heading * (np.pi / 2) + np.pi, 2 * np.pi) - np.pi
    gt = np.stack([pos[:, 0].astype(float), pos[:, 1].astype(float), th], axis=1)
    # landmarks: uniform over the cells within sensor range of the trajectory
    r = int(math.ceil(sensor_range))
    cells = {(int(x) + dx, int(y) + dy) for x, y in pos for dx in range(-r, r + 1) for dy in range(-r, r + 1)}
    cells = sorted(cells)
    nper = rng.poisson(landmarks_per_cell, size=len(cells))
    lm = np.concatenate([np.asarray(c, float)[None] + rng.random((k, 2)) for c, k in zip(cells, nper) if k > 0])
    grid: dict = {}
    for j, (x, y) in enumerate(lm):
        grid.setdefault((int(math.floor(x)), int(math.floor(y))), []).append(j)
    oa, ob = [], []
    for i in range(N):
        px, py = gt[i, 0], gt[i, 1]
        cand = [j for dx in range(-r - 1, r + 2) for dy in range(-r - 1, r + 2)
                for j in grid.get((int(math.floor(px)) + dx, int(math.floor(py)) + dy), ())]
        if not cand:
            continue
        cand = np.asarray(cand)
        d2 = (lm[cand, 0] - px) ** 2 + (lm[cand, 1] - py) ** 2
        keep = cand[d2 <= sensor_range ** 2]
        keep = keep[np.argsort(d2[d2 <= sensor_range ** 2], kind="stable")][:max_obs_per_pose]
        for j in np.sort(keep):
            oa.append(i)
            ob.append(j)
    oa = np.asarray(oa, np.int64)
    ob = np.asarray(ob, np.int64)
    used = np.unique(ob)
    remap = -np.ones(len(lm), np.int64)
    remap[used] = np.arange(len(used))
    lm = lm[used]
    ob = remap[ob]
    L = len(lm)
    # measurements
    c, s_ = np.cos(gt[oa, 2]), np.sin(gt[oa, 2])
    dx, dy = lm[ob, 0] - gt[oa, 0], lm[ob, 1] - gt[oa, 1]
    zo = np.stack([c * dx + s_ * dy, -s_ * dx + c * dy], axis=1) + rng.standard_normal((len(oa), 2)) * np.asarray(point_noise)
    a = np.arange(N - 1)
    rel = _se2_between(gt[a], gt[a + 1])
    zodo = rel + rng.standard_normal((N - 1, 3)) * np.asarray(odo_noise)
    zodo[:, 2] = np.mod(zodo[:, 2] + np.pi, 2 * np.pi) - np.pi
    est = np.empty((N, 3))
    est[0] = gt[0]
    for i in range(1, N):
        est[i] = _se2_compose(est[i - 1], zodo[i - 1])
    lest = np.zeros((L, 2))
    seen = np.zeros(L, bool)
    for k in range(len(oa)):
        j = ob[k]
        if seen[j]:
            continue
        seen[j] = True
        i = oa[k]
        cc, ss = math.cos(est[i, 2]), math.sin(est[i, 2])
        lest[j] = [est[i, 0] + cc * zo[k, 0] - ss * zo[k, 1], est[i, 1] + ss * zo[k, 0] + cc * zo[k, 1]]
    fixed = np.zeros(N, np.int32)
    fixed[0] = 1
    pose_ids = np.arange(N, dtype=np.int32)
    lm_ids = (N + np.arange(L)).astype(np.int32)
    poses = VertexSet(V_SE2, pose_ids, est, fixed, np.zeros(N, np.int32))
    points = VertexSet(V_XY, lm_ids, lest, np.zeros(L, np.int32), np.ones(L, np.int32))
    odo = EdgeSet(E_SE2, pose_ids[a], pose_ids[a + 1], zodo, np.broadcast_to(np.diag(1.0 / np.square(odo_noise)), (N - 1, 3, 3)).copy())
    obs = EdgeSet(E_SE2_XY, pose_ids[oa], lm_ids[ob], zo, np.broadcast_to(np.diag(1.0 / np.square(point_noise)), (len(oa), 2, 2)).copy())
    return Problem(f"slam2d{N}x{L}", [poses, points], [odo, obs], 3, 2)


# ---------------------------------------------------------------- BA
def _small_rot(rng, n, sigma):
    axis = rng.standard_normal((n, 3))
    ang = rng.standard_normal(n) * sigma
    return _axis_angle(axis, ang)


def ba(num_cameras: int = 1000, num_points: int = 100_000, obs_per_point: int = 10, window: int = 64,
       pixel_noise: float = 1.0, cam_rot_noise: float = 0.002, cam_trans_noise: float = 0.01,
       point_noise: float = 0.05, fixed_cameras: int = 2, seed: int = SEED) -> Problem:
    """BAL-style synthetic BA (config C4/C5).  Camera i sits at x = 0.04 i on a line
    (ba_demo.cpp:216-231) with a small random attitude; every point is seen by
    exactly ``obs_per_point`` distinct cameras drawn from a window of ``window``
    consecutive cameras.  fx = fy = 1000, cx = 320, cy = 240, Omega = I2.
    The first ``fixed_cameras`` cameras are fixed: one fixed camera leaves the
    monocular scale unobservable (rank-deficient Schur system), two fix it."""
    rng = _rng(seed, 3)
    C, P, k = num_cameras, num_points, obs_per_point
    W = min(window, C)
    k = min(k, W)
    centers = np.stack([np.arange(C) * 0.04, np.zeros(C), np.zeros(C)], axis=1)
    Rw = _small_rot(rng, C, 0.02)        # world->cam rotation
    tw = -np.einsum("nij,nj->ni", Rw, centers)
    ws = rng.integers(0, C - W + 1, size=P)
    # k distinct cameras of the window: argsort of random keys
    keys = rng.random((P, W))
    sel = np.sort(np.argsort(keys, axis=1)[:, :k], axis=1)
    cams = ws[:, None] + sel              # [P, k] sorted camera indices
    px = centers[ws, 0] + rng.random(P) * (W - 1) * 0.04
    pts = np.stack([px, rng.random(P) * 2 - 1, 3.0 + 2.0 * rng.random(P)], axis=1)
    fx = fy = 1000.0
    cx, cy = 320.0, 240.0
    cflat = cams.reshape(-1)
    pflat = np.repeat(np.arange(P), k)
    pc = np.einsum("nij,nj->ni", Rw[cflat], pts[pflat]) + tw[cflat]
    uv = np.stack([pc[:, 0] / pc[:, 2] * fx + cx, pc[:, 1] / pc[:, 2] * fy + cy], axis=1)
    uv += rng.standard_normal(uv.shape) * pixel_noise
    # initial estimates
    dR = _small_rot(rng, C, cam_rot_noise)
    R0 = dR @ Rw
    t0 = tw + rng.standard_normal((C, 3)) * cam_trans_noise
    nf = min(fixed_cameras, C)
    R0[:nf], t0[:nf] = Rw[:nf], tw[:nf]
    cam_est = np.concatenate([t0, rot_to_quat(R0)], axis=1)
    pt_est = pts + rng.standard_normal(pts.shape) * point_noise
    cam_ids = np.arange(C, dtype=np.int32)
    pt_ids = (C + np.arange(P)).astype(np.int32)
    fixed = np.zeros(C, np.int32)
    fixed[:nf] = 1
    cams_v = VertexSet(V_SE3_EXPMAP, cam_ids, cam_est, fixed, np.zeros(C, np.int32))
    pts_v = VertexSet(V_XYZ, pt_ids, pt_est, np.zeros(P, np.int32), np.ones(P, np.int32))
    m = len(cflat)
    info = np.broadcast_to(np.eye(2), (m, 2, 2)).copy()
    params = np.broadcast_to(np.array([fx, fy, cx, cy]), (m, 4)).copy()
    edges = EdgeSet(E_SE3_PROJECT_XYZ, pt_ids[pflat], cam_ids[cflat], uv, info, params)
    return Problem(f"ba{C}x{P}k{k}w{W}", [cams_v, pts_v], [edges], 6, 3)


def by_name(name: str, scale: str = "full") -> Problem:
    """BASELINE configs.  ``scale='small'`` gives parity-test sizes."""
    small = scale == "small"
    if name == "C1":
        return sphere(10, 10) if small else sphere(50, 50)
    if name == "C2":
        return se2_grid(800 if small else 100_000)
    if name == "C3":
        return sphere(20, 20, extra_lap2=True) if small else sphere(250, 400, extra_lap2=True)
    if name == "C4":
        return ba(40, 1500) if small else ba(1000, 100_000)
    if name == "C5":
        return ba(80, 4000) if small else ba(4000, 1_000_000)
    if name == "C4R":  # C4 with random covisibility (dense reduced camera system)
        return ba(120, 3000, window=120) if small else ba(1000, 100_000, window=1000)
    if name == "S2":  # BlockSolver_3_2: 2D landmark SLAM (not a BASELINE config)
        return slam2d(300) if small else slam2d(100_000)
    raise KeyError(name)


def landmark_shard(prob: Problem, rank: int, nranks: int) -> Problem:
    """Sub-problem of landmark shard ``rank``: every camera, the contiguous landmark range
    [P*rank/nranks, P*(rank+1)/nranks) of the landmark order and the observations of those
    landmarks — the same partition the device engine uses (engine.cpp setup_edges_device)."""
    cams, pts = prob.vertices
    e = prob.edges[0]
    P = pts.ids.size
    a, b = P * rank // nranks, P * (rank + 1) // nranks
    keep = slice(a, b)
    ids = pts.ids[keep]
    m = (e.v0 >= ids[0]) & (e.v0 <= ids[-1]) if ids.size else np.zeros(e.v0.size, bool)
    pv = VertexSet(pts.vtype, ids.copy(), pts.est[keep].copy(), pts.fixed[keep].copy(), pts.marginalized[keep].copy())
    ev = EdgeSet(e.etype, e.v0[m].copy(), e.v1[m].copy(), e.meas[m].copy(), e.info[m].copy(),
                 None if e.params is None else e.params[m].copy())
    return Problem(f"{prob.name}/shard{rank}of{nranks}", [cams, pv], [ev], prob.pose_dim, prob.landmark_dim)


def landmark_subset(prob: Problem, ids, name: str = "subset") -> Problem:
    """Sub-problem of every camera and the landmarks whose ids are in ``ids`` (any subset, e.g. the aligned shard a rank
    holds, SparseOptimizer.local_landmark_ids), with the observations of those landmarks."""
    cams, pts = prob.vertices
    e = prob.edges[0]
    keep = np.isin(pts.ids, np.asarray(ids))
    m = np.isin(e.v0, pts.ids[keep])
    pv = VertexSet(pts.vtype, pts.ids[keep].copy(), pts.est[keep].copy(), pts.fixed[keep].copy(),
                   pts.marginalized[keep].copy())
    ev = EdgeSet(e.etype, e.v0[m].copy(), e.v1[m].copy(), e.meas[m].copy(), e.info[m].copy(),
                 None if e.params is None else e.params[m].copy())
    return Problem(f"{prob.name}/{name}", [cams, pv], [ev], prob.pose_dim, prob.landmark_dim)
