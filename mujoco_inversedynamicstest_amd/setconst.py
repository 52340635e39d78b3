"""Compile-time model constants (mj_setConst, src/engine/engine_setconst.c:580-597).

Evaluates the model once at qpos0 (and once at qpos_spring) on the host to fill the
constant fields the inverse path reads:

  body_subtreemass                      engine_setconst.c:582-588
  dof_M0 (used by simple dofs in crb)   engine_setconst.c:37-59  (mj_setM0)
  body_invweight0, dof_invweight0       engine_setconst.c:124-210 (constraint diagApprox)
  tendon_invweight0, actuator_acc0      engine_setconst.c:212-300
  tendon_length0, actuator_length0      engine_setconst.c:108-111
  cam_pos0/poscom0/mat0, light_*0       engine_setconst.c:346-373
  tendon_lengthspring (if -1)           engine_setconst.c:560-575 (setSpring)

This runs once per model load, never per instance: it is the model compiler's job (the
reference runs it inside mj_compile), not a CPU path for mj_inverse. Dense numpy linear
algebra is used where the reference solves with its sparse LTDL; the constants therefore
match the reference's to rounding, not bit-for-bit (compiled-model parity is unpinned,
DESIGN.md).
"""
from __future__ import annotations

import numpy as np

from . import mjcf


def _quat2mat(q):
  return np.array(mjcf.quat2mat(list(q))).reshape(3, 3)


def _mulquat(a, b):
  return np.array([a[0]*b[0] - a[1]*b[1] - a[2]*b[2] - a[3]*b[3],
                   a[0]*b[1] + a[1]*b[0] + a[2]*b[3] - a[3]*b[2],
                   a[0]*b[2] - a[1]*b[3] + a[2]*b[0] + a[3]*b[1],
                   a[0]*b[3] + a[1]*b[2] - a[2]*b[1] + a[3]*b[0]])


def _rot(v, q):
  return _quat2mat(q) @ np.asarray(v)


def _axis_angle_quat(axis, ang):
  if ang == 0:
    return np.array([1.0, 0, 0, 0])
  s = np.sin(ang*0.5)
  return np.array([np.cos(ang*0.5), axis[0]*s, axis[1]*s, axis[2]*s])


def _quat_neg(q):
  return np.array([q[0], -q[1], -q[2], -q[3]])


def _rot_vec_quat(v, q):
  return _rot(v, q)


def _quat2vel(q):
  """mju_quat2Vel with dt = 1 (engine_util_spatial.c): the expmap axis*angle."""
  axis = np.array(q[1:4], dtype=np.float64)
  n = np.linalg.norm(axis)
  axis = axis / n if n >= 1e-15 else np.array([1.0, 0, 0])
  speed = 2 * np.arctan2(n, q[0])
  if speed > np.pi:
    speed -= 2 * np.pi
  return axis * speed


def _normq(q):
  n = np.linalg.norm(q)
  return q / n if n > 1e-15 else np.array([1.0, 0, 0, 0])


class _Eval:
  """qpos-dependent quantities of one configuration (mj_kinematics/mj_comPos/mj_crb)."""

  def __init__(self, m, qpos):
    nb = m.nbody
    self.xpos = np.zeros((nb, 3))
    self.xquat = np.zeros((nb, 4))
    self.xquat[0, 0] = 1
    self.xmat = np.zeros((nb, 3, 3))
    self.xmat[0] = np.eye(3)
    self.xanchor = np.zeros((m.njnt, 3))
    self.xaxis = np.zeros((m.njnt, 3))
    for i in range(1, nb):
      ja, jn = m.body_jntadr[i], m.body_jntnum[i]
      if jn == 1 and m.jnt_type[ja] == 0:
        qa = m.jnt_qposadr[ja]
        xpos = qpos[qa:qa+3].copy()
        xquat = _normq(qpos[qa+3:qa+7].copy())
        self.xanchor[ja] = xpos
        self.xaxis[ja] = m.jnt_axis[ja]
      else:
        pid = m.body_parentid[i]
        if pid:
          xpos = self.xmat[pid] @ m.body_pos[i] + self.xpos[pid]
          xquat = _mulquat(self.xquat[pid], m.body_quat[i])
        else:
          xpos = m.body_pos[i].copy()
          xquat = m.body_quat[i].copy()
        for j in range(ja, ja + jn):
          qa = m.jnt_qposadr[j]
          xaxis = _rot(m.jnt_axis[j], xquat)
          xanchor = _rot(m.jnt_pos[j], xquat) + xpos
          t = m.jnt_type[j]
          if t == 2:
            xpos = xpos + xaxis * (qpos[qa] - m.qpos0[qa])
          else:
            qloc = _normq(qpos[qa:qa+4].copy()) if t == 1 else \
                _axis_angle_quat(m.jnt_axis[j], qpos[qa] - m.qpos0[qa])
            xquat = _mulquat(xquat, qloc)
            xpos = xanchor - _rot(m.jnt_pos[j], xquat)
          self.xanchor[j] = xanchor
          self.xaxis[j] = xaxis
      xquat = _normq(xquat)
      self.xquat[i] = xquat
      self.xpos[i] = xpos
      self.xmat[i] = _quat2mat(xquat)
    self.xipos = np.zeros((nb, 3))
    self.ximat = np.zeros((nb, 3, 3))
    self.ximat[0] = np.eye(3)
    for i in range(1, nb):
      self.xipos[i] = self.xmat[i] @ m.body_ipos[i] + self.xpos[i]
      self.ximat[i] = _quat2mat(_mulquat(self.xquat[i], m.body_iquat[i]))
    # subtree com (smooth.c:183-215)
    com = np.zeros((nb, 3))
    ms = np.zeros(nb)
    for i in range(nb - 1, -1, -1):
      com[i] += self.xipos[i] * m.body_mass[i]
      ms[i] += m.body_mass[i]
      if i:
        j = m.body_parentid[i]
        com[j] += com[i]
        ms[j] += ms[i]
      com[i] = self.xipos[i] if ms[i] < 1e-15 else com[i] / max(1e-15, ms[i])
    self.subtree_com = com
    # cdof (smooth.c:225-266)
    self.cdof = np.zeros((m.nv, 6))
    for j in range(m.njnt):
      da = m.jnt_dofadr[j]
      bi = m.jnt_bodyid[j]
      off = com[m.body_rootid[bi]] - self.xanchor[j]
      t = m.jnt_type[j]
      if t in (0, 1):
        skip = 0
        if t == 0:
          for k in range(3):
            self.cdof[da + k, 3 + k] = 1
          skip = 3
        for k in range(3):
          ax = self.xmat[bi][:, k]
          self.cdof[da + skip + k, :3] = ax
          self.cdof[da + skip + k, 3:] = np.cross(ax, off)
      elif t == 2:
        self.cdof[da, 3:] = self.xaxis[j]
      else:
        self.cdof[da, :3] = self.xaxis[j]
        self.cdof[da, 3:] = np.cross(self.xaxis[j], off)
    # spatial inertia at subtree com (6x6) per body
    self.I6 = np.zeros((nb, 6, 6))
    for i in range(1, nb):
      R = self.ximat[i]
      Ic = R @ np.diag(m.body_inertia[i]) @ R.T
      c = self.xipos[i] - com[m.body_rootid[i]]
      mass = m.body_mass[i]
      cx = np.array([[0, -c[2], c[1]], [c[2], 0, -c[0]], [-c[1], c[0], 0]])
      I6 = np.zeros((6, 6))
      I6[:3, :3] = Ic - mass * cx @ cx
      I6[:3, 3:] = mass * cx
      I6[3:, :3] = -mass * cx
      I6[3:, 3:] = mass * np.eye(3)
      self.I6[i] = I6
    # composite inertia and dense M
    crb = self.I6.copy()
    for i in range(nb - 1, 0, -1):
      if m.body_parentid[i] > 0:
        crb[m.body_parentid[i]] += crb[i]
    self.crb = crb
    M = np.zeros((m.nv, m.nv))
    for i in range(m.nv):
      buf = crb[m.dof_bodyid[i]] @ self.cdof[i]
      j = i
      while j >= 0:
        M[i, j] = M[j, i] = self.cdof[j] @ buf
        j = m.dof_parentid[j]
      M[i, i] += m.dof_armature[i]
    self.M = M

  def jac_point(self, m, body, point):
    """mj_jac (engine_support.c:389-441): 3 x nv translation and rotation Jacobians."""
    jacp = np.zeros((3, m.nv))
    jacr = np.zeros((3, m.nv))
    if m.body_dofnum[body] == 0:
      # walk up to the first ancestor with dofs
      b = body
      while b > 0 and m.body_dofnum[b] == 0:
        b = m.body_parentid[b]
      if b == 0:
        return jacp, jacr
      j = m.body_dofadr[b] + m.body_dofnum[b] - 1
    else:
      j = m.body_dofadr[body] + m.body_dofnum[body] - 1
    off = point - self.subtree_com[m.body_rootid[body]]
    while j >= 0:
      c = self.cdof[j]
      jacr[:, j] = c[:3]
      jacp[:, j] = c[3:] + np.cross(c[:3], off)
      j = m.dof_parentid[j]
    return jacp, jacr


_MINVAL = 1e-15


def _ancestor_dof(m, body, dof):
  """dof belongs to body or one of its ancestors."""
  b = int(body)
  while b > 0:
    if m.body_dofadr[b] <= dof < m.body_dofadr[b] + m.body_dofnum[b]:
      return True
    b = int(m.body_parentid[b])
  return False


def _subquat(qa, qb):
  """mju_subQuat (engine_util_spatial.c): expmap of qb^-1 * qa."""
  return _quat2vel(_mulquat(_quat_neg(qb), qa))


def _norm2(v):
  n = np.sqrt(v[0]*v[0] + v[1]*v[1])
  return np.array([1.0, 0.0]) if n < _MINVAL else v / n


def _intersect(p1, p2, p3, p4):
  """is_intersect (engine_util_misc.c:33-50)."""
  det = (p4[1]-p3[1])*(p2[0]-p1[0]) - (p4[0]-p3[0])*(p2[1]-p1[1])
  if abs(det) < _MINVAL:
    return False
  a = ((p4[0]-p3[0])*(p1[1]-p3[1]) - (p4[1]-p3[1])*(p1[0]-p3[0])) / det
  b = ((p2[0]-p1[0])*(p1[1]-p3[1]) - (p2[1]-p1[1])*(p1[0]-p3[0])) / det
  return 0 <= a <= 1 and 0 <= b <= 1


def _wrap_circle(e0, e1, side, r):
  """wrap_circle + length_circle (engine_util_misc.c:55-151): tangent points, arc length."""
  sq0, sq1, sqr = e0 @ e0, e1 @ e1, r * r
  if sq0 < sqr or sq1 < sqr or r < _MINVAL:
    return None
  dif = e1 - e0
  dd = dif @ dif
  if dd < _MINVAL:
    return None
  a = min(max(-(dif @ e0) / dd, 0.0), 1.0)
  near = a * dif + e0
  if near @ near > sqr and (side is None or side @ near >= 0):
    return None
  s0, s1 = np.sqrt(sq0 - sqr), np.sqrt(sq1 - sqr)
  sols, good = [], []
  for sgn in (1, -1):
    t0 = np.array([e0[0]*sqr + sgn*r*e0[1]*s0, e0[1]*sqr - sgn*r*e0[0]*s0]) / sq0
    t1 = np.array([e1[0]*sqr - sgn*r*e1[1]*s1, e1[1]*sqr + sgn*r*e1[0]*s1]) / sq1
    g = _norm2(t0 + t1) @ side if side is not None else -((t0 - t1) @ (t0 - t1))
    if _intersect(e0, t0, e1, t1):
      g = -10000
    sols.append((t0, t1))
    good.append(g)
  i = 0 if good[0] > good[1] else 1
  t0, t1 = sols[i]
  if _intersect(e0, t0, e1, t1):
    return None
  ang = np.arccos(_norm2(t0) @ _norm2(t1))
  cr = t0[1]*t1[0] - t0[0]*t1[1]
  if (cr > 0 and i) or (cr < 0 and not i):
    ang = 2 * np.pi - ang
  return t0, t1, r * ang


def _wrap_inside(e0, e1, r):
  """wrap_inside (engine_util_misc.c:157-272): the side site inside the circle."""
  l0, l1 = np.sqrt(e0 @ e0), np.sqrt(e1 @ e1)
  dif = e1 - e0
  dd = dif @ dif
  if l0 <= r or l1 <= r or r < _MINVAL or l0 < _MINVAL or l1 < _MINVAL:
    return None
  if dd > _MINVAL:
    a = -(dif @ e0) / dd
    if 0 < a < 1 and np.linalg.norm(e0 + a * dif) <= r:
      return None
  p = _norm2(0.5 * (e0 + e1)) * r
  A, B = r / l0, r / l1
  cosG = (l0*l0 + l1*l1 - dd) / (2*l0*l1)
  if cosG < -1 + _MINVAL:
    return None
  if cosG > 1 - _MINVAL:
    return p, p, 0.0
  G = np.arccos(cosG)
  z = 1 - 1e-7
  f = np.arcsin(A*z) + np.arcsin(B*z) - 2*np.arcsin(z) + G
  if f > 0:
    return p, p, 0.0
  it = 0
  while it < 20 and abs(f) > 1e-6:
    df = (A / max(_MINVAL, np.sqrt(1 - z*z*A*A)) + B / max(_MINVAL, np.sqrt(1 - z*z*B*B))
          - 2 / max(_MINVAL, np.sqrt(1 - z*z)))
    if df > -_MINVAL:
      return p, p, 0.0
    z1 = z - f / df
    if z1 > z:
      return p, p, 0.0
    z = z1
    f = np.arcsin(A*z) + np.arcsin(B*z) - 2*np.arcsin(z) + G
    if f > 1e-6:
      return p, p, 0.0
    it += 1
  if it >= 20:
    return p, p, 0.0
  if e0[0]*e1[1] - e0[1]*e1[0] > 0:
    vec, ang = _norm2(e0), np.arcsin(z) - np.arcsin(A*z)
  else:
    vec, ang = _norm2(e1), np.arcsin(z) - np.arcsin(B*z)
  p = r * np.array([np.cos(ang)*vec[0] - np.sin(ang)*vec[1],
                    np.sin(ang)*vec[0] + np.cos(ang)*vec[1]])
  return p, p, 0.0


def wrap(x0, x1, xpos, xmat, r, wtype, side):
  """mju_wrap (engine_util_misc.c:282-418): (tangent point 0, tangent point 1, length) of
  the segment x0-x1 around a sphere (wtype 4) or cylinder (5), or None when it clears."""
  p0, p1 = xmat.T @ (x0 - xpos), xmat.T @ (x1 - xpos)
  if np.linalg.norm(p0) < _MINVAL or np.linalg.norm(p1) < _MINVAL:
    return None
  if wtype == 4:
    ax0 = p0 / max(np.linalg.norm(p0), _MINVAL)
    n = np.cross(p0, p1)
    if np.linalg.norm(n) < _MINVAL:
      a = np.abs(ax0)
      i = 2 if a[2] > a[0] and a[2] > a[1] else (1 if a[1] > a[0] and a[1] > a[2] else 0)
      ax1 = np.ones(3)
      ax1[i] = 0
      n = np.cross(ax0, ax1)
    n = n / np.linalg.norm(n)
    ax1 = np.cross(n, ax0)
    ax1 = ax1 / np.linalg.norm(ax1)
  else:
    ax0, ax1 = np.array([1.0, 0, 0]), np.array([0, 1.0, 0])
  e0, e1 = np.array([p0 @ ax0, p0 @ ax1]), np.array([p1 @ ax0, p1 @ ax1])
  if side is not None:
    s = xmat.T @ (side - xpos)
    sd = _norm2(np.array([s @ ax0, s @ ax1])) * r
    out = _wrap_inside(e0, e1, r) if np.linalg.norm(s) < r else _wrap_circle(e0, e1, sd, r)
  else:
    out = _wrap_circle(e0, e1, None, r)
  if out is None:
    return None
  t0, t1, wlen = out
  r0, r1 = ax0 * t0[0] + ax1 * t0[1], ax0 * t1[0] + ax1 * t1[1]
  if wtype == 5:
    L0 = np.hypot(p0[0] - r0[0], p0[1] - r0[1])
    L1 = np.hypot(p1[0] - r1[0], p1[1] - r1[1])
    r0[2] = p0[2] + (p1[2] - p0[2]) * L0 / (L0 + wlen + L1)
    r1[2] = p0[2] + (p1[2] - p0[2]) * (L0 + wlen) / (L0 + wlen + L1)
    wlen = np.sqrt(wlen * wlen + (r1[2] - r0[2]) ** 2)
  return xmat @ r0 + xpos, xmat @ r1 + xpos, wlen


def set_const(m):
  """Fill the compile-time constants of `m` in place (mj_setConst subset)."""
  nv, nb = m.nv, m.nbody
  # subtree mass
  stm = m.body_mass.astype(np.float64).copy()
  for i in range(nb - 1, 0, -1):
    stm[m.body_parentid[i]] += stm[i]
  m.body_subtreemass[:] = stm
  e = _Eval(m, m.qpos0.astype(np.float64))
  # dof_M0 (mj_setM0): armature + cdof_i . (crb_i cdof_i)
  for i in range(nv):
    m.dof_M0[i] = m.dof_armature[i] + e.cdof[i] @ (e.crb[m.dof_bodyid[i]] @ e.cdof[i])
  Minv = np.linalg.inv(e.M) if nv else np.zeros((0, 0))
  # body_invweight0
  m.body_invweight0[:] = 0
  for i in range(1, nb):
    if m.body_weldid[i] == 0:
      continue
    if m.body_simple[i] == 2:
      m.body_invweight0[i] = [1 / max(1e-15, m.body_mass[i]), 0]
      continue
    jacp, jacr = e.jac_point(m, i, e.xipos[i])
    J = np.vstack([jacp, jacr])
    A = J @ Minv @ J.T if nv else np.zeros((6, 6))
    m.body_invweight0[i, 0] = (A[0, 0] + A[1, 1] + A[2, 2]) / 3
    m.body_invweight0[i, 1] = (A[3, 3] + A[4, 4] + A[5, 5]) / 3
  # dof_invweight0
  for j in range(m.njnt):
    da = m.jnt_dofadr[j]
    bi = m.jnt_bodyid[j]
    if m.body_simple[bi] == 2:
      m.dof_invweight0[da] = 1 / max(1e-15, m.body_mass[bi])
      continue
    t = m.jnt_type[j]
    dn = {0: 6, 1: 3}.get(int(t), 1)
    A = Minv[da:da+dn, da:da+dn]
    if dn == 6:
      m.dof_invweight0[da:da+3] = np.trace(A[:3, :3]) / 3
      m.dof_invweight0[da+3:da+6] = np.trace(A[3:, 3:]) / 3
    elif dn == 3:
      m.dof_invweight0[da:da+3] = np.trace(A) / 3
    else:
      m.dof_invweight0[da] = A[0, 0]
  # tendons: length and dense J (mj_tendon, engine_core_smooth.c:651-860; spatial paths
  # through sites and pulleys)
  def tendon(q, ev):
    L = np.zeros(m.ntendon)
    J = np.zeros((m.ntendon, nv))
    for t in range(m.ntendon):
      adr, num = m.tendon_adr[t], m.tendon_num[t]
      if m.wrap_type[adr] == 1:
        for w in range(adr, adr + num):
          k = m.wrap_objid[w]
          L[t] += m.wrap_prm[w] * q[m.jnt_qposadr[k]]
          J[t, m.jnt_dofadr[k]] = m.wrap_prm[w]
        continue
      divisor = 1.0
      site = lambda s: ev.xmat[m.site_bodyid[s]] @ m.site_pos[s] + ev.xpos[m.site_bodyid[s]]
      w = adr
      while w < adr + num - 1:
        if m.wrap_type[w] == 2 or m.wrap_type[w + 1] == 2:
          if m.wrap_type[w] == 2:
            divisor = m.wrap_prm[w]
          w += 1
          continue
        wrapped = m.wrap_type[w + 1] in (4, 5)
        s0, s1 = m.wrap_objid[w], m.wrap_objid[w + (2 if wrapped else 1)]
        pts, bodies = [site(s0)], [m.site_bodyid[s0]]
        out = None
        if wrapped:
          g = m.wrap_objid[w + 1]
          gb = m.geom_bodyid[g]
          gpos = ev.xmat[gb] @ m.geom_pos[g] + ev.xpos[gb]
          gmat = _quat2mat(_normq(_mulquat(ev.xquat[gb], m.geom_quat[g])))
          sid = int(round(m.wrap_prm[w + 1]))
          out = wrap(pts[0], site(s1), gpos, gmat, m.geom_size[g, 0], m.wrap_type[w + 1],
                     site(sid) if sid >= 0 else None)
        if out is None:
          pts.append(site(s1))
          bodies.append(m.site_bodyid[s1])
          L[t] += np.linalg.norm(pts[1] - pts[0]) / divisor
        else:
          pts += [out[0], out[1], site(s1)]
          bodies += [gb, gb, m.site_bodyid[s1]]
          L[t] += (np.linalg.norm(pts[1] - pts[0]) + out[2]
                   + np.linalg.norm(pts[3] - pts[2])) / divisor
        for k in range(len(pts) - 1):
          if bodies[k] == bodies[k + 1]:
            continue
          dif = pts[k + 1] - pts[k]
          n = np.linalg.norm(dif)
          dif = dif / n if n >= 1e-15 else np.array([1.0, 0, 0])
          j0, _ = ev.jac_point(m, bodies[k], pts[k])
          j1, _ = ev.jac_point(m, bodies[k + 1], pts[k + 1])
          J[t] += (dif @ (j1 - j0)) / divisor
        w += 2 if wrapped else 1
    return L, J
  L0, J0 = tendon(m.qpos0, e)
  m.tendon_length0[:] = L0
  for t in range(m.ntendon):
    m.tendon_invweight0[t] = J0[t] @ Minv @ J0[t] if nv else 0.0
  # actuators: mj_transmission at qpos0 (engine_core_smooth.c:884-1081), dense moment
  for a in range(m.nu):
    tid = m.actuator_trnid[a, 0]
    gear = m.actuator_gear[a]
    mom = np.zeros(nv)
    if m.actuator_trntype[a] in (0, 1):
      jt, qa, da = m.jnt_type[tid], m.jnt_qposadr[tid], m.jnt_dofadr[tid]
      inparent = m.actuator_trntype[a] == 1
      if jt in (2, 3):
        length = m.qpos0[qa] * gear[0]
        mom[da] = gear[0]
      elif jt == 1:
        quat = m.qpos0[qa:qa + 4] / np.linalg.norm(m.qpos0[qa:qa + 4])
        ga = _rot_vec_quat(gear[:3], _quat_neg(quat)) if inparent else gear[:3]
        length = float(_quat2vel(quat) @ ga)
        mom[da:da + 3] = ga
      else:
        quat = m.qpos0[qa + 3:qa + 7] / np.linalg.norm(m.qpos0[qa + 3:qa + 7])
        ga = _rot_vec_quat(gear[3:], _quat_neg(quat)) if inparent else gear[3:]
        length = 0.0
        mom[da:da + 3] = gear[:3]
        mom[da + 3:da + 6] = ga
    elif m.actuator_trntype[a] == 2:   # slider-crank (:1000-1052)
      def site(s):
        b = m.site_bodyid[s]
        return e.xmat[b] @ m.site_pos[s] + e.xpos[b], \
            _quat2mat(_mulquat(e.xquat[b], m.site_quat[s]))
      sl = m.actuator_trnid[a, 1]
      ps, ms = site(sl)
      pc, _ = site(tid)
      axis = ms[:, 2]
      vec = pc - ps
      av = vec @ axis
      rod = m.actuator_cranklength[a]
      det = av * av + rod * rod - vec @ vec
      if det <= 0:
        length, dlda, dldv = av, vec, axis
      else:
        sdet = np.sqrt(det)
        length = av - sdet
        dldv = axis * (1 - av / sdet) + vec / sdet
        dlda = vec * (1 - av / sdet)
      jS, jr = e.jac_point(m, m.site_bodyid[sl], ps)
      jA = np.cross(jr.T, axis).T                       # mj_jacPointAxis
      jC, _ = e.jac_point(m, m.site_bodyid[tid], pc)
      length = length * gear[0]
      mom = (dlda @ jA + dldv @ (jC - jS)) * gear[0]
    elif m.actuator_trntype[a] == 4 and m.actuator_trnid[a, 1] < 0:   # site (:1092-1102)
      b = m.site_bodyid[tid]
      p = e.xmat[b] @ m.site_pos[tid] + e.xpos[b]
      R = _quat2mat(_mulquat(e.xquat[b], m.site_quat[tid]))
      jp, jr = e.jac_point(m, b, p)
      length = 0.0
      mom = jp.T @ (R @ gear[:3]) + jr.T @ (R @ gear[3:])
    elif m.actuator_trntype[a] == 4:   # site relative to a reference site (:1105-1212)
      rid = m.actuator_trnid[a, 1]
      b, br = m.site_bodyid[tid], m.site_bodyid[rid]
      p = e.xmat[b] @ m.site_pos[tid] + e.xpos[b]
      pr = e.xmat[br] @ m.site_pos[rid] + e.xpos[br]
      q = _mulquat(m.site_quat[tid], e.xquat[b])
      qr = _mulquat(m.site_quat[rid], e.xquat[br])
      Rr = _quat2mat(_mulquat(e.xquat[br], m.site_quat[rid]))
      jp, jr = e.jac_point(m, b, p)
      jpr, jrr = e.jac_point(m, br, pr)
      chain = lambda body: {d for d in range(nv) if _ancestor_dof(m, body, d)}
      shared = sorted(chain(b) & chain(br))
      djp, djr = jp - jpr, jr - jrr
      djp[:, shared] = 0
      djr[:, shared] = 0
      length = (Rr.T @ (p - pr)) @ gear[:3] + _subquat(q, qr) @ gear[3:]
      mom = djp.T @ (Rr @ gear[:3]) + djr.T @ (Rr @ gear[3:])
    elif m.actuator_trntype[a] == 5:   # body (adhesion): no length; the moment needs the
      length = 0.0                     # contacts at qpos0, which the compiler does not make
      mom = np.zeros(nv)
    else:
      length = L0[tid] * gear[0]
      mom = J0[tid] * gear[0]
    m.actuator_length0[a] = length
    m.actuator_acc0[a] = np.linalg.norm(Minv @ mom) if nv else 0.0
  # missing eq_data of body constraints (engine_setconst.c:289-340)
  for i in range(m.sizes.get("neq", 0)):
    id1, id2 = m.eq_obj1id[i], m.eq_obj2id[i]
    data = m.eq_data[i]
    if m.eq_type[i] == 0:                   # connect
      if m.eq_objtype[i] == 1:
        pos = e.xmat[id1] @ data[0:3] + e.xpos[id1]
        data[3:6] = e.xmat[id2].T @ (pos - e.xpos[id2])
      else:
        data[:] = 0
    elif m.eq_type[i] == 1 and m.eq_objtype[i] == 1:   # weld, body semantic
      if np.any(data[6:10] != 0):
        data[6:10] = data[6:10] / np.linalg.norm(data[6:10])
        continue
      pos = e.xmat[id2] @ data[0:3] + e.xpos[id2]
      data[3:6] = e.xmat[id1].T @ (pos - e.xpos[id1])
      q1 = e.xquat[id1] * np.array([1, -1, -1, -1])
      data[6:10] = _mulquat(q1, e.xquat[id2])
  # cameras / lights at qpos0 in fixed mode (engine_setconst.c:346-373)
  for c in range(m.ncam):
    b = m.cam_bodyid[c]
    pos = e.xmat[b] @ m.cam_pos[c] + e.xpos[b]
    mat = _quat2mat(_mulquat(e.xquat[b], m.cam_quat[c]))
    t = m.cam_targetbodyid[c]
    m.cam_pos0[c] = pos - e.xpos[b]
    m.cam_poscom0[c] = pos - e.subtree_com[t if t >= 0 else b]
    m.cam_mat0[c] = mat.reshape(9)
  for l in range(m.nlight):
    b = m.light_bodyid[l]
    pos = e.xmat[b] @ m.light_pos[l] + e.xpos[b]
    d = _rot(m.light_dir[l], e.xquat[b])
    n = np.linalg.norm(d)
    d = d / n if n >= 1e-15 else np.array([1.0, 0, 0])
    t = m.light_targetbodyid[l]
    m.light_pos0[l] = pos - e.xpos[b]
    m.light_poscom0[l] = pos - e.subtree_com[t if t >= 0 else b]
    m.light_dir0[l] = d
  # tendon spring length at qpos_spring (setSpring)
  Ls, _ = tendon(m.qpos_spring, _Eval(m, m.qpos_spring.astype(np.float64)))
  for t in range(m.ntendon):
    if m.tendon_lengthspring[t, 0] == -1 and m.tendon_lengthspring[t, 1] == -1:
      m.tendon_lengthspring[t] = Ls[t]
  return m
