"""MJCF-subset model compiler: XML -> compiled model arrays with mjModel field names.

The reference's model compiler (src/user, src/xml) cannot be built offline (it needs
tinyxml2/qhull/lodepng/... that CMake would fetch: SURVEY.md §8c), so this module restates
the compiler semantics the inverse-dynamics path depends on, for the MJCF subset used by
model/humanoid/humanoid.xml, src/inverse/test.xml and the reference's inverse/inertia/
derivative test models. Reference semantics followed:

  * default classes / childclass resolution         src/xml/xml_native_reader.cc
  * body tree, rootid/weldid, sameframe, simple       src/user/user_model.cc:2174-2380
  * qpos0 / qpos_spring                               src/user/user_model.cc:2300-2325
  * dof_Madr, nM, nD, dof_simplenum, nC               src/user/user_model.cc:2539-2617
  * joint compile (limits deg->rad, axis normalize)   src/user/user_objects.cc:2149-2260
  * geom fromto / orientation / volume / inertia      src/user/user_objects.cc:2384-2560, 2911-3080
  * body inertial frame from geoms (+eig3)            src/user/user_objects.cc:1507-1575, 1637-1735
  * orientation alternatives                          src/user/user_objects.cc:240-350
  * math helpers (z2quat, frame2quat, eig3, ...)      src/user/user_util.cc:149-800
  * nJmom                                              src/user/user_model.cc:2703-2750
  * C sparse structure, mapM2C                        src/engine/engine_io.c:929-1018, 1135-1259

Model constants computed by mj_setConst (dof_M0, *_invweight0, tendon_length0,
lengthspring, cam/light offsets) are filled by setconst.py.

Compiled-model parity against MuJoCo's own compiler is UNPINNED: no reference test pins
compiled humanoid masses/inertias and the compiler cannot run here.
"""
from __future__ import annotations

import math
import os
import xml.etree.ElementTree as ET

import numpy as np

from . import fields

mjPI = 3.14159265358979323846
mjEPS = 1e-14          # src/user/user_util.h:25
kFrameEps = 1e-6       # src/user/user_model.cc:62
kEigEPS = 1e-12        # src/user/user_util.cc:649

JNT = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}
# mjtObj (mjmodel.h) as mju_str2Type (engine_util_misc.c:1133-1236) spells them
OBJ = {"body": 1, "xbody": 2, "joint": 3, "dof": 4, "geom": 5, "site": 6, "camera": 7,
       "light": 8, "tendon": 18, "actuator": 19}
# MJCF sensor element -> (mjtSensor, object attribute, mjtObj, dim, mjtDataType, mjtStage),
# per xml_native_reader.cc:3864-4180 (element -> type/objtype) and user_objects.cc:6250-6580
# (dim, datatype, needstage). Stages: 1 POS, 2 VEL, 3 ACC. Datatypes: 0 REAL, 1 POSITIVE,
# 2 AXIS, 3 QUATERNION. Frame sensors read objtype/objname (+ reftype/refname).
SENSORS = {
    "touch": (0, "site", 6, 1, 1, 3), "rangefinder": (7, "site", 6, 1, 1, 1),
    "camprojection": (8, "site", 6, 2, 0, 1),
    # geom distance (geom1|body1, geom2|body2; xml_native_reader.cc:4105-4116)
    "distance": (37, "geom1", None, 1, 1, 1), "normal": (38, "geom1", None, 3, 2, 1),
    "fromto": (39, "geom1", None, 6, 0, 1),
    "accelerometer": (1, "site", 6, 3, 0, 3), "velocimeter": (2, "site", 6, 3, 0, 2),
    "gyro": (3, "site", 6, 3, 0, 2), "force": (4, "site", 6, 3, 0, 3),
    "torque": (5, "site", 6, 3, 0, 3), "magnetometer": (6, "site", 6, 3, 0, 1),
    "jointpos": (9, "joint", 3, 1, 0, 1), "jointvel": (10, "joint", 3, 1, 0, 2),
    "tendonpos": (11, "tendon", 18, 1, 0, 1), "tendonvel": (12, "tendon", 18, 1, 0, 2),
    "actuatorpos": (13, "actuator", 19, 1, 0, 1), "actuatorvel": (14, "actuator", 19, 1, 0, 2),
    "actuatorfrc": (15, "actuator", 19, 1, 0, 3),
    "jointactuatorfrc": (16, "joint", 3, 1, 0, 3),
    "ballquat": (17, "joint", 3, 4, 3, 1), "ballangvel": (18, "joint", 3, 3, 0, 2),
    "jointlimitpos": (19, "joint", 3, 1, 0, 1), "jointlimitvel": (20, "joint", 3, 1, 0, 2),
    "jointlimitfrc": (21, "joint", 3, 1, 0, 3),
    "tendonlimitpos": (22, "tendon", 18, 1, 0, 1), "tendonlimitvel": (23, "tendon", 18, 1, 0, 2),
    "tendonlimitfrc": (24, "tendon", 18, 1, 0, 3),
    "framepos": (25, None, None, 3, 0, 1), "framequat": (26, None, None, 4, 3, 1),
    "framexaxis": (27, None, None, 3, 2, 1), "frameyaxis": (28, None, None, 3, 2, 1),
    "framezaxis": (29, None, None, 3, 2, 1), "framelinvel": (30, None, None, 3, 0, 2),
    "frameangvel": (31, None, None, 3, 0, 2), "framelinacc": (32, None, None, 3, 0, 3),
    "frameangacc": (33, None, None, 3, 0, 3),
    "subtreecom": (34, "body", 1, 3, 0, 1), "subtreelinvel": (35, "body", 1, 3, 0, 2),
    "subtreeangmom": (36, "body", 1, 3, 0, 2),
    "e_potential": (40, None, 0, 1, 0, 1), "e_kinetic": (41, None, 0, 1, 0, 1),
    "clock": (42, None, 0, 1, 0, 1),
}
SENSORS_NEXT = ("user", "plugin")
GEOM = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4,
        "cylinder": 5, "box": 6, "mesh": 7, "sdf": 8}
CAMLIGHT = {"fixed": 0, "track": 1, "trackcom": 2, "targetbody": 3, "targetbodycom": 4}
INTEGRATOR = {"Euler": 0, "RK4": 1, "implicit": 2, "implicitfast": 3}
JACOBIAN = {"dense": 0, "sparse": 1, "auto": 2}
CONE = {"pyramidal": 0, "elliptic": 1}
DISABLE = {"constraint": 0, "equality": 1, "frictionloss": 2, "limit": 3, "contact": 4,
           "passive": 5, "gravity": 6, "clampctrl": 7, "warmstart": 8, "filterparent": 9,
           "actuation": 10, "refsafe": 11, "sensor": 12, "midphase": 13, "eulerdamp": 14,
           "autoreset": 15, "nativeccd": 16}
ENABLE = {"override": 0, "energy": 1, "fwdinv": 2, "invdiscrete": 3, "multiccd": 4,
          "island": 5}


class MJCFError(ValueError):
  pass


#--------------------------------- compiler math (src/user/user_util.cc) -------------------

def normvec(v):
  """mjuu_normvec (user_util.cc:149): normalize unless within mjEPS of unit length."""
  nrm = 0.0
  for x in v:
    nrm += x * x
  if nrm < mjEPS:
    return 0.0
  nrm = math.sqrt(nrm)
  if abs(nrm - 1) > mjEPS:
    for i in range(len(v)):
      v[i] /= nrm
  return nrm


def quat2mat(q):
  """mjuu_quat2mat (user_util.cc:196)."""
  if q[0] == 1 and q[1] == 0 and q[2] == 0 and q[3] == 0:
    return [1.0, 0, 0, 0, 1.0, 0, 0, 0, 1.0]
  q00 = q[0]*q[0]; q01 = q[0]*q[1]; q02 = q[0]*q[2]; q03 = q[0]*q[3]
  q11 = q[1]*q[1]; q12 = q[1]*q[2]; q13 = q[1]*q[3]
  q22 = q[2]*q[2]; q23 = q[2]*q[3]; q33 = q[3]*q[3]
  r = [0.0] * 9
  r[0] = q00 + q11 - q22 - q33
  r[4] = q00 - q11 + q22 - q33
  r[8] = q00 - q11 - q22 + q33
  r[1] = 2*(q12 - q03)
  r[2] = 2*(q13 + q02)
  r[3] = 2*(q12 + q03)
  r[5] = 2*(q23 - q01)
  r[6] = 2*(q13 - q02)
  r[7] = 2*(q23 + q01)
  return r


def mulquat(qa, qb):
  """mjuu_mulquat (user_util.cc:239): product, normalized."""
  t = [qa[0]*qb[0] - qa[1]*qb[1] - qa[2]*qb[2] - qa[3]*qb[3],
       qa[0]*qb[1] + qa[1]*qb[0] + qa[2]*qb[3] - qa[3]*qb[2],
       qa[0]*qb[2] - qa[1]*qb[3] + qa[2]*qb[0] + qa[3]*qb[1],
       qa[0]*qb[3] + qa[1]*qb[2] - qa[2]*qb[1] + qa[3]*qb[0]]
  normvec(t)
  return t


def crossvec(a, b):
  return [a[1]*b[2] - a[2]*b[1], a[2]*b[0] - a[0]*b[2], a[0]*b[1] - a[1]*b[0]]


def z2quat(vec):
  """mjuu_z2quat (user_util.cc:384): minimal rotation from (0,0,1) to vec."""
  q = [0.0] + crossvec([0.0, 0.0, 1.0], vec)
  v = q[1:]
  s = normvec(v)
  q[1:] = v
  if s < 1e-10:
    q[1] = 1.0
    q[2] = q[3] = 0.0
  ang = math.atan2(s, vec[2])
  q[0] = math.cos(ang/2)
  q[1] *= math.sin(ang/2)
  q[2] *= math.sin(ang/2)
  q[3] *= math.sin(ang/2)
  return q


def frame2quat(x, y, z):
  """mjuu_frame2quat (user_util.cc:401); axes are matrix columns."""
  mat = [x, y, z]
  q = [0.0] * 4
  if mat[0][0] + mat[1][1] + mat[2][2] > 0:
    q[0] = 0.5 * math.sqrt(1 + mat[0][0] + mat[1][1] + mat[2][2])
    q[1] = 0.25 * (mat[1][2] - mat[2][1]) / q[0]
    q[2] = 0.25 * (mat[2][0] - mat[0][2]) / q[0]
    q[3] = 0.25 * (mat[0][1] - mat[1][0]) / q[0]
  elif mat[0][0] > mat[1][1] and mat[0][0] > mat[2][2]:
    q[1] = 0.5 * math.sqrt(1 + mat[0][0] - mat[1][1] - mat[2][2])
    q[0] = 0.25 * (mat[1][2] - mat[2][1]) / q[1]
    q[2] = 0.25 * (mat[1][0] + mat[0][1]) / q[1]
    q[3] = 0.25 * (mat[2][0] + mat[0][2]) / q[1]
  elif mat[1][1] > mat[2][2]:
    q[2] = 0.5 * math.sqrt(1 - mat[0][0] + mat[1][1] - mat[2][2])
    q[0] = 0.25 * (mat[2][0] - mat[0][2]) / q[2]
    q[1] = 0.25 * (mat[1][0] + mat[0][1]) / q[2]
    q[3] = 0.25 * (mat[2][1] + mat[1][2]) / q[2]
  else:
    q[3] = 0.5 * math.sqrt(1 - mat[0][0] - mat[1][1] + mat[2][2])
    q[0] = 0.25 * (mat[0][1] - mat[1][0]) / q[3]
    q[1] = 0.25 * (mat[2][0] + mat[0][2]) / q[3]
    q[2] = 0.25 * (mat[2][1] + mat[1][2]) / q[3]
  normvec(q)
  return q


def mulvecmat(vec, mat):
  """mjuu_mulvecmat (user_util.cc:251): mat * vec (3x3 row-major)."""
  return [mat[0]*vec[0] + mat[1]*vec[1] + mat[2]*vec[2],
          mat[3]*vec[0] + mat[4]*vec[1] + mat[5]*vec[2],
          mat[6]*vec[0] + mat[7]*vec[1] + mat[8]*vec[2]]


def rotvecquat(vec, quat):
  """mjuu_rotVecQuat (user_util.cc:572): v + 2 q_xyz x (q_w v + q_xyz x v)."""
  if vec[0] == 0 and vec[1] == 0 and vec[2] == 0:
    return [0.0, 0.0, 0.0]
  if quat[0] == 1 and quat[1] == 0 and quat[2] == 0 and quat[3] == 0:
    return list(vec)
  t = [quat[0]*vec[0] + quat[2]*vec[2] - quat[3]*vec[1],
       quat[0]*vec[1] + quat[3]*vec[0] - quat[1]*vec[2],
       quat[0]*vec[2] + quat[1]*vec[1] - quat[2]*vec[0]]
  return [vec[0] + 2 * (quat[2]*t[2] - quat[3]*t[1]),
          vec[1] + 2 * (quat[3]*t[0] - quat[1]*t[2]),
          vec[2] + 2 * (quat[1]*t[1] - quat[2]*t[0])]


def frameaccum(pos, quat, childpos, childquat):
  """mjuu_frameaccum (user_util.cc:458): the child frame expressed through (pos, quat);
  returns the new (pos, quat). mjuu_frameaccumChild (:472) is the same with the result
  stored in the child."""
  vec = mulvecmat(childpos, quat2mat(quat))
  return [pos[0] + vec[0], pos[1] + vec[1], pos[2] + vec[2]], mulquat(quat, childquat)


def globalinertia(local, quat):
  """mjuu_globalinertia (user_util.cc:498)."""
  mat = quat2mat(quat)
  tmp = [mat[0]*local[0], mat[3]*local[0], mat[6]*local[0],
         mat[1]*local[1], mat[4]*local[1], mat[7]*local[1],
         mat[2]*local[2], mat[5]*local[2], mat[8]*local[2]]
  return [mat[0]*tmp[0] + mat[1]*tmp[3] + mat[2]*tmp[6],
          mat[3]*tmp[1] + mat[4]*tmp[4] + mat[5]*tmp[7],
          mat[6]*tmp[2] + mat[7]*tmp[5] + mat[8]*tmp[8],
          mat[0]*tmp[1] + mat[1]*tmp[4] + mat[2]*tmp[7],
          mat[0]*tmp[2] + mat[1]*tmp[5] + mat[2]*tmp[8],
          mat[3]*tmp[2] + mat[4]*tmp[5] + mat[5]*tmp[8]]


def offcenter(mass, vec):
  """mjuu_offcenter (user_util.cc:519)."""
  return [mass*(vec[1]*vec[1] + vec[2]*vec[2]),
          mass*(vec[0]*vec[0] + vec[2]*vec[2]),
          mass*(vec[0]*vec[0] + vec[1]*vec[1]),
          -mass*vec[0]*vec[1],
          -mass*vec[0]*vec[2],
          -mass*vec[1]*vec[2]]


def _mulmat(a, b):
  return [sum(a[3*i+k]*b[3*k+j] for k in range(3)) for i in range(3) for j in range(3)]


def _mulmat_ordered(a, b):
  # mjuu_mulmat: res[i,j] = a[i,0]*b[0,j] + a[i,1]*b[1,j] + a[i,2]*b[2,j]
  r = [0.0] * 9
  for i in range(3):
    for j in range(3):
      r[3*i+j] = a[3*i]*b[j] + a[3*i+1]*b[3+j] + a[3*i+2]*b[6+j]
  return r


def _transpose(a):
  return [a[0], a[3], a[6], a[1], a[4], a[7], a[2], a[5], a[8]]


def eig3(mat):
  """mjuu_eig3 (user_util.cc:650): Jacobi eigen-decomposition, eigenvalues descending."""
  quat = [1.0, 0.0, 0.0, 0.0]
  eigval = [0.0] * 3
  for _ in range(500):
    eigvec = quat2mat(quat)
    tmp = _mulmat_ordered(_transpose(eigvec), mat)
    D = _mulmat_ordered(tmp, eigvec)
    eigval = [D[0], D[4], D[8]]
    if abs(D[1]) > abs(D[2]) and abs(D[1]) > abs(D[5]):
      rk, ck, rotk = 0, 1, 2
    elif abs(D[2]) > abs(D[5]):
      rk, ck, rotk = 0, 2, 1
    else:
      rk, ck, rotk = 1, 2, 0
    if abs(D[3*rk+ck]) < kEigEPS:
      break
    tau = (D[4*ck] - D[4*rk]) / (2*D[3*rk+ck])
    if tau >= 0:
      t = 1.0/(tau + math.sqrt(1 + tau*tau))
    else:
      t = -1.0/(-tau + math.sqrt(1 + tau*tau))
    c = 1.0/math.sqrt(1 + t*t)
    if c > 1.0 - kEigEPS:
      break
    q = [0.0, 0.0, 0.0, 0.0]
    q[rotk+1] = -math.sqrt(0.5-0.5*c) if tau >= 0 else math.sqrt(0.5-0.5*c)
    if rotk == 1:
      q[rotk+1] = -q[rotk+1]
    q[0] = math.sqrt(1.0 - q[rotk+1]*q[rotk+1])
    normvec(q)
    quat = mulquat(quat, q)
    normvec(quat)
  for j in range(3):
    j1 = j % 2
    if eigval[j1] + kEigEPS < eigval[j1+1]:
      eigval[j1], eigval[j1+1] = eigval[j1+1], eigval[j1]
      q = [0.707106781186548, 0.0, 0.0, 0.0]
      q[(j1+2) % 3 + 1] = q[0]
      quat = mulquat(quat, q)
      normvec(quat)
  return eigval, quat


def full_inertia(full6):
  """mjuu_fullInertia (user_util.cc:774)."""
  full = [full6[0], full6[3], full6[4],
          full6[3], full6[1], full6[5],
          full6[4], full6[5], full6[2]]
  eigval, quat = eig3(full)
  if eigval[2] < mjEPS:
    raise MJCFError("inertia must have positive eigenvalues")
  return quat, eigval


def is_same_vec(a, b):
  return all(abs(a[i] - b[i]) < kFrameEps for i in range(3))


def is_same_quat(a, b):
  minus = all(abs(a[i] - b[i]) < kFrameEps for i in range(4))
  plus = all(abs(a[i] + b[i]) < kFrameEps for i in range(4))
  return minus or plus


def is_same_pose(p1, p2, q1, q2):
  """IsSamePose (user_model.cc:95)."""
  if p1 is not None and p2 is not None and not is_same_vec(p1, p2):
    return False
  if q1 is not None and q2 is not None and not is_same_quat(q1, q2):
    return False
  return True


def is_null_pose(p, q):
  return is_same_pose(p, [0, 0, 0] if p is not None else None, q,
                      [1, 0, 0, 0] if q is not None else None)


#--------------------------------- XML helpers ---------------------------------------------

def _floats(s):
  return [float(x) for x in s.split()]


class _Defaults:
  """One default class: per-element attribute dicts, inheriting from the parent class."""

  def __init__(self, name, parent=None):
    self.name = name
    self.parent = parent
    self.attrs = {}  # element tag -> {attr: str}

  def get(self, tag):
    out = dict(self.parent.get(tag)) if self.parent else {}
    out.update(self.attrs.get(tag, {}))
    return out


ACTUATOR_TAGS = ("general", "motor", "position", "velocity", "intvelocity", "adhesion")

# name references of the referencing elements an <attach>/<replicate> namespaces (attribute
# -> kind of object it names; mjCEquality/mjCActuator/mjCSensor::NameSpace,
# user_objects.cc:5119, 5811, 6147)
EQ_REFS = {"body1": "body", "body2": "body", "joint1": "joint", "joint2": "joint",
           "tendon1": "tendon", "tendon2": "tendon", "site1": "site", "site2": "site"}
ACT_REFS = {"joint": "joint", "jointinparent": "joint", "tendon": "tendon", "site": "site",
            "refsite": "site", "body": "body", "cranksite": "site", "slidersite": "site"}
SENSOR_REFS = {"site": "site", "joint": "joint", "tendon": "tendon", "actuator": "actuator",
               "body": "body", "geom1": "geom", "geom2": "geom", "body1": "body",
               "body2": "body", "objname": "any", "refname": "any"}


def _prefixed(a, prefix, keys, suffix=""):
  """A copy of attribute dict `a` with the non-empty names under `keys` namespaced
  (mjCBase::NameSpace, user_objects.cc:707-714)."""
  return {k: (prefix + v + suffix if k in keys and isinstance(v, str) and v else v)
          for k, v in a.items()}


def _namespace(b, prefix, suffix, own=True):
  """mjCBody::NameSpace_ (user_objects.cc:1129-1175) over a parsed subtree, in place: the
  body's name (unless own=False), its elements' names and its descendants'."""
  if own and b.name:
    b.name = prefix + b.name + suffix
    b.attrs["name"] = b.name
  for lst in (b.joints, b.geoms, b.sites, b.cams, b.lights):
    for a in lst:
      if a.get("name"):
        a["name"] = prefix + a["name"] + suffix
  for c in b.children:
    _namespace(c, prefix, suffix)


def _resolve_orientation(attrs, degree, eulerseq, quat):
  """ResolveOrientation (user_objects.cc:240) for axisangle/xyaxes/zaxis/euler."""
  if "axisangle" in attrs:
    aa = _floats(attrs["axisangle"])
    if degree:
      aa[3] = aa[3] / 180.0 * mjPI
    ax = aa[:3]
    if normvec(ax) < mjEPS:
      raise MJCFError("axisangle too small")
    ang2 = aa[3]/2
    return [math.cos(ang2), math.sin(ang2)*ax[0], math.sin(ang2)*ax[1], math.sin(ang2)*ax[2]]
  if "xyaxes" in attrs:
    xy = _floats(attrs["xyaxes"])
    x = xy[:3]
    y = xy[3:]
    if normvec(x) < mjEPS:
      raise MJCFError("xaxis too small")
    d = x[0]*y[0] + x[1]*y[1] + x[2]*y[2]
    y[0] -= x[0]*d
    y[1] -= x[1]*d
    y[2] -= x[2]*d
    if normvec(y) < mjEPS:
      raise MJCFError("yaxis too small")
    z = crossvec(x, y)
    if normvec(z) < mjEPS:
      raise MJCFError("cross(xaxis, yaxis) too small")
    return frame2quat(x, y, z)
  if "zaxis" in attrs:
    z = _floats(attrs["zaxis"])
    if normvec(z) < mjEPS:
      raise MJCFError("zaxis too small")
    return z2quat(z)
  if "euler" in attrs:
    return _euler_quat(_floats(attrs["euler"]), degree, eulerseq)
  return quat


def _euler_quat(eu, degree, eulerseq):
  """The euler branch of ResolveOrientation (user_objects.cc:300-330)."""
  if degree:
    eu = [e / 180.0 * mjPI for e in eu]
  q = [1.0, 0.0, 0.0, 0.0]
  for i in range(3):
    qrot = [math.cos(eu[i]/2), 0.0, 0.0, 0.0]
    sa = math.sin(eu[i]/2)
    ax = eulerseq[i]
    qrot["xyz".index(ax.lower()) + 1] = sa
    if ax.islower():   # moving axes: post-multiply
      q = mulquat(q, qrot)
    else:              # fixed axes: pre-multiply
      q = mulquat(qrot, q)
  return q


#--------------------------------- compiled objects ----------------------------------------

class Body:
  def __init__(self, parent, attrs, cls, childclass):
    self.parent = parent
    self.attrs = attrs
    self.cls = cls
    self.childclass = childclass
    self.children = []
    self.joints = []
    self.geoms = []
    self.sites = []
    self.cams = []
    self.lights = []
    self.inertial = None
    self.id = -1
    self.name = attrs.get("name", "")
    self.frame = None              # the <frame> (or replicate/attach frame) it sits in


class Frame:
  """A coordinate frame around body children (mjCFrame): a <frame> element, one copy of a
  <replicate> (explicit pos/quat) or an <attach> point. Elements inside one carry it (bodies
  in .frame, element attribute dicts under "__frame") and compose it into their own pose at
  the end of their compile, as mjuu_frameaccumChild does (user_objects.cc:1739, 2222-2243,
  3104, 3260, 3368, 3504)."""

  def __init__(self, parent, attrs=None, pos=None, quat=None):
    self.parent = parent
    self.attrs = attrs or {}
    self._pos, self._quat = pos, quat
    self.pose = None

  def compile(self, c):
    """mjCFrame::Compile (user_objects.cc:2001-2019): own orientation, then the parent frame
    accumulated, then normalized; once."""
    if self.pose is None:
      a = self.attrs
      pos = list(self._pos) if self._pos is not None else (
          _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0])
      quat = list(self._quat) if self._quat is not None else (
          _floats(a["quat"]) if "quat" in a else [1.0, 0.0, 0.0, 0.0])
      quat = _resolve_orientation(a, c.degree, c.eulerseq, quat)
      if self.parent is not None:
        ppos, pquat = self.parent.compile(c)
        pos, quat = frameaccum(ppos, pquat, pos, quat)
      normvec(quat)
      self.pose = (pos, quat)
    return self.pose


class Model:
  """A compiled model: sizes + numpy arrays named as in mjModel (see include/mjhip_fields.h).

  ``sizes`` maps size names to ints, ``opt`` is a dict of mjOption values and every model
  field of the field table is an attribute holding a numpy array of shape (dim0, dim1).
  """

  def __init__(self):
    self.sizes = {}
    self.opt = {}
    self.names = {}

  def __getitem__(self, k):
    return getattr(self, k)

  # convenience
  def __getattr__(self, k):
    sizes = self.__dict__.get("sizes", {})
    if k in sizes:
      return sizes[k]
    raise AttributeError(k)

  def save(self, path):
    """Save as .npz (numeric arrays only: loadable with allow_pickle=False)."""
    arrs = {"__sizes_keys": np.array(list(self.sizes.keys())),
            "__sizes_vals": np.array(list(self.sizes.values()), dtype=np.int64)}
    for k, v in self.opt.items():
      arrs["__opt_" + k] = np.asarray(v)
    for f in fields.MODEL_FIELDS:
      arrs[f.name] = getattr(self, f.name)
    for k, v in self.names.items():
      arrs["__names_" + k] = np.array(v if v else [""])
    np.savez(path, **arrs)

  @staticmethod
  def load(path):
    z = np.load(path, allow_pickle=False)
    m = Model()
    m.sizes = {str(k): int(v) for k, v in zip(z["__sizes_keys"], z["__sizes_vals"])}
    for k in z.files:
      if k.startswith("__opt_"):
        v = z[k]
        m.opt[k[6:]] = v.tolist() if v.ndim else (int(v) if v.dtype.kind == "i" else float(v))
      elif k.startswith("__names_"):
        lst = [str(x) for x in z[k]]
        m.names[k[8:]] = [] if lst == [""] and m.sizes.get(_NAME_SIZE.get(k[8:], ""), 0) == 0 else lst
    m.opt.setdefault("o_friction", [1.0, 1.0, 0.005, 0.0001, 0.0001])   # mjOption default
    m.opt.setdefault("magnetic", [0.0, -0.5, 0.0])                      # mjOption default
    m.opt.setdefault("ccd_tolerance", 1e-6)                             # engine_io.c:128
    m.opt.setdefault("ccd_iterations", 50)                              # engine_io.c:160
    for k in fields.MODEL_SIZES:               # sizes added to the table after the file
      m.sizes.setdefault(k, 0)
    for f in fields.MODEL_FIELDS:
      if f.name in z.files:
        setattr(m, f.name, np.ascontiguousarray(z[f.name]))
      else:                                    # a field added after the file: its empty value
        shape = f.shape(m.sizes)
        fill = -1 if f.name == "geom_dataid" or f.name == "mesh_graphadr" else 0
        a = np.full(shape if shape[1] != 1 else shape[:1], fill, dtype=fields.NPTYPE[f.ctype])
        setattr(m, f.name, a)
    return m


_NAME_SIZE = {"body": "nbody", "jnt": "njnt", "geom": "ngeom", "site": "nsite", "cam": "ncam",
              "light": "nlight", "tendon": "ntendon", "actuator": "nu", "key": "nkey",
              "sensor": "nsensor"}


class MJCFCompiler:
  """Compile an MJCF file/string into a Model (subset; raises MJCFError otherwise)."""

  def __init__(self):
    self.degree = True
    self.inertiafromgeom = "auto"
    self.autolimits = True
    self.eulerseq = "xyz"
    self.boundmass = 0.0
    self.boundinertia = 0.0
    self.balanceinertia = False
    self.inertiagrouprange = (0, 5)
    self.opt = {"timestep": 0.002, "impratio": 1.0, "gravity": [0.0, 0.0, -9.81],
                "wind": [0.0, 0.0, 0.0], "magnetic": [0.0, -0.5, 0.0], "density": 0.0, "viscosity": 0.0, "o_margin": 0.0,
                "o_solref": [0.02, 1.0], "o_solimp": [0.9, 0.95, 0.001, 0.5, 2.0],
                "o_friction": [1.0, 1.0, 0.005, 0.0001, 0.0001],
                "integrator": 0, "cone": 0, "jacobian": 2, "disableflags": 0,
                "enableflags": 0, "ccd_tolerance": 1e-6, "ccd_iterations": 50}
    self.classes = {}
    self.bodies = []
    self.tendons = []
    self.actuators = []
    self.sensors = []
    self.materials = {}                 # name -> rgba (<asset><material>)
    self.meshes = {}                    # name -> meshes.Mesh (<asset><mesh>)
    self.hfields = {}                   # name -> meshes.HField (<asset><hfield>)
    self.equalities = []
    self.excludes = []
    self.pairs = []                     # <contact><pair> attribute dicts (class defaults applied)
    self.keys = []
    self.models = {}                    # name -> MJCFCompiler (<asset><model>, parsed only)
    self.basedir = None

  def _compile_pairs(self, arr, s, geoms):
    """Predefined geom pairs: mjs_defaultPair (user_init.c:298-307) under the class chain's
    defaults, root first, and the element's attributes (mjXReader::OnePair,
    xml_native_reader.cc:1866-1893, applied to each default class's copy of its parent's
    mjsPair and then to the element's; ReadAttr copies only the values given, xml_util.cc:681,
    so a partial vector keeps the rest of the level below), the geoms swapped so that body1 <= body2 and the
    body signature (mjCPair::ResolveReferences, user_objects.cc:4777-4817), condim checked
    (mjCPair::Compile :4822-4828), then stably sorted by signature (user_model.cc:4321-4324)
    and written as in mjCModel::CopyObjects (:3153-3164). The pair's values are always
    defined in this version, so Compile's fall-backs to the geoms' parameters never apply."""
    gid = {g["name"]: i for i, g in enumerate(geoms) if g.get("name")}
    recs = []
    for a in self.pairs:
      vals = {"condim": 3, "solref": [0.02, 1.0], "solreffriction": [0.0, 0.0],
              "solimp": [0.9, 0.95, 0.001, 0.5, 2.0], "margin": [0.0], "gap": [0.0],
              "friction": [1.0, 1.0, 0.005, 0.0001, 0.0001]}
      for layer in a.get("_layers", [a]):
        for k in ("solref", "solreffriction", "solimp", "margin", "gap", "friction"):
          if k in layer:
            v = _floats(layer[k])
            if len(v) > len(vals[k]):
              raise MJCFError(f"pair attribute '{k}' has too many values")
            vals[k][:len(v)] = v
        if "condim" in layer:
          vals["condim"] = int(layer["condim"])
      if vals["condim"] not in (1, 3, 4, 6):
        raise MJCFError("invalid condim in contact pair")
      n1, n2 = a.get("geom1"), a.get("geom2")
      for n in (n1, n2):
        if n not in gid:
          raise MJCFError(f"geom '{n}' not found in collision")
      g1, g2 = gid[n1], gid[n2]
      if geoms[g1]["body"] > geoms[g2]["body"]:
        g1, g2 = g2, g1
      recs.append(((geoms[g1]["body"] << 16) + geoms[g2]["body"], g1, g2, vals))
    recs.sort(key=lambda r: r[0])            # list.sort is stable
    npair = len(recs)
    pdim, pg1, pg2, psig = (arr("pair_" + k, npair, np.int32)
                            for k in ("dim", "geom1", "geom2", "signature"))
    psolref = arr("pair_solref", (npair, 2), np.float64)
    psolreffriction = arr("pair_solreffriction", (npair, 2), np.float64)
    psolimp = arr("pair_solimp", (npair, 5), np.float64)
    pmargin = arr("pair_margin", npair, np.float64)
    pgap = arr("pair_gap", npair, np.float64)
    pfriction = arr("pair_friction", (npair, 5), np.float64)
    for i, (sig, g1, g2, v) in enumerate(recs):
      pdim[i], pg1[i], pg2[i], psig[i] = v["condim"], g1, g2, sig
      psolref[i], psolreffriction[i], psolimp[i] = v["solref"], v["solreffriction"], v["solimp"]
      pmargin[i], pgap[i], pfriction[i] = v["margin"][0], v["gap"][0], v["friction"]
    s.update(npair=npair)

  # ---------------------------------------------------------------- parsing
  def _parse_defaults(self, el, parent):
    name = el.get("class", "main")
    d = _Defaults(name, parent)
    self.classes[name] = d
    for ch in el:
      if ch.tag == "default":
        self._parse_defaults(ch, d)
      else:
        tag = "joint" if ch.tag == "freejoint" else ch.tag
        d.attrs.setdefault(tag, {}).update(ch.attrib)

  def _elem_attrs(self, el, tag, childclass):
    cls = el.get("class", childclass or "main")
    if cls not in self.classes:
      raise MJCFError(f"unknown default class '{cls}'")
    a = self.classes[cls].get(tag)
    a.update(el.attrib)
    return a

  def _parse_body(self, el, parent, childclass, frame=None):
    attrs = dict(el.attrib)
    cc = attrs.get("childclass", childclass)
    b = Body(parent, attrs, attrs.get("class", childclass), cc)
    b.frame = frame
    self.bodies.append(b)
    self._parse_children(el, b, cc, None)
    return b

  def _parse_children(self, el, b, cc, frame):
    """The child elements of a body (or of a <frame>/<replicate> inside it): mjXReader::Body
    (xml_native_reader.cc:3380-3640). Elements inside a frame carry it."""
    world = b.parent is None and b.name == "world"

    def framed(a):
      if frame is not None:
        a["__frame"] = frame
      return a
    for ch in el:
      t = ch.tag
      if t == "body":
        b.children.append(self._parse_body(ch, b, cc, frame))
      elif t in ("joint", "freejoint", "inertial") and world:
        raise MJCFError(f"<{t}> is not allowed in the world body")
      elif t == "joint":
        b.joints.append(framed(self._elem_attrs(ch, "joint", cc)))
      elif t == "freejoint":
        a = {"type": "free"}
        for k in ("name", "align", "group"):
          if k in ch.attrib:
            a[k] = ch.attrib[k]
        b.joints.append(framed(a))
      elif t == "geom":
        b.geoms.append(framed(self._elem_attrs(ch, "geom", cc)))
      elif t == "site":
        b.sites.append(framed(self._elem_attrs(ch, "site", cc)))
      elif t == "camera":
        b.cams.append(framed(self._elem_attrs(ch, "camera", cc)))
      elif t == "light":
        b.lights.append(framed(self._elem_attrs(ch, "light", cc)))
      elif t == "inertial":
        b.inertial = dict(ch.attrib)
      elif t == "frame":                    # xml_native_reader.cc:3477-3500
        fcc = ch.get("childclass", cc)
        if fcc is not None and fcc not in self.classes:
          raise MJCFError(f"unknown default childclass '{fcc}'")
        self._parse_children(ch, b, fcc, Frame(frame, dict(ch.attrib)))
      elif t == "replicate":
        self._parse_replicate(ch, b, cc, frame)
      elif t == "attach":
        self._parse_attach(ch, b, frame)
      else:
        raise MJCFError(f"unsupported body child element <{t}>")

  def _parse_replicate(self, el, b, cc, frame):
    """<replicate> (xml_native_reader.cc:3503-3572): `count` copies of the children, copy i
    in a frame at the accumulated offset, rotated by i*euler, its element names suffixed
    with sep + i zero-padded to the digits of count (UpdateString, :83-91). The reference
    parses the children once into a scratch body and attaches copies of its frame; each copy
    here is parsed afresh into a scratch body with its own frame objects, which yields the
    same elements, order and names (inner copies of nested replicates get their suffix
    first). As the reference's self-attach, each copy also appends the suffixed copies of
    the referencing elements parsed so far whose suffixed references resolve."""
    if "count" not in el.attrib:
      raise MJCFError("replicate needs a count")
    count = int(el.get("count"))
    offset = _floats(el.get("offset", "0 0 0"))
    euler = _floats(el.get("euler", "0 0 0"))
    sep = el.get("sep", "")
    rcc = el.get("childclass", cc)
    if rcc is not None and rcc not in self.classes:
      raise MJCFError(f"unknown default childclass '{rcc}'")
    rotation = _euler_quat(euler, self.degree, self.eulerseq)
    pos, quat = [0.0, 0.0, 0.0], [1.0, 0.0, 0.0, 0.0]
    for i in range(count):
      fpos = list(pos)
      pos, quat = frameaccum(pos, quat, offset, rotation)
      quat = _euler_quat([i * e for e in euler], self.degree, self.eulerseq)
      suffix = sep + str(i).zfill(len(str(count)))
      scratch = Body(b.parent, {"name": b.name}, b.cls, rcc)
      self._parse_children(el, scratch, rcc, Frame(frame, pos=fpos, quat=list(quat)))
      if scratch.inertial is not None:
        raise MJCFError("<inertial> inside <replicate>")
      _namespace(scratch, "", suffix, own=False)
      for lst in ("joints", "geoms", "sites", "cams", "lights"):
        getattr(b, lst).extend(getattr(scratch, lst))
      for c in scratch.children:
        c.parent = b
        b.children.append(c)
      self._append_referencing(self, "", suffix)

  def _parse_attach(self, el, b, frame):
    """<attach model body prefix> (xml_native_reader.cc:3621-3646, mjCBody::operator+=
    user_objects.cc:865-955, mjCModel::operator+= user_model.cc:404-464): a copy of body
    `body` of the <asset><model> `model`, with its subtree, at the enclosing frame (a new
    identity frame without one); every name prefixed. The model's assets follow with
    prefixed names, and its excludes, tendons, equalities, actuators and sensors whose
    (prefixed) references all resolve in this model are appended in that order. The
    attached model's keyframes are not carried over (keyframes are not on the path)."""
    for k in ("model", "body", "prefix"):
      if k not in el.attrib:
        raise MJCFError(f"attach needs '{k}'")
    name, bname, prefix = el.get("model"), el.get("body"), el.get("prefix")
    sub = self.models.get(name)
    if sub is None:
      raise MJCFError(f"could not find model '{name}'")
    if any(x.name == prefix + bname for x in self.bodies):
      raise MJCFError("attach to an existing body (frame only) is not in the supported subset")
    for k in ("degree", "eulerseq", "inertiafromgeom", "autolimits", "boundmass",
              "boundinertia", "balanceinertia", "inertiagrouprange"):
      if getattr(sub, k) != getattr(self, k):
        raise MJCFError(f"attached model '{name}' has a different compiler {k}")
    src = next((x for x in sub.bodies if x.name == bname and x.parent is not None), None)
    if src is None:
      raise MJCFError(f"could not find body '{bname}' in model '{name}'")
    top = self._clone_body(src, b, prefix)
    top.frame = frame if frame is not None else Frame(None)
    b.children.append(top)
    # assets (all of them, as the reference's CopyList), then the referencing elements
    for nm, rgba in sub.materials.items():
      self.materials[prefix + nm] = rgba
    for nm, mesh in sub.meshes.items():
      self.meshes[prefix + nm] = mesh
    for nm, hf in sub.hfields.items():
      self.hfields[prefix + nm] = hf
    self._append_referencing(sub, prefix, "")

  def _append_referencing(self, src, prefix, suffix):
    """mjCModel::operator+= (user_model.cc:427-432) over CopyList (:223-261): each exclude,
    tendon, equality, actuator and sensor of `src` (another model for attach, this one for a
    replicate copy) is namespaced -- its name and references -- and appended when every
    reference resolves in this model; the others are skipped."""
    names = self._names()
    p = lambda s: None if s is None else prefix + s + suffix
    ns = lambda a, keys: {k: (p(v) if k in keys and isinstance(v, str) and v else v)
                          for k, v in a.items()}
    lists = [list(src.excludes), list(src.tendons), list(src.equalities),
             list(src.actuators), list(src.sensors)]
    for a in list(src.pairs):            # CopyList(pairs_) precedes the excludes (:427)
      a = ns(a, ("name", "geom1", "geom2"))
      if a.get("geom1") in names["geom"] and a.get("geom2") in names["geom"]:
        self.pairs.append(a)
    for b1, b2 in lists[0]:
      if p(b1) in names["body"] and p(b2) in names["body"]:
        self.excludes.append((p(b1), p(b2)))
    for a, path in lists[1]:
      a = ns(a, ("name",))
      if a.get("__kind") == "fixed":
        path = [(p(j), c) for j, c in path]
        ok = all(j in names["joint"] for j, _ in path)
      else:
        path = [(k, p(v) if k == "site" else (p(v[0]), p(v[1])) if k == "geom" else v)
                for k, v in path]
        ok = all((k != "site" or v in names["site"]) and
                 (k != "geom" or (v[0] in names["geom"] and
                                  (v[1] is None or v[1] in names["site"]))) for k, v in path)
      if ok:
        self.tendons.append((a, path))
        names["tendon"].add(a.get("name"))
    for lst, refs, dst in ((lists[2], EQ_REFS, self.equalities),
                           (lists[3], ACT_REFS, self.actuators)):
      for a in lst:
        a = ns(a, ("name",) + tuple(refs))
        if all(a[k] in names[kind] for k, kind in refs.items() if k in a):
          dst.append(a)
          if dst is self.actuators:
            names["actuator"].add(a.get("name"))
    for tag, a in lists[4]:
      a = ns(a, ("name",) + tuple(SENSOR_REFS))
      if all(a[k] in names[kind] for k, kind in SENSOR_REFS.items() if k in a):
        self.sensors.append((tag, a))

  def _clone_body(self, src, parent, prefix):
    """A copy of an attached model's body subtree with prefixed names (mjCBody copy +
    NameSpace, user_objects.cc:1122-1175, 2365-2379, 3180-3185); frames inside the subtree
    are shared with the source (they are not modified)."""
    nb = Body(parent, _prefixed(src.attrs, prefix, ("name",)), src.cls, src.childclass)
    nb.frame = src.frame
    nb.inertial = dict(src.inertial) if src.inertial is not None else None
    nb.joints = [_prefixed(a, prefix, ("name",)) for a in src.joints]
    nb.geoms = [_prefixed(a, prefix, ("name", "material", "mesh", "hfield")) for a in src.geoms]
    nb.sites = [_prefixed(a, prefix, ("name", "material")) for a in src.sites]
    nb.cams = [_prefixed(a, prefix, ("name", "target")) for a in src.cams]
    nb.lights = [_prefixed(a, prefix, ("name", "target")) for a in src.lights]
    self.bodies.append(nb)
    nb.children = [self._clone_body(c, nb, prefix) for c in src.children]
    return nb

  def _names(self):
    """Names of the elements parsed so far, per kind (reference resolution of attached
    referencing elements)."""
    out = {"body": set(), "joint": set(), "geom": set(), "site": set(), "camera": set(),
           "tendon": {a.get("name") for a, _ in self.tendons},
           "actuator": {a.get("name") for a in self.actuators}}
    for b in self.bodies:
      out["body"].add(b.name)
      for kind, lst in (("joint", b.joints), ("geom", b.geoms), ("site", b.sites),
                        ("camera", b.cams)):
        out[kind].update(a.get("name") for a in lst)
    for v in out.values():
      v.discard(None)
      v.discard("")
    out["any"] = set().union(*out.values())
    return out

  def parse(self, root):
    if root.tag != "mujoco":
      raise MJCFError("root element must be <mujoco>")
    self.model_name = root.get("model", "")
    self.classes["main"] = _Defaults("main")
    for el in root:
      if el.tag == "default":
        # top-level <default> is class "main"; its children are classes
        top = self.classes["main"]
        for ch in el:
          if ch.tag == "default":
            self._parse_defaults(ch, top)
          else:
            tag = "joint" if ch.tag == "freejoint" else ch.tag
            top.attrs.setdefault(tag, {}).update(ch.attrib)
    for el in root:
      t = el.tag
      if t == "compiler":
        a = el.attrib
        if "angle" in a:
          self.degree = a["angle"] == "degree"
        self.inertiafromgeom = a.get("inertiafromgeom", self.inertiafromgeom)
        if "autolimits" in a:
          self.autolimits = a["autolimits"] == "true"
        self.eulerseq = a.get("eulerseq", self.eulerseq)
        self.boundmass = float(a.get("boundmass", self.boundmass))
        self.boundinertia = float(a.get("boundinertia", self.boundinertia))
        if "balanceinertia" in a:
          self.balanceinertia = a["balanceinertia"] == "true"
        if "inertiagrouprange" in a:
          self.inertiagrouprange = tuple(int(x) for x in a["inertiagrouprange"].split())
      elif t == "option":
        self._parse_option(el)
      elif t == "worldbody":
        self._parse_worldbody(el)
      elif t == "tendon":
        for ch in el:
          if ch.tag not in ("fixed", "spatial"):
            raise MJCFError(f"unsupported tendon <{ch.tag}>")
          a = self._elem_attrs(ch, "tendon", None)
          a["__kind"] = ch.tag
          if ch.tag == "fixed":
            path = [(j.get("joint"), float(j.get("coef", "1"))) for j in ch if j.tag == "joint"]
          else:                             # xml_native_reader.cc:3780-3820
            path = []
            for w in ch:
              if w.tag == "site":
                path.append(("site", w.get("site")))
              elif w.tag == "pulley":
                path.append(("pulley", float(w.get("divisor", "0"))))
              elif w.tag == "geom":
                path.append(("geom", (w.get("geom"), w.get("sidesite"))))
              else:
                raise MJCFError(f"unsupported spatial tendon element <{w.tag}>")
          self.tendons.append((a, path))
      elif t == "actuator":
        for ch in el:
          if ch.tag not in ACTUATOR_TAGS:
            raise MJCFError(f"unsupported actuator <{ch.tag}>")
          a = self._elem_attrs(ch, ch.tag, None)
          a["__tag"] = ch.tag
          self.actuators.append(a)
      elif t == "contact":
        for ch in el:
          if ch.tag == "exclude":
            self.excludes.append((ch.get("body1"), ch.get("body2")))
          elif ch.tag == "pair":           # mjXReader::OnePair (xml_native_reader.cc:1866)
            a = self._elem_attrs(ch, "pair", None)
            # the class chain's own pair attributes, root first, then the element's: vectors
            # overlay element-wise level by level (a default class holds a whole mjsPair)
            chain, d = [], self.classes[ch.get("class", "main")]
            while d is not None:
              chain.append(dict(d.attrs.get("pair", {})))
              d = d.parent
            a["_layers"] = chain[::-1] + [dict(ch.attrib)]
            self.pairs.append(a)
          else:
            raise MJCFError(f"unsupported contact element <{ch.tag}>")
      elif t == "keyframe":
        for ch in el:
          self.keys.append(dict(ch.attrib))
      elif t == "equality":
        for ch in el:
          if ch.tag not in ("connect", "weld", "joint", "tendon"):
            raise MJCFError(f"equality <{ch.tag}> is not in the supported subset")
          a = self._elem_attrs(ch, "equality", None)
          a["__tag"] = ch.tag
          self.equalities.append(a)
      elif t == "sensor":
        for ch in el:
          if ch.tag in SENSORS_NEXT:
            raise MJCFError(f"sensor <{ch.tag}> is not in the supported subset (next)")
          if ch.tag not in SENSORS:
            raise MJCFError(f"unknown sensor <{ch.tag}>")
          self.sensors.append((ch.tag, dict(ch.attrib)))
      elif t == "asset":
        # materials matter to mj_ray's visibility test (engine_ray.c:76-84); meshes and height
        # fields are collision geometry (meshes.py); textures have no effect on the path
        for ch in el:
          if ch.tag == "material":
            a = self._elem_attrs(ch, "material", None)
            rgba = [1.0, 1.0, 1.0, 1.0]                 # user_objects.cc mjCMaterial
            v = _floats(a["rgba"]) if "rgba" in a else []
            rgba[:len(v)] = v
            self.materials[a.get("name", f"__material{len(self.materials)}")] = rgba
          elif ch.tag == "mesh":
            self._parse_mesh(ch)
          elif ch.tag == "hfield":
            self._parse_hfield(ch)
          elif ch.tag == "texture":
            continue
          elif ch.tag == "model":
            self._parse_model_asset(ch)
          else:
            raise MJCFError(f"unsupported asset <{ch.tag}>")
      elif t in ("visual", "statistic", "default", "compiler", "size", "extension", "custom"):
        continue  # no effect on the inverse-dynamics path
      else:
        raise MJCFError(f"unsupported top-level element <{t}>")

  def _parse_model_asset(self, el):
    """<asset><model file name> (xml_native_reader.cc:3307-3336): another MJCF file, parsed
    (not compiled) for <attach>; named by `name`, else by its own model name."""
    if el.get("content_type", "text/xml") != "text/xml":
      raise MJCFError(f"unsupported content_type: {el.get('content_type')}")
    if "file" not in el.attrib:
      raise MJCFError("model asset needs a file")
    if self.basedir is None:
      raise MJCFError("a model asset needs the directory of the including file (load_xml)")
    path = os.path.join(self.basedir, el.get("file"))
    sub = MJCFCompiler()
    sub.basedir = os.path.dirname(os.path.abspath(path))
    try:
      sub.parse(ET.parse(path).getroot())
    except (OSError, ET.ParseError) as e:
      raise MJCFError(f"could not parse model file: {e}") from e
    self.models[el.get("name", sub.model_name)] = sub

  def _parse_mesh(self, el):
    """<mesh> with inline vertex (and optional face) data (xml_native_reader.cc:1405-1480);
    mesh files are not read (no file assets on the path)."""
    from . import meshes
    a = self._elem_attrs(el, "mesh", None)
    if "file" in a:
      raise MJCFError("mesh files are not in the supported subset (give vertex data)")
    if "vertex" not in a:
      raise MJCFError("mesh needs vertex data")
    name = a.get("name", f"__mesh{len(self.meshes)}")
    inertia = a.get("inertia", "legacy")
    if inertia not in ("convex", "legacy", "exact", "shell"):
      raise MJCFError(f"invalid mesh inertia '{inertia}'")
    cls = el.get("class", "main")
    try:
      self.meshes[name] = meshes.Mesh(
          name, np.array(a["vertex"].split(), dtype=np.float32),
          face=[int(x) for x in a["face"].split()] if "face" in a else None,
          scale=_floats(a["scale"]) if "scale" in a else (1, 1, 1),
          refpos=_floats(a["refpos"]) if "refpos" in a else (0, 0, 0),
          refquat=_floats(a["refquat"]) if "refquat" in a else (1, 0, 0, 0),
          inertia=inertia, maxhullvert=int(a.get("maxhullvert", -1)))
    except meshes.MeshError as e:
      raise MJCFError(str(e)) from e
    # Process() weighs the mesh with its class's default geom density (user_mesh.cc:1466)
    self.meshes[name].density = float(self.classes[cls].get("geom").get("density", "1000"))

  def _parse_hfield(self, el):
    """<hfield> with inline elevation (xml_native_reader.cc:3249-3300)."""
    from . import meshes
    a = dict(el.attrib)
    if "file" in a:
      raise MJCFError("hfield files are not in the supported subset (give elevation data)")
    name = a.get("name", f"__hfield{len(self.hfields)}")
    try:
      self.hfields[name] = meshes.HField(
          name, int(a.get("nrow", 0)), int(a.get("ncol", 0)), _floats(a.get("size", "")),
          np.array(a["elevation"].split(), dtype=np.float32) if "elevation" in a else None)
    except meshes.MeshError as e:
      raise MJCFError(str(e)) from e

  def _parse_option(self, el):
    a = el.attrib
    o = self.opt
    for k in ("timestep", "impratio", "density", "viscosity", "o_margin", "ccd_tolerance"):
      if k in a:
        o[k] = float(a[k])
    if "ccd_iterations" in a:
      o["ccd_iterations"] = int(a["ccd_iterations"])
    for k in ("gravity", "wind", "magnetic", "o_solref", "o_solimp", "o_friction"):
      if k in a:
        o[k] = _floats(a[k])
    if "integrator" in a:
      o["integrator"] = INTEGRATOR[a["integrator"]]
    if "jacobian" in a:
      o["jacobian"] = JACOBIAN[a["jacobian"]]
    if "cone" in a:
      o["cone"] = CONE[a["cone"]]
    for ch in el:
      if ch.tag == "flag":
        for k, v in ch.attrib.items():
          if k in DISABLE:
            bit = 1 << DISABLE[k]
            if v == "disable":
              o["disableflags"] |= bit
            else:
              o["disableflags"] &= ~bit
          elif k in ENABLE:
            bit = 1 << ENABLE[k]
            if v == "enable":
              o["enableflags"] |= bit
            else:
              o["enableflags"] &= ~bit
          else:
            raise MJCFError(f"unknown flag '{k}'")

  def _parse_worldbody(self, el):
    world = Body(None, {"name": "world"}, None, None)
    self.bodies.insert(0, world)
    self._parse_children(el, world, None, None)

  # ---------------------------------------------------------------- compile
  def _order_bodies(self):
    # depth-first pre-order (mjCModel body list order)
    order = []

    def rec(b):
      order.append(b)
      for c in b.children:
        rec(c)
    rec(self.bodies[0])
    for i, b in enumerate(order):
      b.id = i
    self.bodies = order

  def _compile_geom(self, a, inferinertia):
    g = {}
    g["type"] = GEOM[a.get("type", "sphere")]
    size = [0.0, 0.0, 0.0]
    if "size" in a:
      s = _floats(a["size"])
      size[:len(s)] = s
    pos = _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0]
    quat = _floats(a["quat"]) if "quat" in a else [1.0, 0.0, 0.0, 0.0]
    normvec(quat)
    if "fromto" in a:
      if g["type"] not in (GEOM["capsule"], GEOM["cylinder"], GEOM["ellipsoid"], GEOM["box"]):
        raise MJCFError("fromto requires capsule, cylinder, box or ellipsoid in geom")
      if pos[0] or pos[1] or pos[2]:
        raise MJCFError("both pos and fromto defined in geom")
      ft = _floats(a["fromto"])
      vec = [ft[0]-ft[3], ft[1]-ft[4], ft[2]-ft[5]]
      size[1] = normvec(vec)/2
      if size[1] < mjEPS:
        raise MJCFError("fromto points too close in geom")
      if g["type"] in (GEOM["ellipsoid"], GEOM["box"]):
        size[2] = size[1]
        size[1] = size[0]
      pos = [(ft[0]+ft[3])/2, (ft[1]+ft[4])/2, (ft[2]+ft[5])/2]
      quat = z2quat(vec)
    else:
      quat = _resolve_orientation(a, self.degree, self.eulerseq, quat)
    t = g["type"]
    if t == GEOM["sdf"]:
      raise MJCFError("sdf geoms are not in the supported subset")
    # mesh and height-field references (mjCGeom::Compile, user_objects.cc:2932-3041)
    mesh = hfield = None
    g["dataid"] = -1
    if "mesh" in a:
      if a["mesh"] not in self.meshes:
        raise MJCFError(f"mesh '{a['mesh']}' not found in geom")
      mesh = self.meshes[a["mesh"]]
      if t != GEOM["mesh"]:
        raise MJCFError("fitting a primitive geom to a mesh is not in the supported subset")
      if "fromto" in a:
        raise MJCFError("fromto cannot be used with mesh geom")
      g["dataid"] = list(self.meshes).index(a["mesh"])
    if t == GEOM["mesh"] and mesh is None:
      raise MJCFError("mesh geom must have valid meshid")
    if "hfield" in a:
      if a["hfield"] not in self.hfields:
        raise MJCFError(f"hfield '{a['hfield']}' not found in geom")
      hfield = self.hfields[a["hfield"]]
      g["dataid"] = list(self.hfields).index(a["hfield"])
    if (t == GEOM["hfield"]) != (hfield is not None):
      raise MJCFError("hfield geom must have valid hfieldid")
    if mesh is not None:                 # mjuu_frameaccum(pos, quat, mesh pos, mesh quat)
      mat = quat2mat(quat)
      mp = mesh.pos
      vec = mulvecmat(mp, mat)
      pos = [pos[0] + vec[0], pos[1] + vec[1], pos[2] + vec[2]]
      quat = mulquat(quat, mesh.quat)
      aamm = mesh.aamm
      size = [max(abs(aamm[0]), abs(aamm[3])), max(abs(aamm[1]), abs(aamm[4])),
              max(abs(aamm[2]), abs(aamm[5]))]
    elif hfield is not None:
      hs = hfield.size
      size = [hs[0], hs[1], 0.25*hs[2] + 0.5*hs[3]]
    g["size"] = size
    g["pos"] = pos
    g["quat"] = quat
    g["group"] = int(a.get("group", 0))
    g["contype"] = int(a.get("contype", 1))
    g["conaffinity"] = int(a.get("conaffinity", 1))
    g["condim"] = int(a.get("condim", 3))
    g["priority"] = int(a.get("priority", 0))
    fr = _floats(a["friction"]) if "friction" in a else []
    g["friction"] = [1.0, 0.005, 0.0001]
    g["friction"][:len(fr)] = fr
    g["solmix"] = float(a.get("solmix", 1.0))
    shape = a.get("fluidshape", "none")        # xml_native_reader.cc:1701-1704
    if shape not in ("none", "ellipsoid"):
      raise MJCFError(f"invalid fluidshape '{shape}'")
    g["fluid_ellipsoid"] = 1.0 if shape == "ellipsoid" else 0.0
    coefs = [0.5, 0.25, 1.5, 1.0, 1.0]         # user_init.c:143-147
    fc = _floats(a["fluidcoef"]) if "fluidcoef" in a else []
    coefs[:len(fc)] = fc
    g["fluid_coefs"] = coefs
    g["solref"] = _floats(a["solref"]) if "solref" in a else [0.02, 1.0]
    si = _floats(a["solimp"]) if "solimp" in a else []
    g["solimp"] = [0.9, 0.95, 0.001, 0.5, 2.0]
    g["solimp"][:len(si)] = si
    g["margin"] = float(a.get("margin", 0.0))
    g["gap"] = float(a.get("gap", 0.0))
    g["name"] = a.get("name", "")
    rgba = [0.5, 0.5, 0.5, 1.0]                  # user_init.c mjs_defaultGeom
    v = _floats(a["rgba"]) if "rgba" in a else []
    rgba[:len(v)] = v
    g["rgba"] = rgba
    g["material"] = a.get("material")
    # mass and inertia (user_objects.cc:3052-3080), typeinertia = volume
    g["mass"] = 0.0
    g["inertia"] = [0.0, 0.0, 0.0]
    if inferinertia:
      vol = mesh.volume if mesh is not None else _geom_volume(t, size)

      def inertia(mass):
        if mesh is None:
          return _geom_inertia(t, size, mass)
        bs = mesh.boxsz                   # the mesh's equivalent inertia box
        return [mass * (bs[1]*bs[1] + bs[2]*bs[2]) / 3, mass * (bs[0]*bs[0] + bs[2]*bs[2]) / 3,
                mass * (bs[0]*bs[0] + bs[1]*bs[1]) / 3]
      if "mass" in a:
        mass = float(a["mass"])
        if mass == 0:
          g["mass"] = 0.0
        elif vol > mjEPS:
          g["mass"] = mass
          g["inertia"] = inertia(mass)
      else:
        density = float(a.get("density", 1000.0))
        if density != 0:
          g["mass"] = density * vol
          g["inertia"] = inertia(g["mass"])
    if mesh is not None:                 # GetRBound (user_objects.cc:2723-2729)
      aamm = mesh.aamm
      h = [max(abs(aamm[0]), abs(aamm[3])), max(abs(aamm[1]), abs(aamm[4])),
           max(abs(aamm[2]), abs(aamm[5]))]
      g["rbound"] = math.sqrt(h[0]*h[0] + h[1]*h[1] + h[2]*h[2])
    elif hfield is not None:             # (:2703-2706)
      hs = hfield.size
      g["rbound"] = math.sqrt(hs[0]*hs[0] + hs[1]*hs[1] + max(hs[2]*hs[2], hs[3]*hs[3]))
    else:
      g["rbound"] = _geom_rbound(t, size)
    # fluid-interaction coefficients (user_objects.cc:3081-3084)
    g["fluid"] = _fluid_coefs(t, size, g["fluid_ellipsoid"], g["fluid_coefs"]) \
        if g["fluid_ellipsoid"] > 0 else [0.0] * 12
    if "__frame" in a:                   # end of mjCGeom::Compile (user_objects.cc:3102-3105)
      fpos, fquat = a["__frame"].compile(self)
      g["pos"], g["quat"] = frameaccum(fpos, fquat, g["pos"], g["quat"])
    return g

  def compile(self) -> Model:
    if not self.bodies:                 # no <worldbody>: the world body alone
      self._parse_worldbody(ET.Element("worldbody"))
    self._order_bodies()
    bodies = self.bodies
    nbody = len(bodies)
    # meshes before geoms (mjCModel::TryCompile, user_model.cc:4269-4290): a mesh gets its
    # convex-hull graph when a collidable mesh geom uses it or its inertia is "convex"
    from . import meshes
    for b in bodies:
      for ga in b.geoms:
        if ga.get("type") == "mesh" and ga.get("mesh") in self.meshes:
          mesh = self.meshes[ga["mesh"]]
          if (int(ga.get("contype", 1)) or int(ga.get("conaffinity", 1)) or
              mesh.inertia == "convex"):
            mesh.needhull = True
    for mesh in self.meshes.values():
      try:
        mesh.compile(mesh.density)
      except meshes.MeshError as e:
        raise MJCFError(str(e)) from e
    # ---- per-body compile (mjCBody::Compile)
    jnts, geoms, sites, cams, lights = [], [], [], [], []
    for b in bodies:
      a = b.attrs
      b.pos = _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0]
      b.quat = _floats(a["quat"]) if "quat" in a else [1.0, 0.0, 0.0, 0.0]
      normvec(b.quat)
      b.quat = _resolve_orientation(a, self.degree, self.eulerseq, b.quat)
      b.mocap = a.get("mocap", "false") == "true"
      if b.mocap and (b.parent is None or b.parent.name != "world" or b.joints):
        raise MJCFError("mocap body must be a child of the world body and have no joints")
      b.gravcomp = float(a.get("gravcomp", 0.0))
      b.ipos = None
      b.iquat = [1.0, 0.0, 0.0, 0.0]
      b.mass = 0.0
      b.inertia = [0.0, 0.0, 0.0]
      explicit = b.inertial is not None
      if explicit:
        ia = b.inertial
        b.ipos = _floats(ia["pos"])
        b.mass = float(ia["mass"])
        if "fullinertia" in ia:
          b.iquat, b.inertia = full_inertia(_floats(ia["fullinertia"]))
        else:
          b.inertia = _floats(ia.get("diaginertia", "0 0 0"))
          q = _floats(ia["quat"]) if "quat" in ia else [1.0, 0.0, 0.0, 0.0]
          normvec(q)
          b.iquat = _resolve_orientation(ia, self.degree, self.eulerseq, q)
      b.cgeoms = []
      for ga in b.geoms:
        infer = (b.id > 0 and (not explicit or self.inertiafromgeom == "true") and
                 self.inertiagrouprange[0] <= int(ga.get("group", 0)) <= self.inertiagrouprange[1])
        b.cgeoms.append(self._compile_geom(ga, infer))
      if b.id > 0 and (self.inertiafromgeom == "true" or
                       (b.ipos is None and self.inertiafromgeom == "auto")):
        self._inertia_from_geom(b)
      if b.ipos is None:
        b.ipos = list(b.pos)
        b.iquat = list(b.quat)
      if b.frame is not None:           # after the inertial copy (user_objects.cc:1737-1740)
        fpos, fquat = b.frame.compile(self)
        b.pos, b.quat = frameaccum(fpos, fquat, b.pos, b.quat)
      if b.id > 0:
        b.mass = max(b.mass, self.boundmass)
        b.inertia = [max(x, self.boundinertia) for x in b.inertia]
        I = b.inertia
        if I[0] + I[1] < I[2] or I[0] + I[2] < I[1] or I[1] + I[2] < I[0]:
          if self.balanceinertia:
            b.inertia = [(I[0] + I[1] + I[2])/3.0] * 3
          else:
            raise MJCFError("inertia must satisfy A + B >= C")
      # free-joint alignment (user_objects.cc:1751-1776): only with align="true"
      if (len(b.joints) == 1 and b.joints[0].get("type") == "free" and not b.children and
          b.joints[0].get("align", "auto") == "true"):
        raise MJCFError("free-joint alignment is not in the supported subset")
    # weldid (mjCBody::Compile sets children's weldid)
    for b in bodies:
      if b.id == 0:
        b.weldid = 0
      for c in b.children:
        c.weldid = c.id if c.joints else b.weldid
    # ---- joints
    for b in bodies:
      b.cjoints = []
      for ja in b.joints:
        j = self._compile_joint(ja)
        j["body"] = b.id
        b.cjoints.append(j)
        jnts.append(j)
      b.dofnum = sum(_jnt_nv(j["type"]) for j in b.cjoints)
    # ---- assign ids: joints, geoms, sites, cams, lights in body order
    for b in bodies:
      for g in b.cgeoms:
        g["body"] = b.id
        geoms.append(g)
      for sa in b.sites:
        sites.append(self._compile_site(sa, b.id))
      for ca in b.cams:
        cams.append(self._compile_cam(ca, b.id))
      for la in b.lights:
        lights.append(self._compile_light(la, b.id))
    return self._emit(jnts, geoms, sites, cams, lights)

  def _inertia_from_geom(self, b):
    sel = [g for g in b.cgeoms
           if self.inertiagrouprange[0] <= g["group"] <= self.inertiagrouprange[1]]
    if len(sel) == 1:
      g = sel[0]
      b.ipos = list(g["pos"])
      b.iquat = list(g["quat"])
      b.mass = g["mass"]
      b.inertia = list(g["inertia"])
    elif len(sel) > 1:
      mass = 0.0
      com = [0.0, 0.0, 0.0]
      for g in sel:
        mass += g["mass"]
        com[0] += g["mass"] * g["pos"][0]
        com[1] += g["mass"] * g["pos"][1]
        com[2] += g["mass"] * g["pos"][2]
      if mass < mjEPS:
        raise MJCFError("body mass is too small, cannot compute center of mass")
      ipos = [com[0]/mass, com[1]/mass, com[2]/mass]
      toti = [0.0] * 6
      for g in sel:
        dpos = [g["pos"][0] - ipos[0], g["pos"][1] - ipos[1], g["pos"][2] - ipos[2]]
        i0 = globalinertia(g["inertia"], g["quat"])
        i1 = offcenter(g["mass"], dpos)
        for j in range(6):
          toti[j] = toti[j] + i0[j] + i1[j]
      b.mass = mass
      b.ipos = ipos
      b.iquat, b.inertia = full_inertia(toti)

  def _compile_joint(self, a):
    t = JNT[a.get("type", "hinge")]
    j = {"type": t, "name": a.get("name", "")}
    rng = _floats(a["range"]) if "range" in a else [0.0, 0.0]
    lim = a.get("limited", "auto")
    if t == JNT["free"]:
      limited = False
    elif lim == "auto":
      hasrange = not (rng[0] == 0 and rng[1] == 0)
      if not self.autolimits and hasrange:
        raise MJCFError("joint has range but limited is auto and autolimits is false")
      limited = hasrange if self.autolimits else False
    else:
      limited = lim == "true"
    if limited:
      if rng[0] >= rng[1] and t != JNT["ball"]:
        raise MJCFError("range[0] should be smaller than range[1] in joint")
      if self.degree and t in (JNT["hinge"], JNT["ball"]):
        if rng[0]:
          rng[0] *= mjPI/180.0
        if rng[1]:
          rng[1] *= mjPI/180.0
    axis = _floats(a["axis"]) if "axis" in a else [0.0, 0.0, 1.0]
    frame = a["__frame"].compile(self) if "__frame" in a else None
    if t in (JNT["free"], JNT["ball"]):
      axis = [0.0, 0.0, 1.0]
    elif frame is not None:              # user_objects.cc:2220-2223
      axis = rotvecquat(axis, frame[1])
    if normvec(axis) < mjEPS:
      raise MJCFError("axis too small in joint")
    pos = _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0]
    if t == JNT["free"]:
      pos = [0.0, 0.0, 0.0]
    elif frame is not None:              # (:2240-2244)
      pos = frameaccum(frame[0], frame[1], pos, [1.0, 0.0, 0.0, 0.0])[0]
    ref = float(a.get("ref", 0.0))
    springref = float(a.get("springref", 0.0))
    if t == JNT["hinge"] and self.degree:
      ref *= mjPI/180.0
      springref *= mjPI/180.0
    j.update(limited=limited, range=rng, axis=axis, pos=pos, ref=ref, springref=springref,
             stiffness=float(a.get("stiffness", 0.0)), damping=float(a.get("damping", 0.0)),
             armature=float(a.get("armature", 0.0)),
             frictionloss=float(a.get("frictionloss", 0.0)),
             margin=float(a.get("margin", 0.0)), group=int(a.get("group", 0)),
             actgravcomp=a.get("actuatorgravcomp", "false") == "true")
    sr = _floats(a["solreflimit"]) if "solreflimit" in a else [0.02, 1.0]
    si = [0.9, 0.95, 0.001, 0.5, 2.0]
    if "solimplimit" in a:
      v = _floats(a["solimplimit"])
      si[:len(v)] = v
    j["solref"] = sr
    j["solimp"] = si
    fsr = _floats(a["solreffriction"]) if "solreffriction" in a else [0.02, 1.0]
    fsi = [0.9, 0.95, 0.001, 0.5, 2.0]
    if "solimpfriction" in a:
      v = _floats(a["solimpfriction"])
      fsi[:len(v)] = v
    j["solref_f"] = fsr
    j["solimp_f"] = fsi
    return j

  def _compile_site(self, a, bid):
    pos = _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0]
    quat = _floats(a["quat"]) if "quat" in a else [1.0, 0.0, 0.0, 0.0]
    normvec(quat)
    quat = _resolve_orientation(a, self.degree, self.eulerseq, quat)
    if "__frame" in a:                   # user_objects.cc:3258-3264
      fpos, fquat = a["__frame"].compile(self)
      pos, quat = frameaccum(fpos, fquat, pos, quat)
      normvec(quat)
    size = [0.005, 0.005, 0.005]
    if "size" in a:
      s = _floats(a["size"])
      size[:len(s)] = s
    return {"body": bid, "pos": pos, "quat": quat, "size": size,
            "type": GEOM[a.get("type", "sphere")], "name": a.get("name", "")}

  def _compile_cam(self, a, bid):
    pos = _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0]
    quat = _floats(a["quat"]) if "quat" in a else [1.0, 0.0, 0.0, 0.0]
    normvec(quat)
    quat = _resolve_orientation(a, self.degree, self.eulerseq, quat)
    if "__frame" in a:                   # user_objects.cc:3366-3372
      fpos, fquat = a["__frame"].compile(self)
      pos, quat = frameaccum(fpos, fquat, pos, quat)
      normvec(quat)
    # intrinsics (user_objects.cc mjCCamera::Compile :3383-3420, float arithmetic)
    f32 = np.float32
    fovy = float(a.get("fovy", 45.0))
    if fovy >= 180:
      raise MJCFError("fovy too large in camera")
    res = [int(x) for x in a["resolution"].split()] if "resolution" in a else [1, 1]
    size = [f32(x) for x in _floats(a["sensorsize"])] if "sensorsize" in a else [f32(0)] * 2

    def pair(name):
      return [f32(x) for x in _floats(a[name])] if name in a else [f32(0)] * 2
    fl, fp, pl, pp = pair("focal"), pair("focalpixel"), pair("principal"), pair("principalpixel")
    if (pl[0] and pp[0]) or (pl[1] and pp[1]):
      raise MJCFError("principal length duplicated in camera")
    if (fl[0] and fp[0]) or (fl[1] and fp[1]):
      raise MJCFError("focal length duplicated in camera")
    if size[0] > 0 and size[1] > 0:
      dens = [f32(res[0]) / size[0], f32(res[1]) / size[1]]
      intr = [fp[0] / dens[0] + fl[0], fp[1] / dens[1] + fl[1],
              pp[0] / dens[0] + pl[0], pp[1] / dens[1] + pl[1]]
      fovy = float(np.arctan2(float(size[1]) / 2, float(intr[1])) * 360.0 / np.pi)
    else:
      znear = f32(0.01)                        # visual.map.znear (the <visual> element is not read)
      intr = [znear, znear, f32(0), f32(0)]
    return {"body": bid, "pos": pos, "quat": quat, "mode": CAMLIGHT[a.get("mode", "fixed")],
            "target": a.get("target"), "name": a.get("name", ""), "fovy": fovy,
            "resolution": res, "sensorsize": size, "intrinsic": intr}

  def _compile_light(self, a, bid):
    pos = _floats(a["pos"]) if "pos" in a else [0.0, 0.0, 0.0]
    d = _floats(a["dir"]) if "dir" in a else [0.0, 0.0, -1.0]
    if "__frame" in a:                   # user_objects.cc:3500-3508
      fpos, fquat = a["__frame"].compile(self)
      pos = frameaccum(fpos, fquat, pos, [1.0, 0.0, 0.0, 0.0])[0]
      d = rotvecquat(d, fquat)
    normvec(d)
    return {"body": bid, "pos": pos, "dir": d, "mode": CAMLIGHT[a.get("mode", "fixed")],
            "target": a.get("target"), "name": a.get("name", "")}

  # ---------------------------------------------------------------- emit mjModel arrays
  def _emit(self, jnts, geoms, sites, cams, lights) -> Model:
    bodies = self.bodies
    nbody, njnt = len(bodies), len(jnts)
    nq = sum(_jnt_nq(j["type"]) for j in jnts)
    nv = sum(_jnt_nv(j["type"]) for j in jnts)
    bname = {b.name: b.id for b in bodies if b.name}
    jname = {j["name"]: i for i, j in enumerate(jnts) if j["name"]}
    m = Model()
    s = m.sizes
    s.update(nq=nq, nv=nv, nbody=nbody, njnt=njnt, ngeom=len(geoms), nsite=len(sites),
             ncam=len(cams), nlight=len(lights), na=0, nmocap=0)
    A = {}

    def arr(name, shape, dtype, fill=0):
      a = np.full(shape, fill, dtype=dtype)
      A[name] = a
      return a

    # bodies
    parentid = arr("body_parentid", nbody, np.int32)
    rootid = arr("body_rootid", nbody, np.int32)
    weldid = arr("body_weldid", nbody, np.int32)
    mocapid = arr("body_mocapid", nbody, np.int32, -1)
    nmocap = 0
    for b in bodies:                  # user_model.cc: mocapid in body order
      if getattr(b, "mocap", False):
        mocapid[b.id] = nmocap
        nmocap += 1
    s["nmocap"] = nmocap
    jntnum = arr("body_jntnum", nbody, np.int32)
    jntadr = arr("body_jntadr", nbody, np.int32, -1)
    dofnum = arr("body_dofnum", nbody, np.int32)
    dofadr = arr("body_dofadr", nbody, np.int32, -1)
    geomnum = arr("body_geomnum", nbody, np.int32)
    geomadr = arr("body_geomadr", nbody, np.int32, -1)
    simple = arr("body_simple", nbody, np.uint8)
    sameframe = arr("body_sameframe", nbody, np.uint8)
    bpos = arr("body_pos", (nbody, 3), np.float64)
    bquat = arr("body_quat", (nbody, 4), np.float64)
    bipos = arr("body_ipos", (nbody, 3), np.float64)
    biquat = arr("body_iquat", (nbody, 4), np.float64)
    bmass = arr("body_mass", nbody, np.float64)
    binertia = arr("body_inertia", (nbody, 3), np.float64)
    bgrav = arr("body_gravcomp", nbody, np.float64)
    bmargin = arr("body_margin", nbody, np.float64)
    bcontype = arr("body_contype", nbody, np.int32)
    bconaff = arr("body_conaffinity", nbody, np.int32)
    # joints / dofs
    jtype = arr("jnt_type", njnt, np.int32)
    jqadr = arr("jnt_qposadr", njnt, np.int32)
    jdadr = arr("jnt_dofadr", njnt, np.int32)
    jbody = arr("jnt_bodyid", njnt, np.int32)
    jgroup = arr("jnt_group", njnt, np.int32)
    jlim = arr("jnt_limited", njnt, np.uint8)
    jagc = arr("jnt_actgravcomp", njnt, np.uint8)
    jsolref = arr("jnt_solref", (njnt, 2), np.float64)
    jsolimp = arr("jnt_solimp", (njnt, 5), np.float64)
    jpos = arr("jnt_pos", (njnt, 3), np.float64)
    jaxis = arr("jnt_axis", (njnt, 3), np.float64)
    jstiff = arr("jnt_stiffness", njnt, np.float64)
    jrange = arr("jnt_range", (njnt, 2), np.float64)
    jmargin = arr("jnt_margin", njnt, np.float64)
    qpos0 = arr("qpos0", nq, np.float64)
    qspring = arr("qpos_spring", nq, np.float64)
    dbody = arr("dof_bodyid", nv, np.int32)
    djnt = arr("dof_jntid", nv, np.int32)
    dparent = arr("dof_parentid", nv, np.int32)
    dsolref = arr("dof_solref", (nv, 2), np.float64)
    dsolimp = arr("dof_solimp", (nv, 5), np.float64)
    dfloss = arr("dof_frictionloss", nv, np.float64)
    darm = arr("dof_armature", nv, np.float64)
    ddamp = arr("dof_damping", nv, np.float64)
    arr("dof_invweight0", nv, np.float64)
    arr("dof_M0", nv, np.float64)

    jadr = qadr = dadr = 0
    lastdof = {}
    jid_of = {}
    for b in bodies:
      i = b.id
      par = b.parent
      parentid[i] = par.id if par else 0
      weldid[i] = b.weldid
      jntnum[i] = len(b.cjoints)
      jntadr[i] = jadr if b.cjoints else -1
      dofnum[i] = b.dofnum
      dofadr[i] = dadr if b.dofnum else -1
      geomnum[i] = len(b.cgeoms)
      bpos[i] = b.pos
      bquat[i] = b.quat
      bipos[i] = b.ipos
      biquat[i] = b.iquat
      bmass[i] = b.mass
      binertia[i] = b.inertia
      bgrav[i] = b.gravcomp
      nfree = sum(1 for j in b.cjoints if j["type"] == JNT["free"])
      if nfree > 1 or (nfree == 1 and len(b.cjoints) > 1):
        raise MJCFError("free joint can only appear by itself")
      if nfree and par and par.id != 0:
        raise MJCFError("free joint can only be used on top level")
      rootid[i] = i if (i == 0 or (par and par.id == 0)) else rootid[par.id]
      lastdof[i] = lastdof[par.id] if par else -1
      if is_null_pose(b.ipos, b.iquat):
        sf = 1  # BODY
      elif is_null_pose(None, b.iquat):
        sf = 3  # BODYROT
      else:
        sf = 0
      sameframe[i] = sf
      pid = parentid[i]
      simple[i] = 1 if (sf == 1 and (rootid[i] == i or
                                     (parentid[pid] == 0 and dofnum[pid] == 0))) else 0
      if parentid[i] > 0:
        simple[parentid[i]] = 0
      rotfound = False
      for j in b.cjoints:
        t = j["type"]
        jtype[jadr] = t
        jgroup[jadr] = j["group"]
        jlim[jadr] = 1 if j["limited"] else 0
        jagc[jadr] = 1 if j["actgravcomp"] else 0
        jqadr[jadr] = qadr
        jdadr[jadr] = dadr
        jbody[jadr] = i
        jpos[jadr] = j["pos"]
        jaxis[jadr] = j["axis"]
        jstiff[jadr] = j["stiffness"]
        jrange[jadr] = j["range"]
        jsolref[jadr] = j["solref"]
        jsolimp[jadr] = j["solimp"]
        jmargin[jadr] = j["margin"]
        jid_of[id(j)] = jadr
        ax = j["axis"]
        aligned = ((abs(ax[0]) > mjEPS) + (abs(ax[1]) > mjEPS) + (abs(ax[2]) > mjEPS)) == 1
        if (rotfound or not is_null_pose(j["pos"], None) or
            (t in (JNT["hinge"], JNT["slide"]) and not aligned)):
          simple[i] = 0
        if t in (JNT["ball"], JNT["hinge"]):
          rotfound = True
        if t == JNT["free"]:
          qpos0[qadr:qadr+3] = b.pos
          qpos0[qadr+3:qadr+7] = b.quat
          qspring[qadr:qadr+7] = qpos0[qadr:qadr+7]
        elif t == JNT["ball"]:
          qpos0[qadr:qadr+4] = [1, 0, 0, 0]
          qspring[qadr:qadr+4] = qpos0[qadr:qadr+4]
        else:
          qpos0[qadr] = j["ref"]
          qspring[qadr] = j["springref"]
        for _ in range(_jnt_nv(t)):
          dbody[dadr] = i
          djnt[dadr] = jadr
          dsolref[dadr] = j["solref_f"]
          dsolimp[dadr] = j["solimp_f"]
          dfloss[dadr] = j["frictionloss"]
          darm[dadr] = j["armature"]
          ddamp[dadr] = j["damping"]
          dparent[dadr] = lastdof[i]
          lastdof[i] = dadr
          dadr += 1
        jadr += 1
        qadr += _jnt_nq(t)
      if simple[i] and dofnum[i]:
        simple[i] = 2
        for j in b.cjoints:
          if j["type"] != JNT["slide"]:
            simple[i] = 1
            break
    # geoms
    ng = len(geoms)
    g_int = {k: arr("geom_" + k, ng, np.int32) for k in
             ("type", "contype", "conaffinity", "condim", "bodyid", "group", "priority")}
    gsf = arr("geom_sameframe", ng, np.uint8)
    g_f = {"solmix": arr("geom_solmix", ng, np.float64),
           "rbound": arr("geom_rbound", ng, np.float64),
           "margin": arr("geom_margin", ng, np.float64),
           "gap": arr("geom_gap", ng, np.float64)}
    gsolref = arr("geom_solref", (ng, 2), np.float64)
    gsolimp = arr("geom_solimp", (ng, 5), np.float64)
    gsize = arr("geom_size", (ng, 3), np.float64)
    gpos = arr("geom_pos", (ng, 3), np.float64)
    gquat = arr("geom_quat", (ng, 4), np.float64)
    gfric = arr("geom_friction", (ng, 3), np.float64)
    gfluid = arr("geom_fluid", (ng, 12), np.float64)
    gmatid = arr("geom_matid", ng, np.int32, -1)
    grgba = arr("geom_rgba", (ng, 4), np.float32)
    matnames = list(self.materials)
    s.update(nmat=len(matnames))
    matrgba = arr("mat_rgba", (len(matnames), 4), np.float32)
    for mi, name in enumerate(matnames):
      matrgba[mi] = self.materials[name]
    gdataid = arr("geom_dataid", ng, np.int32, -1)
    for gi, g in enumerate(geoms):
      b = bodies[g["body"]]
      gdataid[gi] = g["dataid"]
      if geomadr[b.id] < 0:
        geomadr[b.id] = gi
      g_int["type"][gi] = g["type"]
      g_int["contype"][gi] = g["contype"]
      g_int["conaffinity"][gi] = g["conaffinity"]
      g_int["condim"][gi] = g["condim"]
      g_int["bodyid"][gi] = g["body"]
      g_int["group"][gi] = g["group"]
      g_int["priority"][gi] = g["priority"]
      if g["type"] == GEOM["plane"] and b.weldid != 0:
        raise MJCFError("plane only allowed in static bodies")
      g_f["solmix"][gi] = g["solmix"]
      g_f["rbound"][gi] = g["rbound"]
      g_f["margin"][gi] = g["margin"]
      g_f["gap"][gi] = g["gap"]
      gsolref[gi] = g["solref"]
      gsolimp[gi] = g["solimp"]
      gsize[gi] = g["size"]
      gpos[gi] = g["pos"]
      gquat[gi] = g["quat"]
      gfric[gi] = g["friction"]
      gfluid[gi] = g["fluid"]
      grgba[gi] = g["rgba"]
      if g["material"] is not None:
        if g["material"] not in self.materials:
          raise MJCFError(f"unknown material '{g['material']}' in geom")
        gmatid[gi] = matnames.index(g["material"])
      gsf[gi] = _sameframe(g["pos"], g["quat"], b.ipos, b.iquat)
      bcontype[b.id] |= g["contype"]
      bconaff[b.id] |= g["conaffinity"]
      bmargin[b.id] = max(bmargin[b.id], g["margin"])
    # meshes and height fields (user_model.cc:2785-2830, hfield arrays alike)
    mlist, hlist = list(self.meshes.values()), list(self.hfields.values())
    s.update(nmesh=len(mlist), nmeshvert=sum(x.nvert for x in mlist),
             nmeshface=sum(x.nface for x in mlist),
             nmeshgraph=sum(len(x.graph) if x.graph else 0 for x in mlist),
             nmeshpoly=sum(len(x.polygons) for x in mlist),
             nmeshpolyvert=sum(len(p) for x in mlist for p in x.polygons),
             nmeshpolymap=sum(len(p) for x in mlist for p in x.polygon_map),
             nhfield=len(hlist), nhfielddata=sum(x.nrow*x.ncol for x in hlist))
    mva = arr("mesh_vertadr", len(mlist), np.int32)
    mvn = arr("mesh_vertnum", len(mlist), np.int32)
    mfa = arr("mesh_faceadr", len(mlist), np.int32)
    mfn = arr("mesh_facenum", len(mlist), np.int32)
    mga = arr("mesh_graphadr", len(mlist), np.int32, -1)
    mvert = arr("mesh_vert", (s["nmeshvert"], 3), np.float32)
    mface = arr("mesh_face", (s["nmeshface"], 3), np.int32)
    mgraph = arr("mesh_graph", s["nmeshgraph"], np.int32)
    # the polygons (CopyPolygonNormals / CopyPolygons / CopyPolygonMap, user_mesh.cc:715-750,
    # user_model.cc:2794-2829): global addresses, mesh-local vertex and polygon ids
    mpn = arr("mesh_polynum", len(mlist), np.int32)
    mpa = arr("mesh_polyadr", len(mlist), np.int32)
    pnormal = arr("mesh_polynormal", (s["nmeshpoly"], 3), np.float64)
    pva = arr("mesh_polyvertadr", s["nmeshpoly"], np.int32)
    pvn = arr("mesh_polyvertnum", s["nmeshpoly"], np.int32)
    pvert = arr("mesh_polyvert", s["nmeshpolyvert"], np.int32)
    pma = arr("mesh_polymapadr", s["nmeshvert"], np.int32)
    pmn = arr("mesh_polymapnum", s["nmeshvert"], np.int32)
    pmap = arr("mesh_polymap", s["nmeshpolymap"], np.int32)
    poly_adr = polyvert_adr = polymap_adr = 0
    vadr = 0
    for mi, x in enumerate(mlist):
      mpa[mi], mpn[mi] = poly_adr, len(x.polygons)
      for i, (p, n) in enumerate(zip(x.polygons, x.polygon_normals)):
        pnormal[poly_adr + i] = n
        pva[poly_adr + i], pvn[poly_adr + i] = polyvert_adr, len(p)
        pvert[polyvert_adr:polyvert_adr + len(p)] = p
        polyvert_adr += len(p)
      for v, lst in enumerate(x.polygon_map):
        pma[vadr + v], pmn[vadr + v] = polymap_adr, len(lst)
        pmap[polymap_adr:polymap_adr + len(lst)] = lst
        polymap_adr += len(lst)
      poly_adr += len(x.polygons)
      vadr += x.nvert
    va = fa = ga_ = 0
    for mi, x in enumerate(mlist):
      mva[mi], mvn[mi], mfa[mi], mfn[mi] = va, x.nvert, fa, x.nface
      mvert[va:va + x.nvert] = x.vert.reshape(-1, 3)
      mface[fa:fa + x.nface] = x.face.reshape(-1, 3)
      if x.graph:
        mga[mi] = ga_
        mgraph[ga_:ga_ + len(x.graph)] = x.graph
        ga_ += len(x.graph)
      va += x.nvert
      fa += x.nface
    hsz = arr("hfield_size", (len(hlist), 4), np.float64)
    hnr = arr("hfield_nrow", len(hlist), np.int32)
    hnc = arr("hfield_ncol", len(hlist), np.int32)
    hadr = arr("hfield_adr", len(hlist), np.int32)
    hdata = arr("hfield_data", s["nhfielddata"], np.float32)
    da = 0
    for hi, x in enumerate(hlist):
      hsz[hi], hnr[hi], hnc[hi], hadr[hi] = x.size, x.nrow, x.ncol, da
      hdata[da:da + x.nrow*x.ncol] = x.data
      da += x.nrow*x.ncol
    # sites
    ns = len(sites)
    stype = arr("site_type", ns, np.int32)
    sbody = arr("site_bodyid", ns, np.int32)
    ssf = arr("site_sameframe", ns, np.uint8)
    ssize = arr("site_size", (ns, 3), np.float64)
    spos = arr("site_pos", (ns, 3), np.float64)
    squat = arr("site_quat", (ns, 4), np.float64)
    for si_, st in enumerate(sites):
      b = bodies[st["body"]]
      stype[si_] = st["type"]
      sbody[si_] = st["body"]
      ssize[si_] = st["size"]
      spos[si_] = st["pos"]
      squat[si_] = st["quat"]
      ssf[si_] = _sameframe(st["pos"], st["quat"], b.ipos, b.iquat)
    # cameras / lights
    nc = len(cams)
    cmode = arr("cam_mode", nc, np.int32)
    cbody = arr("cam_bodyid", nc, np.int32)
    ctarget = arr("cam_targetbodyid", nc, np.int32, -1)
    cpos = arr("cam_pos", (nc, 3), np.float64)
    cquat = arr("cam_quat", (nc, 4), np.float64)
    arr("cam_poscom0", (nc, 3), np.float64)
    arr("cam_pos0", (nc, 3), np.float64)
    arr("cam_mat0", (nc, 9), np.float64)
    cfovy = arr("cam_fovy", nc, np.float64)
    cres = arr("cam_resolution", (nc, 2), np.int32)
    csize = arr("cam_sensorsize", (nc, 2), np.float32)
    cintr = arr("cam_intrinsic", (nc, 4), np.float32)
    for ci, c in enumerate(cams):
      cfovy[ci] = c["fovy"]
      cres[ci] = c["resolution"]
      csize[ci] = c["sensorsize"]
      cintr[ci] = c["intrinsic"]
      cmode[ci] = c["mode"]
      cbody[ci] = c["body"]
      cpos[ci] = c["pos"]
      cquat[ci] = c["quat"]
      if c["target"]:
        ctarget[ci] = bname[c["target"]]
    nl = len(lights)
    lmode = arr("light_mode", nl, np.int32)
    lbody = arr("light_bodyid", nl, np.int32)
    ltarget = arr("light_targetbodyid", nl, np.int32, -1)
    lpos = arr("light_pos", (nl, 3), np.float64)
    ldir = arr("light_dir", (nl, 3), np.float64)
    arr("light_poscom0", (nl, 3), np.float64)
    arr("light_pos0", (nl, 3), np.float64)
    arr("light_dir0", (nl, 3), np.float64)
    for li, l in enumerate(lights):
      lmode[li] = l["mode"]
      lbody[li] = l["body"]
      lpos[li] = l["pos"]
      ldir[li] = l["dir"]
      if l["target"]:
        ltarget[li] = bname[l["target"]]
    # tendons (fixed only)
    nt = len(self.tendons)
    nwrap = sum(len(jl) for _, jl in self.tendons)
    tadr = arr("tendon_adr", nt, np.int32)
    tnum = arr("tendon_num", nt, np.int32)
    tlim = arr("tendon_limited", nt, np.uint8)
    tsolref = arr("tendon_solref_lim", (nt, 2), np.float64)
    tsolimp = arr("tendon_solimp_lim", (nt, 5), np.float64)
    trange = arr("tendon_range", (nt, 2), np.float64)
    tmargin = arr("tendon_margin", nt, np.float64)
    tstiff = arr("tendon_stiffness", nt, np.float64)
    tdamp = arr("tendon_damping", nt, np.float64)
    tfloss = arr("tendon_frictionloss", nt, np.float64)
    tsolref_f = arr("tendon_solref_fri", (nt, 2), np.float64)
    tsolimp_f = arr("tendon_solimp_fri", (nt, 5), np.float64)
    tls = arr("tendon_lengthspring", (nt, 2), np.float64)
    arr("tendon_length0", nt, np.float64)
    arr("tendon_invweight0", nt, np.float64)
    wtype = arr("wrap_type", nwrap, np.int32)
    wobj = arr("wrap_objid", nwrap, np.int32)
    wprm = arr("wrap_prm", nwrap, np.float64)
    w = 0
    sitename_t = {x["name"]: i for i, x in enumerate(sites) if x["name"]}
    geomname_t = {g["name"]: i for i, g in enumerate(geoms) if g["name"]}
    for ti, (ta, jl) in enumerate(self.tendons):
      tadr[ti] = w
      tnum[ti] = len(jl)
      rng = _floats(ta["range"]) if "range" in ta else [0.0, 0.0]
      lim = ta.get("limited", "auto")
      if lim == "auto":
        limited = self.autolimits and not (rng[0] == 0 and rng[1] == 0)
      else:
        limited = lim == "true"
      if limited and rng[0] >= rng[1]:
        raise MJCFError("invalid tendon range")
      tlim[ti] = limited
      trange[ti] = rng
      tsolref[ti] = _floats(ta["solreflimit"]) if "solreflimit" in ta else [0.02, 1.0]
      si = [0.9, 0.95, 0.001, 0.5, 2.0]
      if "solimplimit" in ta:
        v = _floats(ta["solimplimit"])
        si[:len(v)] = v
      tsolimp[ti] = si
      tmargin[ti] = float(ta.get("margin", 0.0))
      tstiff[ti] = float(ta.get("stiffness", 0.0))
      tdamp[ti] = float(ta.get("damping", 0.0))
      # friction loss (mj_instantiateFriction's FRICTION_TENDON rows) and its solver
      # parameters, defaults as mjCTendon's (solreffriction / solimpfriction)
      tfloss[ti] = float(ta.get("frictionloss", 0.0))
      if tfloss[ti] < 0:
        raise MJCFError(f"tendon '{ta.get('name', '')}' (id = {ti}): frictionloss must be "
                        "nonnegative")
      tsolref_f[ti] = _floats(ta["solreffriction"]) if "solreffriction" in ta else [0.02, 1.0]
      si = [0.9, 0.95, 0.001, 0.5, 2.0]
      if "solimpfriction" in ta:
        v = _floats(ta["solimpfriction"])
        si[:len(v)] = v
      tsolimp_f[ti] = si
      sl = _floats(ta["springlength"]) if "springlength" in ta else [-1.0, -1.0]
      if len(sl) == 1:
        sl = [sl[0], sl[0]]
      tls[ti] = sl
      if ta["__kind"] == "spatial":
        # mjCTendon::Compile (user_objects.cc:5448-5570): path rules; wraps compiled as
        # user_model.cc:3215-3222 (site: prm 0; pulley: prm = divisor, objid -1)
        sz = len(jl)
        if sz < 2:
          raise MJCFError(f"tendon '{ta.get('name', '')}' (id = {ti}): spatial path must "
                          "contain at least two objects")
        if float(ta.get("width", 0.003)) <= 0:
          raise MJCFError(f"tendon '{ta.get('name', '')}' (id = {ti}) must have positive width")
        for i, (kind, val) in enumerate(jl):
          if kind == "pulley":
            if i > 0 and jl[i - 1][0] == "pulley":
              raise MJCFError(f"tendon (id = {ti}): consecutive pulleys (pos {i})")
            if i == sz - 1:
              raise MJCFError(f"tendon (id = {ti}): path ends with pulley")
            wtype[w], wobj[w], wprm[w] = 2, -1, val     # mjWRAP_PULLEY
          elif kind == "geom":
            # mjCWrap::Compile (user_objects.cc:5647-5676): sphere or cylinder geom, optional
            # side site; wrap_prm = side site id or -1 (user_model.cc:3219-3221)
            gname, side = val
            if gname not in geomname_t:
              raise MJCFError(f"geom '{gname}' not found in tendon {ti}, wrap {i}")
            gi = geomname_t[gname]
            gt = geoms[gi]["type"]
            if gt not in (GEOM["sphere"], GEOM["cylinder"]):
              raise MJCFError(f"geom '{gname}' in tendon {ti}, wrap {i} is not sphere or "
                              "cylinder")
            sid = -1
            if side is not None:
              if side not in sitename_t:
                raise MJCFError(f"side site '{side}' not found in tendon {ti}, wrap {i}")
              sid = sitename_t[side]
            if i == 0 or i == sz - 1 or jl[i - 1][0] != "site" or jl[i + 1][0] != "site":
              raise MJCFError(f"tendon '{ta.get('name', '')}' (id = {ti}): geom at pos {i} "
                              "not bracketed by sites")
            wtype[w] = 4 if gt == GEOM["sphere"] else 5   # mjWRAP_SPHERE / mjWRAP_CYLINDER
            wobj[w], wprm[w] = gi, float(sid)
          else:
            if val not in sitename_t:
              raise MJCFError(f"unknown site '{val}' in tendon")
            if (i == 0 or jl[i - 1][0] == "pulley") and (i == sz - 1 or jl[i + 1][0] == "pulley"):
              raise MJCFError(f"tendon (id = {ti}): site {i} needs a neighbor that is not a "
                              "pulley")
            if i < sz - 1 and jl[i + 1][0] == "site" and jl[i + 1][1] == val:
              raise MJCFError(f"tendon (id = {ti}): site {i} is repeated")
            wtype[w], wobj[w], wprm[w] = 3, sitename_t[val], 0.0   # mjWRAP_SITE
          w += 1
        if sl[0] > sl[1]:
          raise MJCFError("invalid springlength in tendon")
        continue
      for jn, coef in jl:
        if jn not in jname:
          raise MJCFError(f"unknown joint '{jn}' in tendon")
        wtype[w] = 1  # mjWRAP_JOINT
        wobj[w] = jname[jn]
        wprm[w] = coef
        w += 1
    # actuators (joint transmission)
    nu = len(self.actuators)
    atrn = arr("actuator_trntype", nu, np.int32)
    adyn = arr("actuator_dyntype", nu, np.int32)
    again = arr("actuator_gaintype", nu, np.int32)
    abias = arr("actuator_biastype", nu, np.int32)
    atrnid = arr("actuator_trnid", (nu, 2), np.int32, -1)
    actl = arr("actuator_ctrllimited", nu, np.uint8)
    afl = arr("actuator_forcelimited", nu, np.uint8)
    adynprm = arr("actuator_dynprm", (nu, 10), np.float64)
    againprm = arr("actuator_gainprm", (nu, 10), np.float64)
    abiasprm = arr("actuator_biasprm", (nu, 10), np.float64)
    actr = arr("actuator_ctrlrange", (nu, 2), np.float64)
    afr = arr("actuator_forcerange", (nu, 2), np.float64)
    agear = arr("actuator_gear", (nu, 6), np.float64)
    acrank = arr("actuator_cranklength", nu, np.float64)
    arr("actuator_length0", nu, np.float64)
    arr("actuator_acc0", nu, np.float64)
    na_count = 0                        # activation states (dyntype != none)
    for ai, a in enumerate(self.actuators):
      tag = a["__tag"]
      sitename = {x["name"]: i for i, x in enumerate(sites) if x["name"]}
      tname = {"joint": jname, "jointinparent": jname, "cranksite": sitename, "site": sitename,
               "tendon": {ta.get("name"): i for i, (ta, _) in enumerate(self.tendons)
                          if ta.get("name")},
               "body": {b.name: b.id for b in self.bodies if b.name}}
      trn = [k for k in ("joint", "jointinparent", "tendon", "cranksite", "site", "body")
             if k in a]
      if len(trn) != 1:
        raise MJCFError("actuator has no transmission target" if not trn
                        else "actuator has more than one transmission target")
      if "refsite" in a and trn[0] != "site":
        raise MJCFError("reference site is only allowed with a site transmission")
      if a[trn[0]] not in tname[trn[0]]:
        raise MJCFError(f"unknown {trn[0]} '{a[trn[0]]}' in actuator")
      atrn[ai] = {"joint": 0, "jointinparent": 1, "cranksite": 2, "tendon": 3,
                  "site": 4, "body": 5}[trn[0]]
      atrnid[ai, 0] = tname[trn[0]][a[trn[0]]]
      if trn[0] == "cranksite":         # mjCActuator::ResolveReferences (user_objects.cc:5858-5877)
        if not a.get("slidersite"):
          raise MJCFError("missing base site for slider-crank")
        if a["slidersite"] not in sitename:
          raise MJCFError(f"base site '{a['slidersite']}' not found")
        atrnid[ai, 1] = sitename[a["slidersite"]]
        acrank[ai] = float(a.get("cranklength", 0.0))
        if acrank[ai] <= 0:
          raise MJCFError("crank length must be positive")
      if trn[0] == "site" and "refsite" in a:   # user_objects.cc ResolveReferences
        if a["refsite"] not in sitename:
          raise MJCFError(f"reference site '{a['refsite']}' not found")
        atrnid[ai, 1] = sitename[a["refsite"]]
      gear = [1.0, 0, 0, 0, 0, 0]
      if "gear" in a:
        g = _floats(a["gear"])
        gear[:len(g)] = g
      agear[ai] = gear
      adynprm[ai, 0] = 1.0
      againprm[ai, 0] = 1.0
      if tag == "general":
        if "gainprm" in a:
          v = _floats(a["gainprm"])
          againprm[ai, :len(v)] = v
        if "biasprm" in a:
          v = _floats(a["biasprm"])
          abiasprm[ai, :len(v)] = v
        again[ai] = {"fixed": 0, "affine": 1}[a.get("gaintype", "fixed")]
        abias[ai] = {"none": 0, "affine": 1}[a.get("biastype", "none")]
        dyn = a.get("dyntype", "none")
        if dyn not in ("none", "integrator", "filter", "filterexact"):
          raise MJCFError(f"actuator dyntype '{dyn}' is not in the supported subset")
        adyn[ai] = {"none": 0, "integrator": 1, "filter": 2, "filterexact": 3}[dyn]
        if adyn[ai] and again[ai] == 1 and againprm[ai, 2] != 0:
          # mjd_actuator_vel (engine_derivative.c:855-863) multiplies the velocity gain by
          # mjData.act[last] for such an actuator; act is not an input of this path
          raise MJCFError("an affine velocity gain with activation dynamics is not in the "
                          "supported subset")
        if "dynprm" in a:
          v = _floats(a["dynprm"])
          adynprm[ai, :len(v)] = v
        na_count += adyn[ai] != 0
      elif tag == "position":          # xml_native_reader.cc:2190-2240
        kp = float(a.get("kp", 1.0))
        kv = float(a.get("kv", -1.0))
        dampratio = float(a.get("dampratio", -1.0))
        if "kv" in a and kv < 0:
          raise MJCFError("kv cannot be negative")
        if dampratio > 0 and kv > 0:
          raise MJCFError("kv and dampratio cannot both be defined")
        againprm[ai, 0] = kp
        abias[ai] = 1
        abiasprm[ai, 1] = -kp
        if kv > 0:
          abiasprm[ai, 2] = -kv
        if dampratio > 0:
          raise MJCFError("position actuator dampratio (resolved by mj_setConst) is not in "
                          "the supported subset")
        inherit = float(a.get("inheritrange", 0.0))
        if inherit > 0:
          if "ctrlrange" in a and any(_floats(a["ctrlrange"])):
            raise MJCFError("ctrlrange and inheritrange cannot both be defined")
          # mjCActuator::Compile (user_objects.cc:5940-5982): the compiled (radian) range of
          # the hinge/slide joint or tendon, scaled about its mean
          if trn[0] in ("joint", "jointinparent"):
            jt = jtype[atrnid[ai, 0]]
            if jt not in (JNT["hinge"], JNT["slide"]):
              raise MJCFError("inheritrange can only be used with hinge and slide joints, "
                              "actuator")
            rng = jrange[atrnid[ai, 0]]
          elif trn[0] == "tendon":
            rng = trange[atrnid[ai, 0]]
          else:
            raise MJCFError("inheritrange can only be used with joint and tendon "
                            "transmission, actuator")
          if rng[0] == rng[1]:
            raise MJCFError(f"inheritrange used but target '{a[trn[0]]}' has no range "
                            f"defined in actuator {ai}")
          mean = 0.5 * (rng[1] + rng[0])
          radius = 0.5 * (rng[1] - rng[0]) * inherit
          a = dict(a, ctrlrange=f"{float(mean - radius)!r} {float(mean + radius)!r}")
      elif tag == "velocity":
        kv = float(a.get("kv", 1.0))
        againprm[ai, 0] = kv
        abias[ai] = 1
        abiasprm[ai, 2] = -kv
      elif tag == "intvelocity":        # mjs_setToIntVelocity: an integrator driving a
        kp = float(a.get("kp", 1.0))    # position servo on the activation
        kv = float(a.get("kv", 0.0))
        adyn[ai] = 1
        againprm[ai, 0] = kp
        abias[ai] = 1
        abiasprm[ai, 1] = -kp
        abiasprm[ai, 2] = -kv
        na_count += 1
      elif tag == "adhesion":           # xml_native_reader.cc:2341-2356
        againprm[ai, 0] = float(a.get("gain", 1.0))
        if againprm[ai, 0] < 0:
          raise MJCFError("adhesion gain cannot be negative")
        cr = _floats(a["ctrlrange"]) if "ctrlrange" in a else [0.0, 0.0]
        if cr[0] < 0 or cr[1] < 0:
          raise MJCFError("adhesion control range cannot be negative")
        a = dict(a, ctrllimited="true")
      cr = _floats(a["ctrlrange"]) if "ctrlrange" in a else [0.0, 0.0]
      cl = a.get("ctrllimited", "auto")
      actl[ai] = (not (cr[0] == 0 and cr[1] == 0)) if cl == "auto" else (cl == "true")
      actr[ai] = cr
      fr = _floats(a["forcerange"]) if "forcerange" in a else [0.0, 0.0]
      fl = a.get("forcelimited", "auto")
      afl[ai] = (not (fr[0] == 0 and fr[1] == 0)) if fl == "auto" else (fl == "true")
      afr[ai] = fr
    # equality constraints (xml_native_reader.cc:1898-2035, user_objects.cc:5139-5220;
    # eq_data defaults mjs_defaultEquality user_init.c:312-319; missing body-constraint
    # data are filled by setconst.py as mj_setConst does, engine_setconst.c:289-340)
    neq = len(self.equalities)
    eqt = arr("eq_type", neq, np.int32)
    eq1 = arr("eq_obj1id", neq, np.int32, -1)
    eq2 = arr("eq_obj2id", neq, np.int32, -1)
    eqo = arr("eq_objtype", neq, np.int32)
    eqa = arr("eq_active0", neq, np.uint8)
    eqsr = arr("eq_solref", (neq, 2), np.float64)
    eqsi = arr("eq_solimp", (neq, 5), np.float64)
    eqd = arr("eq_data", (neq, 11), np.float64)
    sitename = {x["name"]: i for i, x in enumerate(sites) if x["name"]}
    tendonname = {ta.get("name"): i for i, (ta, _) in enumerate(self.tendons) if ta.get("name")}
    for ei, a in enumerate(self.equalities):
      tag = a["__tag"]
      data = np.zeros(11)
      data[1] = 1
      data[10] = 1
      if tag in ("connect", "weld"):
        site = "site1" in a or "site2" in a
        if site and ("body1" in a or "body2" in a or "anchor" in a or "relpose" in a):
          raise MJCFError("body and site semantics cannot be mixed")
        if "anchor" in a:
          data[0:3] = _floats(a["anchor"])
        elif tag == "weld" and not site:
          data[0:3] = 0
        if tag == "weld":
          if "relpose" in a:
            data[3:10] = _floats(a["relpose"])
          if "torquescale" in a:
            data[10] = float(a["torquescale"])
        if site:
          if "site1" not in a or "site2" not in a:
            raise MJCFError("both site1 and site2 must be defined")
          eqo[ei] = 6
          n1, n2, table = a["site1"], a["site2"], sitename
        else:
          if "body1" not in a or (tag == "connect" and "anchor" not in a):
            raise MJCFError("body1 (and anchor for connect) must be defined")
          eqo[ei] = 1
          n1, n2, table = a["body1"], a.get("body2"), bname
        eqt[ei] = 0 if tag == "connect" else 1
      else:
        eqt[ei] = 2 if tag == "joint" else 3
        eqo[ei] = 3 if tag == "joint" else 18
        n1, n2 = a.get(tag + "1"), a.get(tag + "2")
        table = jname if tag == "joint" else tendonname
        if "polycoef" in a:
          v = _floats(a["polycoef"])
          data[:len(v)] = v
      if n1 not in table or (n2 is not None and n2 not in table):
        raise MJCFError(f"unknown element in equality constraint ({n1}, {n2})")
      eq1[ei] = table[n1]
      eq2[ei] = table[n2] if n2 is not None else (0 if eqo[ei] == 1 else -1)
      if eq1[ei] == eq2[ei]:
        raise MJCFError("element is repeated in equality constraint")
      if tag == "joint":
        for jj in (eq1[ei], eq2[ei]):
          if jj >= 0 and int(jtype[jj]) not in (2, 3):
            raise MJCFError("only scalar joints can be coupled")
      eqa[ei] = a.get("active", "true") == "true"
      eqsr[ei] = _floats(a["solref"]) if "solref" in a else [0.02, 1.0]
      si = [0.9, 0.95, 0.001, 0.5, 2.0]
      if "solimp" in a:
        v = _floats(a["solimp"])
        si[:len(v)] = v
      eqsi[ei] = si
      eqd[ei] = data
    s.update(neq=neq)
    # sensors (user_objects.cc mjCSensor::Compile :6250-6580, user_model.cc:3265-3286)
    ns_ = len(self.sensors)
    stype = arr("sensor_type", ns_, np.int32)
    sdtype = arr("sensor_datatype", ns_, np.int32)
    sstage = arr("sensor_needstage", ns_, np.int32)
    sobjt = arr("sensor_objtype", ns_, np.int32)
    sobj = arr("sensor_objid", ns_, np.int32, -1)
    sreft = arr("sensor_reftype", ns_, np.int32)
    sref = arr("sensor_refid", ns_, np.int32, -1)
    sdim = arr("sensor_dim", ns_, np.int32)
    sadr = arr("sensor_adr", ns_, np.int32)
    scut = arr("sensor_cutoff", ns_, np.float64)
    lookup = {1: bname, 2: bname, 3: jname,
              5: {g["name"]: i for i, g in enumerate(geoms) if g["name"]},
              6: {x["name"]: i for i, x in enumerate(sites) if x["name"]},
              7: {c["name"]: i for i, c in enumerate(cams) if c["name"]},
              18: {ta.get("name"): i for i, (ta, _) in enumerate(self.tendons) if ta.get("name")},
              19: {a.get("name"): i for i, a in enumerate(self.actuators) if a.get("name")}}

    def find(ot, name, what):
      if not name:
        raise MJCFError(f"missing name of {what} in sensor")
      if name not in lookup.get(ot, {}):
        raise MJCFError(f"unrecognized name '{name}' of {what} in sensor")
      return lookup[ot][name]
    sensadr = 0
    for si_, (tag, a) in enumerate(self.sensors):
      tp, attr, ot, dim, dt, st = SENSORS[tag]
      cut = float(a.get("cutoff", 0.0))
      if cut < 0 or float(a.get("noise", 0.0)) < 0:
        raise MJCFError("negative noise/cutoff in sensor")
      rt, rid = 0, -1
      if tp in (37, 38, 39):                       # geom distance: (geom1|body1, geom2|body2)
        sides = []
        for k in ("1", "2"):
          hb, hg = f"body{k}" in a, f"geom{k}" in a
          if hb == hg:
            raise MJCFError(f"exactly one of (geom{k}, body{k}) must be specified")
          t_ = 1 if hb else 5
          sides.append((t_, find(t_, a[f"body{k}" if hb else f"geom{k}"], "sensorized object")))
        (ot, oid), (rt, rid) = sides
        if (ot, oid) == (rt, rid):
          raise MJCFError("1st body/geom must be different from 2nd body/geom")
        for t_, i_ in sides:
          if t_ == 5 and g_int["type"][i_] == GEOM["hfield"]:
            raise MJCFError("height fields are not supported in geom distance sensors")
      elif attr is None and ot is None:              # frame sensors
        ot = OBJ.get(a.get("objtype", ""), None)
        if ot not in (1, 2, 5, 6, 7):
          raise MJCFError("sensor must be attached to (x)body, geom, site or camera")
        oid = find(ot, a.get("objname"), "sensorized object")
        if "reftype" in a and tp <= 31:
          rt = OBJ.get(a["reftype"], None)
          if rt not in (1, 2, 5, 6, 7):
            raise MJCFError("reference frame object must be (x)body, geom, site or camera")
          rid = find(rt, a.get("refname"), "reference frame object")
        elif "refname" in a and tp <= 31:
          raise MJCFError("refname given but reftype is missing")
      elif attr is None:                           # global sensors
        oid = -1
      else:
        oid = find(ot, a.get(attr), "sensorized object")
        if tp == 8:                                # camprojection: the camera is the reference
          rt, rid = 7, find(7, a.get("camera"), "camera")
        if ot == 3:
          jt = int(jtype[oid])
          if tp in (9, 10, 16) and jt not in (2, 3):
            raise MJCFError("joint must be slide or hinge in sensor")
          if tp in (17, 18) and jt != 1:
            raise MJCFError("joint must be ball in sensor")
          if tp in (19, 20, 21) and not jlim[oid]:
            raise MJCFError("joint must be limited in sensor")
        if ot == 18 and tp in (22, 23, 24) and not tlim[oid]:
          raise MJCFError("tendon must be limited in sensor")
      stype[si_], sdtype[si_], sstage[si_], sobjt[si_], sobj[si_] = tp, dt, st, ot, oid
      sreft[si_], sref[si_], sdim[si_], sadr[si_], scut[si_] = rt, rid, dim, sensadr, cut
      sensadr += dim
    s.update(nsensor=ns_, nsensordata=sensadr)
    # exclude pairs: signature = (body1 << 16) + body2 with body1 < body2, stably sorted by
    # signature (user_model.cc:4321-4324)
    nex = len(self.excludes)
    exs = arr("exclude_signature", nex, np.int32)
    sigs = []
    for b1, b2 in self.excludes:
      i1, i2 = bname[b1], bname[b2]
      sigs.append((min(i1, i2) << 16) + max(i1, i2))
    exs[:] = sorted(sigs)
    self._compile_pairs(arr, s, geoms)
    # keyframes
    nkey = len(self.keys)
    kq = arr("key_qpos", (nkey, nq), np.float64)
    for ki, k in enumerate(self.keys):
      kq[ki] = qpos0
      if "qpos" in k:
        kq[ki] = _floats(k["qpos"])
    s.update(nu=nu, ntendon=nt, nwrap=nwrap, nexclude=nex, nkey=nkey, na=int(na_count))
    # ---- dof tree quantities (user_model.cc:2441-2617)
    ntree = 0
    dtree = arr("dof_treeid", nv, np.int32)
    for i in range(nv):
      if dparent[i] == -1:
        ntree += 1
      dtree[i] = ntree - 1
    btree = arr("body_treeid", nbody, np.int32, -1)
    for i in range(nbody):
      wid = weldid[i]
      if dofnum[wid]:
        btree[i] = dtree[dofadr[wid]]
    s["ntree"] = ntree
    s["ngravcomp"] = int(np.sum(bgrav > 0))
    Madr = arr("dof_Madr", nv, np.int32)
    nM = 0
    for i in range(nv):
      Madr[i] = nM
      j = i
      while j >= 0:
        nM += 1
        j = dparent[j]
    s["nM"] = nM
    s["nD"] = 2*nM - nv
    simplenum = arr("dof_simplenum", nv, np.int32)
    count = 0
    for i in range(nv - 1, -1, -1):
      count = count + 1 if simple[dbody[i]] else 0
      simplenum[i] = count
    nOD = 0
    for i in range(nv):
      if not simplenum[i]:
        j = i
        while j >= 0:
          if j != i:
            nOD += 1
          j = dparent[j]
    s["nC"] = nC = nOD + nv
    # nJmom as CountNJmom (user_model.cc:2703-2750): 1/3/6 per joint transmission, nv per
    # tendon, slider-crank or site transmission, so actuator_moment has the reference's size
    s["nJmom"] = sum({0: 6, 1: 3, 2: 1, 3: 1}[int(jtype[atrnid[ai, 0]])] if atrn[ai] in (0, 1)
                     else nv for ai in range(nu))
    A.update(sparse_structures(s, A, jacobian=int(self.opt["jacobian"])))
    # scalars and names
    m.opt = {k: (list(v) if isinstance(v, list) else v) for k, v in self.opt.items()}
    for k, v in A.items():
      setattr(m, k, v)
    arr("body_subtreemass", nbody, np.float64)
    arr("body_invweight0", (nbody, 2), np.float64)
    setattr(m, "body_subtreemass", A["body_subtreemass"])
    setattr(m, "body_invweight0", A["body_invweight0"])
    m.names = {"body": [b.name for b in bodies], "jnt": [j["name"] for j in jnts],
               "geom": [g["name"] for g in geoms], "site": [x["name"] for x in sites],
               "cam": [c["name"] for c in cams], "light": [l["name"] for l in lights],
               "tendon": [ta.get("name", "") for ta, _ in self.tendons],
               "actuator": [a.get("name", "") for a in self.actuators],
               "sensor": [a.get("name", "") for _, a in self.sensors],
               "key": [k.get("name", "") for k in self.keys]}
    m.model_name = getattr(self, "model_name", "")
    # check every field of the table is present with the right shape
    for f in fields.MODEL_FIELDS:
      a = getattr(m, f.name)
      want = f.shape(m.sizes)
      if want[1] == 1:
        want = want[:1]
      setattr(m, f.name, np.ascontiguousarray(a.reshape(want).astype(fields.NPTYPE[f.ctype])))
    return m


def sparse_structures(sizes: dict, A, jacobian: int = 2) -> dict:
  """The model-constant sparse structures the reference keeps in mjData (mj_makeData):
  C (reduced LTDL pattern) and mapM2C, D (dof x dof) and mapM2D, B (body x dof), and the
  actuator moment pattern. `A` maps mjModel field names to arrays (the compiler's, or an
  imported .mjb's, mjb.py); sizes needs nv, nbody, nu, nM, nC, nD, nB, nJmom. Returns the
  new arrays by field name; raises MJCFError on an inconsistent model."""
  nv, nbody, nu = sizes["nv"], sizes["nbody"], sizes["nu"]
  nC, nD, nJmom = sizes["nC"], sizes["nD"], sizes["nJmom"]
  sparse_jac = jacobian == 1 or (jacobian == 2 and nv >= 60)     # mj_isSparse
  dparent = np.asarray(A["dof_parentid"]).reshape(-1)
  simplenum = np.asarray(A["dof_simplenum"]).reshape(-1)
  Madr = np.asarray(A["dof_Madr"]).reshape(-1)
  dbody = np.asarray(A["dof_bodyid"]).reshape(-1)
  parentid = np.asarray(A["body_parentid"]).reshape(-1)
  dofadr = np.asarray(A["body_dofadr"]).reshape(-1)
  dofnum = np.asarray(A["body_dofnum"]).reshape(-1)
  atrn = np.asarray(A["actuator_trntype"]).reshape(-1)
  atrnid = np.asarray(A["actuator_trnid"]).reshape(-1, 2)
  agear = np.asarray(A["actuator_gear"]).reshape(-1, 6)
  jtype = np.asarray(A["jnt_type"]).reshape(-1)
  jdadr = np.asarray(A["jnt_dofadr"]).reshape(-1)
  sbody = np.asarray(A["site_bodyid"]).reshape(-1)
  tadr = np.asarray(A["tendon_adr"]).reshape(-1)
  tnum = np.asarray(A["tendon_num"]).reshape(-1)
  wobj = np.asarray(A["wrap_objid"]).reshape(-1)
  wprm = np.asarray(A["wrap_prm"]).reshape(-1)
  out = {}

  def arr(name, shape, dtype, fill=0):
    out[name] = np.full(shape, fill, dtype=dtype)
    return out[name]

  # C sparse structure and mapM2C (engine_io.c:929-1018, 1135-1259; reduced=1)
  rownnz = arr("C_rownnz", nv, np.int32)
  rowadr = arr("C_rowadr", nv, np.int32)
  colind = arr("C_colind", nC, np.int32)
  mapM2C = arr("mapM2C", nC, np.int32, -1)
  for i in range(nv - 1, -1, -1):
    rownnz[i] += 1
    if not simplenum[i]:
      j = i
      while True:
        j = dparent[j]
        if j < 0:
          break
        rownnz[i] += 1
  for i in range(1, nv):
    rowadr[i] = rowadr[i-1] + rownnz[i-1]
  remaining = rownnz.copy()
  for i in range(nv - 1, -1, -1):
    remaining[i] -= 1
    colind[rowadr[i] + remaining[i]] = i
    adr = Madr[i]
    mapM2C[rowadr[i] + remaining[i]] = adr
    adr += 1
    if not simplenum[i]:
      j = i
      while True:
        j = dparent[j]
        if j < 0:
          break
        remaining[i] -= 1
        colind[rowadr[i] + remaining[i]] = j
        mapM2C[rowadr[i] + remaining[i]] = adr
        adr += 1
  if nv and (remaining != 0).any():
    raise MJCFError("unexpected remaining")  # SHOULD NOT OCCUR
  # D sparse structure (dof x dof, ancestors and descendants) and mapM2D
  # (engine_io.c:929-1018 with reduced=0, :1135-1232): row i lists every dof on i's chain
  # to the root and in i's subtree, ascending
  cols = [[i] for i in range(nv)]
  for i in range(nv - 1, -1, -1):
    j = dparent[i]
    while j >= 0:
      cols[i].append(j)
      cols[j].append(i)
      j = dparent[j]
  Drownnz = arr("D_rownnz", nv, np.int32)
  Drowadr = arr("D_rowadr", nv, np.int32)
  Dcolind = arr("D_colind", nD, np.int32)
  mapM2D = arr("mapM2D", nD, np.int32, -1)
  for i in range(nv):
    Drownnz[i] = len(cols[i])
    Drowadr[i] = Drowadr[i-1] + Drownnz[i-1] if i else 0
    Dcolind[Drowadr[i]:Drowadr[i] + Drownnz[i]] = sorted(cols[i])
  for i in range(nv):                 # qM element (i, j), j on i's chain, at Madr[i] + k
    adr, j = Madr[i], i
    while j >= 0:
      for r, c in ((i, j), (j, i)):
        row = Dcolind[Drowadr[r]:Drowadr[r] + Drownnz[r]]
        mapM2D[Drowadr[r] + int(np.searchsorted(row, c))] = adr
      adr += 1
      j = dparent[j]
  if nv and ((mapM2D < 0).any() or Drowadr[-1] + Drownnz[-1] != nD):
    raise MJCFError("D sparsity mismatch")  # SHOULD NOT OCCUR
  # B sparse structure (body x dof: ancestor and subtree dofs, ascending),
  # engine_io.c:1021-1106 makeBSparse
  bcols = [set() for _ in range(nbody)]
  for i in range(nbody - 1, 0, -1):
    bcols[i].update(range(dofadr[i], dofadr[i] + dofnum[i]))
    bcols[parentid[i]].update(bcols[i])
  for i in range(nbody):
    p = parentid[i] if i else -1
    while p > 0:
      bcols[i].update(range(dofadr[p], dofadr[p] + dofnum[p]))
      p = parentid[p]
  nB = sum(len(c) for c in bcols)
  if nB != sizes.setdefault("nB", nB):
    raise MJCFError("B sparsity size mismatch")
  Brownnz = arr("B_rownnz", nbody, np.int32)
  Browadr = arr("B_rowadr", nbody, np.int32)
  Bcolind = arr("B_colind", nB, np.int32)
  for i in range(nbody):
    Brownnz[i] = len(bcols[i])
    Browadr[i] = Browadr[i-1] + Brownnz[i-1] if i else 0
    Bcolind[Browadr[i]:Browadr[i] + Brownnz[i]] = sorted(bcols[i])
  for j in range(nv):                 # checkDBSparse engine_io.c:1111-1130
    b = dbody[j]
    if list(Dcolind[Drowadr[j]:Drowadr[j] + Drownnz[j]]) != \
       list(Bcolind[Browadr[b]:Browadr[b] + Brownnz[b]]):
      raise MJCFError("D and B sparsity differ")  # SHOULD NOT OCCUR
  # actuator moment sparsity (mj_transmission, engine_core_smooth.c:884-1081). For the
  # transmissions in the subset it depends on the model only: a joint's dofs, or the dofs
  # where a fixed tendon's dense ten_J row times gear[0] is nonzero (the dense compress
  # loop :1070-1079; ten_J entries are the wrap coefficients, last one per joint wins,
  # smooth.c mj_tendon dense branch). rowadr is cumulative (:896).
  mrownnz = arr("moment_rownnz", nu, np.int32)
  mrowadr = arr("moment_rowadr", nu, np.int32)
  cols = []
  for ai in range(nu):
    tid = int(atrnid[ai, 0])
    if atrn[ai] in (0, 1):
      cnt = {0: 6, 1: 3, 2: 1, 3: 1}[int(jtype[tid])]
      c = list(range(jdadr[tid], jdadr[tid] + cnt))
    elif atrn[ai] == 5:
      # body (adhesion): the mean normal Jacobian of the body's contacts (:1228-1318); any
      # dof can appear (the other body of a contact), so the row is dense
      c = list(range(nv))
    elif atrn[ai] == 4 and atrnid[ai, 1] >= 0:
      # site relative to a reference site (:1105-1212): the difference of the two sites'
      # Jacobians with the shared ancestral chain cleared, i.e. the symmetric difference of
      # the two dof chains
      chains = []
      for sid in atrnid[ai]:
        c = set()
        b = int(sbody[sid])
        while b > 0:
          c.update(range(dofadr[b], dofadr[b] + dofnum[b]))
          b = int(parentid[b])
        chains.append(c)
      c = [] if not np.any(agear[ai]) else sorted(chains[0] ^ chains[1])
    elif atrn[ai] in (2, 4):
      # slider-crank: the dense moment is the chain rule over the two sites' Jacobians
      # (:1035-1052); its structural nonzeros are the dofs of both sites' body chains
      c = set()
      for sid in atrnid[ai]:
        if sid < 0:
          continue
        b = int(sbody[sid])
        while b > 0:
          c.update(range(dofadr[b], dofadr[b] + dofnum[b]))
          b = int(parentid[b])
      gzero = agear[ai, 0] == 0 if atrn[ai] == 2 else not np.any(agear[ai])
      c = [] if gzero else sorted(c)
    elif int(np.asarray(A["wrap_type"]).reshape(-1)[tadr[tid]]) != 1:
      # spatial tendon: ten_J is nonzero on the dof chains of the path's site and wrap-geom
      # bodies (the reference compresses its dense row by value, :1070-1079; generic states
      # have no exact zeros there)
      wtype = np.asarray(A["wrap_type"]).reshape(-1)
      gbody = np.asarray(A["geom_bodyid"]).reshape(-1)
      c = set()
      for wi in range(tadr[tid], tadr[tid] + tnum[tid]):
        if wtype[wi] not in (3, 4, 5):
          continue
        b = int(sbody[wobj[wi]] if wtype[wi] == 3 else gbody[wobj[wi]])
        while b > 0:
          c.update(range(dofadr[b], dofadr[b] + dofnum[b]))
          b = int(parentid[b])
      c = [] if agear[ai, 0] == 0 else sorted(c)
    elif sparse_jac:
      # fixed tendon of a sparse-mode model (:1060-1067): the tendon's compressed ten_J row,
      # i.e. the merged dofs of its joints (mj_tendon's mju_combineSparse, smooth.c:709-714),
      # whatever the coefficients and gear
      c = sorted({int(jdadr[wobj[wi]]) for wi in range(tadr[tid], tadr[tid] + tnum[tid])})
    else:
      row = np.zeros(nv)
      for wi in range(tadr[tid], tadr[tid] + tnum[tid]):
        row[jdadr[wobj[wi]]] = wprm[wi]
      c = [j for j in range(nv) if row[j] * agear[ai, 0] != 0]
    mrownnz[ai] = len(c)
    mrowadr[ai] = mrowadr[ai - 1] + mrownnz[ai - 1] if ai else 0
    cols.extend(c)
  mcol = arr("moment_colind", nJmom, np.int32)
  if len(cols) > nJmom:
    raise MJCFError("actuator moment pattern exceeds nJmom")
  mcol[:len(cols)] = cols

  return out


def _sameframe(pos, quat, ipos, iquat):
  """Geom/site sameframe (user_model.cc:2404-2416, 2444-2456)."""
  if is_null_pose(pos, quat):
    return 1      # BODY
  if is_null_pose(None, quat):
    return 3      # BODYROT
  if is_same_pose(pos, ipos, quat, iquat):
    return 2      # INERTIA
  if is_same_pose(None, None, quat, iquat):
    return 4      # INERTIAROT
  return 0


def _jnt_nq(t):
  return {0: 7, 1: 4, 2: 1, 3: 1}[t]


def _jnt_nv(t):
  return {0: 6, 1: 3, 2: 1, 3: 1}[t]


def _geom_volume(t, size):
  """mjCGeom::GetVolume, typeinertia = volume (user_objects.cc:2384-2460)."""
  if t == GEOM["sphere"]:
    r = size[0]
    return 4 * mjPI * r * r * r / 3
  if t == GEOM["capsule"]:
    h = 2 * size[1]
    r = size[0]
    return mjPI * (r * r * h + 4 * r * r * r / 3)
  if t == GEOM["cylinder"]:
    h = 2 * size[1]
    r = size[0]
    return mjPI * r * r * h
  if t == GEOM["ellipsoid"]:
    return 4 * mjPI * size[0] * size[1] * size[2] / 3
  if t in (GEOM["box"], GEOM["hfield"]):
    return size[0] * size[1] * size[2] * 8
  return 0.0


def _geom_inertia(t, size, mass):
  """mjCGeom::SetInertia, typeinertia = volume (user_objects.cc:2474-2560)."""
  if t == GEOM["sphere"]:
    v = 2 * mass * size[0] * size[0] / 5
    return [v, v, v]
  if t == GEOM["capsule"]:
    height = 2 * size[1]
    radius = size[0]
    sphere_mass = mass * 4 * radius / (4 * radius + 3 * height)
    cylinder_mass = mass - sphere_mass
    i0 = cylinder_mass * (3 * radius * radius + height * height) / 12
    i2 = cylinder_mass * radius * radius / 2
    sphere_inertia = 2 * sphere_mass * radius * radius / 5
    i0 += sphere_inertia + sphere_mass * height * (3 * radius + 2 * height) / 8
    i1 = i0
    i2 += sphere_inertia
    return [i0, i1, i2]
  if t == GEOM["cylinder"]:
    height = 2 * size[1]
    radius = size[0]
    i0 = mass * (3 * radius * radius + height * height) / 12
    return [i0, i0, mass * radius * radius / 2]
  if t == GEOM["ellipsoid"]:
    s = size
    return [mass * (s[1]*s[1] + s[2]*s[2]) / 5, mass * (s[0]*s[0] + s[2]*s[2]) / 5,
            mass * (s[0]*s[0] + s[1]*s[1]) / 5]
  if t in (GEOM["box"], GEOM["hfield"]):
    s = size
    return [mass * (s[1]*s[1] + s[2]*s[2]) / 3, mass * (s[0]*s[0] + s[2]*s[2]) / 3,
            mass * (s[0]*s[0] + s[1]*s[1]) / 3]
  return [0.0, 0.0, 0.0]


def _added_mass_kappa(dx, dy, dz):
  """mjCGeom::GetAddedMassKappa (user_objects.cc:2738-2785): 15-point Gauss-Kronrod
  quadrature of dx dy dz / sqrt((dx^2 + l)^3 (dy^2 + l)(dz^2 + l)) over l in [0, inf), after
  l = x^3 / (1 - x)^2, in the reference's operation order."""
  w = (0.01146766, 0.03154605, 0.05239501, 0.07032663, 0.08450236, 0.09517529, 0.10221647,
       0.10474107, 0.10221647, 0.09517529, 0.08450236, 0.07032663, 0.05239501, 0.03154605,
       0.01146766)
  ls = (7.865151709349917e-08, 1.7347976913907274e-05, 0.0003548008144506193,
        0.002846636252924549, 0.014094260903596077, 0.053063261727396636,
        0.17041978741317773, 0.5, 1.4036301548686991, 3.9353484827022642,
        11.644841677041734, 39.53187807410903, 177.5711362220801, 1429.4772912937397,
        54087.416549217705)
  ds = (5.538677720489877e-05, 0.002080868285293228, 0.016514126520723166,
        0.07261900344370877, 0.23985243401862602, 0.6868318249020725, 1.8551129519182894,
        5.0, 14.060031152313941, 43.28941239611009, 156.58546376397112, 747.9826085305024,
        5827.4042950027115, 116754.0197944512, 25482945.327264845)
  ix, iy, iz = 1.0 / (dx * dx), 1.0 / (dy * dy), 1.0 / (dz * dz)
  scale = math.pow(dx*dx*dx * dy * dz, 0.4)
  kappa = 0.0
  for i in range(15):
    lam = scale * ls[i]
    denom = (1 + lam*ix) * math.sqrt((1 + lam*ix) * (1 + lam*iy) * (1 + lam*iz))
    kappa += scale * ds[i] / denom * w[i]
  return kappa * ix


def _fluid_coefs(t, size, ellipsoid, coefs):
  """mjCGeom::SetFluidCoefs (user_objects.cc:2788-2849): geom_fluid = [ellipsoid flag, the
  5 coefficients, virtual mass (3), virtual inertia (3)] of the equivalent ellipsoid."""
  if t == GEOM["sphere"]:
    dx = dy = dz = size[0]
  elif t == GEOM["capsule"]:
    dx, dy, dz = size[0], size[0], size[1] + size[0]
  elif t == GEOM["cylinder"]:
    dx, dy, dz = size[0], size[0], size[1]
  else:
    dx, dy, dz = size[0], size[1], size[2]
  volume = 4.0 / 3.0 * mjPI * dx * dy * dz
  kx = _added_mass_kappa(dx, dy, dz)
  ky = _added_mass_kappa(dy, dz, dx)
  kz = _added_mass_kappa(dz, dx, dy)
  p2 = lambda v: v * v                       # noqa: E731
  ixf = p2(dy*dy - dz*dz) * abs(kz - ky) / max(
      mjEPS, abs(2*(dy*dy - dz*dz) + (dy*dy + dz*dz)*(ky - kz)))
  iyf = p2(dz*dz - dx*dx) * abs(kx - kz) / max(
      mjEPS, abs(2*(dz*dz - dx*dx) + (dz*dz + dx*dx)*(kz - kx)))
  izf = p2(dx*dx - dy*dy) * abs(ky - kx) / max(
      mjEPS, abs(2*(dx*dx - dy*dy) + (dx*dx + dy*dy)*(kx - ky)))
  vm = [volume * kx / max(mjEPS, 2 - kx), volume * ky / max(mjEPS, 2 - ky),
        volume * kz / max(mjEPS, 2 - kz)]
  vi = [volume*ixf/5, volume*iyf/5, volume*izf/5]
  return [float(ellipsoid)] + [float(c) for c in coefs] + vm + vi


def _geom_rbound(t, size):
  """mjCGeom::GetRBound (radius of the bounding sphere)."""
  if t == GEOM["sphere"]:
    return size[0]
  if t == GEOM["capsule"]:
    return size[0] + size[1]
  if t == GEOM["cylinder"]:
    return math.sqrt(size[0]*size[0] + size[1]*size[1])
  if t == GEOM["ellipsoid"]:
    return max(size[0], size[1], size[2])
  if t == GEOM["box"]:
    return math.sqrt(size[0]*size[0] + size[1]*size[1] + size[2]*size[2])
  return 0.0


def load_xml_string(text: str, basedir: str | None = None) -> Model:
  """Compile an MJCF string (the LoadModelFromString of test/fixture.h:85-97)."""
  from . import setconst
  root = ET.fromstring(text)
  c = MJCFCompiler()
  c.basedir = basedir
  c.parse(root)
  m = c.compile()
  setconst.set_const(m)
  return m


def load_xml(path: str) -> Model:
  """Compile an MJCF file (mj_loadXML, src/xml/xml_api.cc:97, restricted to the subset)."""
  with open(path) as f:
    return load_xml_string(f.read(), os.path.dirname(os.path.abspath(path)))
