"""ctypes binding of liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference's mj_inverse path (mj_oracle.c) is the parity checker
for the HIP engine. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module; the product package never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from mujoco_inversedynamicstest_amd import fields, host

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: another build of the same source (tests/test_asan.py: the sanitizer build)
_LIB = os.environ.get("ORACLE_LIB", os.path.join(_HERE, "liboracle.so"))
_lib = None

_D = ctypes.POINTER(ctypes.c_double)

# contact arrays of orEfc (mj_oracle.h) and their widths
CON_DOUBLE = (("con_dist", 1), ("con_pos", 3), ("con_frame", 9), ("con_includemargin", 1),
              ("con_friction", 5), ("con_solref", 2), ("con_solreffriction", 2),
              ("con_solimp", 5), ("con_mu", 1))
CON_INT = (("con_dim", 1), ("con_geom", 2), ("con_exclude", 1), ("con_efc_address", 1))


class Efc(ctypes.Structure):
  _fields_ = ([("capacity", ctypes.c_int), ("nefc", ctypes.c_int), ("ne", ctypes.c_int),
               ("nf", ctypes.c_int), ("nl", ctypes.c_int),
               ("efc_type", ctypes.POINTER(ctypes.c_int)),
               ("efc_id", ctypes.POINTER(ctypes.c_int)),
               ("efc_state", ctypes.POINTER(ctypes.c_int))] +
              [(n, _D) for n in ("efc_J", "efc_pos", "efc_margin", "efc_frictionloss",
                                 "efc_diagApprox", "efc_KBIP", "efc_D", "efc_R", "efc_vel",
                                 "efc_aref", "efc_force")] +
              [("con_capacity", ctypes.c_int), ("ncon", ctypes.c_int)] +
              [(n, _D) for n, _ in CON_DOUBLE] +
              [(n, ctypes.POINTER(ctypes.c_int)) for n, _ in CON_INT] +
              [("nJ", ctypes.c_int)] +
              [(n, ctypes.POINTER(ctypes.c_int)) for n in ("efc_J_rownnz", "efc_J_rowadr",
                                                           "efc_J_colind")] +
              [("efc_JT", _D)] +
              [(n, ctypes.POINTER(ctypes.c_int)) for n in ("efc_JT_rownnz", "efc_JT_rowadr",
                                                           "efc_JT_colind")])

# compressed-row arrays of orEfc (sparse-mode models): (name, dtype, size per capacity row or
# per dof)
EFC_SPARSE = (("efc_J_rownnz", np.int32, "row"), ("efc_J_rowadr", np.int32, "row"),
              ("efc_J_colind", np.int32, "row_nv"), ("efc_JT", np.float64, "row_nv"),
              ("efc_JT_rownnz", np.int32, "nv"), ("efc_JT_rowadr", np.int32, "nv"),
              ("efc_JT_colind", np.int32, "row_nv"))


class UnsupportedModel(ValueError):
  pass


def build():
  subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
  global _lib
  if _lib is None:
    if not os.path.exists(_LIB):
      build()
    L = ctypes.CDLL(_LIB)
    M = ctypes.POINTER(fields.CModel)
    Dp = ctypes.POINTER(fields.CData)
    E = ctypes.POINTER(Efc)
    L.or_efcCapacity.argtypes = [M]
    L.or_contactCapacity.argtypes = [M]
    L.or_inverseSkip.argtypes = [M, Dp, E, ctypes.c_int, ctypes.c_int]
    L.or_inverse.argtypes = [M, Dp, E]
    for fn in ("or_kinematics", "or_comPos", "or_crb", "or_factorM"):
      getattr(L, fn).argtypes = [M, Dp]
    L.or_solveM.argtypes = [M, Dp, _D, _D, ctypes.c_int]
    L.or_rne.argtypes = [M, Dp, ctypes.c_int, _D]
    L.or_fullM.argtypes = [M, _D, _D]
    L.or_smoothVel.argtypes = [M, Dp, _D, ctypes.c_int]
    L.or_forward.argtypes = [M, Dp, E]
    L.or_forward.restype = ctypes.c_int
    L.or_xfrcAccumulate.argtypes = [M, Dp, _D]
    L.or_boxBoxRaw.argtypes = [M, Dp, ctypes.c_int, ctypes.c_int, ctypes.c_double, _D]
    L.or_boxBoxRaw.restype = ctypes.c_int
    L.or_rungeKutta4.argtypes = [M, Dp, E]
    L.or_inverseFD.argtypes = [M, Dp, E, ctypes.c_double, _D, _D, _D, _D, _D, _D, _D]
    L.or_inverseFDEx.argtypes = [M, Dp, E, ctypes.c_double, ctypes.c_int, _D, _D, _D, _D, _D,
                                 _D, _D]
    L.or_compareFwdInv.argtypes = [M, Dp, E]
    L.or_inverseBatch.argtypes = [M, ctypes.c_int, _D, _D, _D, _D, ctypes.c_int]
    L.or_ccdPenetration.argtypes = [M, Dp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_int, _D]
    L.or_ccdPenetration.restype = ctypes.c_int
    L.or_ccdGeneral.argtypes = [M, Dp, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_double, _D]
    L.or_ccdGeneral.restype = ctypes.c_double
    L.or_rayTest.argtypes = [M, Dp, _D, _D, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    L.or_rayTest.restype = ctypes.c_double
    L.or_inverseBatch.restype = ctypes.c_double
    _lib = L
  return _lib


def _p(a):
  return None if a is None else a.ctypes.data_as(_D)


class Oracle:
  """Single-instance CPU reference bound to one compiled model."""

  def __init__(self, m):
    self.m = m
    self.cm = host.model_struct(m)
    self.L = lib()
    # the oracle keeps its rows in its own orEfc (below), not in the data's row buffers
    self.d = host.MjData(m, efc_capacity=0, con_capacity=0)
    cap = max(self.L.or_efcCapacity(ctypes.byref(self.cm)), 1)
    nv = max(m.nv, 1)
    self._efc_arrays = {n: np.zeros(cap * k) for n, k in
                        (("efc_J", nv), ("efc_pos", 1), ("efc_margin", 1),
                         ("efc_frictionloss", 1), ("efc_diagApprox", 1), ("efc_KBIP", 4),
                         ("efc_D", 1), ("efc_R", 1), ("efc_vel", 1), ("efc_aref", 1),
                         ("efc_force", 1))}
    self._efc_int = {n: np.zeros(cap, dtype=np.int32) for n in
                     ("efc_type", "efc_id", "efc_state")}
    self.efc = Efc()
    self.efc.capacity = cap
    for n, a in self._efc_arrays.items():
      setattr(self.efc, n, _p(a))
    for n, a in self._efc_int.items():
      setattr(self.efc, n, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    self._efc_sparse = {}
    for n, dt, k in EFC_SPARSE:
      a = np.zeros({"row": cap, "row_nv": cap * nv, "nv": nv}[k], dtype=dt)
      self._efc_sparse[n] = a
      setattr(self.efc, n, a.ctypes.data_as(ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))))
    ncap = max(self.L.or_contactCapacity(ctypes.byref(self.cm)), 1)
    self.efc.con_capacity = ncap
    self._con = {n: np.zeros(ncap * k) for n, k in CON_DOUBLE}
    self._con.update({n: np.zeros(ncap * k, dtype=np.int32) for n, k in CON_INT})
    for n, k in CON_DOUBLE:
      setattr(self.efc, n, _p(self._con[n]))
    for n, k in CON_INT:
      setattr(self.efc, n, self._con[n].ctypes.data_as(ctypes.POINTER(ctypes.c_int)))

  def _args(self):
    return ctypes.byref(self.cm), ctypes.byref(self.d.struct), ctypes.byref(self.efc)

  def set_state(self, qpos=None, qvel=None, qacc=None):
    if qpos is not None:
      self.d.qpos[:] = qpos
    if qvel is not None:
      self.d.qvel[:] = qvel
    if qacc is not None:
      self.d.qacc[:] = qacc

  def inverse(self, qpos=None, qvel=None, qacc=None, skipstage=0, skipsensor=0):
    self.set_state(qpos, qvel, qacc)
    self.L.or_inverseSkip(*self._args(), skipstage, skipsensor)
    return self.d.qfrc_inverse.copy()

  def forward(self):
    return self.L.or_forward(*self._args())

  def rk4(self):
    self.L.or_rungeKutta4(*self._args())

  def xfrc_accumulate(self, qfrc):
    self.L.or_xfrcAccumulate(ctypes.byref(self.cm), ctypes.byref(self.d.struct), _p(qfrc))

  def solveM(self, y):
    y = np.ascontiguousarray(y, dtype=np.float64)
    n = y.size // self.m.nv
    x = np.zeros_like(y)
    self.L.or_solveM(ctypes.byref(self.cm), ctypes.byref(self.d.struct), _p(x), _p(y), n)
    return x

  def fullM(self, M=None):
    M = self.d.qM if M is None else np.ascontiguousarray(M)
    out = np.zeros((self.m.nv, self.m.nv))
    self.L.or_fullM(ctypes.byref(self.cm), _p(out), _p(M))
    return out

  def smooth_vel(self, flg_bias=1):
    """mjd_smooth_vel of the last call's state as a dense nv x nv matrix (D sparsity)."""
    m = self.m
    q = np.zeros(max(m.sizes["nD"], 1))
    self.L.or_smoothVel(ctypes.byref(self.cm), ctypes.byref(self.d.struct), _p(q), flg_bias)
    out = np.zeros((m.nv, m.nv))
    for r in range(m.nv):
      a, n = m.D_rowadr[r], m.D_rownnz[r]
      out[r, m.D_colind[a:a + n]] = q[a:a + n]
    return out

  def contact_field(self, name):
    """Contacts of the last call, one row per contact (width = field width)."""
    k = dict(CON_DOUBLE + CON_INT)[name]
    return self._con[name][:self.efc.ncon * k].reshape(self.efc.ncon, k).squeeze(-1) \
        if k == 1 else self._con[name][:self.efc.ncon * k].reshape(self.efc.ncon, k)

  def efc_field(self, name):
    """Rows of the last call. efc_J: dense nefc x nv rows (flattened), also for a sparse-mode
    model, whose compressed rows are expanded (efc_sparse() has them as they are)."""
    if name == "efc_J" and fields.is_sparse(self.m):
      return self.efc_dense().ravel()
    if name in self._efc_arrays:
      k = self._efc_arrays[name].size // self.efc.capacity
      return self._efc_arrays[name][:self.efc.nefc * k]
    return self._efc_int[name][:self.efc.nefc]

  def efc_sparse(self):
    """Compressed rows of a sparse-mode model's last call: dict of efc_J (nJ values),
    efc_J_rownnz/rowadr (nefc), efc_J_colind (nJ), efc_JT (nJ), efc_JT_rownnz/rowadr (nv),
    efc_JT_colind (nJ)."""
    e, nv = self.efc, self.m.nv
    nJ, nefc = e.nJ, e.nefc
    S = self._efc_sparse
    return {"efc_J": self._efc_arrays["efc_J"][:nJ].copy(),
            "efc_J_rownnz": S["efc_J_rownnz"][:nefc].copy(),
            "efc_J_rowadr": S["efc_J_rowadr"][:nefc].copy(),
            "efc_J_colind": S["efc_J_colind"][:nJ].copy(),
            "efc_JT": S["efc_JT"][:nJ].copy(),
            "efc_JT_rownnz": S["efc_JT_rownnz"][:nv].copy(),
            "efc_JT_rowadr": S["efc_JT_rowadr"][:nv].copy(),
            "efc_JT_colind": S["efc_JT_colind"][:nJ].copy()}

  def efc_dense(self):
    """efc_J of the last call as a dense nefc x nv matrix (a sparse model's rows expanded)."""
    e, nv = self.efc, self.m.nv
    if not fields.is_sparse(self.m):
      return self._efc_arrays["efc_J"][:e.nefc * nv].reshape(e.nefc, nv).copy()
    S = self._efc_sparse
    out = np.zeros((e.nefc, nv))
    for r in range(e.nefc):
      a, n = S["efc_J_rowadr"][r], S["efc_J_rownnz"][r]
      out[r, S["efc_J_colind"][a:a + n]] = self._efc_arrays["efc_J"][a:a + n]
    return out

  def ten_J_dense(self):
    """ten_J of the last call as ntendon x nv (a sparse model's compressed rows expanded)."""
    m, d = self.m, self.d
    nt, nv = m.sizes["ntendon"], m.nv
    if not fields.is_sparse(m):
      return d.ten_J.reshape(nt, nv).copy()
    out = np.zeros((nt, nv))
    for t in range(nt):
      a, n = d.sparse("ten_J_rowadr")[t], d.sparse("ten_J_rownnz")[t]
      out[t, d.sparse("ten_J_colind")[a:a + n]] = d.ten_J[a:a + n]
    return out

  def box_box_raw(self, g1, g2, margin):
    """mjc_BoxBox's raw contacts on the current geom poses (after inverse/forward):
    (dist, pos, normal) arrays, before the driver's bad/duplicate clean-up."""
    out = np.zeros(24 * 7)
    n = self.L.or_boxBoxRaw(ctypes.byref(self.cm), ctypes.byref(self.d.struct), g1, g2,
                            margin, _p(out))
    out = out[:7 * n].reshape(n, 7)
    return out[:, 0], out[:, 1:4], out[:, 4:7]

  def rne(self, flg_acc):
    """mj_rne of the data's current cdof/cinert/cvel/cdof_dot/qvel/qacc."""
    out = np.zeros(self.m.nv)
    self.L.or_rne(ctypes.byref(self.cm), ctypes.byref(self.d.struct), flg_acc, _p(out))
    return out

  def compare_fwd_inv(self):
    """mj_compareFwdInv on the rows of the last call; returns solver_fwdinv."""
    self.L.or_compareFwdInv(*self._args())
    return self.d.solver_fwdinv

  def export(self, d, rows=True):
    """Copy this data's fields (and, with rows, its constraint rows and contacts) into a
    product MjData d, as a forward pass would leave them for the single-instance calls."""
    for f in fields.DATA_FIELDS + fields.FORWARD_FIELDS + fields.AUX_FIELDS:
      src, dst = getattr(self.d, f.name), getattr(d, f.name)
      dst[:] = src
    d.struct.time = self.d.struct.time
    if not rows:
      return
    e = self.efc
    arrays = {}
    for f in fields.EFC_FIELDS:
      arrays[f.name] = self.efc_field(f.name)
    for f in fields.CONTACT_FIELDS:
      arrays[f.name] = self.contact_field(f.name)
    d.set_rows(nefc=e.nefc, ne=e.ne, nf=e.nf, nl=e.nl, ncon=e.ncon, **arrays)

  def inverse_fd(self, eps=1e-6, dmdq=False, sensors=False, flg_actuation=False):
    """mjd_inverseFD: (DfDq, DfDv, DfDa, DmDq), plus (DsDq, DsDv, DsDa) when sensors."""
    nv, nM, ns = self.m.nv, self.m.nM, self.m.sizes.get("nsensordata", 0)
    DfDq = np.zeros((nv, nv))
    DfDv = np.zeros((nv, nv))
    DfDa = np.zeros((nv, nv))
    DmDq = np.zeros((nv, nM)) if dmdq else None
    Ds = [np.zeros((nv, max(ns, 1))) for _ in range(3)] if sensors else [None] * 3
    self.L.or_inverseFDEx(*self._args(), eps, int(bool(flg_actuation)), _p(DfDq), _p(DfDv),
                          _p(DfDa), *map(_p, Ds), _p(DmDq))
    if sensors:
      return DfDq, DfDv, DfDa, DmDq, tuple(x[:, :ns] for x in Ds)
    return DfDq, DfDv, DfDa, DmDq

  def penetration(self, g1, g2, margin=0.0, tol=1e-6, kmax=1000):
    """The reference tests' Penetration helper (engine_collision_gjk_test.cc:86-150) on the
    current frames (run inverse() first): (ncon, dist, dir, pos)."""
    out = np.zeros(7)
    n = self.L.or_ccdPenetration(*self._args()[:2], g1, g2, margin, tol, kmax, _p(out))
    return n, out[0], out[1:4], out[4:7]

  def ccd(self, g1, g2, margin=0.0, tol=1e-6, kmax=1000, max_contacts=1, cutoff=0.0):
    """mjc_ccd (engine_collision_gjk.c:2215-2343) on the current frames with the reference
    tests' config (engine_collision_gjk_test.cc:62-150): (dist, nx, x1, x2); with
    max_contacts > 1, x1 / x2 are [nx, 3] (multicontact)."""
    out = np.zeros(3 + 300)
    dist = self.L.or_ccdGeneral(*self._args()[:2], g1, g2, margin, tol, kmax, max_contacts,
                                cutoff, _p(out))
    if out[2]:
      raise NotImplementedError("multicontact: a feature the restatement does not cover")
    nx = int(out[1])
    if max_contacts <= 1:
      return dist, nx, out[3:6].copy(), out[153:156].copy()
    return dist, nx, out[3:3 + 3*nx].reshape(nx, 3).copy(), out[153:153 + 3*nx].reshape(nx, 3).copy()

  def ray(self, pnt, vec, bodyexclude=-1):
    """mj_ray (geomgroup NULL, flg_static 1) on the current frames: (distance, geomid)."""
    gid = ctypes.c_int(-1)
    pnt = np.ascontiguousarray(pnt, dtype=np.float64)
    vec = np.ascontiguousarray(vec, dtype=np.float64)
    x = self.L.or_rayTest(*self._args()[:2], _p(pnt), _p(vec), bodyexclude, ctypes.byref(gid))
    return x, gid.value

  def inverse_batch(self, qpos, qvel, qacc, nthread=1, lib=None):
    """CPU baseline over B instances; returns (qfrc_inverse [B, nv], seconds). lib: another
    build of the same source (native_baseline_lib()), default the checker build."""
    qpos = np.ascontiguousarray(qpos, dtype=np.float64)
    qvel = np.ascontiguousarray(qvel, dtype=np.float64)
    qacc = np.ascontiguousarray(qacc, dtype=np.float64)
    B = qpos.shape[0]
    out = np.zeros((B, self.m.nv))
    L = lib or self.L
    t = L.or_inverseBatch(ctypes.byref(self.cm), B, _p(qpos), _p(qvel), _p(qacc), _p(out),
                          nthread)
    return out, t


def native_baseline_lib():
  """The oracle compiled for THIS host's CPU (-O3 -march=native, BASELINE.md's CPU plan) into
  a temporary directory, for bench.py's cpu_baseline leg only. ISO C mode keeps gcc from
  contracting multiply-adds, so the arithmetic is the checker build's; only the instruction
  selection and scheduling differ. Built where it runs (the GPU box's host CPU may not be this
  container's), about 6 s. Returns (ctypes library, compiler flags)."""
  import tempfile
  flags = ["-std=c11", "-O3", "-march=native", "-ffp-contract=off", "-fPIC", "-shared"]
  out = os.path.join(tempfile.mkdtemp(prefix="oracle_native_"), "liboracle_native.so")
  subprocess.run([os.environ.get("CC", "gcc"), *flags, "-o", out,
                  os.path.join(_HERE, "mj_oracle.c"), "-lm", "-lpthread"], check=True)
  L = ctypes.CDLL(out)
  L.or_inverseBatch.argtypes = [ctypes.POINTER(fields.CModel), ctypes.c_int, _D, _D, _D, _D,
                                ctypes.c_int]
  L.or_inverseBatch.restype = ctypes.c_double
  return L, " ".join(flags)
