"""Host-side mjModel/mjData views for the C-ABI (ctypes structs over numpy arrays).

``model_struct(m)`` builds the ``mjhipModel`` struct of include/mjhip.h from a compiled
Model (pointer fields alias the Model's numpy arrays, which the struct keeps alive), and
``MjData`` holds one instance's fields in the reference's per-field row-major layout
(include/mujoco/mjdata.h via mjxmacro.h) behind an ``mjhipData`` struct.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import fields


def model_struct(m) -> fields.CModel:
  s = fields.CModel()
  keep = []
  for k in fields.MODEL_SIZES:
    setattr(s, k, int(m.sizes.get(k, 0)))
  o = s.opt
  for k in ("timestep", "impratio", "density", "viscosity", "o_margin"):
    setattr(o, k, float(m.opt[k]))
  o.ccd_tolerance = float(m.opt.get("ccd_tolerance", 1e-6))
  o.ccd_iterations = int(m.opt.get("ccd_iterations", 50))
  for k, n in (("gravity", 3), ("wind", 3), ("magnetic", 3), ("o_solref", 2), ("o_solimp", 5),
               ("o_friction", 5)):
    arr = getattr(o, k)
    for i in range(n):
      arr[i] = float(m.opt[k][i])
  for k in ("integrator", "cone", "jacobian", "disableflags", "enableflags"):
    setattr(o, k, int(m.opt[k]))
  for f in fields.MODEL_FIELDS:
    a = np.ascontiguousarray(getattr(m, f.name), dtype=fields.NPTYPE[f.ctype])
    if a is not getattr(m, f.name):
      setattr(m, f.name, a)
    keep.append(a)
    if a.size:
      setattr(s, f.name, a.ctypes.data_as(ctypes.POINTER(fields.CTYPE[f.ctype])))
  s._keep = keep
  return s


def model_capacity(m):
  """(constraint rows, contacts) one instance of model m can produce on the device path
  (mjhip_modelCapacity: exact for the implemented functions)."""
  from . import engine
  rows, cons = ctypes.c_int(), ctypes.c_int()
  cm = model_struct(m)
  engine.lib().mjhip_modelCapacity(ctypes.byref(cm), ctypes.byref(rows), ctypes.byref(cons))
  return rows.value, cons.value


class MjData:
  """One instance of the per-instance fields (mjData subset), numpy-backed, with buffers for
  the constraint rows and contacts (the reference's d->efc_* / d->contact)."""

  def __init__(self, m, efc_capacity=None, con_capacity=None):
    self.m = m
    sizes = m.sizes
    self._arrays = {}
    for f in fields.DATA_FIELDS + fields.FORWARD_FIELDS + fields.AUX_FIELDS:
      n = f.size(sizes)
      self._arrays[f.name] = np.zeros(max(n, 1))
    if efc_capacity is None or con_capacity is None:
      rows, cons = model_capacity(m)
      efc_capacity = rows if efc_capacity is None else efc_capacity
      con_capacity = cons if con_capacity is None else con_capacity
    self._rows = {}
    for f, cap in ([(f, efc_capacity) for f in fields.EFC_FIELDS] +
                   [(f, con_capacity) for f in fields.CONTACT_FIELDS]):
      self._rows[f.name] = np.zeros(max(cap * f.row_size(sizes), 1),
                                    dtype=fields.NPTYPE[f.ctype])
    # reference defaults (mj_resetData): qpos = qpos0, world body identity frames
    self._arrays["qpos"][:m.nq] = m.qpos0
    for b in range(m.nbody):            # mocap_pos/quat = body_pos/quat (mj_resetData)
      k = int(m.body_mocapid[b])
      if k >= 0:
        self._arrays["mocap_pos"][3*k:3*k + 3] = m.body_pos[b]
        self._arrays["mocap_quat"][4*k:4*k + 4] = m.body_quat[b]
    self.struct = fields.CData()
    for name, a in self._arrays.items():
      setattr(self.struct, name, a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    self.struct.efc_capacity = efc_capacity
    self.struct.con_capacity = con_capacity
    for f in fields.EFC_FIELDS + fields.CONTACT_FIELDS:
      setattr(self.struct, f.name,
              self._rows[f.name].ctypes.data_as(ctypes.POINTER(fields.CTYPE[f.ctype])))
    # compressed-Jacobian structures (sparse-mode models only; NULL otherwise)
    self._sparse = {}
    if fields.is_sparse(m):
      for f in fields.SPARSE_FIELDS:
        a = np.zeros(max(f.size(sizes, efc_capacity), 1), dtype=fields.NPTYPE[f.ctype])
        self._sparse[f.name] = a
        setattr(self.struct, f.name, a.ctypes.data_as(ctypes.POINTER(fields.CTYPE[f.ctype])))

  def __getattr__(self, k):
    arrs = self.__dict__.get("_arrays")
    if arrs is not None and k in arrs:
      f = fields.DATA_FIELD.get(k)
      n = f.size(self.m.sizes) if f else len(arrs[k])
      return arrs[k][:n]
    raise AttributeError(k)

  def sparse(self, name):
    """A compressed-Jacobian array of a sparse-mode model (MJHIP_DATA_SPARSE), whole buffer."""
    return self._sparse[name]

  def efc(self, name):
    """Constraint-row (efc_*) or contact (con_*) array of the current rows / contacts, one
    row per constraint (contact); a writable view of the buffer."""
    f = {x.name: x for x in fields.EFC_FIELDS + fields.CONTACT_FIELDS}[name]
    w = f.row_size(self.m.sizes)
    n = self.struct.ncon if name.startswith("con_") else self.struct.nefc
    return self._rows[name][:n * w].reshape(n, w)

  def set_rows(self, nefc=None, ne=None, nf=None, nl=None, ncon=None, **arrays):
    """Fill the constraint rows / contacts (as a forward pass would leave them)."""
    for k, v in (("nefc", nefc), ("ne", ne), ("nf", nf), ("nl", nl), ("ncon", ncon)):
      if v is not None:
        setattr(self.struct, k, int(v))
    for name, vals in arrays.items():
      vals = np.ravel(vals)
      self._rows[name][:len(vals)] = vals

  @property
  def nefc(self):
    return self.struct.nefc

  @property
  def ncon(self):
    return self.struct.ncon

  @property
  def efc_counts(self):
    """(nefc, ne, nf, nl)"""
    s = self.struct
    return s.nefc, s.ne, s.nf, s.nl

  @property
  def status(self):
    """mjhipInstanceStatus bits of the last call."""
    return self.struct.status

  @property
  def solver_fwdinv(self):
    return np.array(self.struct.solver_fwdinv[:2])

  @property
  def energy(self):
    return np.array(self.struct.energy[:2])

  @property
  def time(self):
    return float(self.struct.time)

  @time.setter
  def time(self, t):
    self.struct.time = float(t)

  def ptr(self):
    return ctypes.byref(self.struct)
