"""Field tables shared with C/HIP: parsed from include/mjhip_fields.h.

The header is the single source of truth for the names, element types and shapes of the
model and per-instance data fields (which follow the reference's
include/mujoco/mjxmacro.h tables). This module turns it into ctypes structures that are
binary-compatible with ``mjhipModel`` / ``mjhipData`` in include/mjhip.h.
"""
from __future__ import annotations

import ctypes
import os
import re
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(_HERE)
INCLUDE_DIR = os.path.join(REPO_ROOT, "include")
FIELDS_HEADER = os.path.join(INCLUDE_DIR, "mjhip_fields.h")

CTYPE = {"mjtNum": ctypes.c_double, "int": ctypes.c_int, "mjtByte": ctypes.c_ubyte,
         "float": ctypes.c_float}
NPTYPE = {"mjtNum": np.float64, "int": np.int32, "mjtByte": np.uint8, "float": np.float32}


@dataclass(frozen=True)
class ModelField:
  ctype: str
  name: str
  dim0: str
  dim1: str  # integer literal or MJ_M(size)

  def shape(self, sizes: dict) -> tuple:
    return (sizes[self.dim0], _dim(self.dim1, sizes))


@dataclass(frozen=True)
class DataField:
  name: str
  dim0: str
  dim1: str
  stage: int  # 0 input, 1 position, 2 velocity, 3 acceleration

  def size(self, sizes: dict) -> int:
    return sizes[self.dim0] * _dim(self.dim1, sizes)


def _dim(tok: str, sizes: dict) -> int:
  m = re.fullmatch(r"MJ_M\((\w+)\)", tok)
  if m:
    return sizes[m.group(1)]
  return int(tok)


def _macro_body(text: str, name: str) -> str:
  m = re.search(r"#define\s+" + name + r"\s*\\\n(.*?)(?:\n\s*\n|\n#)", text, re.S)
  if not m:
    raise RuntimeError(f"macro {name} not found in {FIELDS_HEADER}")
  return m.group(1)


def _parse():
  text = open(FIELDS_HEADER).read()
  sizes = re.findall(r"XS\((\w+)\)", _macro_body(text, "MJHIP_MODEL_SIZES"))
  model = []
  for group in ("MJHIP_MODEL_POINTERS_M", "MJHIP_MODEL_POINTERS_D"):
    for ct, nm, d0, d1 in re.findall(
        r"X\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\w+)\s*,\s*([\w()]+)\s*\)",
        _macro_body(text, group)):
      model.append(ModelField(ct, nm, d0, d1))
  def xd(group):
    return [DataField(nm, d0, d1, int(st)) for nm, d0, d1, st in re.findall(
        r"XD\(\s*(\w+)\s*,\s*(\w+)\s*,\s*([\w()]+)\s*,\s*(\d)\s*\)",
        _macro_body(text, group))]
  data = []
  for group in ("MJHIP_DATA_INPUTS", "MJHIP_DATA_POSITION", "MJHIP_DATA_VELOCITY",
                "MJHIP_DATA_ACCELERATION"):
    data += xd(group)

  def rows(group, tag):
    return [RowField(ct, nm, w, int(st)) for ct, nm, w, st in re.findall(
        tag + r"\(\s*(\w+)\s*,\s*(\w+)\s*,\s*([\w()]+)\s*,\s*(\d)\s*\)",
        _macro_body(text, group))]
  sparse = [SparseField(ct, nm, dim) for ct, nm, dim in re.findall(
      r"XJ\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\w+)\s*\)", _macro_body(text, "MJHIP_DATA_SPARSE"))]
  return (sizes, model, data, xd("MJHIP_DATA_FORWARD"), xd("MJHIP_DATA_SENSOR_AUX"),
          rows("MJHIP_DATA_EFC", "XE"), rows("MJHIP_DATA_CONTACT", "XC"), sparse)


@dataclass(frozen=True)
class RowField:
  """A per-row (efc_*) or per-contact (con_*) array: `width` elements per row."""
  ctype: str
  name: str
  width: str   # integer literal or MJ_M(size)
  stage: int

  def row_size(self, sizes: dict) -> int:
    return _dim(self.width, sizes)


@dataclass(frozen=True)
class SparseField:
  """An array of the compressed Jacobians of sparse-mode models (MJHIP_DATA_SPARSE)."""
  ctype: str
  name: str
  dim: str     # ntendon, ntendon_nv, efc, efc_nv or nv

  def size(self, sizes: dict, efc_capacity: int) -> int:
    nt, nv = sizes["ntendon"], sizes["nv"]
    return {"ntendon": nt, "ntendon_nv": nt * nv, "efc": efc_capacity,
            "efc_nv": efc_capacity * nv, "nv": nv}[self.dim]


(MODEL_SIZES, MODEL_FIELDS, DATA_FIELDS, FORWARD_FIELDS, AUX_FIELDS, EFC_FIELDS,
 CONTACT_FIELDS, SPARSE_FIELDS) = _parse()
MODEL_FIELD = {f.name: f for f in MODEL_FIELDS}
DATA_FIELD = {f.name: f for f in DATA_FIELDS + FORWARD_FIELDS + AUX_FIELDS}


class Option(ctypes.Structure):
  """mjhipOption (include/mjhip.h), the subset of mjOption (mjmodel.h) on the path."""
  _fields_ = [
      ("timestep", ctypes.c_double),
      ("impratio", ctypes.c_double),
      ("gravity", ctypes.c_double * 3),
      ("wind", ctypes.c_double * 3),
      ("magnetic", ctypes.c_double * 3),
      ("density", ctypes.c_double),
      ("viscosity", ctypes.c_double),
      ("o_margin", ctypes.c_double),
      ("o_solref", ctypes.c_double * 2),
      ("o_solimp", ctypes.c_double * 5),
      ("o_friction", ctypes.c_double * 5),
      ("ccd_tolerance", ctypes.c_double),
      ("integrator", ctypes.c_int),
      ("cone", ctypes.c_int),
      ("jacobian", ctypes.c_int),
      ("disableflags", ctypes.c_int),
      ("enableflags", ctypes.c_int),
      ("ccd_iterations", ctypes.c_int),
  ]


class CModel(ctypes.Structure):
  _fields_ = ([(s, ctypes.c_int) for s in MODEL_SIZES] + [("opt", Option)] +
              [(f.name, ctypes.POINTER(CTYPE[f.ctype])) for f in MODEL_FIELDS])


class CData(ctypes.Structure):
  _fields_ = ([("nefc", ctypes.c_int), ("status", ctypes.c_int),
               ("solver_fwdinv", ctypes.c_double * 2), ("energy", ctypes.c_double * 2),
               ("time", ctypes.c_double)] +
              [(f.name, ctypes.POINTER(ctypes.c_double)) for f in DATA_FIELDS] +
              [(f.name, ctypes.POINTER(ctypes.c_double)) for f in FORWARD_FIELDS] +
              [(f.name, ctypes.POINTER(ctypes.c_double)) for f in AUX_FIELDS] +
              [(k, ctypes.c_int) for k in ("efc_capacity", "ne", "nf", "nl", "con_capacity",
                                           "ncon")] +
              [(f.name, ctypes.POINTER(CTYPE[f.ctype])) for f in EFC_FIELDS + CONTACT_FIELDS] +
              [("nJ", ctypes.c_int)] +
              [(f.name, ctypes.POINTER(CTYPE[f.ctype])) for f in SPARSE_FIELDS])


def is_sparse(m) -> bool:
  """mj_isSparse (engine_core_constraint.c:99-106): jacobian="sparse", or "auto" with nv >= 60."""
  jac = int(m.opt["jacobian"])
  return jac == 1 or (jac == 2 and m.sizes["nv"] >= 60)


def output_doubles(sizes: dict) -> int:
  """W of SURVEY.md §8d: fp64 mjData values written by mj_inverseSkip(NONE)."""
  return sum(f.size(sizes) for f in DATA_FIELDS if f.stage > 0)


def input_doubles(sizes: dict) -> int:
  """R of SURVEY.md §8d: fp64 values read per instance (qpos, qvel, qacc)."""
  return sum(f.size(sizes) for f in DATA_FIELDS if f.stage == 0)


def model_signature(m) -> int:
  """FNV-1a 64 over sizes, options and every model array, in field-table order.

  Identical to model_signature() in csrc/mjhip.hip, so a generated straight-line kernel is
  only ever used for a bit-identical model.
  """
  h = 0xcbf29ce484222325
  prime = 0x100000001b3
  mask = (1 << 64) - 1

  def feed(b: bytes):
    nonlocal h
    for byte in b:
      h ^= byte
      h = (h * prime) & mask

  for k in MODEL_SIZES:
    feed(np.int32(m.sizes.get(k, 0)).tobytes())
  o = m.opt
  for k in ("timestep", "impratio"):
    feed(np.float64(o[k]).tobytes())
  for k, n in (("gravity", 3), ("wind", 3), ("magnetic", 3)):
    feed(np.asarray(o[k], dtype=np.float64)[:n].tobytes())
  for k in ("density", "viscosity", "o_margin"):
    feed(np.float64(o[k]).tobytes())
  feed(np.asarray(o["o_solref"], dtype=np.float64)[:2].tobytes())
  feed(np.asarray(o["o_solimp"], dtype=np.float64)[:5].tobytes())
  feed(np.asarray(o["o_friction"], dtype=np.float64)[:5].tobytes())
  for k in ("integrator", "cone", "jacobian", "disableflags", "enableflags"):
    feed(np.int32(o[k]).tobytes())
  feed(np.float64(o.get("ccd_tolerance", 1e-6)).tobytes())
  feed(np.int32(o.get("ccd_iterations", 50)).tobytes())
  for f in MODEL_FIELDS:
    feed(np.ascontiguousarray(getattr(m, f.name), dtype=NPTYPE[f.ctype]).tobytes())
  return h
