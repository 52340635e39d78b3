"""Build/load the test-only CPU compilation of the device pipeline (cpu_kernel_harness.cpp)."""
import ctypes
import os
import subprocess

import numpy as np

from mujoco_inversedynamicstest_amd import fields, host

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
SO = os.path.join(BUILD, "libkernel_cpu.so")
# KERNEL_HARNESS_FLAGS: extra g++ flags, built under another name (tests/test_asan.py)
EXTRA = os.environ.get("KERNEL_HARNESS_FLAGS", "").split()
if EXTRA:
  SO = os.path.join(BUILD, "libkernel_cpu_san.so")
SRC = [os.path.join(HERE, "cpu_kernel_harness.cpp"),
       os.path.join(HERE, "..", "include", "mjhip.h"),
       os.path.join(HERE, "..", "include", "mjhip_fields.h"),
       os.path.join(HERE, "..", "include", "mjhip_contact.h"),
       os.path.join(HERE, "..", "mujoco_inversedynamicstest_amd", "csrc", "engine_device.h"),
       os.path.join(HERE, "..", "mujoco_inversedynamicstest_amd", "csrc", "pair_program.h")]

_lib = None


def lib():
  global _lib
  if _lib is None:
    os.makedirs(BUILD, exist_ok=True)
    if not os.path.exists(SO) or any(os.path.getmtime(s) > os.path.getmtime(SO) for s in SRC):
      # -ffp-contract=off: same rounding as the oracle's scalar C build
      # built under a private name and renamed: parallel test workers never see half a file
      tmp = f"{SO}.{os.getpid()}"
      subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-fPIC", "-shared",
                      *EXTRA, "-o", tmp, SRC[0]], check=True)
      os.replace(tmp, SO)
    L = ctypes.CDLL(SO)
    L.kh_sizes.restype = None
    L.kh_sizes.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                           ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long)]
    L.kh_field.restype = ctypes.c_int
    L.kh_field.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                           ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_long)]
    L.kh_forward.restype = ctypes.c_int
    L.kh_forward.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.kh_inverse.restype = ctypes.c_int
    L.kh_inverse.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int]
    D = ctypes.POINTER(ctypes.c_double)
    L.kh_ccd.restype = ctypes.c_int
    L.kh_ccd.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, D, D, D, D,
                         ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                         ctypes.c_double, D]
    _lib = L
  return _lib


def ccd_host(m, g1, g2, xpos, xmat, margin=0.0, tol=1e-6, kmax=1000, max_contacts=1,
             cutoff=0.0):
  """The device's mjc_ccd (mjh::ccdGeneral) compiled for the host, on geoms g1, g2 at the
  frames xpos [ngeom, 3], xmat [ngeom, 9]: (dist, nx, x1, x2), as Oracle.ccd."""
  cm = host.model_struct(m)
  D = ctypes.POINTER(ctypes.c_double)
  out = np.zeros(2 + 300)
  a = [np.ascontiguousarray(v, dtype=np.float64) for v in (xpos[g1], xmat[g1], xpos[g2],
                                                            xmat[g2])]
  st = lib().kh_ccd(ctypes.byref(cm), g1, g2, *(x.ctypes.data_as(D) for x in a), margin,
                    kmax, tol, max_contacts, cutoff, out.ctypes.data_as(D))
  assert st == 0, f"ccdGeneral status {st}"
  nx = int(out[1])
  if max_contacts <= 1:
    return out[0], nx, out[2:5].copy(), out[152:155].copy()
  return (out[0], nx, out[2:2 + 3*nx].reshape(nx, 3).copy(),
          out[152:152 + 3*nx].reshape(nx, 3).copy())


class KernelCPU:
  """One instance of the device pipeline on the host. Capacities default to the engine's
  (include/mjhip_contact.h, the same functions the oracle uses)."""

  def __init__(self, m, efc_cap=None, con_cap=None):
    from oracle.oracle import lib as olib
    self.m = m
    self.cm = host.model_struct(m)
    self.d = host.MjData(m, efc_capacity=efc_cap, con_capacity=con_cap)
    O = olib()
    self.efc_cap = O.or_efcCapacity(ctypes.byref(self.cm)) if efc_cap is None else efc_cap
    self.con_cap = max(O.or_contactCapacity(ctypes.byref(self.cm)), 0) if con_cap is None \
        else con_cap
    nd, ni = ctypes.c_long(), ctypes.c_long()
    lib().kh_sizes(ctypes.byref(self.cm), self.efc_cap, self.con_cap, ctypes.byref(nd),
                   ctypes.byref(ni))
    self.scratch = np.zeros(nd.value)
    self.iscratch = np.zeros(ni.value, dtype=np.int32)

  def inverse(self, qpos=None, qvel=None, qacc=None, skipstage=0, classic=False):
    """classic=True forces the unfused constraint path (the default follows the GPU)."""
    if qpos is not None:
      self.d.qpos[:] = qpos
    if qvel is not None:
      self.d.qvel[:] = qvel
    if qacc is not None:
      self.d.qacc[:] = qacc
    st = lib().kh_inverse(ctypes.byref(self.cm), ctypes.byref(self.d.struct),
                          self.scratch.ctypes.data, self.iscratch.ctypes.data, self.efc_cap,
                          self.con_cap, skipstage, int(classic))
    return self.d.qfrc_inverse.copy(), st

  def forward(self, qpos, qvel):
    self.d.qpos[:] = qpos
    self.d.qvel[:] = qvel
    st = lib().kh_forward(ctypes.byref(self.cm), ctypes.byref(self.d.struct),
                          self.scratch.ctypes.data, self.iscratch.ctypes.data, self.efc_cap,
                          self.con_cap)
    return self.d.qacc.copy(), st

  def field(self, name):
    """Whole scratch field (efc_* rows, con_* contacts, counts)."""
    off, n = ctypes.c_long(), ctypes.c_long()
    kind = lib().kh_field(ctypes.byref(self.cm), self.efc_cap, self.con_cap, name.encode(),
                          ctypes.byref(off), ctypes.byref(n))
    if kind < 0:
      raise KeyError(name)
    arr = self.iscratch if kind else self.scratch
    return arr[off.value:off.value + n.value]
