"""Python host side of the batched engine: ctypes binding of libmjhip.so (include/mjhip.h).

Mirrors the reference's inverse-dynamics interface (src/engine/engine_inverse.c) for one
mjModel and many states:

  InverseEngine(model).inverse(qpos, qvel, qacc)      batched mj_inverse     (inverse.c:266)
  InverseEngine.inverse(..., skipstage=, skipsensor=) batched mj_inverseSkip (inverse.c:197)
  InverseEngine.field(name)                           any mjData output field, per instance
  InverseEngine.inverse_fd(...)                       batched mjd_inverseFD  (derivative_fd.c:611)
  mj_inverse(m, d) / mj_inverseSkip(m, d, ...)        single-instance drop-ins on host MjData

Every call runs the HIP kernels; there is no CPU fallback. Importing this module on a
machine without a GPU works, but creating an engine raises MJHIPError (MJHIP_ERR_NO_DEVICE).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import fields, host

_HERE = os.path.dirname(os.path.abspath(__file__))
# MJHIP_LIB: an experiment build of the same library (tools/exp_phases.py variants); the
# default is the in-tree build, and a missing library is an error (no fallback path)
LIB_PATH = os.environ.get("MJHIP_LIB") or os.path.join(_HERE, "libmjhip.so")

mjSTAGE_NONE, mjSTAGE_POS, mjSTAGE_VEL = 0, 1, 2
FLAG_DEVICE_PTRS, FLAG_MIRROR_INPUT, FLAG_NO_MIRROR, FLAG_GENERIC = 1, 2, 4, 8
ERR = {0: "OK", -1: "NO_DEVICE", -2: "ARG", -3: "HIP", -4: "MODEL", -5: "CAPACITY",
       1: "INSTANCE"}
INST_BITS = {1: "BADQPOS", 2: "BADQVEL", 4: "BADQACC", 8: "INERTIA", 16: "CNSTRFULL",
             32: "UNSUPPORTED"}

_D = ctypes.POINTER(ctypes.c_double)
_I = ctypes.POINTER(ctypes.c_int)
_V = ctypes.c_void_p

# symbol -> (restype, argtypes): every MJHIP_API entry of include/mjhip.h
SIGNATURES = {
    "mjhip_version": (ctypes.c_char_p, []),
    "mjhip_deviceCount": (ctypes.c_int, []),
    "mjhip_lastError": (ctypes.c_char_p, []),
    "mjhip_setErrorCallback": (None, [_V]),
    "mjhip_fieldSize": (ctypes.c_int, [_V, ctypes.c_char_p]),
    "mjhip_outputDoubles": (ctypes.c_int, [_V]),
    "mjhip_contextCreate": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(_V)]),
    "mjhip_contextCreateCapped": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.POINTER(_V)]),
    "mjhip_contextFree": (None, [_V]),
    "mjhip_contextCapacity": (ctypes.c_int, [_V]),
    "mjhip_contextFastKernel": (ctypes.c_char_p, [_V]),
    "mjhip_contextLoadKernel": (ctypes.c_int, [_V, _V, ctypes.c_size_t, ctypes.c_char_p,
                                               ctypes.c_ulonglong, ctypes.c_int]),
    "mjhip_worklistCount": (ctypes.c_int, [_V]),
    "mjhip_contextLastPath": (ctypes.c_int, [_V]),
    "mjhip_contextConstraintKernel": (ctypes.c_char_p, [_V]),
    "mjhip_contextStream": (_V, [_V]),
    "mjhip_contextSetStream": (ctypes.c_int, [_V, _V]),
    "mjhip_inverseBatch": (ctypes.c_int, [_V, ctypes.c_int, _V, _V, _V, _V, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, _I]),
    "mjhip_forwardBatch": (ctypes.c_int, [_V, ctypes.c_int, _V, _V, _V, _V, ctypes.c_int, _I]),
    "mjhip_mirrorDownload": (ctypes.c_int, [_V, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                            _D]),
    "mjhip_mirrorUpload": (ctypes.c_int, [_V, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                          _D]),
    "mjhip_mirrorDevicePtr": (_V, [_V, ctypes.c_char_p]),
    "mjhip_mirrorDownloadInt": (ctypes.c_int, [_V, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                               _I]),
    "mjhip_fieldSizeInt": (ctypes.c_int, [_V, ctypes.c_char_p]),
    "mjhip_mirrorFieldSize": (ctypes.c_int, [_V, ctypes.c_char_p]),
    "mjhip_statusDownload": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, _I]),
    "mjhip_inverseFDBatch": (ctypes.c_int, [_V, ctypes.c_int, _V, _V, _V, ctypes.c_double,
                                            _V, _V, _V, _V, _V, _V, _V, ctypes.c_int]),
    "mjhip_inverseFDBatchEx": (ctypes.c_int, [_V, ctypes.c_int, _V, _V, _V, _V,
                                              ctypes.c_double, ctypes.c_int, _V, _V, _V, _V,
                                              _V, _V, _V, ctypes.c_int]),
    "mjhip_modelCapacity": (ctypes.c_int, [_V, _I, _I]),
    "mjhip_ccdBatch": (ctypes.c_int, [_V, ctypes.c_int, _I, _I, _D, _D, _D, _D, _D,
                                      ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                      ctypes.c_double, _D, _I, _D, _D]),
    "mjhip_timeInverseKernel": (ctypes.c_int, [_V, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int,
                                               ctypes.POINTER(ctypes.c_float)]),
    "mjhip_contextTimers": (ctypes.c_int, [_V, ctypes.c_int]),
    "mjhip_timerRead": (ctypes.c_int, [_V, _V, ctypes.c_int]),
    "mjhip_setDevice": (None, [ctypes.c_int]),
    "mjhip_inverse": (None, [_V, _V]),
    "mjhip_inverseSkip": (None, [_V, _V, ctypes.c_int, ctypes.c_int]),
    "mjhip_invPosition": (None, [_V, _V]),
    "mjhip_invVelocity": (None, [_V, _V]),
    "mjhip_invConstraint": (None, [_V, _V]),
    "mjhip_rne": (None, [_V, _V, ctypes.c_int, _D]),
    "mjhip_xfrcAccumulate": (None, [_V, _V, _D]),
    "mjhip_compareFwdInv": (None, [_V, _V]),
    "mjhip_inverseFD": (None, [_V, _V, ctypes.c_double, ctypes.c_ubyte, _D, _D, _D, _D, _D,
                               _D, _D]),
    "mjhip_releaseModel": (None, [_V]),
}


class MJHIPError(RuntimeError):
  pass


# the reference's mjtTimer slots (include/mujoco/mjdata.h), mjhipTimer in include/mjhip.h
TIMERS = ("STEP", "FORWARD", "INVERSE", "POSITION", "VELOCITY", "ACTUATION", "CONSTRAINT",
          "ADVANCE", "POS_KINEMATICS", "POS_INERTIA", "POS_COLLISION", "POS_MAKE",
          "POS_PROJECT", "COL_BROAD", "COL_NARROW")


class TimerStat(ctypes.Structure):
  """mjhipTimerStat (= the reference's mjTimerStat)."""
  _fields_ = [("duration", ctypes.c_double), ("number", ctypes.c_int)]


_lib = None


def lib():
  """Load libmjhip.so (built in-tree by __graft_entry__.build()); fail loudly if absent."""
  global _lib
  if _lib is None:
    # One HIP runtime per process: torch ships its own libamdhip64.so (same SONAME as
    # /opt/rocm's). Loading torch first makes libmjhip.so bind to that runtime, so device
    # pointers and streams can be shared with torch (bench.py, tests, RCCL).
    try:
      import torch  # noqa: F401
    except ImportError:
      pass
    if not os.path.exists(LIB_PATH):
      raise MJHIPError(f"{LIB_PATH} not built: run __graft_entry__.build() (the engine has "
                       "no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
      fn = getattr(L, name)
      fn.restype = res
      fn.argtypes = args
    _lib = L
  return _lib


def _check(rc, what):
  if rc < 0:
    msg = lib().mjhip_lastError().decode()
    raise MJHIPError(f"{what}: {ERR.get(rc, rc)}: {msg}")
  return rc


def _dptr(a):
  """Device pointer of a torch tensor, else None."""
  if hasattr(a, "data_ptr") and hasattr(a, "is_cuda"):
    if not a.is_cuda:
      raise MJHIPError("torch tensors passed to the engine must be on the GPU")
    if not a.is_contiguous() or str(a.dtype) != "torch.float64":
      raise MJHIPError("device tensors must be contiguous float64")
    return a.data_ptr()
  return None


class _TorchOrder:
  """Orders a device-pointer call after the work queued on torch's current stream and
  torch's later work after the call: the context's stream waits on an event recorded on
  torch's stream, and torch's stream waits on one recorded after the launch. Nothing is
  added when the context already runs on torch's current stream (set_stream)."""

  def __init__(self, engine):
    self.engine = engine
    self.ts = self.cs = None

  def __enter__(self):
    import torch
    ts = torch.cuda.current_stream(self.engine.device)
    if ts.cuda_stream != (self.engine.stream or 0):
      self.ts = ts
      self.cs = torch.cuda.ExternalStream(self.engine.stream, device=self.engine.device)
      self.cs.wait_stream(ts)
    return self

  def __exit__(self, *exc):
    if self.ts is not None:
      self.ts.wait_stream(self.cs)
    return False


class InverseEngine:
  """Batched mj_inverse for one model on one device (an mjhipContext).

  Calls with torch tensors run asynchronously on the context's stream, ordered with torch's
  current stream (inputs written by earlier torch work are read, and later torch work sees
  the outputs); host-array calls are synchronous."""

  def __init__(self, model, capacity: int, device: int = 0, specialize=None,
               max_contacts: int = 0, max_rows: int = 0):
    """specialize: generate and load a straight-line kernel for a model that has no bundled
    one (specialize.py; compiled once per model, then cached). None = the MJHIP_SPECIALIZE
    environment variable ("1" default, "0" off). max_contacts / max_rows: per-instance caps
    below the exact worst case (mjhip_contextCreateCapped; 0 = no cap)."""
    self.m = model
    self.cm = host.model_struct(model)
    L = lib()
    ctx = _V()
    _check(L.mjhip_contextCreateCapped(ctypes.byref(self.cm), device, capacity, max_contacts,
                                       max_rows, ctypes.byref(ctx)),
           "mjhip_contextCreateCapped")
    self.ctx = ctx
    self.device = device
    self.capacity = L.mjhip_contextCapacity(ctx)
    self.nv, self.nq = model.nv, model.nq
    explicit = specialize is True
    if specialize is None:
      specialize = os.environ.get("MJHIP_SPECIALIZE", "1") != "0"
    if specialize and self.fast_kernel is None and os.environ.get("MJHIP_DISABLE_FAST") != "1":
      from . import codegen
      from . import specialize as spec
      if codegen.fast_path_supported(model) is None:
        try:
          spec.load(self)
        except (spec.SpecializeError, OSError) as e:
          # no compiler, a read-only cache or a failed compile: the generic kernel still
          # serves the model (it did before specialization); only an explicit request fails
          if explicit:
            raise
          import warnings
          warnings.warn(f"run-time kernel specialization unavailable, using the generic "
                        f"kernel: {e}", RuntimeWarning, stacklevel=2)

  def close(self):
    if getattr(self, "ctx", None):
      lib().mjhip_contextFree(self.ctx)
      self.ctx = None

  def __del__(self):
    try:
      self.close()
    except Exception:   # interpreter shutdown
      pass

  @property
  def stream(self):
    return lib().mjhip_contextStream(self.ctx)

  def set_stream(self, stream_handle: int):
    _check(lib().mjhip_contextSetStream(self.ctx, stream_handle), "mjhip_contextSetStream")

  @property
  def fast_kernel(self):
    """Name of the model-specialized kernel in use, or None (generic kernel)."""
    n = lib().mjhip_contextFastKernel(self.ctx)
    return n.decode() if n else None

  @property
  def constraint_kernel(self):
    """The constraint kernel the last straight-line call launched ("none" if none)."""
    n = lib().mjhip_contextConstraintKernel(self.ctx)
    return n.decode() if n else None

  @property
  def last_path(self):
    """Kernels of the last batched inverse: 0 generic, 1 straight-line pipeline, 2 the
    straight-line mj_inverseSkip(POS / VEL) kernels, 3 the straight-line pipeline of a contact
    model split over two streams."""
    return lib().mjhip_contextLastPath(self.ctx)

  def worklist_count(self):
    return lib().mjhip_worklistCount(self.ctx)

  def inverse(self, qpos=None, qvel=None, qacc=None, out=None, skipstage=mjSTAGE_NONE,
              skipsensor=0, mirror_input=False, status=False, generic=False):
    """Batched mj_inverseSkip. numpy arrays (host) or float64 torch tensors (device).

    Returns qfrc_inverse [B, nv] (numpy for host inputs; `out` for device tensors). With
    mirror_input=True the inputs already in the mirror are used (pass B via qpos=int).
    """
    L = lib()
    flags = FLAG_GENERIC if generic else 0
    if mirror_input:
      B = int(qpos)
      flags |= FLAG_MIRROR_INPUT
      pq = pv = pa = None
      # no `out`: the results stay in the device mirror (field()), nothing is copied back
      dev = out is None or _dptr(out) is not None
    else:
      dev = _dptr(qpos) is not None
      if dev:
        B = qpos.shape[0]
        pq, pv, pa = _dptr(qpos), _dptr(qvel), _dptr(qacc)
      else:
        qpos = np.ascontiguousarray(qpos, dtype=np.float64).reshape(-1, self.nq)
        qvel = np.ascontiguousarray(qvel, dtype=np.float64).reshape(-1, self.nv)
        qacc = np.ascontiguousarray(qacc, dtype=np.float64).reshape(-1, self.nv)
        B = qpos.shape[0]
        pq, pv, pa = (qpos.ctypes.data, qvel.ctypes.data, qacc.ctypes.data)
    if dev:
      flags |= FLAG_DEVICE_PTRS
      po = _dptr(out) if out is not None else None
      st = None
    else:
      if out is None:
        out = np.zeros((B, self.nv))
      po = out.ctypes.data
      st = np.zeros(B, dtype=np.int32)
    if dev and (out is not None or not mirror_input):
      with _TorchOrder(self):
        rc = L.mjhip_inverseBatch(self.ctx, B, pq, pv, pa, po, skipstage, skipsensor, flags,
                                  None)
    else:
      rc = L.mjhip_inverseBatch(self.ctx, B, pq, pv, pa, po, skipstage, skipsensor, flags,
                                st.ctypes.data_as(_I) if st is not None else None)
    _check(rc, "mjhip_inverseBatch")
    if status:
      return out, st
    return out

  def forward(self, qpos, qvel, ctrl=None, qfrc_applied=None, xfrc_applied=None, out=None,
              status=False):
    """Batched constraint-free mj_forward (host numpy arrays). Returns qacc [B, nv].

    qfrc_applied [B, nv] / xfrc_applied [B, nbody, 6] are placed in the mirror first (they
    stay there for later calls, as in mjData); instances with constraint rows are flagged
    MJHIP_INST_UNSUPPORTED in the status (the constraint solver is not implemented)."""
    L = lib()
    qpos = np.ascontiguousarray(qpos, dtype=np.float64).reshape(-1, self.nq)
    qvel = np.ascontiguousarray(qvel, dtype=np.float64).reshape(-1, self.nv)
    B = qpos.shape[0]
    pc = None
    if ctrl is not None and self.m.nu:
      ctrl = np.ascontiguousarray(ctrl, dtype=np.float64).reshape(B, self.m.nu)
      pc = ctrl.ctypes.data
    if qfrc_applied is not None:
      self.set_field("qfrc_applied", np.reshape(qfrc_applied, (B, self.nv)))
    if xfrc_applied is not None:
      self.set_field("xfrc_applied", np.reshape(xfrc_applied, (B, 6 * self.m.nbody)))
    if out is None:
      out = np.zeros((B, self.nv))
    st = np.zeros(B, dtype=np.int32)
    rc = L.mjhip_forwardBatch(self.ctx, B, qpos.ctypes.data, qvel.ctypes.data, pc,
                              out.ctypes.data, 0, st.ctypes.data_as(_I))
    _check(rc, "mjhip_forwardBatch")     # per-instance flags come back in `st`
    return (out, st) if status else out

  def field(self, name, first=0, count=None):
    """Mirror field `name` of instances [first, first+count) as [count, size] (numpy)."""
    L = lib()
    S = L.mjhip_mirrorFieldSize(self.ctx, name.encode())
    if S < 0:
      raise MJHIPError(f"unknown field {name}")
    count = self.capacity - first if count is None else count
    out = np.zeros((count, max(S, 1)))
    if S:
      _check(L.mjhip_mirrorDownload(self.ctx, name.encode(), first, count,
                                    out.ctypes.data_as(_D)), "mjhip_mirrorDownload")
    return out[:, :S]

  def field_int(self, name, first=0, count=None):
    """Int per-instance array `name` (efc_type, efc_count, con_count, con_geom, ...)."""
    L = lib()
    S = L.mjhip_fieldSizeInt(self.ctx, name.encode())
    if S < 0:
      raise MJHIPError(f"unknown int field {name}")
    count = self.capacity - first if count is None else count
    out = np.zeros((count, max(S, 1)), dtype=np.int32)
    if S:
      _check(L.mjhip_mirrorDownloadInt(self.ctx, name.encode(), first, count,
                                       out.ctypes.data_as(_I)), "mjhip_mirrorDownloadInt")
    return out[:, :S]

  def set_field(self, name, values, first=0):
    values = np.ascontiguousarray(values, dtype=np.float64)
    count = values.shape[0]
    _check(lib().mjhip_mirrorUpload(self.ctx, name.encode(), first, count,
                                    values.ctypes.data_as(_D)), "mjhip_mirrorUpload")

  def upload_states(self, qpos, qvel, qacc, first=0):
    """Place states in the device mirror (inputs resident in HBM for timed runs)."""
    self.set_field("qpos", qpos, first)
    self.set_field("qvel", qvel, first)
    self.set_field("qacc", qacc, first)

  def ccd(self, g1, g2, pos1, mat1, pos2, mat2, margin=None, max_iterations=1000,
          tolerance=1e-6, max_contacts=1, dist_cutoff=0.0):
    """mjc_ccd on the device over pairs (g1[i], g2[i]) at frames pos (n x 3) / mat (n x 9)
    (mjhip_ccdBatch): (dist [n], nx [n], x1 [n, 3], x2 [n, 3]); with max_contacts > 1, x1 / x2
    are [n, min(max_contacts, 50), 3] (multicontact; the first nx[i] rows hold pair i's)."""
    g1 = np.ascontiguousarray(g1, dtype=np.int32)
    g2 = np.ascontiguousarray(g2, dtype=np.int32)
    n = g1.size
    f = [np.ascontiguousarray(a, dtype=np.float64).reshape(n, -1)
         for a in (pos1, mat1, pos2, mat2)]
    mg = None if margin is None else np.ascontiguousarray(
        np.broadcast_to(margin, (n,)), dtype=np.float64)
    dist, nx = np.zeros(n), np.zeros(n, dtype=np.int32)
    xcap = 1 if max_contacts <= 1 else min(max_contacts, 50)
    x1, x2 = np.zeros((n, xcap, 3)), np.zeros((n, xcap, 3))
    D = lambda a: a.ctypes.data_as(_D)
    _check(lib().mjhip_ccdBatch(self.ctx, n, g1.ctypes.data_as(_I), g2.ctypes.data_as(_I),
                                *map(D, f), D(mg) if mg is not None else None,
                                max_iterations, tolerance, max_contacts, dist_cutoff, D(dist),
                                nx.ctypes.data_as(_I), D(x1), D(x2)), "mjhip_ccdBatch")
    if xcap == 1:
      return dist, nx, x1[:, 0], x2[:, 0]
    return dist, nx, x1, x2

  def timers(self, enable=True):
    """Per-stage timers on or off (mjhip_contextTimers): timed inverse calls synchronize."""
    _check(lib().mjhip_contextTimers(self.ctx, int(bool(enable))), "mjhip_contextTimers")

  def timer_read(self, reset=False):
    """{mjTIMER name: (milliseconds, calls)} accumulated since the last reset."""
    out = (TimerStat * len(TIMERS))()
    _check(lib().mjhip_timerRead(self.ctx, out, int(bool(reset))), "mjhip_timerRead")
    return {n: (out[i].duration, out[i].number) for i, n in enumerate(TIMERS)}

  def time_kernel(self, B, reps=20, skipstage=mjSTAGE_NONE, generic=False):
    """Average ms per launch of the mj_inverse kernels on mirror-resident inputs (HIP
    events on the context's stream; fast path = straight-line kernel + work-list kernel)."""
    ms = ctypes.c_float()
    _check(lib().mjhip_timeInverseKernel(self.ctx, B, reps, skipstage,
                                         FLAG_GENERIC if generic else 0, ctypes.byref(ms)),
           "mjhip_timeInverseKernel")
    return ms.value

  def inverse_fd(self, qpos, qvel, qacc, eps=1e-6, dmdq=False, sensors=False, out=None,
                 ctrl=None, flg_actuation=False):
    """Batched mjd_inverseFD: DfDq, DfDv, DfDa [B, nv, nv], DmDq [B, nv, nM] (or None), plus
    (DsDq, DsDv, DsDa) [B, nv, nsensordata] when sensors. With flg_actuation the forces are
    qfrc_inverse - qfrc_actuator of the base states' controls ctrl [B, nu].

    Host arrays in -> numpy arrays out (PCIe both ways). Contiguous float64 torch tensors on
    the context's GPU in -> torch tensors out on that GPU, asynchronous on the context's
    stream (out: optional preallocated tuple in the same order as the return value)."""
    nv, ns = self.nv, self.m.sizes.get("nsensordata", 0)
    if _dptr(qpos) is not None:
      import torch
      B = qpos.shape[0]
      # the kernels index these by B without bounds: check the shapes before the launch
      if tuple(qpos.shape) != (B, self.nq) or tuple(qvel.shape) != (B, nv) or \
         tuple(qacc.shape) != (B, nv):
        raise MJHIPError(f"inverse_fd: expected qpos [{B}, {self.nq}], qvel and qacc "
                         f"[{B}, {nv}]")
      if ctrl is not None and ctrl.numel() != B * self.m.nu:
        raise MJHIPError(f"inverse_fd: ctrl must hold B x nu = {B * self.m.nu} values")
      if flg_actuation and self.m.nu and ctrl is None:
        raise MJHIPError("inverse_fd: flg_actuation needs ctrl [B, nu]")
      if out is None:
        mk = lambda n: torch.empty((B, nv, n), dtype=torch.float64, device=qpos.device)
        out = (mk(nv), mk(nv), mk(nv), mk(self.m.nM) if dmdq else None)
        if sensors:
          out = out + ((mk(ns), mk(ns), mk(ns)),)
      ptr = lambda t: None if t is None else _dptr(t)
      Ds = out[4] if len(out) > 4 else (None, None, None)
      with _TorchOrder(self):
        rc = lib().mjhip_inverseFDBatchEx(self.ctx, B, _dptr(qpos), _dptr(qvel), _dptr(qacc),
                                          None if ctrl is None else _dptr(ctrl), eps,
                                          int(bool(flg_actuation)), ptr(out[0]), ptr(out[1]),
                                          ptr(out[2]), *map(ptr, Ds), ptr(out[3]),
                                          FLAG_DEVICE_PTRS)
      _check(rc, "mjhip_inverseFDBatchEx")
      return tuple(out)
    qpos = np.ascontiguousarray(qpos, dtype=np.float64).reshape(-1, self.nq)
    qvel = np.ascontiguousarray(qvel, dtype=np.float64).reshape(-1, self.nv)
    qacc = np.ascontiguousarray(qacc, dtype=np.float64).reshape(-1, self.nv)
    B = qpos.shape[0]
    DfDq = np.zeros((B, nv, nv))
    DfDv = np.zeros((B, nv, nv))
    DfDa = np.zeros((B, nv, nv))
    DmDq = np.zeros((B, nv, self.m.nM)) if dmdq else None
    Ds = tuple(np.zeros((B, nv, ns)) for _ in range(3)) if sensors else (None, None, None)
    p = lambda a: None if a is None else a.ctypes.data
    if ctrl is not None:
      ctrl = np.ascontiguousarray(ctrl, dtype=np.float64).reshape(B, -1)
    _check(lib().mjhip_inverseFDBatchEx(self.ctx, B, qpos.ctypes.data, qvel.ctypes.data,
                                        qacc.ctypes.data, p(ctrl), eps,
                                        int(bool(flg_actuation)), p(DfDq), p(DfDv), p(DfDa),
                                        *map(p, Ds), p(DmDq), 0),
           "mjhip_inverseFDBatchEx")
    if sensors:
      return DfDq, DfDv, DfDa, DmDq, Ds
    return DfDq, DfDv, DfDa, DmDq


def output_bytes_per_eval(model) -> int:
  """B_eval of SURVEY.md §8d: 8 * (R + W) for the model's field table."""
  return 8 * (fields.input_doubles(model.sizes) + fields.output_doubles(model.sizes))


def constraint_bytes(model, nefc_total: int, ncon_total: int, B: int) -> int:
  """Algorithmic bytes the constraint part of B evaluations writes on top of B_eval: per row
  the efc_* arrays of MJHIP_DATA_EFC (nv + 13 doubles: J, pos, margin, frictionloss,
  diagApprox, KBIP[4], D, R, vel, aref, force; 3 ints: type, id, state), per contact the
  con_* arrays of MJHIP_DATA_CON (29 doubles, 5 ints), per instance its 4 count words."""
  row = 8 * (model.nv + 13) + 4 * 3
  con = 8 * 29 + 4 * 5
  return row * int(nefc_total) + con * int(ncon_total) + 16 * int(B)


# ---------------------------------------------------------------- single-instance drop-ins
# The model struct is rebuilt per call (its option block is a copy), so edits of the Model
# between calls are seen; the library caches device state by the model's content.


def _cm(m):
  return host.model_struct(m)


def _out(a, n, what):
  """A caller's float64 output vector, written in place (no silent copies)."""
  if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous
          and a.size >= n):
    raise MJHIPError(f"{what}: expected a C-contiguous float64 array of {n} values")
  return a.ctypes.data_as(_D)


def mj_inverse(m, d: host.MjData):
  """mj_inverse(m, d) (engine_inverse.c:266) on the GPU, writing every output into d."""
  lib().mjhip_inverse(ctypes.byref(_cm(m)), d.ptr())


def mj_inverseSkip(m, d: host.MjData, skipstage: int, skipsensor: int):
  """mj_inverseSkip (engine_inverse.c:197) on the GPU: reads the skipped stages' fields and
  constraint rows from d, writes the outputs and rows of the stages that ran."""
  lib().mjhip_inverseSkip(ctypes.byref(_cm(m)), d.ptr(), skipstage, skipsensor)


def mj_invPosition(m, d: host.MjData):
  """mj_invPosition (engine_inverse.c:37-68): position stage only."""
  lib().mjhip_invPosition(ctypes.byref(_cm(m)), d.ptr())


def mj_invVelocity(m, d: host.MjData):
  """mj_invVelocity (engine_inverse.c:73-76): velocity stage only."""
  lib().mjhip_invVelocity(ctypes.byref(_cm(m)), d.ptr())


def mj_invConstraint(m, d: host.MjData):
  """mj_invConstraint (engine_inverse.c:169-192): qfrc_constraint, efc_force, efc_state."""
  lib().mjhip_invConstraint(ctypes.byref(_cm(m)), d.ptr())


def mj_rne(m, d: host.MjData, flg_acc: int, result):
  """mj_rne (engine_core_smooth.c:1969): result = RNE of d's cdof/cinert/cvel/cdof_dot."""
  lib().mjhip_rne(ctypes.byref(_cm(m)), d.ptr(), flg_acc, _out(result, m.nv, "mj_rne"))


def mj_xfrcAccumulate(m, d: host.MjData, qfrc):
  """mj_xfrcAccumulate (engine_support.c:1254): qfrc += J' xfrc_applied, in place."""
  lib().mjhip_xfrcAccumulate(ctypes.byref(_cm(m)), d.ptr(), _out(qfrc, m.nv,
                                                                   "mj_xfrcAccumulate"))


def mj_compareFwdInv(m, d: host.MjData):
  """mj_compareFwdInv (engine_inverse.c:275-316): fills d.solver_fwdinv."""
  lib().mjhip_compareFwdInv(ctypes.byref(_cm(m)), d.ptr())


def mjd_inverseFD(m, d: host.MjData, eps, flg_actuation, DfDq=None, DfDv=None, DfDa=None,
                  DsDq=None, DsDv=None, DsDa=None, DmDq=None):
  """mjd_inverseFD (engine_derivative_fd.c:611-719); outputs are filled in place (None to
  skip), in the reference's transposed layout (nv x nv, nv x nsensordata, nv x nM)."""
  nv, ns, nM = m.nv, m.sizes.get("nsensordata", 0), m.nM
  p = lambda a, n, w: None if a is None else _out(a, n, "mjd_inverseFD " + w)
  lib().mjhip_inverseFD(ctypes.byref(_cm(m)), d.ptr(), float(eps), int(bool(flg_actuation)),
                        p(DfDq, nv * nv, "DfDq"), p(DfDv, nv * nv, "DfDv"),
                        p(DfDa, nv * nv, "DfDa"), p(DsDq, nv * ns, "DsDq"),
                        p(DsDv, nv * ns, "DsDv"), p(DsDa, nv * ns, "DsDa"),
                        p(DmDq, nv * nM, "DmDq"))


def release_model(m):
  """Release the device state the single-instance calls cached for model m."""
  lib().mjhip_releaseModel(ctypes.byref(_cm(m)))
