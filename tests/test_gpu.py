"""GPU parity: the HIP engine vs the CPU oracle (run on an MI355X with -m gpu).

Tolerance (BASELINE.json north_star): bit-exact on indices/counts; fp64 outputs within
1e-10 relative, measured normwise per instance: max_k |gpu_k - cpu_k| <= 1e-10 * max(1,
max_k |cpu_k|). The GPU build contracts multiply-adds into FMAs and uses the device libm
(sin/cos in mju_axisAngle2Quat); the same source compiled without contraction on the host
matches the oracle bit for bit (test_kernel_cpu.py).
"""
import ctypes

import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine, fields, host, models
from mujoco_inversedynamicstest_amd.sampler import sample_contact_states, sample_states
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu
RTOL = 1e-10
OUTPUTS = [f.name for f in fields.DATA_FIELDS if f.stage > 0]


def assert_close(gpu, cpu, what):
  gpu = np.asarray(gpu).reshape(len(gpu), -1)
  cpu = np.asarray(cpu).reshape(len(cpu), -1)
  scale = np.maximum(1.0, np.abs(cpu).max(axis=1))
  err = (np.abs(gpu - cpu).max(axis=1) / scale).max()
  assert err <= RTOL, f"{what}: normwise relative error {err:.3e} > {RTOL}"
  return err


def oracle_batch(m, q, v, a, fields_=("qfrc_inverse",)):
  o = Oracle(m)
  out = {f: [] for f in fields_}
  nefc = []
  for i in range(len(q)):
    o.inverse(q[i], v[i], a[i])
    for f in fields_:
      out[f].append(getattr(o.d, f).copy())
    nefc.append(o.d.nefc)
  return {f: np.array(x) for f, x in out.items()}, np.array(nefc)


@pytest.fixture(scope="module")
def eng(humanoid):
  e = engine.InverseEngine(humanoid, capacity=65536 + 4096)
  yield e
  e.close()


def test_device_present():
  assert engine.lib().mjhip_deviceCount() >= 1


def test_humanoid_config2_parity_4096(humanoid, eng):
  """Config 2: humanoid, contacts disabled, B=4096, every limit inactive (nefc = 0)."""
  q, v, a = sample_states(humanoid, 4096)
  f, st = eng.inverse(q, v, a, status=True)
  assert (st == 0).all()
  ref, nefc = oracle_batch(humanoid, q, v, a)
  assert (nefc == 0).all()
  assert_close(f, ref["qfrc_inverse"], "qfrc_inverse")


def test_humanoid_every_mirror_field(humanoid, eng):
  """All 2,563 mjData doubles of mj_inverse for 256 instances."""
  q, v, a = sample_states(humanoid, 256, first=77)
  eng.inverse(q, v, a)
  ref, _ = oracle_batch(humanoid, q, v, a, OUTPUTS)
  for f in OUTPUTS:
    if fields.DATA_FIELD[f].size(humanoid.sizes):
      assert_close(eng.field(f, 0, 256), ref[f], f)


def test_humanoid_limits_active(humanoid, eng):
  """Limit rows (joint + tendon), impedance and qfrc_constraint on the device."""
  q, v, a = sample_states(humanoid, 512, first=3000, margin=-0.25, resample_tendons=False)
  f = eng.inverse(q, v, a)
  ref, nefc = oracle_batch(humanoid, q, v, a, ("qfrc_inverse", "qfrc_constraint"))
  assert nefc.sum() > 512
  assert_close(f, ref["qfrc_inverse"], "qfrc_inverse")
  assert_close(eng.field("qfrc_constraint", 0, 512), ref["qfrc_constraint"], "qfrc_constraint")


def test_skipstage_chain(humanoid, eng):
  """mj_inverseSkip(VEL) / (POS) reuse the earlier stages kept in the device mirror."""
  q, v, a = sample_states(humanoid, 128, first=11)
  eng.inverse(q, v, a)
  a2 = a + 0.25
  f_vel = eng.inverse(q, v, a2, skipstage=engine.mjSTAGE_VEL)
  v2 = v * 0.9
  f_pos = eng.inverse(q, v2, a2, skipstage=engine.mjSTAGE_POS)
  o = Oracle(humanoid)
  rv, rp = [], []
  for i in range(128):
    o.inverse(q[i], v[i], a[i])
    rv.append(o.inverse(qacc=a2[i], skipstage=2))
    rp.append(o.inverse(qvel=v2[i], skipstage=1))
  assert_close(f_vel, rv, "skip VEL")
  assert_close(f_pos, rp, "skip POS")


@pytest.mark.parametrize("name", ["humanoid", "humanoid_contact", "inverse_test", "linear",
                                  "inertia"])
def test_skipstage_straight_line(name, monkeypatch):
  """Batched mj_inverseSkip(POS / VEL) on the straight-line kernels (k_va for POS, k_acc for
  VEL): the path is asserted (mjhip_contextLastPath = 2), on the humanoid
  a fifth of the instances carry limit rows from the full call (k_skip_rows finishes them), and
  the results match the oracle's serial mj_inverseSkip chain and the generic kernel
  (MJHIP_SKIP_GENERIC=1) to the north-star tolerance, with inputs given for every field."""
  contact = name == "humanoid_contact"
  m = models.load("humanoid" if contact else name, disable_contact=not contact,
                  disable_sensor=(name == "linear"))
  B = 200
  # humanoid_contact (rows on every instance: contacts and their rows from the full call,
  # finished for every instance by k_skip_rows; the reference driver's own call,
  # inverse_test.cpp:93, on a model with contacts)
  q, v, a = sample_contact_states(m, B) if contact else sample_states(m, B, first=21)
  if name == "humanoid":
    j = int(np.flatnonzero(np.asarray(m.jnt_limited))[3])
    q[::5, m.jnt_qposadr[j]] = m.jnt_range[j][1] + 0.2
  a2, v2 = a + 0.25, v * 0.9
  e = engine.InverseEngine(m, capacity=256)
  try:
    assert e.fast_kernel == name
    got = []
    for generic in (False, True):
      if generic:
        monkeypatch.setenv("MJHIP_SKIP_GENERIC", "1")
      e.inverse(q, v, a)
      assert e.last_path == 1
      fv, sv = e.inverse(q, v, a2, skipstage=engine.mjSTAGE_VEL, status=True)
      assert e.last_path == (0 if generic else 2)
      fp, sp = e.inverse(q, v2, a2, skipstage=engine.mjSTAGE_POS, status=True)
      assert e.last_path == (0 if generic else 2)
      assert (sv == 0).all() and (sp == 0).all()
      got.append((fv, fp, e.field("qfrc_constraint", 0, B), e.field("efc_force", 0, B)))
    nefc = e.field_int("efc_count", 0, B)[:, 0]
  finally:
    e.close()
  o = Oracle(m)
  rv, rp, rc = [], [], []
  for i in range(B):
    o.inverse(q[i], v[i], a[i])
    rv.append(o.inverse(qacc=a2[i], skipstage=2))
    rp.append(o.inverse(qvel=v2[i], skipstage=1))
    rc.append(o.d.qfrc_constraint.copy())
    assert o.d.nefc == nefc[i]
  if name == "humanoid":
    assert (nefc[::5] > 0).all()
  if contact:
    assert (nefc > 0).mean() > 0.5 and (nefc == 0).any()
  for (fv, fp, qc, _), what in zip(got, ("straight-line", "generic")):
    assert_close(fv, rv, f"{name} skip VEL ({what})")
    assert_close(fp, rp, f"{name} skip POS ({what})")
    assert_close(qc, rc, f"{name} qfrc_constraint ({what})")
  assert_close(got[0][0], got[1][0], "VEL straight-line vs generic")
  assert_close(got[0][1], got[1][1], "POS straight-line vs generic")


@pytest.mark.parametrize("B", [1, 63, 64, 65, 1000])
def test_ragged_batches(humanoid, eng, B):
  q, v, a = sample_states(humanoid, B, first=500)
  f = eng.inverse(q, v, a)
  ref, _ = oracle_batch(humanoid, q, v, a)
  assert f.shape == (B, humanoid.nv)
  assert_close(f, ref["qfrc_inverse"], f"B={B}")


def test_empty_batch(humanoid, eng):
  out = eng.inverse(np.zeros((0, humanoid.nq)), np.zeros((0, humanoid.nv)),
                    np.zeros((0, humanoid.nv)))
  assert out.shape == (0, humanoid.nv)


@pytest.mark.parametrize("name", ["inverse_test", "linear", "inertia"])
def test_other_models(name):
  m = models.load(name, disable_contact=True)
  q, v, a = sample_states(m, 300)
  e = engine.InverseEngine(m, capacity=512)
  f = e.inverse(q, v, a)
  ref, _ = oracle_batch(m, q, v, a, OUTPUTS)
  assert_close(f, ref["qfrc_inverse"], name)
  for fld in ("qM", "qLD", "cdof", "cinert", "qfrc_bias", "qfrc_passive"):
    if fields.DATA_FIELD[fld].size(m.sizes):
      assert_close(e.field(fld, 0, 300), ref[fld], f"{name}.{fld}")
  e.close()


def test_full_size_properties(humanoid, eng):
  """B = 65,536 (the metric's batch): shard equivalence (bit-exact) and the affine-in-qacc
  identity qfrc_inverse(a) - qfrc_inverse(0) = M(q) a, with M from the device mirror."""
  B = 65536
  q, v, a = sample_states(humanoid, B)
  f = eng.inverse(q, v, a)
  h = B // 2
  f1 = eng.inverse(q[:h], v[:h], a[:h])
  f2 = eng.inverse(q[h:], v[h:], a[h:])
  np.testing.assert_array_equal(np.vstack([f1, f2]), f)
  f0 = eng.inverse(q, v, np.zeros_like(a))
  qM = eng.field("qM", 0, B)
  # dense M from qM (dof_Madr ancestor lists)
  nv = humanoid.nv
  Mx = np.zeros_like(a)
  adr = 0
  for i in range(nv):
    j = i
    while j >= 0:
      Mx[:, i] += qM[:, adr] * a[:, j]
      if j != i:
        Mx[:, j] += qM[:, adr] * a[:, i]
      j = humanoid.dof_parentid[j]
      adr += 1
  scale = np.maximum(1.0, np.abs(f).max(axis=1))
  assert (np.abs((f - f0) - Mx).max(axis=1) / scale).max() < 1e-9
  # a checksum of checksums, for the record
  assert np.isfinite(f).all()


def test_inverse_fd_parity(humanoid):
  """Config 5 at its configured size: batched mjd_inverseFD over 1,024 base states (x 82
  evaluations) vs the oracle's serial mjd_inverseFD on a subsample, and on every base state
  the size-independent property DfDa = M (inverse dynamics is affine in qacc with slope M;
  forward differences of an affine map are exact up to rounding / eps). The stage-skip
  layout puts the centres first and they keep every field: the fields the perturbed
  instances drop (codegen.FD_KEEP) equal a plain mj_inverse of the base states."""
  NB = 1024
  q, v, a = sample_states(humanoid, NB, first=900)
  e = engine.InverseEngine(humanoid, capacity=NB * (3 * humanoid.nv + 1))
  try:
    DfDq, DfDv, DfDa, DmDq = e.inverse_fd(q, v, a, eps=1e-6, dmdq=True)
    centre = {f: e.field(f, 0, NB) for f in ("xpos", "xmat", "crb", "qLD", "cvel", "qfrc_bias")}
    e.inverse(q, v, a)
    qM = e.field("qM", 0, NB)
    for f, x in centre.items():
      np.testing.assert_array_equal(x, e.field(f, 0, NB), err_msg=f)
  finally:
    e.close()
  nv = humanoid.nv
  madr, parent = humanoid.dof_Madr, humanoid.dof_parentid
  for i in range(NB):                   # dense M from the sparse qM of the base state
    M = np.zeros((nv, nv))
    for r in range(nv):
      adr, c = madr[r], r
      while c >= 0:
        M[r, c] = M[c, r] = qM[i, adr]
        adr, c = adr + 1, parent[c]
    np.testing.assert_allclose(DfDa[i], M, rtol=1e-6, atol=1e-6 * np.abs(M).max())
  o = Oracle(humanoid)
  for i in range(0, NB, 64):
    o.set_state(q[i], v[i], a[i])
    rq, rv, ra, rm = o.inverse_fd(1e-6, dmdq=True)
    # FD amplifies last-bit differences of the two builds by 1/eps = 1e6
    np.testing.assert_allclose(DfDa[i], ra, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(DfDv[i], rv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(DfDq[i], rq, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(DmDq[i], rm, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("NB,limits", [(1024, "none"), (64, "all"), (64, "some"),
                                       (48, "some"), (3, "none")])
def test_inverse_fd_stage_skip_bit_exact(humanoid, NB, limits, monkeypatch):
  """mjd_inverseFD's stage skipping (engine_derivative_fd.c:646-699: the qvel perturbations
  run mj_inverseSkip(mjSTAGE_POS), the qacc ones mjSTAGE_VEL) against every perturbation
  through the full pipeline (MJHIP_FD_NOSKIP=1). Layout 1 (both kinds on the va stage over the
  centre's position-stage outputs; the default runs k_all then k_vaskip, MJHIP_FD_FUSED=1 one
  launch, k_fdall, whose skip waves wait for their centres' flags; the perturbed instances
  run the generated bodies without the stores nobody reads, which the compiler contracts
  into multiply-adds a little differently) equals it within the contraction bound; layout 2
  (MJHIP_FD_ACCSKIP=1: the qacc perturbations on the acceleration stage alone over the centre's velocity stage,
  k_fdskip) within it too. NB=1024 takes the skip layouts; with joint limits active on every centre, or on every
  fifth, the work-list model falls back on the device to the full pipeline over the
  perturbations; NB=48 puts 16 qpos perturbations in the centres' block (which stores every
  field); NB=3 (28*3 instances, not a whole wave) never takes them."""
  q, v, a = sample_states(humanoid, NB, first=300)
  if limits != "none":                  # push a limited hinge past its range
    j = int(np.flatnonzero(np.asarray(humanoid.jnt_limited))[3])
    rows = slice(None) if limits == "all" else slice(None, None, 5)
    q[rows, humanoid.jnt_qposadr[j]] = humanoid.jnt_range[j][1] + 0.2
  e = engine.InverseEngine(humanoid, capacity=NB * (3 * humanoid.nv + 1))
  try:
    got1 = e.inverse_fd(q, v, a, eps=1e-6, dmdq=True)      # layout 1, the default
    monkeypatch.setenv("MJHIP_FD_FUSED", "1")               # layout 1 in one launch (k_fdall)
    got1u = e.inverse_fd(q, v, a, eps=1e-6, dmdq=True)
    monkeypatch.delenv("MJHIP_FD_FUSED")
    monkeypatch.setenv("MJHIP_FD_ACCSKIP", "1")             # layout 2
    got = e.inverse_fd(q, v, a, eps=1e-6, dmdq=True)
    monkeypatch.setenv("MJHIP_FD_NOSKIP", "1")
    ref = e.inverse_fd(q, v, a, eps=1e-6, dmdq=True)
  finally:
    e.close()
  for g, g1, g1u, r in zip(got, got1, got1u, ref):
    _assert_fd_contraction_close(g1, r)
    _assert_fd_contraction_close(g1u, r)
    _assert_fd_contraction_close(g, r)


def _assert_fd_contraction_close(g, r, eps=1e-6):
  """A skip layout against the full pipeline: the same operations, but the compiler contracts
  multiply-adds per kernel body (layout 2's acceleration-only stage; layout 1's perturbed
  instances, whose bodies drop the stores nobody reads), so a term of qfrc_inverse can round
  differently by a few ulp; the forward difference scales that by 1/eps. Bound: 16 ulp of the
  largest |qfrc_inverse| (<= 1e3 on these states) over eps."""
  tol = 16 * np.finfo(float).eps * 1e3 / eps
  err = np.abs(g - r).max()
  assert err <= tol, f"DfDa layout 2 vs full pipeline {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("name", ["inverse_test", "linear", "inertia"])
def test_inverse_fd_stage_skip_other_models(name, monkeypatch):
  """The stage-skip layouts on the other bundled models with a k_vaskip kernel (work-list or
  row-free): layout 1 device-resident and back to back (no host wait between calls, each call
  bit-identical to the last) against the full pipeline within the contraction bound (the
  perturbed instances' bodies without their unread stores), layout 2 (k_fdskip) within it
  as well, and both against the oracle's serial mjd_inverseFD."""
  import torch
  m = models.load(name, disable_contact=True, disable_sensor=(name == "linear"))
  NB = 64
  q, v, a = sample_states(m, NB, first=40)
  e = engine.InverseEngine(m, capacity=NB * (3 * m.nv + 1))
  try:
    assert e.fast_kernel == name
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
    tq, tv, ta = t(q), t(v), t(a)
    outs = [e.inverse_fd(tq, tv, ta, eps=1e-6) for _ in range(3)]
    torch.cuda.synchronize()
    got = [x.cpu().numpy() for x in outs[-1][:3]]
    for o in outs[:-1]:
      for x, y in zip(o[:3], got):
        assert np.array_equal(x.cpu().numpy(), y)
    monkeypatch.setenv("MJHIP_FD_ACCSKIP", "1")             # layout 2, k_fdskip
    got2 = e.inverse_fd(q, v, a, eps=1e-6)
    monkeypatch.setenv("MJHIP_FD_NOSKIP", "1")
    ref = e.inverse_fd(q, v, a, eps=1e-6)
  finally:
    e.close()
  for g, g2, r in zip(got, got2, ref[:3]):
    _assert_fd_contraction_close(g, r)
    _assert_fd_contraction_close(g2, r)
  o = Oracle(m)
  for i in range(0, NB, 8):
    o.set_state(q[i], v[i], a[i])
    rq, rv, ra, _ = o.inverse_fd(1e-6)
    np.testing.assert_allclose(got[2][i], ra, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got[1][i], rv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(got[0][i], rq, rtol=1e-5, atol=1e-4)


def test_inverse_fd_device_tensors(humanoid, eng):
  """Device-resident mjd_inverseFD (config 5 bench path) equals the host-array path bit for
  bit: same kernels, only the transfers differ."""
  import torch
  q, v, a = sample_states(humanoid, 8, first=1200)
  hq, hv, ha, hm = eng.inverse_fd(q, v, a, eps=1e-6, dmdq=True)
  t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).cuda()
  tq, tv, ta = t(q), t(v), t(a)
  torch.cuda.synchronize()
  dq, dv, da, dm = eng.inverse_fd(tq, tv, ta, eps=1e-6, dmdq=True)
  torch.cuda.synchronize()
  for h, d in ((hq, dq), (hv, dv), (ha, da), (hm, dm)):
    assert np.array_equal(h, d.cpu().numpy())


def test_linear_system_inverse_on_gpu(linear):
  """LinearSystemInverse (engine_derivative_test.cc:793-868) through the GPU FD path."""
  o = Oracle(linear)
  o.forward()
  e = engine.InverseEngine(linear, capacity=64)
  DfDq, DfDv, DfDa, DmDq = e.inverse_fd(o.d.qpos[None], o.d.qvel[None], o.d.qacc[None],
                                        eps=1e-6, dmdq=True)
  np.testing.assert_allclose(DfDq[0], np.diag(linear.jnt_stiffness), atol=1e-6)
  np.testing.assert_allclose(DfDv[0], np.diag(linear.dof_damping), atol=1e-6)
  np.testing.assert_allclose(DfDa[0], o.fullM(), atol=1e-6)
  np.testing.assert_allclose(DmDq[0], 0, atol=1e-6)
  # LinearSystemInverse's sensor derivatives (engine_derivative_test.cc:843-862)
  _, _, _, _, (DsDq, DsDv, DsDa) = e.inverse_fd(o.d.qpos[None], o.d.qvel[None],
                                                o.d.qacc[None], eps=1e-6, sensors=True)
  ns, adr = linear.nsensordata, linear.sensor_adr
  exp = np.zeros((3, ns)); exp[0, adr[1]] = 1
  np.testing.assert_allclose(DsDq[0], exp, atol=1e-6)
  exp = np.zeros((3, ns)); exp[1, adr[0]] = 1
  np.testing.assert_allclose(DsDv[0], exp, atol=1e-6)
  exp = np.zeros((3, ns)); exp[0, adr[2] + 1] = 1; exp[1, adr[2] + 1] = 1
  np.testing.assert_allclose(DsDa[0], exp, atol=1e-6)
  e.close()


def _sensor_model():
  import sys
  import os
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_sensors_cpu import _all_model
  return _all_model()


def test_sensors_parity():
  """Every supported sensor type (mj_sensorPos/Vel/Acc, mj_subtreeVel,
  mj_rnePostConstraint), limit rows active, time/xfrc/actuator inputs set per instance."""
  m = _sensor_model()
  B = 256
  q, v, a = sample_states(m, B, first=11, margin=-0.3, resample_tendons=False)
  rng = np.random.default_rng(5)
  time = 0.01 * np.arange(B)[:, None]
  xfrc = np.zeros((B, m.nbody * 6))
  xfrc[:, 18:24] = rng.normal(size=(B, 6))
  af = rng.normal(size=(B, m.nu))
  qa = rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  # the run-time straight-line kernel with the sensor pass after it, and the generic kernel
  assert e.fast_kernel and e.fast_kernel.startswith("rt_")
  for name, val in (("time", time), ("xfrc_applied", xfrc), ("actuator_force", af),
                    ("qfrc_actuator", qa)):
    e.set_field(name, val)
  e.inverse(q, v, a)
  got = {f: e.field(f, 0, B) for f in ("sensordata", "qfrc_inverse", "subtree_linvel",
                                        "subtree_angmom", "cfrc_int", "cfrc_ext")}
  e.inverse(q, v, a, generic=True)
  o = Oracle(m)
  ref = {f: [] for f in ("sensordata", "qfrc_inverse", "subtree_linvel", "subtree_angmom",
                         "cfrc_int", "cfrc_ext")}
  for i in range(B):
    o.d.time = time[i, 0]
    o.d.xfrc_applied[:] = xfrc[i]
    o.d.actuator_force[:] = af[i]
    o.d.qfrc_actuator[:] = qa[i]
    o.inverse(q[i], v[i], a[i])
    for f in ref:
      ref[f].append(getattr(o.d, f).copy())
  for f, r in ref.items():
    assert_close(got[f], np.array(r), f + " (straight-line + sensor pass)")
    assert_close(e.field(f, 0, B), np.array(r), f + " (generic)")
  e.close()


def test_touch_sensor_parity():
  """Touch sensors (ray-zone tests on box, cylinder and sphere zones, flipped rays for the
  contacts' second body) over random resting states of a box and a ball on a plane, with
  every contact and constraint row of the instance, vs the oracle."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><worldbody><geom type="plane" size="2 2 1"/>
    <body name="box" pos="0 0 .1"><freejoint/><geom type="box" size=".2 .15 .1"/>
      <site name="zb" type="box" size=".25 .2 .12"/>
      <site name="zt" type="cylinder" size=".1 .05" pos="0 0 .1"/></body>
    <body name="ball" pos="0 0 .29"><freejoint/><geom size=".09"/>
      <site name="zs" type="sphere" size=".12"/></body></worldbody>
    <sensor><touch site="zb"/><touch site="zt"/><touch site="zs"/></sensor></mujoco>""")
  B = 2048
  rng = np.random.default_rng(12)
  q = np.tile(np.asarray(m.qpos0, dtype=float), (B, 1))
  q[:, 2] = 0.1 - 0.002 + 0.001 * rng.normal(size=B)
  q[:, 3:7] += 0.01 * rng.normal(size=(B, 4))
  q[:, 9] = 0.29 - 0.003 + 0.001 * rng.normal(size=B)
  v = 0.05 * rng.normal(size=(B, m.nv))
  a = rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    sd = e.field("sensordata", 0, B)
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  ref, refs = [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    refs.append(o.d.sensordata.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(sd, np.array(refs), "sensordata")
  assert (np.array(refs) > 0).all(axis=0).any() and (np.array(refs) > 0).any(axis=0).all()


def test_sensor_fd_parity():
  """mjd_inverseFD sensor derivatives (stage-skipping semantics) vs the oracle."""
  m = _sensor_model()
  q, v, a = sample_states(m, 6, first=40)
  e = engine.InverseEngine(m, capacity=6 * (3 * m.nv + 1))
  DfDq, DfDv, DfDa, _, (DsDq, DsDv, DsDa) = e.inverse_fd(q, v, a, sensors=True)
  o = Oracle(m)
  for i in range(6):
    o.set_state(q[i], v[i], a[i])
    rq, rv, ra, _, (sq, sv, sa) = o.inverse_fd(1e-6, sensors=True)
    for g, r in ((DfDq[i], rq), (DfDv[i], rv), (DfDa[i], ra), (DsDq[i], sq), (DsDv[i], sv),
                 (DsDa[i], sa)):
      np.testing.assert_allclose(g, r, rtol=1e-5, atol=1e-4)
    # entries the reference never recomputes are exactly zero
    stage = np.repeat(m.sensor_needstage, m.sensor_dim)
    assert (DsDa[i][:, stage < 3] == 0).all() and (DsDv[i][:, stage < 2] == 0).all()
  e.close()


def test_single_instance_dropin_inverse_test_driver(arm2, rng):
  """src/inverse/inverse_test.cpp with the GPU mj_inverseSkip(m, d, mjSTAGE_VEL, 1):
  forward states from the oracle harness, inverse through the single-instance drop-in."""
  o = Oracle(arm2)
  d = host.MjData(arm2)
  worst = 0
  for _ in range(int(1.0 / arm2.opt["timestep"])):
    o.d.qfrc_applied[:] = 0.4 * (rng.random(arm2.nv) - 0.5)
    o.d.xfrc_applied[:] = 0.8 * (rng.random(6 * arm2.nbody) - 0.5)
    assert o.forward() == 0
    expected = (o.d.qfrc_applied + o.d.qfrc_actuator).copy()
    o.xfrc_accumulate(expected)
    for f in [x.name for x in fields.DATA_FIELDS]:
      getattr(d, f)[:] = getattr(o.d, f)
    engine.mj_inverseSkip(arm2, d, engine.mjSTAGE_VEL, 1)
    worst = max(worst, np.linalg.norm(expected - d.qfrc_inverse))
    o.rk4()
  assert worst < 1e-6


def test_single_instance_mj_inverse(humanoid):
  q, v, a = sample_states(humanoid, 3, first=42)
  d = host.MjData(humanoid)
  o = Oracle(humanoid)
  for i in range(3):
    d.qpos[:], d.qvel[:], d.qacc[:] = q[i], v[i], a[i]
    engine.mj_inverse(humanoid, d)
    o.inverse(q[i], v[i], a[i])
    for f in OUTPUTS:
      if fields.DATA_FIELD[f].size(humanoid.sizes):
        assert_close(getattr(d, f)[None], getattr(o.d, f)[None], f)
    assert d.nefc == o.d.nefc


def test_device_tensor_io(humanoid, eng):
  torch = pytest.importorskip("torch")
  q, v, a = sample_states(humanoid, 2048, first=1234)
  dev = torch.device("cuda:0")
  tq, tv, ta = (torch.from_numpy(x).to(dev) for x in (q, v, a))
  out = torch.empty((2048, humanoid.nv), dtype=torch.float64, device=dev)
  torch.cuda.synchronize()
  eng.inverse(tq, tv, ta, out=out)
  torch.cuda.synchronize()
  ref = eng.inverse(q, v, a)
  np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_device_tensor_stream_order(humanoid):
  """Device-tensor calls are ordered with torch's current stream without any explicit
  synchronization: inputs produced by queued torch work on a side stream are read after it,
  and torch work queued after the call sees the outputs (engine._TorchOrder)."""
  torch = pytest.importorskip("torch")
  B = 4096
  q, v, a = sample_states(humanoid, B, first=777)
  ref = None
  e = engine.InverseEngine(humanoid, capacity=B)
  try:
    ref = e.inverse(q, v, a)
    dev = torch.device("cuda:0")
    side = torch.cuda.Stream(dev)
    hq, hv, ha = (torch.from_numpy(x).pin_memory() for x in (q, v, a))
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
      big = torch.randn(4096, 4096, device=dev, dtype=torch.float64)
      for _ in range(4):                 # keep the side stream busy before the inputs land
        big = big @ big * 1e-3
      tq = hq.to(dev, non_blocking=True) + 0 * big[0, 0]
      tv = hv.to(dev, non_blocking=True)
      ta = ha.to(dev, non_blocking=True)
      out = torch.full((B, humanoid.nv), float("nan"), dtype=torch.float64, device=dev)
      e.inverse(tq, tv, ta, out=out)
      res = (out * 1.0).to("cpu", non_blocking=False)
  finally:
    torch.cuda.synchronize()
    e.close()
  np.testing.assert_array_equal(res.numpy(), ref)


def test_fast_kernel_selected(eng):
  """The bundled humanoid runs the model-specialized straight-line kernel (codegen.py)."""
  assert eng.fast_kernel == "humanoid"


def test_fast_vs_generic_and_worklist(humanoid, eng):
  """Fast path (straight-line + work-list) vs the generic kernel on mixed states: every
  instance whose limits are active is recomputed through the work-list."""
  q, v, a = sample_states(humanoid, 2048, first=20000, margin=-0.02, resample_tendons=False)
  f_fast = eng.inverse(q, v, a)
  n_wl = eng.worklist_count()
  f_gen = eng.inverse(q, v, a, generic=True)
  _, nefc = oracle_batch(humanoid, q, v, a)
  assert n_wl == int((nefc > 0).sum()) > 0
  assert_close(f_fast, f_gen, "fast vs generic")
  ref, _ = oracle_batch(humanoid, q, v, a)
  assert_close(f_fast, ref["qfrc_inverse"], "fast vs oracle")


@pytest.fixture(scope="module")
def humanoid_contacts_eng(humanoid_contacts):
  e = engine.InverseEngine(humanoid_contacts, capacity=4096)
  yield e
  e.close()


@pytest.mark.parametrize("generic", [False, True])
def test_contacts_config4_parity(humanoid_contacts, humanoid_contacts_eng, generic):
  """Config 4: keyframe poses + noise, contacts on. Default dispatch: the
  generated kernels plus k_constraint; generic: k_inverse with the fused constraint rows.

  Counts, row types/ids and contact geom pairs bit-exact; fp64 outputs within 1e-10
  normwise relative."""
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
  from oracle.oracle import CON_DOUBLE, CON_INT
  m, e = humanoid_contacts, humanoid_contacts_eng
  assert e.fast_kernel == "humanoid_contact"
  B = 4096                              # config 4's batch
  q, v, a = sample_contact_states(m, B)
  f, st = e.inverse(q, v, a, status=True, generic=generic)
  assert (st == 0).all()
  o = Oracle(m)
  ncon_g = e.field_int("con_count", 0, B)[:, 0]
  efc_g = e.field_int("efc_count", 0, B)[:, 0]
  width = dict(CON_DOUBLE + CON_INT)
  gpu = {n: e.field(n, 0, B) for n in ("qfrc_constraint", "qfrc_bias", "qM", "con_dist",
                                         "con_pos", "efc_force", "efc_R")}
  gint = {n: e.field_int(n, 0, B) for n in ("con_geom", "efc_type", "efc_id", "efc_state")}
  ref_f, ref_c = [], []
  for i in range(B):
    ref_f.append(o.inverse(q[i], v[i], a[i]))
    ref_c.append(o.d.qfrc_constraint.copy())
    ncon, nefc = o.efc.ncon, o.efc.nefc
    assert ncon_g[i] == ncon and efc_g[i] == nefc, i
    np.testing.assert_array_equal(gint["con_geom"][i][:2 * ncon],
                                  o.contact_field("con_geom").ravel())
    for n in ("efc_type", "efc_id", "efc_state"):
      np.testing.assert_array_equal(gint[n][i][:nefc], o.efc_field(n), err_msg=f"{n} {i}")
    np.testing.assert_allclose(gpu["con_dist"][i][:ncon], o.contact_field("con_dist"),
                               rtol=0, atol=1e-12)
    np.testing.assert_allclose(gpu["con_pos"][i][:3 * ncon],
                               o.contact_field("con_pos").ravel(), rtol=0, atol=1e-12)
    fr = o.efc_field("efc_force")
    assert np.abs(gpu["efc_force"][i][:nefc] - fr).max(initial=0) <= \
        RTOL * max(1.0, np.abs(fr).max(initial=0))
  assert_close(f, np.array(ref_f), "qfrc_inverse")
  assert_close(gpu["qfrc_constraint"], np.array(ref_c), "qfrc_constraint")
  assert (ncon_g > 0).mean() > 0.5
  assert width["con_pos"] == 3


@pytest.mark.parametrize("generic", [False, True])
def test_invdiscrete_euler_parity(generic):
  """mjENBL_INVDISCRETE (Euler, implicit damping) on the device, through the run-time
  straight-line kernel with the discrete pass (csrc/post_pass.h) and through the generic
  kernel: matches the oracle, and qacc is restored."""
  m = models.load("humanoid", disable_contact=True)
  m.opt["enableflags"] |= 1 << 3
  B = 512
  q, v, a = sample_states(m, B, first=100)
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None and e.fast_kernel.startswith("rt_")
    f, st = e.inverse(q, v, a, status=True, generic=generic)
    assert (st == 0).all()
    np.testing.assert_array_equal(e.field("qacc", 0, B), a)       # restored
  finally:
    e.close()
  ref, _ = oracle_batch(m, q, v, a)
  assert_close(f, ref["qfrc_inverse"], "qfrc_inverse (INVDISCRETE)")


def test_forward_parity_and_fwdinv_identity(humanoid):
  """Batched constraint-free mj_forward on the device vs the oracle, then the fwd/inv
  identity entirely on the device (mj_compareFwdInv, engine_inverse.c:275-316): inverse
  dynamics of forward's qacc returns qfrc_applied + qfrc_actuator + J'xfrc_applied."""
  m = humanoid
  B = 1024
  q, v, _ = sample_states(m, B, first=300)
  rng = np.random.default_rng(7)
  ctrl = rng.uniform(-1.2, 1.2, (B, m.nu))
  qa = rng.normal(size=(B, m.nv))
  xa = 0.3 * rng.normal(size=(B, m.nbody, 6))
  e = engine.InverseEngine(m, capacity=B)
  try:
    acc, st = e.forward(q, v, ctrl, qfrc_applied=qa, xfrc_applied=xa, status=True)
    assert (st == 0).all()
    smooth = e.field("qfrc_smooth", 0, B)
    f = e.inverse(q, v, acc)
    passive, bias = e.field("qfrc_passive", 0, B), e.field("qfrc_bias", 0, B)
  finally:
    e.close()
  o = Oracle(m)
  ref = np.zeros((B, m.nv))
  for i in range(B):
    o.d.ctrl[:] = ctrl[i]
    o.d.qfrc_applied[:] = qa[i]
    o.d.xfrc_applied[:] = xa[i].ravel()
    o.set_state(q[i], v[i])
    o.forward()
    ref[i] = o.d.qacc
  assert_close(acc, ref, "forward qacc")
  expected = smooth - passive + bias          # qfrc_applied + qfrc_actuator + J'xfrc
  assert_close(f, expected, "fwd/inv identity")


def test_invdiscrete_implicitfast_parity():
  """INVDISCRETE with implicitfast (qDeriv from actuators, dof and tendon damping) on the
  device vs the oracle; ctrl enters through the mirror."""
  import importlib.util, os
  spec = importlib.util.spec_from_file_location(
      "tinv", os.path.join(os.path.dirname(__file__), "test_invdiscrete_cpu.py"))
  tinv = importlib.util.module_from_spec(spec)
  spec.loader.exec_module(tinv)
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(tinv._ARM)
  m.opt["enableflags"] |= 1 << 3
  B = 256
  rng = np.random.default_rng(8)
  q, v, a = rng.normal(size=(B, 3)), rng.normal(size=(B, 3)), rng.normal(size=(B, 3))
  ctrl = rng.uniform(-1, 1, (B, m.nu))
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None
    e.set_field("ctrl", ctrl)
    f, st = e.inverse(q, v, a, status=True)
    assert (st == 0).all()
    g = e.inverse(q, v, a, generic=True)
  finally:
    e.close()
  o = Oracle(m)
  ref = []
  for i in range(B):
    o.d.ctrl[:] = ctrl[i]
    ref.append(o.inverse(q[i], v[i], a[i]))
  assert_close(f, np.array(ref), "qfrc_inverse (implicitfast INVDISCRETE)")
  assert_close(g, np.array(ref), "qfrc_inverse (implicitfast INVDISCRETE, generic)")


def test_invdiscrete_contacts_sensors_parity():
  """INVDISCRETE (implicitfast) with contacts, a spatial tendon and acceleration sensors on
  the straight-line path: tendon pass, discrete pass, unfused constraint kernel, sensor pass
  on the discrete qacc, qacc restored; qfrc_inverse and sensordata vs the oracle."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_codegen_cpu import MIXED_TENDONS
  from mujoco_inversedynamicstest_amd import mjcf
  xml = MIXED_TENDONS.replace('<option density="1.1" viscosity=".2"/>',
                              '<option timestep=".01" integrator="implicitfast">'
                              '<flag invdiscrete="enable"/></option>')
  xml = xml.replace('<tendonpos tendon="fx"/>', '<tendonpos tendon="fx"/>'
                    '<accelerometer site="s1"/><framelinacc objtype="site" objname="s2"/>')
  m = mjcf.load_xml_string(xml)
  B = 1024
  q, v, a = sample_states(m, B, first=7, margin=-0.1)
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None
    f, st = e.inverse(q, v, a, status=True)
    sd = e.field("sensordata", 0, B)
    np.testing.assert_array_equal(e.field("qacc", 0, B), a)       # restored
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  ref, rs = [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    rs.append(o.d.sensordata.copy())
  assert_close(f, np.array(ref), "qfrc_inverse (INVDISCRETE, contacts)")
  assert_close(sd, np.array(rs), "sensordata (INVDISCRETE)")


@pytest.mark.parametrize("name,generic", [("humanoid", False), ("humanoid", True),
                                          ("inertia", False), ("inertia", True)])
def test_invdiscrete_implicit_parity(name, generic):
  """INVDISCRETE with the implicit integrator (mjd_rne_vel on the B/D sparsity, qLU product)
  on the device vs the oracle, straight-line + discrete pass and generic; the inertia model
  covers free and ball joints."""
  m = models.load(name, disable_contact=True)
  m.opt["enableflags"] |= 1 << 3
  m.opt["integrator"] = 2
  B = 512
  q, v, a = sample_states(m, B, first=400)
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None
    f, st = e.inverse(q, v, a, status=True, generic=generic)
    assert (st == 0).all()
    np.testing.assert_array_equal(e.field("qacc", 0, B), a)       # restored
  finally:
    e.close()
  ref, _ = oracle_batch(m, q, v, a)
  assert_close(f, ref["qfrc_inverse"], "qfrc_inverse (implicit INVDISCRETE)")


def test_energy_parity():
  """mjENBL_ENERGY (mj_energyPos/Vel) on the device: energy in the mirror vs the oracle."""
  m = models.load("humanoid", disable_contact=True)
  m.opt["enableflags"] |= 1 << 1
  B = 512
  q, v, a = sample_states(m, B, first=500)
  e = engine.InverseEngine(m, capacity=B)
  try:
    # the humanoid with ENERGY has its own signature: a run-time straight-line kernel, the
    # energy terms in the pass after it; then the generic kernel
    assert e.fast_kernel and e.fast_kernel.startswith("rt_")
    f = e.inverse(q, v, a)
    en = e.field("energy", 0, B)
    g = e.inverse(q, v, a, generic=True)
    eg = e.field("energy", 0, B)
  finally:
    e.close()
  o = Oracle(m)
  ref_f, ref_e = [], []
  for i in range(B):
    ref_f.append(o.inverse(q[i], v[i], a[i]))
    ref_e.append(o.d.energy)
  assert_close(f, np.array(ref_f), "qfrc_inverse (ENERGY)")
  assert_close(en, np.array(ref_e), "energy")
  assert_close(g, np.array(ref_f), "qfrc_inverse (ENERGY, generic)")
  assert_close(eg, np.array(ref_e), "energy (generic)")


def test_single_instance_sensors_dropin():
  """mj_inverse(m, d) drop-in with sensors: sensordata and the on-demand mjData fields
  (subtree_linvel/angmom, cacc, cfrc_int/ext) come back into d; skipstage keeps the skipped
  stages' sensor values (engine_inverse.c:203-242)."""
  m = _sensor_model()
  q, v, a = sample_states(m, 3, first=7, margin=-0.3, resample_tendons=False)
  d = host.MjData(m)
  o = Oracle(m)
  for dd in (d, o.d):
    dd.time = 1.5
    dd.xfrc_applied[18:24] = [0.1, -0.2, 0.3, 0.01, 0.02, -0.03]
    dd.actuator_force[:] = [0.4, -0.5]
  d.qpos[:], d.qvel[:], d.qacc[:] = q[0], v[0], a[0]
  engine.mj_inverse(m, d)
  o.inverse(q[0], v[0], a[0])
  for f in ("sensordata", "subtree_linvel", "subtree_angmom", "cacc", "cfrc_int",
            "cfrc_ext", "qfrc_inverse"):
    assert_close(getattr(d, f)[None], getattr(o.d, f)[None], f)
  d.qacc[:] = a[1]
  engine.mj_inverseSkip(m, d, engine.mjSTAGE_VEL, 0)
  o.inverse(qacc=a[1], skipstage=2)
  assert_close(d.sensordata[None], o.d.sensordata[None], "sensordata (skip VEL)")


@pytest.mark.parametrize("name", ["weld", "connect", "equality_site", "equality_compare"])
def test_equality_parity(name):
  """Equality constraints (connect, weld; body and site semantics; force/torque sensors
  through mj_rnePostConstraint's equality branch) on the device vs the oracle. The test
  models' viscosity is zeroed (fluid forces are outside the subset)."""
  m = models.load(name)
  m.opt["viscosity"] = 0.0
  B = 512
  q, v, a = sample_states(m, B, first=17)
  e = engine.InverseEngine(m, capacity=B)
  f, st = e.inverse(q, v, a, status=True)
  assert (st == 0).all()
  efc_g = e.field_int("efc_count", 0, B)
  gforce = e.field("efc_force", 0, B)
  gint = {n: e.field_int(n, 0, B) for n in ("efc_type", "efc_id", "efc_state")}
  o = Oracle(m)
  ref = {k: [] for k in ("qfrc_inverse", "qfrc_constraint", "sensordata")}
  for i in range(B):
    o.inverse(q[i], v[i], a[i])
    for k in ref:
      ref[k].append(getattr(o.d, k).copy())
    assert efc_g[i, 0] == o.efc.nefc and efc_g[i, 1] == o.efc.ne
    for n in gint:
      np.testing.assert_array_equal(gint[n][i][:o.efc.nefc], o.efc_field(n))
    fr = o.efc_field("efc_force")
    assert np.abs(gforce[i][:o.efc.nefc] - fr).max() <= RTOL * max(1.0, np.abs(fr).max())
  assert_close(f, np.array(ref["qfrc_inverse"]), "qfrc_inverse")
  assert_close(e.field("qfrc_constraint", 0, B), np.array(ref["qfrc_constraint"]),
               "qfrc_constraint")
  if m.nsensordata:
    assert_close(e.field("sensordata", 0, B), np.array(ref["sensordata"]), "sensordata")
  e.close()


def test_plane_box_cylinder_contacts_parity():
  """mjc_PlaneBox / mjc_PlaneCylinder contacts (up to 4 per pair) on the device."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><default><geom contype="1" conaffinity="2"/></default>
    <worldbody><geom type="plane" size="3 3 .1" contype="2" conaffinity="1"/>
    <body pos="0 0 .1"><freejoint/><geom type="box" size=".2 .1 .05" condim="1"/></body>
    <body pos=".8 0 .1"><freejoint/><geom type="cylinder" size=".1 .15" condim="6"/></body>
    <body pos="-.8 0 .1"><freejoint/><geom type="box" size=".1 .1 .1"/>
      <body pos="0 0 .2"><joint axis="1 0 0"/><geom type="cylinder" size=".05 .1"
        pos="0 0 .1"/></body></body>
  </worldbody></mujoco>""")
  B = 1024
  rng = np.random.default_rng(11)
  q = np.tile(m.qpos0, (B, 1))
  for b in range(3):
    q[:, 7 * b + 2] = 0.05 + 0.1 * rng.random(B)
    qq = rng.normal(size=(B, 4))
    q[:, 7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  q[:, 21] = rng.normal(size=B)
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  f, st = e.inverse(q, v, a, status=True)
  assert (st == 0).all()
  ncon_g = e.field_int("con_count", 0, B)[:, 0]
  o = Oracle(m)
  ref = []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    assert ncon_g[i] == o.efc.ncon
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert ncon_g.sum() > B
  e.close()


def test_sphere_cylinder_contacts_parity():
  """mjc_SphereCylinder contacts (side, caps, rims, deep penetration) on the device."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="cylinder" size=".12 .2"/></body>
    <body pos=".3 0 .5"><freejoint/><geom size=".06" condim="1"/></body>
    <body pos="-.3 0 .5"><freejoint/><geom size=".08" condim="4"/></body>
    </worldbody></mujoco>""")
  B = 2048
  rng = np.random.default_rng(21)
  q = np.tile(m.qpos0, (B, 1))
  qq = rng.normal(size=(B, 4))
  q[:, 3:7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  for b in (1, 2):
    q[:, 7 * b:7 * b + 3] = q[:, :3] + rng.uniform(-0.25, 0.25, size=(B, 3))
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    ncon_g = e.field_int("con_count", 0, B)[:, 0]
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  ref = []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    assert ncon_g[i] == o.efc.ncon
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert ncon_g.sum() > B // 4


def test_box_box_contacts_parity():
  """mjc_BoxBox contacts (face and edge-edge separating axes, up to 24 raw contacts per pair,
  bad and repeated ones removed) on the device: the cooperative kernel (positions staged in
  LDS) and the generic pipeline (positions in the contact list's free tail)."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="box" size=".2 .15 .1"/></body>
    <body pos=".4 0 .5"><freejoint/><geom type="box" size=".1 .12 .08" condim="1"/></body>
    <body pos="-.4 0 .5"><freejoint/><geom type="box" size=".25 .05 .06" margin=".01"/></body>
    </worldbody></mujoco>""")
  B = 4096
  rng = np.random.default_rng(41)
  q = np.tile(m.qpos0, (B, 1))
  for b in range(3):
    qq = rng.normal(size=(B, 4))
    q[:, 7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  for b in (1, 2):
    q[:, 7 * b:7 * b + 3] = q[:, :3] + rng.uniform(-0.3, 0.3, size=(B, 3))
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    ncon_g = e.field_int("con_count", 0, B)[:, 0]
    pos_g = e.field("con_pos", 0, B)
    g = e.inverse(q, v, a, generic=True)
    ncon_gen = e.field_int("con_count", 0, B)[:, 0]
  finally:
    e.close()
  assert (st == 0).all()
  np.testing.assert_array_equal(ncon_gen, ncon_g)
  o = Oracle(m)
  ref = []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    assert ncon_g[i] == o.efc.ncon
    if i % 16 == 0 and ncon_g[i]:
      rp = o.contact_field("con_pos").reshape(-1)
      assert np.abs(pos_g[i][:rp.size] - rp).max() <= 1e-10 * max(1.0, np.abs(rp).max())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(g, np.array(ref), "qfrc_inverse (generic)")
  assert ncon_g.sum() > B // 4


def test_capsule_box_contacts_parity():
  """mjc_CapsuleBox contacts (face, edge and corner closest; one or two per pair) on the
  device."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="box" size=".2 .15 .1"/></body>
    <body pos=".4 0 .5"><freejoint/><geom type="capsule" size=".05 .15" condim="1"/></body>
    <body pos="-.4 0 .5"><freejoint/><geom type="capsule" size=".03 .25"/></body>
    </worldbody></mujoco>""")
  B = 4096
  rng = np.random.default_rng(31)
  q = np.tile(m.qpos0, (B, 1))
  for b in range(3):
    qq = rng.normal(size=(B, 4))
    q[:, 7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  for b in (1, 2):
    q[:, 7 * b:7 * b + 3] = q[:, :3] + rng.uniform(-0.3, 0.3, size=(B, 3))
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    ncon_g = e.field_int("con_count", 0, B)[:, 0]
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  ref = []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    assert ncon_g[i] == o.efc.ncon
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert ncon_g.sum() > B // 8


def test_mocap_parity():
  """Mocap bodies: per-instance mocap_pos/mocap_quat mirror inputs drive the kinematics."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_mocap_cpu import MOCAP
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(MOCAP)
  B = 256
  q, v, a = sample_states(m, B, first=5)
  rng = np.random.default_rng(8)
  mp, mq = rng.normal(size=(B, 3)), rng.normal(size=(B, 4))
  e = engine.InverseEngine(m, capacity=B)
  # the run-time straight-line kernel reads the mocap inputs; then the generic kernel
  assert e.fast_kernel and e.fast_kernel.startswith("rt_")
  e.set_field("mocap_pos", mp)
  e.set_field("mocap_quat", mq)
  f = e.inverse(q, v, a)
  sf = e.field("sensordata", 0, B)
  g = e.inverse(q, v, a, generic=True)
  sg = e.field("sensordata", 0, B)
  o = Oracle(m)
  ref, sref = [], []
  for i in range(B):
    o.d.mocap_pos[:], o.d.mocap_quat[:] = mp[i], mq[i]
    ref.append(o.inverse(q[i], v[i], a[i]))
    sref.append(o.d.sensordata.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(sf, np.array(sref), "sensordata")
  assert_close(g, np.array(ref), "qfrc_inverse (generic)")
  assert_close(sg, np.array(sref), "sensordata (generic)")
  e.close()


@pytest.mark.parametrize("path", ["generic", "straight-line"])
def test_transmission_parity(path):
  """Ball/free-joint, fixed-tendon and site transmissions: actuator_length/moment on the
  device, through the generic kernel and through the run-time straight-line kernel (the site
  transmission in its post pass)."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_transmission_cpu import XML
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(XML)
  B = 256
  q, v, a = sample_states(m, B, first=5)
  e = engine.InverseEngine(m, capacity=B)
  assert e.fast_kernel is not None
  f = e.inverse(q, v, a, generic=(path == "generic"))
  o = Oracle(m)
  ref, lref, mref = [], [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    lref.append(o.d.actuator_length.copy())
    mref.append(o.d.actuator_moment.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(e.field("actuator_length", 0, B), np.array(lref), "actuator_length")
  assert_close(e.field("actuator_moment", 0, B), np.array(mref), "actuator_moment")
  e.close()


def test_site_refsite_transmission_parity():
  """Site transmissions relative to a reference site (translation, rotation, both; refsite
  in the world, on a shared ancestor and on a sibling branch) on the device."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_transmission_cpu import REFSITE
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(REFSITE)
  B = 1024
  rng = np.random.default_rng(3)
  q = rng.uniform(-1, 1, (B, m.nq))
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f = e.inverse(q, v, a)
    lg = e.field("actuator_length", 0, B)
    mg = e.field("actuator_moment", 0, B)
  finally:
    e.close()
  o = Oracle(m)
  ref, lref, mref = [], [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    lref.append(o.d.actuator_length.copy())
    mref.append(o.d.actuator_moment.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(lg, np.array(lref), "actuator_length")
  assert_close(mg, np.array(mref), "actuator_moment")


@pytest.mark.parametrize("cone,condim", [("pyramidal", 3), ("elliptic", 6), ("pyramidal", 1)])
def test_adhesion_transmission_parity(cone, condim):
  """Body (adhesion) transmissions: the moment from the body's contact rows and in-gap
  contacts, on the device."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_transmission_cpu import _adhesion
  m = _adhesion(cone, condim, 0.01, 0.005, 0.1)
  B = 1024
  rng = np.random.default_rng(19)
  q = np.tile(m.qpos0, (B, 1))
  q[:, 2] = 0.1 + 0.03 * rng.normal(size=B)
  qq = np.array([1, 0, 0, 0]) + 0.15 * rng.normal(size=(B, 4))
  q[:, 3:7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  q[:, 7:9] = q[:, 0:2] + rng.uniform(-0.4, 0.4, (B, 2))
  q[:, 9] = 0.1 + 0.05 * rng.normal(size=B)
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    mg = e.field("actuator_moment", 0, B)
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  ref, mref = [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    mref.append(o.d.actuator_moment.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(mg, np.array(mref), "actuator_moment")
  assert np.abs(np.array(mref)).max() > 0.5


def test_slider_crank_parity():
  """BASELINE.json config 1 model: slider-crank transmissions and its capsule-cylinder pair
  (mjc_Convex on native GJK/EPA): every uniform state is computed, none flagged."""
  m = models.load("slider_crank")
  B = 256
  rng = np.random.default_rng(11)
  q, v, a = rng.uniform(-np.pi, np.pi, (B, 3)), rng.normal(size=(B, 3)), rng.normal(size=(B, 3))
  e = engine.InverseEngine(m, capacity=B)
  f, st = e.inverse(q, v, a, status=True)
  o = Oracle(m)
  ref, lref, mref, oref = [], [], [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    oref.append(o.d.status)
    lref.append(o.d.actuator_length.copy())
    mref.append(o.d.actuator_moment.copy())
  np.testing.assert_array_equal(st, oref)
  assert np.count_nonzero(st) == 0
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(e.field("actuator_length", 0, B), np.array(lref), "actuator_length")
  assert_close(e.field("actuator_moment", 0, B), np.array(mref), "actuator_moment")
  e.close()


def test_fluid_parity():
  """Inertia-box fluid forces (viscosity and density, with wind) on the device."""
  m = models.load("equality_site")
  m.opt["density"] = 1.3
  m.opt["wind"] = [0.2, -0.1, 0.3]
  B = 512
  q, v, a = sample_states(m, B, first=21)
  e = engine.InverseEngine(m, capacity=B)
  assert e.fast_kernel is not None        # straight-line kernel + the fluid pass
  f = e.inverse(q, v, a)
  o = Oracle(m)
  ref, fl = [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    fl.append(o.d.qfrc_fluid.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(e.field("qfrc_fluid", 0, B), np.array(fl), "qfrc_fluid")
  e.close()


def test_ellipsoid_fluid_parity():
  """The ellipsoid fluid model (added mass, Magnus and Kutta lift, viscous drag; density,
  viscosity and wind) on box/capsule/cylinder/ellipsoid geoms next to an inertia-box body."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><option density="1.2" viscosity=".3" wind=".4 -.2 .1">
    <flag contact="disable"/></option><worldbody>
    <body pos="0 0 1"><freejoint/><geom type="box" size=".2 .1 .05" fluidshape="ellipsoid"
      fluidcoef=".4 .3 1.2 .9 1.1"/><geom type="capsule" size=".05 .1" pos=".2 0 0"
      fluidshape="ellipsoid"/>
      <body pos="0 .3 0"><joint axis="1 0 0"/><geom type="cylinder" size=".05 .2"
        fluidshape="ellipsoid"/>
        <body pos="0 .3 0"><joint axis="0 1 1"/><geom type="ellipsoid" size=".1 .05 .2"
          fluidshape="ellipsoid"/></body></body></body>
    <body pos="1 0 1"><freejoint/><geom type="box" size=".1 .2 .3"/></body>
    </worldbody></mujoco>""")
  B = 1024
  q, v, a = sample_states(m, B, first=3)
  v = 2 * v
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None      # straight-line kernel + the fluid pass
    f = e.inverse(q, v, a)
    fl_gpu = e.field("qfrc_fluid", 0, B)
    fg = e.inverse(q, v, a, generic=True)
  finally:
    e.close()
  assert_close(f, fg, "straight-line vs generic qfrc_inverse")
  o = Oracle(m)
  ref, fl = [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    fl.append(o.d.qfrc_fluid.copy())
  assert np.abs(np.array(fl)).max() > 1e-2
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(fl_gpu, np.array(fl), "qfrc_fluid")


def test_rangefinder_parity():
  """Rangefinders on moving bodies among every primitive type (one geom half transparent, one
  invisible, one sensor with a cutoff): sensordata on the device vs the oracle."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_rangefinder_cpu import SCENE
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(SCENE)
  B = 1024
  rng = np.random.default_rng(8)
  q = np.tile(m.qpos0, (B, 1))
  q[:, :3] = rng.uniform(-1, 1, (B, 3)) + [0, 0, 1]
  qq = rng.normal(size=(B, 4))
  q[:, 3:7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  q[:, 7:] = rng.uniform(-2, 2, (B, 2))
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f = e.inverse(q, v, a)
    sd = e.field("sensordata", 0, B)
  finally:
    e.close()
  o = Oracle(m)
  ref, rsd = [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    rsd.append(o.d.sensordata.copy())
  rsd = np.array(rsd)
  assert (rsd >= 0).sum() > 1000 and (rsd < 0).sum() > 200
  np.testing.assert_array_equal(sd < 0, rsd < 0)        # hit or miss, exactly
  assert_close(sd, rsd, "sensordata")
  assert_close(f, np.array(ref), "qfrc_inverse")


def test_camprojection_parity():
  """Camera projections from cameras on a free body and a hinge body (fovy and pinhole
  intrinsics) on the device vs the oracle."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_camprojection_cpu import MOVING
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(MOVING)
  B = 1024
  rng = np.random.default_rng(12)
  q = np.tile(m.qpos0, (B, 1))
  q[:, :3] += rng.uniform(-.3, .3, (B, 3))
  qq = rng.normal(size=(B, 4))
  q[:, 3:7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  q[:, 7] = rng.uniform(-3, 3, B)
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    e.inverse(q, v, a)
    sd = e.field("sensordata", 0, B)
  finally:
    e.close()
  o = Oracle(m)
  rsd = []
  for i in range(B):
    o.inverse(q[i], v[i], a[i])
    rsd.append(o.d.sensordata.copy())
  assert_close(sd, np.array(rsd), "sensordata")


def test_geom_distance_parity():
  """Geom-distance sensors (distance, normal, fromto; primitive pairs, the native solver's
  pairs and a body-level sensor) on the device vs the oracle. The native solver's pairs are
  iterative (test_convex_gpu.py explains their conditioning): distances are held to
  10 ccd_tolerance, everything else to the north-star bar."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_geomdist_cpu import SCENE
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(SCENE)
  B = 1024
  rng = np.random.default_rng(14)
  q = np.tile(m.qpos0, (B, 1))
  q[:, :3] = rng.uniform(-.6, .6, (B, 3)) + [0, 0, 1]
  qq = rng.normal(size=(B, 4))
  q[:, 3:7] = qq / np.linalg.norm(qq, axis=1, keepdims=True)
  q[:, 7] = rng.uniform(-3, 3, B)
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    sd = e.field("sensordata", 0, B)
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  rsd = []
  for i in range(B):
    o.inverse(q[i], v[i], a[i])
    rsd.append(o.d.sensordata.copy())
  rsd = np.array(rsd)
  err = np.abs(sd - rsd).max()
  print(f"geom distance sensors: max abs difference {err:.2e}")
  assert err <= 10 * m.opt["ccd_tolerance"]
  # the primitive pairs (ball-floor: sensor 0; blk-floor: the last) to the north-star bar
  for k in (0, m.nsensordata - 1):
    assert_close(sd[:, k:k + 1], rsd[:, k:k + 1], f"sensordata[{k}]")


def test_elliptic_cone_parity():
  """Elliptic friction cones (classic constraint passes) on the device: humanoid config-4
  states with cone="elliptic"."""
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
  m = models.load("humanoid")
  m.opt["cone"] = 1
  B = 512
  q, v, a = sample_contact_states(m, B, first=3)
  e = engine.InverseEngine(m, capacity=B)
  f, st = e.inverse(q, v, a, status=True)
  assert (st == 0).all()
  nefc_g = e.field_int("efc_count", 0, B)[:, 0]
  o = Oracle(m)
  ref = []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    assert nefc_g[i] == o.efc.nefc
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert nefc_g.sum() > 0
  e.close()


@pytest.mark.parametrize("lanes", ["0", "16"])
def test_constraint_coop_lanes(humanoid_contacts, lanes, monkeypatch):
  """The cooperative constraint kernel (16 lanes per instance: sphere filter and collision
  pairs, rows and J'force split over the group) against the one-lane kernel and the oracle,
  config-4 states with limits and contacts: counts, row types/ids and contact pairs exact."""
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
  m = humanoid_contacts
  monkeypatch.setenv("MJHIP_COOP_LANES", lanes)
  B = 2048
  q, v, a = sample_contact_states(m, B, first=10000)
  e = engine.InverseEngine(m, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    ints = {n: e.field_int(n, 0, B) for n in ("con_count", "efc_count", "con_geom", "efc_type",
                                              "efc_id", "efc_state", "con_efc_address")}
    force = e.field("efc_force", 0, B)
    qc = e.field("qfrc_constraint", 0, B)
  finally:
    e.close()
  assert (st == 0).all()
  o = Oracle(m)
  ref, refc = [], []
  for i in range(0, B, 4):
    ref.append(o.inverse(q[i], v[i], a[i]))
    refc.append(o.d.qfrc_constraint.copy())
    ncon, nefc = o.efc.ncon, o.efc.nefc
    assert ints["con_count"][i, 0] == ncon and ints["efc_count"][i, 0] == nefc
    np.testing.assert_array_equal(ints["con_geom"][i][:2 * ncon],
                                  o.contact_field("con_geom").ravel())
    np.testing.assert_array_equal(ints["con_efc_address"][i][:ncon],
                                  o.contact_field("con_efc_address"))
    for n in ("efc_type", "efc_id", "efc_state"):
      np.testing.assert_array_equal(ints[n][i][:nefc], o.efc_field(n))
    fr = o.efc_field("efc_force")
    assert np.abs(force[i][:nefc] - fr).max(initial=0) <= RTOL * max(1.0, np.abs(fr).max(initial=0))
  assert_close(f[::4], np.array(ref), "qfrc_inverse")
  assert_close(qc[::4], np.array(refc), "qfrc_constraint")
  assert (ints["con_count"][:, 0] > 0).mean() > 0.5


def _bad_inputs(m, B, first):
  q, v, a = sample_states(m, B, first=first)
  q[3, 5] = np.nan                      # BADQPOS (and a NaN pivot: INERTIA)
  v[5, 2] = 2e10                        # BADQVEL
  a[7, 0] = np.inf                      # BADQACC
  a[9, 1] = -1e11
  return q, v, a


@pytest.mark.parametrize("generic", [False, True])
def test_status_bits_bad_inputs(humanoid, eng, generic):
  """mj_checkPos/Vel/Acc (engine_forward.c:53-102) and the INERTIA pivot test as per-instance
  status bits, identical to the oracle's, on the straight-line and the generic kernels; good
  instances stay at 0 and nothing aborts the batch."""
  q, v, a = _bad_inputs(humanoid, 64, 50)
  _, st = eng.inverse(q, v, a, status=True, generic=generic)
  o = Oracle(humanoid)
  ref = []
  for i in range(64):
    o.inverse(q[i], v[i], a[i])
    ref.append(o.d.status)
  np.testing.assert_array_equal(st, ref)
  assert st[3] & 1 and st[3] & 8 and st[5] == 2 and st[7] == 4 and st[9] == 4
  assert (np.delete(st, [3, 5, 7, 9]) == 0).all()


def test_config3_full_batch_one_gpu(humanoid):
  """Config 3's whole global batch (262,144 humanoid states) on one GPU: 8 contiguous
  32,768-instance shards (one per rank of the 8-GPU run) equal the single batch bit for bit,
  the affine-in-qacc identity holds at full size, and an oracle subsample matches."""
  B, world = 262144, 8
  from mujoco_inversedynamicstest_amd import parallel
  q, v, a = sample_states(humanoid, B)
  e = engine.InverseEngine(humanoid, capacity=B)
  try:
    f, st = e.inverse(q, v, a, status=True)
    assert (st == 0).all()
    for r in range(world):
      first, count = parallel.shard(B, world, r)
      fr = e.inverse(q[first:first + count], v[first:first + count], a[first:first + count])
      np.testing.assert_array_equal(fr, f[first:first + count])
    sub = np.arange(0, B, B // 1024)
    f0 = e.inverse(q[sub], v[sub], np.zeros_like(a[sub]))
    qM = e.field("qM", 0, len(sub))
  finally:
    e.close()
  nv = humanoid.nv
  Mx = np.zeros((len(sub), nv))
  adr = 0
  for i in range(nv):
    j = i
    while j >= 0:
      Mx[:, i] += qM[:, adr] * a[sub, j]
      if j != i:
        Mx[:, j] += qM[:, adr] * a[sub, i]
      j = humanoid.dof_parentid[j]
      adr += 1
  scale = np.maximum(1.0, np.abs(f[sub]).max(axis=1))
  assert (np.abs((f[sub] - f0) - Mx).max(axis=1) / scale).max() < 1e-9
  ref, _ = oracle_batch(humanoid, q[sub[:256]], v[sub[:256]], a[sub[:256]])
  assert_close(f[sub[:256]], ref["qfrc_inverse"], "qfrc_inverse (config 3 subsample)")


@pytest.mark.parametrize("which,path", [("sites", "fast"), ("wrap", "fast"),
                                        ("sites", "onelane"), ("wrap", "onelane"),
                                        ("sites", "generic"), ("wrap", "generic")])
def test_spatial_tendon_parity(which, path, monkeypatch):
  """Spatial tendons through sites and pulleys, and wrapping around spheres and cylinders
  (with side sites outside and inside the wrap geom, and without one): lengths, Jacobians,
  limit rows, spring-damper, tendon actuators on the device vs the oracle, through the
  run-time straight-line kernel with the tendon pass (csrc/post_pass.h) and the cooperative
  or the one-lane constraint kernel, and through the generic kernel."""
  if path == "onelane":
    monkeypatch.setenv("MJHIP_COOP_LANES", "0")
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  import test_tendon_cpu as T
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(T.ARM if which == "sites" else T.WRAP)
  st = (T._states if which == "sites" else T._wrap_states)(m, 2048, 5)
  q = np.array([x[0] for x in st])
  v = np.array([x[1] for x in st])
  a = np.array([x[2] for x in st])
  e = engine.InverseEngine(m, capacity=len(q))
  try:
    assert e.fast_kernel is not None
    f, status = e.inverse(q, v, a, status=True, generic=path == "generic")
    vel = e.field("ten_velocity", 0, len(q))
    sd = e.field("qfrc_passive", 0, len(q))
    am = e.field("actuator_moment", 0, len(q))
    tl = e.field("ten_length", 0, len(q))
    tj = e.field("ten_J", 0, len(q))
    nefc = e.field_int("efc_count", 0, len(q))[:, 0]
  finally:
    e.close()
  assert (status == 0).all()
  o = Oracle(m)
  ref, rl, rj, rv, rp, rm = [], [], [], [], [], []
  for i in range(len(q)):
    ref.append(o.inverse(q[i], v[i], a[i]))
    rl.append(o.d.ten_length.copy())
    rj.append(o.d.ten_J.copy())
    rv.append(o.d.ten_velocity.copy())
    rp.append(o.d.qfrc_passive.copy())
    rm.append(o.d.actuator_moment.copy())
    assert nefc[i] == o.d.nefc
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(tl, np.array(rl), "ten_length")
  assert_close(tj, np.array(rj), "ten_J")
  assert_close(vel, np.array(rv), "ten_velocity")
  assert_close(sd, np.array(rp), "qfrc_passive")
  assert_close(am, np.array(rm), "actuator_moment")
  assert nefc.sum() > 0


def test_spatial_tendon_mixed_parity():
  """A fixed and a spatial tendon (limits, friction loss, spring-damper, transmissions,
  tendon and actuator sensors) with contacts, fluid and gravity compensation: the run-time
  straight-line kernel, the tendon pass and the cooperative constraint kernel vs the oracle
  on qfrc_inverse, qfrc_passive and the sensors."""
  import os
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  from test_codegen_cpu import MIXED_TENDONS
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(MIXED_TENDONS)
  B = 2048
  q, v, a = sample_states(m, B, first=3, margin=-0.1)
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None
    f, status = e.inverse(q, v, a, status=True)
    pas = e.field("qfrc_passive", 0, B)
    sd = e.field("sensordata", 0, B)
    ncon = e.field_int("efc_count", 0, B)
  finally:
    e.close()
  assert (status == 0).all()
  o = Oracle(m)
  ref, rp, rs = [], [], []
  for i in range(B):
    ref.append(o.inverse(q[i], v[i], a[i]))
    rp.append(o.d.qfrc_passive.copy())
    rs.append(o.d.sensordata.copy())
  assert_close(f, np.array(ref), "qfrc_inverse")
  assert_close(pas, np.array(rp), "qfrc_passive")
  assert_close(sd, np.array(rs), "sensordata")
  assert ncon[:, 0].sum() > 0


@pytest.mark.parametrize("integ", ["Euler", "implicit", "implicitfast"])
def test_invdiscrete_trn_after_parity(integ):
  """INVDISCRETE with slider-crank and site transmissions now on the straight-line path
  (run-time specialized kernel, the transmissions formed by the discrete pass): qfrc_inverse
  and the actuator moments vs the oracle, the generic kernel alike, qacc restored."""
  from test_codegen_cpu import TRN_AFTER_XML
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string(TRN_AFTER_XML.format(integ=integ))
  B = 256
  rng = np.random.default_rng(13)
  q = rng.uniform(-1, 1, (B, m.nq)) * 0.5
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  e = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel is not None and e.fast_kernel.startswith("rt_")
    f, st = e.inverse(q, v, a, status=True)
    assert (st == 0).all()
    np.testing.assert_array_equal(e.field("qacc", 0, B), a)       # restored
    mom = e.field("actuator_moment", 0, B)
    g = e.inverse(q, v, a, generic=True)
  finally:
    e.close()
  ref, _ = oracle_batch(m, q, v, a, ("qfrc_inverse", "actuator_moment"))
  assert_close(f, ref["qfrc_inverse"], f"qfrc_inverse (INVDISCRETE {integ}, TRN_AFTER)")
  assert_close(g, ref["qfrc_inverse"], f"qfrc_inverse (INVDISCRETE {integ}, generic)")
  assert_close(mom, ref["actuator_moment"], "actuator_moment")
