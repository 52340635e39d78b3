"""The reference's 627-dof benchmark model (model/humanoid/humanoid100.xml)
on the GPU: the humanoid plus 100 free primitives in contact with the floor and each other
(tests/humanoid100_states.py), through a context capped at 1,024 contacts / 4,096 rows per
instance (mjhip_contextCreateCapped; the exact worst case is 344 MB of efc_J per instance).
Jacobian "auto" with nv = 627 is the reference's sparse path (mj_isSparse): the generic
kernel builds the compressed rows over the bodies' dof chains, their transpose, and the
position-grouped sums of mju_mulMatVecSparse, as the oracle restates them (sparse
Jacobians); the compressed structure is compared exactly.

Floating point: the generic kernel's unit rounds every operation as the oracle does (no
multiply-add contraction, DESIGN.md build), so, as for tests/test_reference_model_gpu.py, the
bar is exact: every contact equal to the oracle's bit for bit (the ellipsoid and cylinder
pairs run the iterative native solver) and every qfrc_inverse within the north-star 1e-10
(measured equal). Counts, statuses and contact geoms exact."""
import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine

import humanoid100_states as H

pytestmark = pytest.mark.gpu

RTOL = 1e-10


def _oracle(m, q, v, a, perturb=False):
  from oracle.oracle import Oracle
  o = Oracle(m)
  rng = np.random.default_rng(0)
  out = dict(f=[], st=[], nefc=[], ncon=[], geom=[], dist=[], pf=[])
  for i in range(len(q)):
    qi = q[i] * (1 + (rng.random(len(q[i])) - 0.5) * 2e-16) if perturb else q[i]
    out["f"].append(o.inverse(qi, v[i], a[i]).copy())
    out["st"].append(o.d.status)
    out["nefc"].append(o.d.nefc)
    out["ncon"].append(o.efc.ncon)
    out["geom"].append(o.contact_field("con_geom").ravel().copy())
    out["dist"].append(o.contact_field("con_dist").ravel().copy())
    out["pf"].append(np.concatenate([o.contact_field("con_pos").ravel(),
                                     o.contact_field("con_frame").ravel()]))
    if not perturb:
      out.setdefault("sp", []).append(o.efc_sparse())
  out["f"] = np.array(out["f"])
  return out


def _err(f, ref):
  return np.abs(f - ref).max(axis=1) / np.maximum(1.0, np.abs(ref).max(axis=1))


def test_humanoid100_vs_oracle():
  m = H.model()
  B = 128
  q, v, a = H.states(m, B, seed=5)
  e = engine.InverseEngine(m, capacity=B, max_contacts=H.MAX_CONTACTS, max_rows=H.MAX_ROWS)
  try:
    assert e.fast_kernel is None                  # nv >= 60: the generic kernel
    f, st = e.inverse(q, v, a, status=True)
    nefc = e.field_int("efc_count", 0, B)[:, 0]
    ncon = e.field_int("con_count", 0, B)[:, 0]
    geom = e.field_int("con_geom", 0, B)
    dist = e.field("con_dist", 0, B)
    pos, frame = e.field("con_pos", 0, B), e.field("con_frame", 0, B)
    nJ = e.field_int("nJ", 0, B)[:, 0]
    J = e.field("efc_J", 0, B)
    ints = {n: e.field_int(n, 0, B) for n in ("efc_J_rownnz", "efc_J_colind",
                                             "efc_JT_rownnz", "efc_JT_colind")}
  finally:
    e.close()
  o = _oracle(m, q, v, a)
  # the compressed rows (mj_isSparse): structure exact, values to the bar
  jerr = 0.0
  for i in range(B):
    sp = o["sp"][i]
    assert nJ[i] == sp["efc_J"].size
    np.testing.assert_array_equal(ints["efc_J_rownnz"][i, :nefc[i]], sp["efc_J_rownnz"])
    np.testing.assert_array_equal(ints["efc_J_colind"][i, :nJ[i]], sp["efc_J_colind"])
    np.testing.assert_array_equal(ints["efc_JT_rownnz"][i, :m.nv], sp["efc_JT_rownnz"])
    np.testing.assert_array_equal(ints["efc_JT_colind"][i, :nJ[i]], sp["efc_JT_colind"])
    jerr = max(jerr, np.abs(J[i, :nJ[i]] - sp["efc_J"]).max() / max(1, np.abs(sp["efc_J"]).max()))
  print(f"humanoid100: {int(nJ.sum())} compressed Jacobian entries (dense rows would hold "
        f"{int(nefc.sum()) * m.nv}), max efc_J error {jerr:.2e}")
  assert jerr <= RTOL
  np.testing.assert_array_equal(st, o["st"])
  assert (st == 0).all()
  np.testing.assert_array_equal(ncon, o["ncon"])
  np.testing.assert_array_equal(nefc, o["nefc"])
  derr, cerr = np.zeros(B), np.zeros(B)
  for i in range(B):
    n = o["ncon"][i]
    np.testing.assert_array_equal(geom[i, :2*n], o["geom"][i])
    derr[i] = np.abs(dist[i, :n] - o["dist"][i]).max()
    cerr[i] = max(derr[i], np.abs(np.concatenate([pos[i, :3*n], frame[i, :9*n]]) -
                                  o["pf"][i]).max())
  err = _err(f, o["f"])
  spread = _err(_oracle(m, q, v, a, perturb=True)["f"], o["f"])
  same = cerr <= 1e-12
  frac, self_frac = float((err > RTOL).mean()), float((spread > RTOL).mean())
  print(f"humanoid100: {int(np.sum(o['ncon']))} contacts, {int(np.sum(o['nefc']))} rows over "
        f"{B} instances; {int(same.sum())}/{B} with contacts matching to 1e-12, max error "
        f"there {err[same].max(initial=0):.2e}; above {RTOL}: device {frac:.3f}, oracle "
        f"under a one-ulp qpos change {self_frac:.3f}; max depth error {derr.max():.2e}")
  assert np.min(o["ncon"]) > 100
  assert derr.max() == 0                      # every depth bit for bit
  assert same.all()
  assert err.max() <= RTOL


def test_humanoid100_cap_flags_overflow():
  """A cap below what an instance needs flags it MJHIP_INST_CNSTRFULL (mjWARN_CONTACTFULL /
  mjWARN_CNSTRFULL), it does not write past the rows."""
  m = H.model()
  q, v, a = H.states(m, 64, seed=6)
  e = engine.InverseEngine(m, capacity=64, max_contacts=64, max_rows=256)
  try:
    _, st = e.inverse(q, v, a, status=True)
  finally:
    e.close()
  assert (st & 16).all()                          # MJHIP_INST_CNSTRFULL
