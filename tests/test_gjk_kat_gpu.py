"""MjGjkTest known answers (test/engine/engine_collision_gjk_test.cc) on the device: the
native GJK/EPA solver through mjhip_ccdBatch (mjh::ccdGeneral, one lane per pair) against the
values the reference's own tests assert (tests/gjk_cases.py), and against the oracle bit for
bit (the solver's region is compiled without multiply-add contraction, as the oracle is).
CylinderBoxMargin runs the whole device pipeline (one contact, efc_address < 0, no row).
"""
import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine, mjcf
from oracle.oracle import Oracle

import gjk_cases as K

pytestmark = pytest.mark.gpu


def test_gjk_known_answers_device():
  for name, xml, key, overrides, call, geoms, kw, expected in K.CASES:
    m = mjcf.load_xml_string(xml)
    o = Oracle(m)
    xpos, xmat = K.frames(m, o, key, overrides)
    g1, g2 = (m.names["geom"].index(g) for g in geoms)
    margin, maxc, cutoff = K.call_args(call, kw)
    e = engine.InverseEngine(m, capacity=64)
    try:
      # the same pair 64 times (one full wave) and once more: every lane answers alike
      n = 65
      dist, nx, x1, x2 = e.ccd([g1] * n, [g2] * n, [xpos[g1]] * n, [xmat[g1]] * n,
                               [xpos[g2]] * n, [xmat[g2]] * n, margin, K.KMAX, K.KTOL, maxc,
                               cutoff)
    finally:
      e.close()
    assert (dist == dist[0]).all() and (nx == nx[0]).all(), name
    K.check(name + " (device)", expected, K.report(call, dist[0], nx[0], x1[0], x2[0]))
    o.d.geom_xpos[:] = xpos.ravel()
    o.d.geom_xmat[:] = xmat.ravel()
    ro = o.ccd(g1, g2, margin, K.KTOL, K.KMAX, maxc, cutoff)
    assert dist[0] == ro[0] and nx[0] == ro[1], (name, dist[0], ro[0])
    if ro[1]:
      np.testing.assert_array_equal(x1[0], ro[2], err_msg=name)
      np.testing.assert_array_equal(x2[0], ro[3], err_msg=name)


def test_ccd_batch_arguments():
  """Bad arguments fail loudly (no launch): geom ids out of range, a negative max_contacts."""
  m = mjcf.load_xml_string(K.SPHERES)
  e = engine.InverseEngine(m, capacity=64)
  try:
    f = np.zeros((1, 3)), np.eye(3).reshape(1, 9)
    with pytest.raises(engine.MJHIPError):
      e.ccd([0], [5], f[0], f[1], f[0], f[1])
    with pytest.raises(engine.MJHIPError):
      e.ccd([0], [1], f[0], f[1], f[0], f[1], max_contacts=-1)
  finally:
    e.close()


def test_cylinder_box_margin_device():
  """CylinderBoxMargin (:1571-1600) on the device pipeline: one contact, efc_address < 0,
  no constraint row, qfrc_inverse as the oracle's."""
  m = mjcf.load_xml_string(K.CYLINDER_BOX_MARGIN)
  o = Oracle(m)
  z = np.zeros((1, m.nv))
  ref = o.inverse(m.qpos0, z[0], z[0])
  e = engine.InverseEngine(m, capacity=64)
  try:
    f = e.inverse(m.qpos0[None], z, z)
    assert e.field_int("con_count", 0, 1)[0, 0] == 1
    assert e.field_int("efc_count", 0, 1)[0, 0] == 0
    assert e.field_int("con_efc_address", 0, 1)[0, 0] < 0
  finally:
    e.close()
  np.testing.assert_allclose(f[0], ref, rtol=0, atol=1e-12)


def test_gjk_multicontact_known_answers_device():
  """Multicontact on the device (max_contacts > 1, box and mesh pairs; mjhip_ccdBatch): the
  reference's BoxBoxMultiCCD*, BoxEdge*, BoxMesh*, MeshMesh*, MeshEdge and LongBox known
  answers, and the oracle's contacts bit for bit."""
  for name, xml, overrides, geoms, maxc, expected in K.MULTI_CASES + K.MESH_MULTI_CASES:
    m = mjcf.load_xml_string(xml)
    o = Oracle(m)
    xpos, xmat = K.frames(m, o, None, overrides)
    g1, g2 = (m.names["geom"].index(g) for g in geoms)
    e = engine.InverseEngine(m, capacity=64)
    try:
      n = 3
      dist, nx, x1, x2 = e.ccd([g1] * n, [g2] * n, [xpos[g1]] * n, [xmat[g1]] * n,
                               [xpos[g2]] * n, [xmat[g2]] * n, 0.0, K.KMAX, K.KTOL, maxc, 0.0)
    finally:
      e.close()
    assert (dist == dist[0]).all() and (nx == nx[0]).all(), name
    k = nx[0]
    K.check(name + " (device)", expected, K.report_multi(dist[0], k, x1[0, :k], x2[0, :k]))
    o.d.geom_xpos[:] = xpos.ravel()
    o.d.geom_xmat[:] = xmat.ravel()
    ro = o.ccd(g1, g2, 0.0, K.KTOL, K.KMAX, maxc, 0.0)
    assert dist[0] == ro[0] and k == ro[1], (name, dist[0], ro[0], k, ro[1])
    np.testing.assert_array_equal(x1[0, :k], ro[2], err_msg=name)
    np.testing.assert_array_equal(x2[0, :k], ro[3], err_msg=name)
