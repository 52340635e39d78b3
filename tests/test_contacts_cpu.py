"""Contacts on the CPU.

* The oracle's collision / contact-constraint restatement is pinned by the reference's own
  tests, restated: test/engine/engine_collision_driver_test.cc (ContactCount, FilterParent,
  FilterParentDoesntAffectWorldBody) and test/engine/engine_core_constraint_test.cc
  (RestPenetration), plus analytic answers of the primitive pairs.
* The device pipeline compiled for the host (tests/cpu_kernel_harness.cpp) must equal the
  oracle bit for bit on every output, constraint row and contact.
"""
import ctypes

import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import fields, host, mjcf, models
from mujoco_inversedynamicstest_amd.sampler import sample_contact_states
from oracle.oracle import CON_DOUBLE, CON_INT, Oracle, UnsupportedModel, lib as olib

from kernel_harness import KernelCPU

mjDSBL_FILTERPARENT = 1 << 9


def _geom_pairs(m, o):
  names = m.names["geom"]
  return [tuple(names[g] for g in pair) for pair in o.contact_field("con_geom")]


def test_contact_count():
  """engine_collision_driver_test.cc:99-132 — 8 spheres resting on a plane in a body."""
  m = mjcf.load_xml_string("""
  <mujoco><worldbody>
    <body><geom type="plane" size="5 5 .01"/></body>
    <body pos="0 0 0.9"><freejoint/>
      <geom type="sphere" size="1" pos="-1 -1 0"/><geom type="sphere" size="1" pos="-1  1 0"/>
      <geom type="sphere" size="1" pos=" 1 -1 0"/><geom type="sphere" size="1" pos=" 1  1 0"/>
      <geom type="sphere" size="1" pos="-2 -2 0"/><geom type="sphere" size="1" pos="-2  2 0"/>
      <geom type="sphere" size="1" pos=" 2 -2 0"/><geom type="sphere" size="1" pos=" 2  2 0"/>
    </body></worldbody></mujoco>""")
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert o.efc.ncon == 8
  # midphase order (body with 8 geoms): sorted by geom id
  assert list(o.contact_field("con_geom")[:, 1]) == list(range(1, 9))
  np.testing.assert_allclose(o.contact_field("con_dist"), -0.1, atol=1e-12)


_FILTER_PARENT = """
  <mujoco><worldbody>
    <body pos="0 0 0"><freejoint/>
      <geom name="colliding1" size="1" pos="0 0 100"/>
      <body><geom size="1"/>
        <body><joint axis="1 0 0"/><geom size="1" pos="0 0 50"/>
          <body><geom name="colliding2" size="1" pos="0 0 99.5"/></body>
        </body>
      </body>
    </body></worldbody></mujoco>"""


def test_filter_parent():
  """engine_collision_driver_test.cc:134-175."""
  m = mjcf.load_xml_string(_FILTER_PARENT)
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert o.efc.ncon == 0
  m.opt["disableflags"] |= mjDSBL_FILTERPARENT
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert _geom_pairs(m, o) == [("colliding1", "colliding2")]


def test_filter_parent_doesnt_affect_world_body():
  """engine_collision_driver_test.cc:177-203."""
  m = mjcf.load_xml_string("""
  <mujoco><worldbody>
    <geom name="colliding1" size="1" pos="0 0 100"/>
    <body pos="0 0 0"><joint axis="1 0 0"/><geom name="colliding2" size="1" pos="0 0 99.5"/>
    </body></worldbody></mujoco>""")
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert _geom_pairs(m, o) == [("colliding1", "colliding2")]


@pytest.mark.parametrize("reference", [-100.0, -10.0, 0.1, 0.01])
@pytest.mark.parametrize("impedance", [0.3, 0.9, 0.99])
def test_rest_penetration(reference, impedance):
  """engine_core_constraint_test.cc:161-229, restated for inverse dynamics.

  The reference simulates a sphere on a slide joint until it rests and checks its
  penetration depth: g(1-imp)/-ref (direct solref) or g(1-imp)(timeconst*dampratio)^2. At
  that depth, at rest (qvel = qacc = 0), the soft contact force holds the weight exactly,
  so the inverse dynamics must need no applied force: qfrc_inverse = 0.
  """
  m = mjcf.load_xml_string("""
  <mujoco><worldbody>
    <geom type="plane" size="1 1 1"/>
    <body pos="0 0 .2"><joint type="slide" axis="0 0 1"/><geom size=".1"/></body>
  </worldbody></mujoco>""")
  g = -m.opt["gravity"][2]
  dr = 0.8
  m.geom_solimp[:, 0] = impedance
  m.geom_solimp[:, 1] = impedance
  m.geom_solref[:, 0] = reference
  m.geom_solref[:, 1] = -10 if reference < 0 else dr
  depth = g * (1 - impedance) / -reference if reference < 0 else \
      g * (1 - impedance) * (reference * dr) ** 2
  o = Oracle(m)
  q = np.array([-0.1 - depth])            # sphere bottom at -depth
  f = o.inverse(q, np.zeros(1), np.zeros(1))
  assert o.efc.ncon == 1
  assert -o.contact_field("con_dist")[0] == pytest.approx(depth, rel=1e-12, abs=1e-15)
  weight = m.body_mass[1] * g
  assert abs(f[0]) <= 1e-9 * weight, (f, weight)


def _one_contact(xml):
  m = mjcf.load_xml_string(xml)
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  return m, o


def test_plane_sphere_known_answer():
  """mjraw_PlaneSphere: dist = height - r, point midway into the gap, normal = plane z."""
  m, o = _one_contact("""<mujoco><worldbody><geom type="plane" size="1 1 1"/>
    <body pos=".3 -.2 .25"><freejoint/><geom size=".3"/></body></worldbody></mujoco>""")
  assert o.efc.ncon == 1
  assert o.contact_field("con_dist")[0] == pytest.approx(-0.05, abs=1e-15)
  np.testing.assert_allclose(o.contact_field("con_pos")[0], [0.3, -0.2, -0.025], atol=1e-15)
  np.testing.assert_allclose(o.contact_field("con_frame")[0][:3], [0, 0, 1])


def test_plane_capsule_two_contacts():
  """mjc_PlaneCapsule: a horizontal capsule touches the plane at both segment ends."""
  m, o = _one_contact("""<mujoco><worldbody><geom type="plane" size="1 1 1"/>
    <body pos="0 0 .09"><freejoint/><geom type="capsule" fromto="-.2 0 0 .2 0 0" size=".1"/>
    </body></worldbody></mujoco>""")
  assert o.efc.ncon == 2
  np.testing.assert_allclose(o.contact_field("con_dist"), [-0.01, -0.01], atol=1e-15)
  xs = sorted(o.contact_field("con_pos")[:, 0])
  np.testing.assert_allclose(xs, [-0.2, 0.2], atol=1e-15)
  # pyramidal condim 3: four rows per contact
  assert o.efc.nefc == 8


def test_capsule_capsule_crossing_and_sphere_sphere():
  """mjraw_CapsuleCapsule (crossing axes -> one contact between the axes) and
  mjraw_SphereSphere (normal from sphere 1 to sphere 2)."""
  m, o = _one_contact("""<mujoco><option gravity="0 0 0"/><worldbody>
    <body><freejoint/><geom type="capsule" fromto="-.5 0 0 .5 0 0" size=".1"/></body>
    <body pos="0 0 .15"><freejoint/><geom type="capsule" fromto="0 -.5 0 0 .5 0" size=".1"/>
    </body>
    <body pos="2 0 0"><freejoint/><geom size=".2"/></body>
    <body pos="2 0 .3"><freejoint/><geom size=".2"/></body>
  </worldbody></mujoco>""")
  assert o.efc.ncon == 2
  np.testing.assert_allclose(o.contact_field("con_dist"), [-0.05, -0.1], atol=1e-14)
  np.testing.assert_allclose(o.contact_field("con_frame")[:, :3], [[0, 0, 1], [0, 0, 1]],
                             atol=1e-15)
  np.testing.assert_allclose(o.contact_field("con_pos")[0], [0, 0, 0.075], atol=1e-15)
  np.testing.assert_allclose(o.contact_field("con_pos")[1], [2, 0, 0.15], atol=1e-15)


def test_plane_box_four_lowest_corners():
  """mjc_PlaneBox (engine_collision_primitive.c:200-243): a level box below its half height
  touches at its 4 bottom corners, each midway into the gap; a tilted box at the corners
  under the margin, at most 4."""
  m, o = _one_contact("""<mujoco><worldbody><geom type="plane" size="1 1 1"/>
    <body pos=".1 .2 .08"><freejoint/><geom type="box" size=".3 .2 .1"/></body>
    </worldbody></mujoco>""")
  assert o.efc.ncon == 4
  np.testing.assert_allclose(o.contact_field("con_dist"), [-0.02] * 4, atol=1e-15)
  pos = o.contact_field("con_pos")
  np.testing.assert_allclose(sorted(map(tuple, np.round(pos, 12))),
                             sorted((0.1 + sx * 0.3, 0.2 + sy * 0.2, -0.01)
                                    for sx in (-1, 1) for sy in (-1, 1)), atol=1e-12)
  m, o = _one_contact("""<mujoco><worldbody><geom type="plane" size="1 1 1"/>
    <body pos="0 0 .15" euler="0 30 0"><freejoint/><geom type="box" size=".3 .2 .1"/></body>
    </worldbody></mujoco>""")
  # the two corners of the lowered edge: z = .15 - .3 sin30 - .1 cos30 < 0
  assert o.efc.ncon == 2
  np.testing.assert_allclose(o.contact_field("con_dist"),
                             [0.15 - 0.3 * 0.5 - 0.1 * np.cos(np.pi / 6)] * 2, atol=1e-12)


def test_plane_cylinder_disk_triangle():
  """mjc_PlaneCylinder (engine_collision_primitive.c:95-195): an upright cylinder sinking
  into the plane touches at a rim point and the two triangle points (3 contacts)."""
  m, o = _one_contact("""<mujoco><worldbody><geom type="plane" size="1 1 1"/>
    <body pos="0 0 .18"><freejoint/><geom type="cylinder" size=".1 .2"/></body>
    </worldbody></mujoco>""")
  assert o.efc.ncon == 3
  np.testing.assert_allclose(o.contact_field("con_dist"), [-0.02] * 3, atol=1e-15)
  r = 0.1
  np.testing.assert_allclose(o.contact_field("con_pos"),
                             [[r, 0, -0.01], [-r / 2, r * np.sqrt(3) / 2, -0.01],
                              [-r / 2, -r * np.sqrt(3) / 2, -0.01]], atol=1e-15)
  # lying on its side: both rim ends of the lowest line, no triangle points
  m, o = _one_contact("""<mujoco><worldbody><geom type="plane" size="1 1 1"/>
    <body pos="0 0 .09" euler="90 0 0"><freejoint/><geom type="cylinder" size=".1 .2"/></body>
    </worldbody></mujoco>""")
  assert o.efc.ncon == 2
  np.testing.assert_allclose(o.contact_field("con_dist"), [-0.01, -0.01], atol=1e-15)


def test_box_sphere_reference():
  """BoxSphere (engine_collision_box_test.cc:247-273): a sphere at the top face of a box
  that sits under a plane touches both, with equal distances, at every depth; the device
  code equals the oracle bit for bit."""
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <geom type="plane" size="0.05 0.05 0.001"/>
    <geom type="box" pos="0 0 -0.025" size="0.05 0.05 .025"/>
    <body><freejoint/><geom type="sphere" mass="1" size="0.005"/></body>
    </worldbody></mujoco>""")
  o = Oracle(m)
  k = KernelCPU(m, o.efc.capacity)
  for z in (-.015, -.00501, -.005, -.00499, 0.0, 0.004):
    q = m.qpos0.copy()
    q[2] = z
    o.inverse(q, np.zeros(6), np.zeros(6))
    k.inverse(q, np.zeros(6), np.zeros(6))
    assert o.efc.ncon == 2
    d = o.contact_field("con_dist")
    assert abs(d[0] - d[1]) < 1e-8
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name))


def test_box_cylinder_device_bitexact():
  """Random poses of boxes and cylinders over a plane (condim 1/3/6): the device code on the
  host equals the oracle bit for bit on every contact, row and output."""
  m = mjcf.load_xml_string("""<mujoco><default><geom contype="1" conaffinity="2"/></default>
    <worldbody><geom type="plane" size="3 3 .1" contype="2" conaffinity="1"/>
    <body pos="0 0 .1"><freejoint/><geom type="box" size=".2 .1 .05" condim="1"/></body>
    <body pos=".8 0 .1"><freejoint/><geom type="cylinder" size=".1 .15" condim="6"/></body>
    <body pos="-.8 0 .1"><freejoint/><geom type="box" size=".1 .1 .1"/>
      <body pos="0 0 .2"><joint axis="1 0 0"/><geom type="cylinder" size=".05 .1"
        pos="0 0 .1"/></body></body>
  </worldbody></mujoco>""")
  rng = np.random.default_rng(11)
  o, k = Oracle(m), KernelCPU(m)
  total = 0
  for i in range(40):
    q = m.qpos0.copy()
    for b in range(3):
      q[7 * b + 2] = 0.05 + 0.1 * rng.random()
      qq = rng.normal(size=4)
      q[7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq)
    q[21] = rng.normal()
    v, a = rng.normal(size=m.nv), rng.normal(size=m.nv)
    o.inverse(q, v, a)
    k.inverse(q, v, a)
    ncon = o.efc.ncon
    total += ncon
    assert k.field("con_count")[0] == ncon
    width = dict(CON_DOUBLE + CON_INT)
    for name in CON_FIELDS:
      ref = o.contact_field(name).reshape(ncon, width[name])
      np.testing.assert_array_equal(k.field(name)[:ref.size].reshape(ncon, width[name]), ref,
                                    err_msg=f"{name} inst {i}")
    for name in EFC_FIELDS:
      ref = o.efc_field(name)
      np.testing.assert_array_equal(k.field(name)[:ref.size], ref, err_msg=f"{name} inst {i}")
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name))
  assert total > 60


def test_unimplemented_pair_flagged_per_instance():
  """A cylinder-box pair under mjDSBL_NATIVECCD (mjc_Convex on libccd's MPR, outside the
  subset) adds no capacity; an instance whose pair passes the bounding-sphere filter is
  flagged MJHIP_INST_UNSUPPORTED, the others are exact (here: the plane-sphere contact of the
  same instance is still made)."""
  m = mjcf.load_xml_string("""<mujoco><option><flag nativeccd="disable"/></option><worldbody>
    <geom type="plane" size="5 5 .1"/>
    <geom type="box" size=".5 .5 .5" pos="0 0 2" contype="3" conaffinity="3"/>
    <body pos="0 0 2"><freejoint/><geom type="cylinder" size=".1 .1" contype="2"
      conaffinity="2"/><geom type="sphere" size=".1" pos="0 0 -.1" contype="1"
      conaffinity="1"/></body></worldbody></mujoco>""")
  cm = host.model_struct(m)
  assert olib().or_contactCapacity(ctypes.byref(cm)) == 2       # plane-sphere, sphere-box
  o = Oracle(m)
  k = KernelCPU(m, o.efc.capacity)
  outs = [f.name for f in fields.DATA_FIELDS if f.stage > 0]
  for z, flag in ((0.05, 0), (2.3, 32)):   # far from the world box / overlapping it
    q = np.array([0, 0, z, 1, 0, 0, 0.0])
    v, a = np.zeros(6), np.zeros(6)
    o.inverse(q, v, a)
    _, st = k.inverse(q, v, a)
    assert o.d.status == st == flag
    assert o.efc.ncon == 1                 # plane-sphere low, sphere-box high
    for f in outs:
      np.testing.assert_array_equal(getattr(k.d, f), getattr(o.d, f), err_msg=f)


def test_capacity_exact():
  m = models.load("humanoid", disable_contact=False)
  cm = host.model_struct(m)
  L = olib()
  ncap = L.or_contactCapacity(ctypes.byref(cm))
  assert ncap > 0 and L.or_efcCapacity(ctypes.byref(cm)) > ncap
  q, v, a = sample_contact_states(m, 48)
  o = Oracle(m)
  for i in range(48):
    o.inverse(q[i], v[i], a[i])
    assert o.efc.ncon <= ncap


CON_FIELDS = ("con_dist", "con_pos", "con_frame", "con_includemargin", "con_friction",
              "con_solref", "con_solreffriction", "con_solimp", "con_mu", "con_dim",
              "con_geom", "con_exclude", "con_efc_address")
EFC_FIELDS = ("efc_J", "efc_pos", "efc_margin", "efc_frictionloss", "efc_diagApprox",
              "efc_KBIP", "efc_D", "efc_R", "efc_vel", "efc_aref", "efc_force", "efc_type",
              "efc_id", "efc_state")


def test_device_code_bitexact_with_contacts():
  """Config-4 humanoid states: every output, row and contact equals the oracle's."""
  m = models.load("humanoid", disable_contact=False)
  q, v, a = sample_contact_states(m, 48, first=7)
  o, k = Oracle(m), KernelCPU(m)
  seen = 0
  for i in range(48):
    o.inverse(q[i], v[i], a[i])
    k.inverse(q[i], v[i], a[i])
    ncon, nefc = o.efc.ncon, o.efc.nefc
    seen += ncon > 0
    assert k.field("con_count")[0] == ncon and k.field("efc_count")[0] == nefc
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name),
                                      err_msg=f"{f.name} inst {i}")
    width = dict(CON_DOUBLE + CON_INT)
    for name in CON_FIELDS:
      ref = o.contact_field(name).reshape(ncon, width[name])
      got = k.field(name)[:ref.size].reshape(ncon, width[name])
      np.testing.assert_array_equal(got, ref, err_msg=f"{name} inst {i}")
    for name in EFC_FIELDS:
      ref = o.efc_field(name)
      np.testing.assert_array_equal(k.field(name)[:ref.size], ref, err_msg=f"{name} inst {i}")
  assert seen > 30


_MIXED = """<mujoco><worldbody><geom type="plane" size="3 3 .1" condim="1"/>
  <body pos="0 0 .1"><freejoint/><geom size=".11" condim="1"/></body>
  <body pos=".6 0 .1"><freejoint/><geom type="capsule" fromto="-.1 0 0 .1 0 0" size=".105"
    condim="4"/></body>
  <body pos="1.2 0 .1"><freejoint/><geom size=".105" condim="6"/></body>
  <body pos="-.6 0 .5"><joint type="hinge" axis="0 1 0" range="-.1 .1" limited="true"
      frictionloss=".3"/>
    <geom type="capsule" fromto="0 0 0 0 0 -.45" size=".06" condim="3"/></body>
</worldbody></mujoco>"""


def test_fused_equals_classic_and_oracle():
  """The fused constraint path (rows finished at creation) against the classic passes and
  the oracle: condim 1, 3, 4 and 6 contacts, a friction-loss row and joint limits."""
  m = mjcf.load_xml_string(_MIXED)
  o, kf, kc = Oracle(m), KernelCPU(m), KernelCPU(m)
  rng = np.random.default_rng(3)
  dims = set()
  for t in range(40):
    q = m.qpos0.copy()
    for b in range(3):                       # free bodies: height and small tilt
      q[7*b + 2] = 0.1 + rng.uniform(-0.03, 0.03)
      q[7*b + 3:7*b + 7] = [1, *rng.normal(scale=0.1, size=3)]
      q[7*b + 3:7*b + 7] /= np.linalg.norm(q[7*b + 3:7*b + 7])
    q[21] = rng.uniform(-0.3, 0.3)          # hinge across its limits
    v, a = rng.normal(size=m.nv), rng.normal(size=m.nv)
    f_o = o.inverse(q, v, a)
    f_f, _ = kf.inverse(q, v, a)
    f_c, _ = kc.inverse(q, v, a, classic=True)
    np.testing.assert_array_equal(f_f, f_o)
    np.testing.assert_array_equal(f_c, f_o)
    nefc = o.efc.nefc
    for name in EFC_FIELDS:
      ref = o.efc_field(name)
      np.testing.assert_array_equal(kf.field(name)[:ref.size], ref, err_msg=f"{name} {t}")
      np.testing.assert_array_equal(kc.field(name)[:ref.size], ref, err_msg=f"{name} {t}")
    np.testing.assert_array_equal(kf.field("con_mu")[:o.efc.ncon], o.contact_field("con_mu"))
    dims.update(int(x) for x in o.contact_field("con_dim"))
    assert kf.field("efc_count")[0] == nefc
  assert dims == {1, 3, 4, 6}


@pytest.mark.parametrize("impedance", [0.3, 0.9, 0.99])
def test_rest_penetration_elliptic(impedance):
  """RestPenetration with an elliptic cone: the normal row of the cone holds the weight at
  the reference's rest depth exactly as the pyramid does (mj_makeImpedance keeps the
  normal R of the elliptic cone; friction rows carry no load at rest)."""
  m = mjcf.load_xml_string("""
  <mujoco><option cone="elliptic"/><worldbody>
    <geom type="plane" size="1 1 1"/>
    <body pos="0 0 .2"><joint type="slide" axis="0 0 1"/><geom size=".1"/></body>
  </worldbody></mujoco>""")
  g, dr, reference = -m.opt["gravity"][2], 0.8, 0.01
  m.geom_solimp[:, 0] = impedance
  m.geom_solimp[:, 1] = impedance
  m.geom_solref[:, 0] = reference
  m.geom_solref[:, 1] = dr
  depth = g * (1 - impedance) * (reference * dr) ** 2
  o = Oracle(m)
  f = o.inverse(np.array([-0.1 - depth]), np.zeros(1), np.zeros(1))
  assert o.efc.nefc == 3 and list(o.efc_field("efc_type")) == [7, 7, 7]
  assert abs(f[0]) <= 1e-9 * m.body_mass[1] * g


_ELLIPTIC = _MIXED.replace("<mujoco>", '<mujoco><option cone="elliptic" impratio="3"/>').replace(
    'condim="6"/>', 'condim="6" solreffriction=".05 1"/>')


def test_elliptic_cone_states_and_device_bitexact():
  """Elliptic cones (condim 1, 3, 4, 6; solreffriction; impratio): every cone state occurs;
  in the CONE state the force lies on the cone, |f_T / mu| = f_N; the device code on the
  host equals the oracle bit for bit."""
  m = mjcf.load_xml_string(_ELLIPTIC)
  o, k = Oracle(m), KernelCPU(m)
  rng = np.random.default_rng(13)
  states = set()
  for i in range(60):
    q = m.qpos0.copy()
    for b in range(3):
      q[7 * b + 2] = 0.09 + 0.02 * rng.random()
      qq = np.array([1, 0, 0, 0]) + 0.2 * rng.normal(size=4)
      q[7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq)
    q[21] = 0.2 * rng.normal()
    v, a = 0.5 * rng.normal(size=m.nv), 3 * rng.normal(size=m.nv)
    o.inverse(q, v, a)
    k.inverse(q, v, a)
    st, tp = o.efc_field("efc_state"), o.efc_field("efc_type")
    fr = o.efc_field("efc_force")
    states |= set(st[tp == 7].tolist())
    for c in range(o.efc.ncon):
      adr, dim = o.contact_field("con_efc_address")[c], o.contact_field("con_dim")[c]
      if adr >= 0 and dim > 1 and st[adr] == 4:       # CONE
        mu = o.contact_field("con_friction")[c][:dim - 1]
        np.testing.assert_allclose(np.linalg.norm(fr[adr + 1:adr + dim] / mu), fr[adr],
                                   rtol=1e-10)
    for name in EFC_FIELDS:
      ref = o.efc_field(name)
      np.testing.assert_array_equal(k.field(name)[:ref.size], ref, err_msg=f"{name} inst {i}")
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name))
  assert {0, 1, 4} <= states, states


@pytest.mark.parametrize("where,pos,dist,normal", [
    # side: sphere beside the upright cylinder (r=.1, half-height .2), sphere r=.05
    ("side", (0.14, 0.0, 0.05), -0.01, (1.0, 0.0, 0.0)),
    # top cap: sphere above the top face, inside the radius
    ("cap", (0.03, 0.02, 0.24), -0.01, (0.0, 0.0, 1.0)),
    # bottom cap: the flipped frame
    ("bottom", (0.0, -0.04, -0.24), -0.01, (0.0, 0.0, -1.0)),
    # rim corner: beyond both the radius and the top
    ("rim", (0.13, 0.0, 0.23), np.hypot(0.03, 0.03) - 0.05, (np.sqrt(.5), 0.0, np.sqrt(.5)))])
def test_sphere_cylinder_known_answers(where, pos, dist, normal):
  """mjc_SphereCylinder (engine_collision_primitive.c:323-391): side contacts are
  sphere-sphere with the nearest axis point, cap contacts plane-sphere on the cap plane
  (the bottom cap through the flipped frame) with the normal flipped, rim contacts
  sphere-sphere with the corner point. The frame normal points from geom 1 (the sphere)
  into geom 2 (the cylinder): minus the face normal `normal` listed here."""
  m = mjcf.load_xml_string(f"""<mujoco><worldbody>
    <geom type="cylinder" size=".1 .2" contype="1" conaffinity="1"/>
    <body pos="{pos[0]} {pos[1]} {pos[2]}"><freejoint/><geom size=".05"/></body>
    </worldbody></mujoco>""")
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert o.efc.ncon == 1
  assert o.contact_field("con_dist")[0] == pytest.approx(dist, abs=1e-15)
  # contact frame normal points from geom 1 (sphere) to geom 2 (cylinder)
  np.testing.assert_allclose(o.contact_field("con_frame")[0][:3], -np.asarray(normal),
                             atol=1e-15)
  k = KernelCPU(m)
  k.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  for name in ("con_dist", "con_pos", "con_frame"):
    np.testing.assert_array_equal(k.field(name)[:o.contact_field(name).size],
                                  o.contact_field(name).ravel())


def test_sphere_cylinder_device_bitexact():
  """Random poses of spheres around a free cylinder (side, caps, rims, deep penetration):
  the device code on the host equals the oracle bit for bit on contacts, rows and outputs."""
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="cylinder" size=".12 .2"/></body>
    <body pos=".3 0 .5"><freejoint/><geom size=".06" condim="1"/></body>
    <body pos="-.3 0 .5"><freejoint/><geom size=".08" condim="4"/></body>
    </worldbody></mujoco>""")
  rng = np.random.default_rng(21)
  o, k = Oracle(m), KernelCPU(m)
  total = 0
  for i in range(60):
    q = m.qpos0.copy()
    qq = rng.normal(size=4)
    q[3:7] = qq / np.linalg.norm(qq)
    for b in (1, 2):
      q[7 * b:7 * b + 3] = q[:3] + rng.uniform(-0.25, 0.25, size=3)
    v, a = rng.normal(size=m.nv), rng.normal(size=m.nv)
    o.inverse(q, v, a)
    _, st = k.inverse(q, v, a)
    assert st == o.d.status == 0
    ncon = o.efc.ncon
    total += ncon
    assert k.field("con_count")[0] == ncon
    width = dict(CON_DOUBLE + CON_INT)
    for name in CON_FIELDS:
      ref = o.contact_field(name).reshape(ncon, width[name])
      np.testing.assert_array_equal(k.field(name)[:ref.size].reshape(ncon, width[name]), ref,
                                    err_msg=f"{name} inst {i}")
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name))
  assert total > 30


def test_capsule_box_known_answers():
  """mjraw_CapsuleBox (engine_collision_box.c:121-594): a capsule lying on a box's top face
  touches it at both segment ends (two sphere-box contacts, normal along the face normal); a
  capsule standing on its end touches once; one crossing a box edge diagonally touches at
  the edge point."""
  def contacts(cap_pos, cap_euler):
    m = mjcf.load_xml_string(f"""<mujoco><worldbody>
      <geom type="box" size=".5 .5 .1"/>
      <body pos="{cap_pos}" euler="{cap_euler}"><freejoint/>
        <geom type="capsule" size=".05 .2"/></body></worldbody></mujoco>""")
    o = Oracle(m)
    o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
    k = KernelCPU(m)
    k.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
    for name in ("con_dist", "con_pos", "con_frame"):
      np.testing.assert_array_equal(k.field(name)[:o.contact_field(name).size],
                                    o.contact_field(name).ravel())
    return o.contact_field("con_dist"), o.contact_field("con_pos"), o.contact_field("con_frame")
  # lying along x on the top face, 0.01 deep: both ends
  d, p, f = contacts("0 0 .14", "0 90 0")
  assert len(d) == 2
  np.testing.assert_allclose(d, [-0.01, -0.01], atol=1e-15)
  np.testing.assert_allclose(sorted(p[:, 0]), [-0.2, 0.2], atol=1e-12)
  np.testing.assert_allclose(np.abs(f[:, 2]), [1, 1], atol=1e-15)
  # standing on its lower end, 0.01 deep: one contact below the lower end
  d, p, f = contacts("0.1 -0.2 .34", "0 0 0")
  assert len(d) == 1
  assert d[0] == pytest.approx(-0.01, abs=1e-15)
  np.testing.assert_allclose(p[0][:2], [0.1, -0.2], atol=1e-15)
  # crossing the edge x = .5 (along y) horizontally above its top corner line
  d, p, f = contacts(".5 0 .14", "90 0 0")
  assert len(d) >= 1
  assert min(d) == pytest.approx(-0.01, abs=1e-12)


def test_capsule_box_device_bitexact():
  """Random poses of capsules around a free box (faces, edges and corners closest, every
  second-point branch): the device code on the host equals the oracle bit for bit on
  contacts, rows and outputs."""
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="box" size=".2 .15 .1"/></body>
    <body pos=".4 0 .5"><freejoint/><geom type="capsule" size=".05 .15" condim="1"/></body>
    <body pos="-.4 0 .5"><freejoint/><geom type="capsule" size=".03 .25"/></body>
    </worldbody></mujoco>""")
  rng = np.random.default_rng(31)
  o, k = Oracle(m), KernelCPU(m)
  total, two = 0, 0
  for i in range(200):
    q = m.qpos0.copy()
    for b in range(3):
      qq = rng.normal(size=4)
      q[7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq)
    for b in (1, 2):
      q[7 * b:7 * b + 3] = q[:3] + rng.uniform(-0.3, 0.3, size=3)
    v, a = rng.normal(size=m.nv), rng.normal(size=m.nv)
    o.inverse(q, v, a)
    _, st = k.inverse(q, v, a)
    assert st == o.d.status == 0
    ncon = o.efc.ncon
    total += ncon
    g = o.contact_field("con_geom").reshape(ncon, 2)
    for b in (1, 2):
      two += int(((g == b).any(axis=1)).sum() == 2)
    assert k.field("con_count")[0] == ncon
    width = dict(CON_DOUBLE + CON_INT)
    for name in CON_FIELDS:
      ref = o.contact_field(name).reshape(ncon, width[name])
      np.testing.assert_array_equal(k.field(name)[:ref.size].reshape(ncon, width[name]), ref,
                                    err_msg=f"{name} inst {i}")
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name))
  assert total > 50 and two > 5


# ---- box : box (mjc_BoxBox, engine_collision_box.c:607-1343, with mj_collideGeoms' clean-up
# at engine_collision_driver.c:1522-1588). The models below are the reference's own test
# fixtures (test/engine/testdata/collision_box/*.xml), held here as data.
BOXBOX_BAD0 = """<mujoco><default><geom rgba="1 1 1 1" margin="1e-3" gap="1e-3"/></default>
  <worldbody>
    <geom name="ground" pos="0 0 0" quat="1 0 0 0" size="50 50 1" type="plane"/>
    <body name="block01" pos="-0.9 0 1.5" quat="1 0 0 0"><freejoint/>
      <geom mass="1" name="geom01" size="0.5 0.5 1.5" type="box"/></body>
    <body name="block02" pos="-0.7 0 3.5" quat="1 0 0 0"><freejoint/>
      <geom mass="1" name="geom02" size="1.5 0.5 0.5" type="box"/></body>
    <body name="block03" pos="0.3 0 5.5" quat="1 0 0 0"><freejoint/>
      <geom mass="1" name="geom03" size="0.5 0.5 1.5" type="box"/></body>
    <body name="block04" pos="0.200 1e-9 7.5" quat="1 0 0 0"><freejoint/>
      <geom mass="1" name="geom04" size="1.5 0.5 0.5" type="box"/></body>
  </worldbody>
  <contact><exclude body1="world" body2="block01"/><exclude body1="block03" body2="block02"/>
  </contact></mujoco>"""
BOXBOX_DUPLICATE = """<mujoco><worldbody><geom type="box" size="1 1 1"/>
  <body pos="0 0 2"><freejoint/><geom type="box" size="1 1 1"/></body></worldbody></mujoco>"""
BOXBOX_DEEP = """<mujoco><worldbody><geom type="box" size="1 1 1"/>
  <body pos=".1 .2 .3"><freejoint/><geom type="box" size=".2 .2 .2"/></body></worldbody>
  </mujoco>"""


def _box_pairs(m, o):
  g = o.contact_field("con_geom").reshape(-1, 2)
  out = []
  for g1, g2 in g:
    if m.geom_type[g1] == 6 and m.geom_type[g2] == 6 and (g1, g2) not in out:
      out.append((int(g1), int(g2)))
  return out


def _outside(point, pos, mat, size, inflate):
  """mju_outsideBox (engine_util_misc.c:911-950), restated in numpy for the test."""
  v = mat.reshape(3, 3).T @ (point - pos)
  big = size * inflate
  if (v > big).any() or (v < -big).any():
    return 1
  small = size / inflate
  return -1 if ((v < small) & (v > -small)).all() else 0


def _raw_vs_kept(m, o):
  """Per box pair: the raw mjc_BoxBox contacts and which of them survive in the list."""
  pos = o.contact_field("con_pos").reshape(-1, 3)
  g = o.contact_field("con_geom").reshape(-1, 2)
  for g1, g2 in _box_pairs(m, o):
    margin = max(m.geom_margin[g1], m.geom_margin[g2])
    _, raw, _ = o.box_box_raw(g1, g2, margin)
    kept = pos[(g[:, 0] == g1) & (g[:, 1] == g2)]
    matched = np.zeros(len(raw), bool)
    used = np.zeros(len(kept), bool)
    for i, p in enumerate(raw):
      for j, q in enumerate(kept):
        if not used[j] and (p == q).all():
          matched[i] = used[j] = True
          break
    assert used.all()                       # every kept contact is a raw one
    yield g1, g2, margin, raw, matched


def test_boxbox_bad_contacts():
  """BadContacts (engine_collision_box_test.cc:34-133): some raw contacts are removed, and
  every removed one lies outside one box (by 1%) without being inside the other."""
  m = mjcf.load_xml_string(BOXBOX_BAD0)
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  npairs = 0
  for g1, g2, margin, raw, matched in _raw_vs_kept(m, o):
    npairs += 1
    assert matched.sum() < len(raw)
    gx = o.d.geom_xpos.reshape(-1, 3)
    gm = o.d.geom_xmat.reshape(-1, 9)
    s1 = m.geom_size[g1] + margin
    s2 = m.geom_size[g2] + margin
    for i in np.flatnonzero(~matched):
      o1 = _outside(raw[i], gx[g1], gm[g1], s1, 1.01)
      o2 = _outside(raw[i], gx[g2], gm[g2], s2, 1.01)
      assert (o1 == 1 and o2 != -1) or (o2 == 1 and o1 != -1)
  assert npairs == 2


def test_boxbox_duplicate_contacts():
  """DuplicateContacts (engine_collision_box_test.cc:138-227): a box resting exactly on an
  equal box; removed raw contacts are repeats of another raw contact."""
  m = mjcf.load_xml_string(BOXBOX_DUPLICATE)
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  for g1, g2, margin, raw, matched in _raw_vs_kept(m, o):
    assert matched.sum() < len(raw)
    for i in np.flatnonzero(~matched):
      assert any((raw[i] == raw[j]).all() for j in range(len(raw)) if j != i)
  assert o.efc.ncon == 4


def test_boxbox_deep_penetration():
  """DeepPenetration (engine_collision_box_test.cc:233-245): 4 contacts."""
  m = mjcf.load_xml_string(BOXBOX_DEEP)
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert o.efc.ncon == 4


def test_boxbox_resting_known_answer():
  """A level box 0.01 into a wide slab: the face path gives the small box's 4 bottom corners,
  midway into the overlap, normal +z; the reference reports half the face depth as dist."""
  m = mjcf.load_xml_string("""<mujoco><worldbody><geom type="box" size="1 1 .1"/>
    <body pos=".1 .2 .29"><freejoint/><geom type="box" size=".2 .2 .2"/></body></worldbody>
    </mujoco>""")
  o = Oracle(m)
  o.inverse(m.qpos0, np.zeros(m.nv), np.zeros(m.nv))
  assert o.efc.ncon == 4
  np.testing.assert_allclose(o.contact_field("con_dist"), [-0.005] * 4, atol=1e-15)
  pos = o.contact_field("con_pos").reshape(4, 3)
  np.testing.assert_allclose(sorted(map(tuple, np.round(pos, 12))),
                             sorted((0.1 + sx * 0.2, 0.2 + sy * 0.2, 0.095)
                                    for sx in (-1, 1) for sy in (-1, 1)), atol=1e-12)
  np.testing.assert_allclose(o.contact_field("con_frame").reshape(4, 9)[:, :3],
                             [[0, 0, 1]] * 4, atol=1e-15)


def test_boxbox_device_bitexact():
  """Random poses of boxes around a free box (face-face, face-edge and edge-edge separating
  axes, the clean-up of bad and repeated contacts): the device code on the host equals the
  oracle bit for bit on contacts, rows and outputs."""
  m = mjcf.load_xml_string("""<mujoco><worldbody>
    <body pos="0 0 .5"><freejoint/><geom type="box" size=".2 .15 .1"/></body>
    <body pos=".4 0 .5"><freejoint/><geom type="box" size=".1 .12 .08" condim="1"/></body>
    <body pos="-.4 0 .5"><freejoint/><geom type="box" size=".25 .05 .06" margin=".01"/></body>
    </worldbody></mujoco>""")
  rng = np.random.default_rng(41)
  o, k = Oracle(m), KernelCPU(m)
  total, many = 0, 0
  for i in range(300):
    q = m.qpos0.copy()
    for b in range(3):
      qq = rng.normal(size=4)
      q[7 * b + 3:7 * b + 7] = qq / np.linalg.norm(qq)
    for b in (1, 2):
      q[7 * b:7 * b + 3] = q[:3] + rng.uniform(-0.3, 0.3, size=3)
    v, a = rng.normal(size=m.nv), rng.normal(size=m.nv)
    o.inverse(q, v, a)
    _, st = k.inverse(q, v, a)
    assert st == o.d.status == 0
    ncon = o.efc.ncon
    total += ncon
    many += ncon > 4
    assert k.field("con_count")[0] == ncon
    width = dict(CON_DOUBLE + CON_INT)
    for name in CON_FIELDS:
      ref = o.contact_field(name).reshape(ncon, width[name])
      np.testing.assert_array_equal(k.field(name)[:ref.size].reshape(ncon, width[name]), ref,
                                    err_msg=f"{name} inst {i}")
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        np.testing.assert_array_equal(getattr(k.d, f.name), getattr(o.d, f.name))
  assert total > 100 and many > 5
