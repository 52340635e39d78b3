"""MJCF <frame>, <replicate> and <asset><model>/<attach> (the reference's
627-dof model/humanoid/humanoid100.xml). The compiled poses are checked against an
independent restatement with scipy rotations (the reference's own arithmetic is
mjuu_frameaccum; tolerance 1e-12), the names and counts against the reference's semantics
(xml_native_reader.cc:83-91, 3477-3646; user_objects.cc:707-714, 865-955), and the attached
humanoid against humanoid.xml compiled alone (bit-identical arrays). Compiled-model parity
with MuJoCo's own compiler stays unpinned: the header of humanoid100.xml
("Degree of Freedom: 627, Actuators: 21") is the one number the reference states."""
import os

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

from mujoco_inversedynamicstest_amd import mjcf, models

import humanoid100_states as H

REF = "/root/reference"


def _rot(euler_deg=None, quat=None):
  # MJCF eulerseq "xyz" rotates about the moving axes: scipy's intrinsic "XYZ"
  if euler_deg is not None:
    return Rotation.from_euler("XYZ", euler_deg, degrees=True)
  w, x, y, z = quat
  return Rotation.from_quat([x, y, z, w])


def _compose(frames):
  """frames: outermost first, each (pos, Rotation). Returns (pos, Rotation)."""
  pos, rot = np.zeros(3), Rotation.identity()
  for p, r in frames:
    pos = pos + rot.apply(p)
    rot = rot * r
  return pos, rot


def _same_pose(pos, quat, epos, erot, tol=1e-12):
  np.testing.assert_allclose(pos, epos, atol=tol)
  d = (_rot(quat=quat).inv() * erot).magnitude()
  assert d < tol, d


FRAMES = """
<mujoco><worldbody>
  <frame pos="0.1 0.2 0.3" euler="10 20 30">
    <frame pos="0 0 0.5" quat="0.9 0.1 0.2 0.3">
      <body name="b" pos="0.3 0 0" euler="0 30 0">
        <joint name="jb" type="hinge" axis="1 0 0" pos="0 0 0.1"/>
        <geom name="gb" type="capsule" size="0.05 0.1" pos="0 0.1 0" euler="5 0 0"/>
      </body>
      <geom name="g0" type="box" size=".1 .1 .1" pos="1 0 0" euler="0 0 45"/>
      <site name="s0" pos="0 1 0"/>
    </frame>
  </frame>
  <body name="c" pos="0 0 1">
    <frame euler="0 0 90" pos="0 0 0.2">
      <joint name="jc" type="slide" axis="1 0 0" pos="0.1 0 0"/>
      <geom name="gc" type="sphere" size=".1" pos="0.2 0 0"/>
    </frame>
  </body>
</worldbody></mujoco>
"""


def test_frames_compose_like_nested_transforms():
  m = mjcf.load_xml_string(FRAMES)
  n = m.names
  F1 = (np.array([0.1, 0.2, 0.3]), _rot([10, 20, 30]))
  q2 = np.array([0.9, 0.1, 0.2, 0.3])
  F2 = (np.array([0, 0, 0.5]), _rot(quat=q2 / np.linalg.norm(q2)))
  b = n["body"].index("b")
  _same_pose(m.body_pos[b], m.body_quat[b], *_compose([F1, F2, (np.array([0.3, 0, 0]),
                                                                   _rot([0, 30, 0]))]))
  # elements inside a frame in the world body: the frames' composition
  g0 = n["geom"].index("g0")
  _same_pose(m.geom_pos[g0], m.geom_quat[g0],
             *_compose([F1, F2, (np.array([1.0, 0, 0]), _rot([0, 0, 45]))]))
  s0 = n["site"].index("s0")
  _same_pose(m.site_pos[s0], m.site_quat[s0],
             *_compose([F1, F2, (np.array([0, 1.0, 0]), Rotation.identity())]))
  # elements of a body outside any frame are untouched by the frames of its ancestors
  gb = n["geom"].index("gb")
  _same_pose(m.geom_pos[gb], m.geom_quat[gb], np.array([0, 0.1, 0]), _rot([5, 0, 0]))
  jb = n["jnt"].index("jb")
  np.testing.assert_allclose(m.jnt_axis[jb], [1, 0, 0], atol=1e-15)
  # a frame inside a body moves its joint (axis rotated, pos framed) and geom
  jc, gc = n["jnt"].index("jc"), n["geom"].index("gc")
  Fc = (np.array([0, 0, 0.2]), _rot([0, 0, 90]))
  np.testing.assert_allclose(m.jnt_axis[jc], [0, 1, 0], atol=1e-15)
  np.testing.assert_allclose(m.jnt_pos[jc], _compose([Fc, (np.array([0.1, 0, 0]),
                                                           Rotation.identity())])[0], atol=1e-15)
  _same_pose(m.geom_pos[gc], m.geom_quat[gc],
             *_compose([Fc, (np.array([0.2, 0, 0]), Rotation.identity())]))


REPLICATE = """
<mujoco>
  <actuator><motor name="a" joint="jp"/></actuator>
  <worldbody>
    <replicate count="4" offset="1 0 0" euler="0 0 90" sep="-">
      <body name="r"><joint name="j" type="hinge"/><geom name="g" size=".1"/></body>
    </replicate>
    <body name="p" pos="0 0 2">
      <joint name="jp" type="hinge"/>
      <replicate count="12" offset="0 0 .1">
        <geom name="h" size=".01"/>
      </replicate>
      <geom name="after" size=".01"/>
    </body>
    <frame pos="0 5 0">
      <replicate count="2" offset="0 1 0">
        <frame pos="0 0 1">
          <replicate count="3" offset="0 0 1">
            <body name="n"><freejoint/><geom size=".1"/></body>
          </replicate>
        </frame>
      </replicate>
    </frame>
  </worldbody>
  <tendon><fixed name="t"><joint joint="j-2" coef="1"/></fixed></tendon>
</mujoco>
"""


def _replicate_frames(count, offset, euler):
  """The copy frames of xml_native_reader.cc:3540-3557 restated: copy i sits at the offsets
  accumulated under the previous copies' rotations, rotated by i*euler."""
  out, pos, rot = [], np.zeros(3), Rotation.identity()
  for i in range(count):
    out.append((pos.copy(), _rot(np.multiply(i, euler))))
    pos = pos + rot.apply(offset)
    rot = _rot(np.multiply(i, euler))
  return out


def test_replicate_names_order_and_frames():
  m = mjcf.load_xml_string(REPLICATE)
  n = m.names
  assert n["body"][1:5] == ["r-0", "r-1", "r-2", "r-3"]
  assert n["jnt"][:4] == ["j-0", "j-1", "j-2", "j-3"]
  p = n["body"].index("p")
  names = [n["geom"][g] for g in range(m.sizes["ngeom"]) if m.geom_bodyid[g] == p]
  assert names == [f"h{i:02d}" for i in range(12)] + ["after"]   # copies in place, padded
  for i, (fp, fr) in enumerate(_replicate_frames(4, [1, 0, 0], [0, 0, 90])):
    _same_pose(m.body_pos[1 + i], m.body_quat[1 + i], fp, fr)
  hg = [g for g in range(m.sizes["ngeom"]) if m.geom_bodyid[g] == p][:12]
  np.testing.assert_allclose(m.geom_pos[hg][:, 2], 0.1 * np.arange(12), atol=1e-15)
  # nested: inner suffix first, then the outer one; outer copies stay contiguous
  nested = [b for b in n["body"] if b.startswith("n")]
  assert nested == ["n00", "n10", "n20", "n01", "n11", "n21"]
  for k, b in enumerate(nested):
    i, j = divmod(k, 3)
    bid = n["body"].index(b)
    np.testing.assert_allclose(m.body_pos[bid], [0, 5 + i, 1 + j], atol=1e-15)
  # referencing elements resolve against the suffixed names; the actuator declared before
  # the world body names an unreplicated joint, so no suffixed copy of it appears
  assert n["actuator"] == ["a"]
  assert n["tendon"] == ["t"]
  assert m.sizes["nu"] == 1


def test_replicate_count_required():
  with pytest.raises(mjcf.MJCFError):
    mjcf.load_xml_string("<mujoco><worldbody><replicate><geom size='.1'/></replicate>"
                         "</worldbody></mujoco>")


def test_attach_needs_a_model_asset():
  with pytest.raises(mjcf.MJCFError, match="could not find model"):
    mjcf.load_xml_string("<mujoco><worldbody><attach model='x' body='b' prefix='p'/>"
                         "</worldbody></mujoco>")


def test_humanoid100_counts():
  m = H.model()
  s = m.sizes
  assert (m.nv, s["nu"]) == (627, 21)              # the file's header
  assert (s["nbody"], m.nq, s["ntendon"], s["nexclude"]) == (117, 728, 2, 2)
  n = m.names
  assert n["body"][1] == "humanoid_torso" and n["body"][16] == "humanoid_hand_left"
  assert n["actuator"][0] == "humanoid_abdomen_z" and n["tendon"] == [
      "humanoid_hamstring_right", "humanoid_hamstring_left"]
  assert all(b == "" for b in n["body"][H.FIRST_OBJECT:])
  types = m.geom_type[[m.body_geomadr[b] for b in range(H.FIRST_OBJECT, 117)]]
  # capsule, ellipsoid, box, cylinder, sphere columns of 20
  np.testing.assert_array_equal(types, np.repeat([3, 4, 6, 5, 2], 20))


def test_humanoid100_attached_humanoid_matches_humanoid_alone():
  """The attached subtree compiles to the same arrays as humanoid.xml alone (its attach
  frame is the identity): bodies, joints, dofs, geoms, actuators, tendons."""
  m, h = H.model(), models.load("humanoid")
  nb, nj, nv, ng = 17, h.sizes["njnt"], h.nv, h.sizes["ngeom"]
  for f in ("body_pos", "body_quat", "body_ipos", "body_iquat", "body_mass", "body_inertia"):
    np.testing.assert_array_equal(getattr(m, f)[1:nb], getattr(h, f)[1:nb], err_msg=f)
  for f in ("jnt_type", "jnt_pos", "jnt_axis", "jnt_range", "jnt_stiffness", "jnt_limited"):
    np.testing.assert_array_equal(getattr(m, f)[:nj], getattr(h, f)[:nj], err_msg=f)
  for f in ("dof_armature", "dof_damping", "dof_parentid"):
    np.testing.assert_array_equal(getattr(m, f)[:nv], getattr(h, f)[:nv], err_msg=f)
  # humanoid.xml's floor is not attached (body="torso"): its geoms follow the 9 world geoms
  off = m.sizes["ngeom"] - 100 - (ng - 1)
  for f in ("geom_type", "geom_size", "geom_pos", "geom_quat", "geom_friction", "geom_solimp",
            "geom_condim"):
    np.testing.assert_array_equal(getattr(m, f)[off:off + ng - 1], getattr(h, f)[1:ng],
                                  err_msg=f)
  for f in ("actuator_gear", "actuator_ctrlrange", "actuator_trnid", "tendon_range",
            "wrap_prm"):
    np.testing.assert_array_equal(getattr(m, f), getattr(h, f), err_msg=f)


def test_humanoid100_object_poses():
  """Body k of the 100: column frame, outer copy (offset 0 1 0, euler of the column), inner
  frame (0 0 -1.5), inner copy (offset 0 0 1, euler 0 0 60 except the spheres), the body's own
  euler (humanoid100.xml:84-147)."""
  m = H.model()
  cols = [((-2, -2, 2.5), (0, 180, 0), (0, 0, 60), (30, 40, 0)),
          ((-1, -2, 2.5), (0, 180, 0), (0, 0, 60), (20, 40, 60)),
          ((0, -2, 3.5), (0, 180, 0), (0, 0, 60), (30, 70, 110)),
          ((1, -2, 2.5), (0, 180, 0), (0, 0, 60), (60, 30, 0)),
          ((2, -2, 2.5), (0, 0, 0), (0, 0, 0), (0, 0, 0))]
  for c, (cpos, oeul, ieul, beul) in enumerate(cols):
    outer = _replicate_frames(5, [0, 1, 0], oeul)
    inner = _replicate_frames(4, [0, 0, 1], ieul)
    for i in range(5):
      for j in range(4):
        b = H.FIRST_OBJECT + 20 * c + 4 * i + j
        _same_pose(m.body_pos[b], m.body_quat[b], *_compose(
            [(np.array(cpos, float), Rotation.identity()), outer[i],
             (np.array([0, 0, -1.5]), Rotation.identity()), inner[j],
             (np.zeros(3), _rot(beul))]), tol=1e-12)


@pytest.mark.skipif(not os.path.isdir(REF), reason="needs the reference sources")
def test_humanoid100_bundle_is_the_compiled_file():
  a = mjcf.load_xml(os.path.join(REF, models.SOURCES["humanoid100"]))
  b = H.model()
  for f in ("body_pos", "body_quat", "geom_size", "geom_pos", "geom_quat", "body_mass"):
    np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)


def test_humanoid100_oracle_decouples_the_trees():
  """With every primitive in the air and apart, the humanoid's forces equal humanoid.xml's
  alone on the same state (its tree shares nothing with the others), and each free body's
  are its Newton-Euler equation: m (a - g) for the translation of a body at rest."""
  from oracle.oracle import Oracle
  m, h = H.model(), models.load("humanoid")
  rng = np.random.default_rng(3)
  q = np.asarray(m.qpos0, dtype=np.float64).ravel().copy()
  q[2] += 0.1                           # humanoid off the floor, below the box column
  q[7:28] += 0.05 * rng.normal(size=21)
  v, a = np.zeros(m.nv), rng.normal(size=m.nv)
  v[:27] = 0.3 * rng.normal(size=27)
  f = Oracle(m).inverse(q, v, a)
  oh = Oracle(h)
  fh = oh.inverse(q[:28], v[:27], a[:27])
  np.testing.assert_allclose(f[:27], fh, rtol=0, atol=1e-10 * max(1, np.abs(fh).max()))
  g = np.array(m.opt["gravity"])
  for k in range(100):
    b, d = H.FIRST_OBJECT + k, 27 + 6 * k
    exp = m.body_mass[b] * (a[d:d + 3] - g)
    np.testing.assert_allclose(f[d:d + 3], exp, rtol=1e-12, atol=1e-12)


def test_humanoid100_device_code_bitexact():
  """The device pipeline compiled for the host (tests/cpu_kernel_harness.cpp, the generic
  kernel's code) on humanoid100 contact states, capped like the GPU test: identical to the
  oracle bit for bit (same operation order, no contraction on either side)."""
  from kernel_harness import KernelCPU
  from oracle.oracle import Oracle
  m = H.model()
  q, v, a = H.states(m, 3, seed=2)
  k = KernelCPU(m, efc_cap=H.MAX_ROWS, con_cap=H.MAX_CONTACTS)
  o = Oracle(m)
  for i in range(3):
    f, st = k.inverse(q[i], v[i], a[i])
    ref = o.inverse(q[i], v[i], a[i])
    assert st == o.d.status == 0
    assert k.field("con_count")[0] == o.efc.ncon > 100
    np.testing.assert_array_equal(f, ref)
