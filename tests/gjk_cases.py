"""The reference's own known answers for the native GJK/EPA solver mjc_ccd
(test/engine/engine_collision_gjk_test.cc, MjGjkTest), restated as data: each case's model,
the geom frames the test overrides after mj_forward, the call (the test file's GeomDist
helper, :62-84, or its Penetration helper, :86-150) and the expected values at the test's
tolerance. Test data only: the expected numbers are the ones that file asserts.

Shared by tests/test_gjk_kat_cpu.py (oracle and the device code compiled for the host) and
tests/test_gjk_kat_gpu.py (mjhip_ccdBatch on the device).

The helpers' config (:43-44, :65-71, :123-131): max_iterations 1000 (kMaxIterations),
tolerance 1e-6 (kTolerance); GeomDist: margin 0, max_contacts 0, dist_cutoff (default
mjMAXVAL); Penetration: object margin `margin` on both geoms, max_contacts 1, dist_cutoff 0,
and the reported contact is dir = normalize(x1 - x2), pos = (x1 + x2) / 2 when dist < 0.
"""
import numpy as np

KTOL = 1e-6            # kTolerance (:43)
KMAX = 1000            # kMaxIterations (:44)
MAXVAL = 1e10          # mjMAXVAL

# kEllipoid (:45-60)
ELLIPSOID = """<mujoco model="Ellipsoid Test">
  <compiler angle="radian"/>
  <size nkey="1"/>
  <worldbody>
    <geom name="geom1" size="0.1 0.1 0.1" pos="0 0 -0.1" type="ellipsoid"/>
    <body pos="0 0 0.1">
      <joint type="free" limited="false"/>
      <geom name="geom2" size="0.01 0.02 0.1" type="ellipsoid"/>
    </body>
  </worldbody>
  <keyframe>
    <key time="1.446"
      qpos="0.000886189 -0.0303047 0.0951303 0.98783 0.155468 0.00454524 1.60038e-06"
      qvel="0.00769267 -0.258656 -0.0775641 2.73712 0.0813998 -0.000166485"/>
  </keyframe>
</mujoco>"""

SPHERES = """<mujoco><worldbody>
  <geom name="geom1" type="sphere" pos="-1.5 0 0" size="1"/>
  <geom name="geom2" type="sphere" pos="1.5 0 0" size="1"/>
</worldbody></mujoco>"""

BOX_MESHES = """<mujoco><asset>
  <mesh name="box" scale=".5 .5 .1" vertex="-1 -1 -1  1 -1 -1  1 1 -1  1 1 1  1 -1 1
        -1 1 -1  -1 1 1  -1 -1 1"/>
  <mesh name="smallbox" scale=".1 .1 .1" vertex="-1 -1 -1  1 -1 -1  1 1 -1  1 1 1  1 -1 1
        -1 1 -1  -1 1 1  -1 -1 1"/></asset>
  <worldbody>
    <geom name="geom2" pos="0 0 .1" size=".1 .1 .1" type="mesh" mesh="smallbox"/>
    <geom name="geom1" pos="0 0 -.099999999" size=".5 .5 .1" type="mesh" mesh="box"/>
  </worldbody></mujoco>"""

ELLIPSOIDS = """<mujoco><worldbody>
  <geom name="geom1" type="ellipsoid" pos="1.5 0 -.5" size=".15 .30 .20"/>
  <geom name="geom2" type="ellipsoid" pos="1.5 .5 .5" size=".10 .10 .15"/>
</worldbody></mujoco>"""

LONG_BOX = """<mujoco><asset>
  <mesh name="long_box" vertex="-1 -1 -1 1 -1 -1 1 1 -1 1 1 1 1 -1 1 -1 1 -1 -1 1 1 -1 -1 1"
        scale=".6 .03 .03"/></asset>
  <worldbody>
    <geom name="geom1" type="box" size="1 1 .3" pos="0 0 -.3"/>
    <geom name="geom2" type="mesh" mesh="long_box" pos="0 0 .02" euler="0 0 40"/>
  </worldbody></mujoco>"""


def _boxes(size1, pos1, size2, pos2):
  return (f'<mujoco><worldbody><geom name="geom1" type="box" pos="{pos1}" size="{size1}"/>'
          f'<geom name="geom2" type="box" pos="{pos2}" size="{size2}"/></worldbody></mujoco>')


# BoxBoxDepth2 (:318-332): geom 1's frame after mj_forward
DEPTH2_FRAMES = {1: ([-0.000171208577507291721461757383, -0.000171208577507290908310128019,
                      1.067119586248553853025100579544],
                     [0.999999966039443077825410455262, -0.000000033960556969622165789148,
                      -0.000260616790777324182967061850, -0.000000033960556972087627235699,
                      0.999999966039443077825410455262, -0.000260616790777321797722282382,
                      0.000260616790777324182967061850, 0.000260616790777321797722282382,
                      0.999999932078886044628518448008])}

# BoxBoxDepth3 (:368-404): both frames
DEPTH3_FRAMES = {0: ([-0.015346499999999199323474918799, -0.023505500000000002086553152481,
                      -4.562296442400120888294168253196],
                     [0.965925826289068201191412299522, -0.258819045102520739476403832668,
                      0.000000000000000006339100926609, 0.258819045102520739476403832668,
                      0.965925826289068201191412299522, -0.000000000000000214827792362716,
                      0.000000000000000049478422780336, 0.000000000000000209148392896446,
                      1.000000000000000000000000000000]),
                 1: ([-0.015346499999999797803074130798, -0.023505499999999998617106200527,
                      -4.659230360891631228525966434972],
                     [0.866025403784438707610604524234, -0.499999999999999944488848768742,
                      0.000000000000000018716705841316, 0.499999999999999944488848768742,
                      0.866025403784438707610604524234, -0.000000000000000263161736875730,
                      0.000000000000000115371725704125, 0.000000000000000237263102359077,
                      1.000000000000000000000000000000])}

# name, model, key (keyframe index or None), frame overrides, call, geoms (by name), kwargs,
# expected. call "dist": GeomDist -> checks on dist (and x1/x2); "pen": Penetration -> checks
# on ncon, dist, dir, pos. Expected entries: ("eq", value) is EXPECT_EQ, ("near", value, tol)
# is EXPECT_NEAR; "x1"/"x2"/"dir"/"pos" take 3-vectors; "abspos0" is |pos[0]|; "if1" applies
# the checks only when ncon == 1 (BoxBoxDepth2's `if (ncons == 1)`).
CASES = [
    ("SphereSphereDist", SPHERES, None, {}, "dist", ("geom1", "geom2"), {},     # :155-181
     {"dist": ("eq", 1.0), "x1": ("eq", [-.5, 0, 0]), "x2": ("eq", [.5, 0, 0])}),
    ("SphereSphereDistCutoff", SPHERES, None, {}, "dist", ("geom1", "geom2"),   # :183-206
     {"cutoff": .999999}, {"dist": ("eq", MAXVAL)}),
    ("SphereSphereNoDist", SPHERES, None, {}, "pen", ("geom1", "geom2"), {},    # :208-233
     {"ncon": ("eq", 0)}),
    ("SphereSphereIntersect",                                                   # :235-274
     SPHERES.replace('pos="-1.5 0 0" size="1"', 'pos="-1 0 0" size="3"')
            .replace('pos="1.5 0 0" size="1"', 'pos="3 0 0" size="3"'),
     None, {}, "pen", ("geom1", "geom2"), {},
     {"ncon": ("eq", 1), "dist": ("near", -2, KTOL), "dir": ("near", [1, 0, 0], KTOL),
      "pos": ("near", [1, 0, 0], KTOL)}),
    ("BoxBoxDepth", _boxes("2.5 2.5 2.5", "-1 0 0", "1 1 1", "1.5 0 0"), None, {},  # :276-308
     "pen", ("geom1", "geom2"), {},
     {"ncon": ("eq", 1), "dist": ("near", -1, KTOL), "dir": ("near", [1, 0, 0], KTOL)}),
    ("BoxBoxDepth2", _boxes("5 5 .1", "0 0 0", "1 1 1", "0 0 0"), None, DEPTH2_FRAMES,  # :310-358
     "pen", ("geom1", "geom2"), {},
     {"if1": True, "dist": ("near", -0.033401579411886845, KTOL),
      "dir": ("near", [0, 0, 1], KTOL)}),
    ("BoxBoxDepth3", _boxes("0.25 0.25 0.05", "0 0 0", "0.25 0.25 0.05", "0 0 0"), None,  # :360-424
     DEPTH3_FRAMES, "pen", ("geom1", "geom2"), {},
     {"ncon": ("eq", 1), "dist": ("near", -0.003066, KTOL), "dir": ("near", [0, 0, -1], KTOL)}),
    ("BoxBoxTouching", _boxes("1 1 1", "0 0 1.859913200000001376466229885409", "1 1 1",  # :426-452
                              "0 2 1.859913200000001376466229885409"), None, {}, "pen",
     ("geom1", "geom2"), {}, {"ncon": ("eq", 0)}),
    ("SmallBoxMesh", BOX_MESHES, None, {}, "pen", ("geom1", "geom2"), {},       # :942-999
     {"ncon": ("eq", 1), "dist": ("near", 0, KTOL), "dir": ("near", [0, 0, 1], KTOL),
      "abspos0": ("near", 0.08333333, KTOL), "pos12": ("near", [0, 0], KTOL)}),
    ("EllipsoidEllipsoidPenetrating", ELLIPSOID, 0, {}, "pen", ("geom1", "geom2"), {},  # :1401-1420
     {"ncon": ("eq", 1), "dist": ("near", -0.00022548856248122027, KTOL)}),
    ("EllipsoidEllipsoid", ELLIPSOIDS, None, {}, "dist", ("geom1", "geom2"), {},  # :1422-1445
     {"dist": ("near", 0.7542, 1e-4)}),
    ("BoxBox", _boxes("1 1 1", "-1.5 .5 0", "1 1 1", "1.5 0 0"), None, {}, "dist",  # :1447-1470
     ("geom1", "geom2"), {}, {"dist": ("eq", 1.0)}),
    ("LongBox", LONG_BOX, None, {}, "pen", ("geom1", "geom2"), {},              # :1472-1516
     {"ncon": ("eq", 1), "dist": ("near", -0.01, KTOL), "dir": ("near", [0, 0, 1], KTOL),
      "pos": ("near", [0, 0, -0.005], KTOL)}),
    ("EllipsoidEllipsoidIntersect", ELLIPSOIDS, None, {}, "pen", ("geom1", "geom2"),  # :1518-1544
     {"margin": 15}, {"ncon": ("eq", 1), "dist": ("near", -14.245732934582151, KTOL)}),
    ("CapsuleCapsule",                                                          # :1546-1569
     """<mujoco><worldbody>
       <geom name="geom1" type="capsule" pos="-.3 .2 -.4" size=".15 .30"/>
       <geom name="geom2" type="capsule" pos=".3 .2 .4" size=".10 .10"/>
     </worldbody></mujoco>""", None, {}, "dist", ("geom1", "geom2"), {},
     {"dist": ("near", 0.4711, 1e-4)}),
]

# CylinderBoxMargin (:1571-1600) is a whole-pipeline case: mj_forward on this model gives one
# contact whose efc_address is negative (its distance lies between margin - gap and margin).
CYLINDER_BOX_MARGIN = """<mujoco>
  <option><flag gravity="disable"/></option>
  <worldbody>
    <body pos="0 0 .265"><freejoint/>
      <geom type="box" size=".05 .05 .05" margin="0.1" gap="0.1"/></body>
    <body mocap="true"><geom name="geom2" type="cylinder" size=".2 .2"/></body>
  </worldbody></mujoco>"""


def frames(m, oracle, key, overrides):
  """geom_xpos [ngeom, 3], geom_xmat [ngeom, 9] after mj_forward (the oracle's kinematics at
  qpos0 or the keyframe), then the test's overrides (geom id -> (pos, mat))."""
  q = m.qpos0 if key is None else m.key_qpos.reshape(-1, m.nq)[key]
  oracle.inverse(q, np.zeros(m.nv), np.zeros(m.nv))
  xpos = oracle.d.geom_xpos.reshape(-1, 3).copy()
  xmat = oracle.d.geom_xmat.reshape(-1, 9).copy()
  for g, (p, r) in overrides.items():
    xpos[g] = p
    xmat[g] = r
  return xpos, xmat


def call_args(call, kw):
  """(margin, max_contacts, cutoff) of the helper the case calls."""
  if call == "dist":
    return 0.0, 0, kw.get("cutoff", MAXVAL)
  return float(kw.get("margin", 0.0)), 1, 0.0


def report(call, dist, nx, x1, x2):
  """What the helper returns: GeomDist -> {dist, x1, x2 (when nx > 0)}; Penetration ->
  {ncon, dist, dir, pos} (engine_collision_gjk_test.cc:77-82, :134-146)."""
  if call == "dist":
    r = {"dist": dist}
    if nx > 0:
      r["x1"], r["x2"] = np.asarray(x1), np.asarray(x2)
    return r
  if not dist < 0:
    return {"ncon": 0}
  d = np.asarray(x1) - np.asarray(x2)
  d = d / np.sqrt(d @ d)
  pos = 0.5 * (np.asarray(x1) + np.asarray(x2))
  return {"ncon": nx, "dist": dist, "dir": d, "pos": pos}


def check(name, expected, got):
  """The case's EXPECT_* lines on a helper report; raises AssertionError naming the case."""
  if expected.get("if1") and got.get("ncon") != 1:
    return
  for k, e in expected.items():
    if k == "if1":
      continue
    if k == "abspos0":
      val = abs(got["pos"][0])
    elif k == "pos12":
      val = got["pos"][1:]
    else:
      assert k in got, f"{name}: helper reported no {k} ({got})"
      val = got[k]
    if e[0] == "eq":
      assert np.array_equal(np.asarray(val, dtype=float), np.asarray(e[1], dtype=float)), \
          f"{name}: {k} = {val}, expected exactly {e[1]}"
    else:
      assert np.all(np.abs(np.asarray(val, dtype=float) - np.asarray(e[1])) <= e[2]), \
          f"{name}: {k} = {val}, expected {e[1]} +- {e[2]}"
