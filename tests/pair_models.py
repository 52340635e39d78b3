"""Models with predefined <contact><pair> elements and their states (test data).

COLLISIONS has the structure of the reference's collision-driver test model
(test/engine/testdata/collisions.xml used by engine_collision_driver_test.cc:52-67): a box,
a sphere that touches it, a sphere that touches it only through a predefined pair's geoms, a
sphere within bounding-sphere reach but not touching, a far sphere, and an excluded body.

MIXED exercises every rule of the merge (engine_collision_driver.c:316-327, :432-437,
mj_collideGeomPair :499-523, mj_collideGeoms :1440-1632):
* the floor has contype = conaffinity = 0, so it touches nothing except through pairs (no
  bitmask filter for a predefined pair);
* pairs from the default class (solreffriction) and from a child class (solref, condim,
  friction, margin, gap);
* a pair between bodies whose body pair is excluded (pairs are merged before the filters);
* a pair whose geoms the body-pair sweep would also test (left to the pair: condim 6 there);
* a body with two geoms (the midphase sort of the dynamic contacts after the merged pairs);
* plane-box (up to 4 contacts) and plane-capsule through a pair, elliptic cones.
"""
import numpy as np

from mujoco_inversedynamicstest_amd import mjcf

COLLISIONS = """<mujoco model="collisions"><worldbody>
  <body name="box"><geom name="box" type="box" size="1 1 1"/></body>
  <body pos="1.2 1.2 0.0"><joint/><geom name="sphere_collides" type="sphere" size="1"/></body>
  <body pos="-0.9 -0.9 0.0"><joint/><geom name="sphere_predefined" type="sphere" size="0.1"/>
  </body>
  <body pos="1.8 -1.8 0.0"><joint/><geom name="sphere_narrowphase" type="sphere" size="1"/>
  </body>
  <body pos="-2.1 -2.1 0.0"><joint/><geom name="sphere_broadphase" type="sphere" size="1"/>
  </body>
  <body name="sphere_excluded"><joint/>
    <geom name="sphere_excluded" type="sphere" pos="0 0 0" size="0.2"/></body>
</worldbody><contact>
  <exclude body1="box" body2="sphere_excluded"/>
  <pair geom1="box" geom2="sphere_predefined"/>
</contact></mujoco>"""

MIXED = """<mujoco model="pairs"><option cone="elliptic" impratio="2"/>
<default>
  <pair solreffriction=".04 1"/>
  <default class="soft">
    <pair solref=".05 1.2" condim="4" friction=".7 .7 .01 .001 .001" margin=".02" gap=".005"/>
  </default>
</default>
<worldbody>
  <geom name="floor" type="plane" size="3 3 .1" contype="0" conaffinity="0"/>
  <body name="a" pos="0 0 .1"><freejoint/><geom name="ball" size=".1"/></body>
  <body name="b" pos=".3 0 .1"><freejoint/>
    <geom name="cap" type="capsule" fromto="-.1 0 0 .1 0 0" size=".1"/>
    <geom name="box" type="box" size=".05 .05 .05" pos="-.12 .08 -.05"/></body>
  <body name="c" pos="-.21 0 .1"><freejoint/><geom name="ball2" size=".1"/></body>
</worldbody>
<contact>
  <exclude body1="a" body2="c"/>
  <pair geom1="ball" geom2="floor"/>
  <pair geom1="floor" geom2="cap" class="soft"/>
  <pair geom1="ball2" geom2="ball" condim="1"/>
  <pair geom1="cap" geom2="ball" condim="6" friction="1 1 .02 .002 .002"/>
  <pair geom1="box" geom2="floor" margin=".01"/>
</contact></mujoco>"""


def collisions():
  return mjcf.load_xml_string(COLLISIONS)


def mixed():
  return mjcf.load_xml_string(MIXED)


def mixed_states(m, n, seed=0):
  """Three free bodies resting near the floor and each other: heights, lateral offsets and
  tilts jittered so that every pair touches in some states and not in others."""
  rng = np.random.default_rng(seed)
  q = np.tile(m.qpos0, (n, 1))
  for b, x0 in enumerate((0.0, 0.3, -0.21)):
    q[:, 7*b] = x0 + rng.uniform(-0.04, 0.04, n)
    q[:, 7*b + 1] = rng.uniform(-0.03, 0.03, n)
    q[:, 7*b + 2] = 0.1 + rng.uniform(-0.02, 0.03, n)
    quat = np.array([1.0, 0, 0, 0]) + 0.15 * rng.normal(size=(n, 4))
    q[:, 7*b + 3:7*b + 7] = quat / np.linalg.norm(quat, axis=1, keepdims=True)
  v = 0.5 * rng.normal(size=(n, m.nv))
  a = 3.0 * rng.normal(size=(n, m.nv))
  return q, v, a
