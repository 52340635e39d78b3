"""Generated straight-line kernels (codegen.py), compiled for the host, vs the oracle.

With -ffp-contract=off every mjData output of the generated code must equal the oracle's
BIT FOR BIT, including instances whose limits are active (those take the work-list path
through the generic pipeline).
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import codegen, fields, host, mjcf, models
from mujoco_inversedynamicstest_amd.sampler import sample_contact_states, sample_states
from oracle.oracle import Oracle

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")


def build(m, name):
  src = codegen.generate(m, name)
  h = hashlib.sha1(src.encode())
  # the harness also compiles the device header and the field tables: key the cache on them
  for dep in (os.path.join(HERE, "..", "mujoco_inversedynamicstest_amd", "csrc", "engine_device.h"),
              os.path.join(HERE, "..", "include", "mjhip.h"),
              os.path.join(HERE, "..", "include", "mjhip_fields.h"),
              os.path.join(HERE, "..", "include", "mjhip_contact.h"),
              os.path.join(HERE, "..", "mujoco_inversedynamicstest_amd", "csrc", "post_pass.h"),
              os.path.join(HERE, "..", "mujoco_inversedynamicstest_amd", "csrc", "pair_program.h"),
              os.path.join(HERE, "codegen_harness.cpp")):
    h.update(open(dep, "rb").read())
  tag = h.hexdigest()[:10]
  os.makedirs(BUILD, exist_ok=True)
  inc = os.path.join(BUILD, f"gen_{name}_{tag}.inc")
  so = os.path.join(BUILD, f"libcg_{name}_{tag}.so")
  if not os.path.exists(so):
    # private file names, then an atomic rename (parallel test workers)
    inc = f"{inc}.{os.getpid()}"
    open(inc, "w").write(src)
    tmp = f"{so}.{os.getpid()}"
    subprocess.run(["g++", "-std=c++17", "-O1", "-ffp-contract=off", "-fPIC", "-shared",
                    f'-DGEN_INC="{inc}"', f"-DFAST_BODY=fast_body_{name}", "-o", tmp,
                    os.path.join(HERE, "codegen_harness.cpp")], check=True)
    os.replace(tmp, so)
    os.remove(inc)
  L = ctypes.CDLL(so)
  L.cg_run.restype = ctypes.c_int
  L.cg_run.argtypes = [ctypes.c_void_p, ctypes.c_int] + [ctypes.c_void_p] * 4 + \
      [ctypes.c_int] * 3
  L.cg_set_full_blk.restype = None
  L.cg_set_full_blk.argtypes = [ctypes.c_int]
  return L


def run_and_compare(m, name, q, v, a, full_blk=-1):
  """full_blk >= 0: Mirror::fd_elide set, instance blocks from full_blk on store only what
  mjd_inverseFD's later kernels read (codegen.FD_KEEP and every re-read field); those are
  compared, and the elided fields must stay untouched (zero)."""
  L = build(m, name)
  L.cg_set_full_blk(full_blk)
  o = Oracle(m)
  cm = host.model_struct(m)
  B = len(q)
  sizes = {f.name: f.size(m.sizes) for f in fields.DATA_FIELDS}
  out = np.zeros(sum(sizes.values()) * B)
  q, v, a = (np.ascontiguousarray(x) for x in (q, v, a))
  cmode = codegen.CONSTRAINT_MODES[codegen.constraint_mode(m)]
  con_cap = o.efc.con_capacity if cmode == 2 and o.L.or_contactCapacity(ctypes.byref(cm)) > 0 \
      else 0
  nwl = L.cg_run(ctypes.byref(cm), B, q.ctypes.data, v.ctypes.data, a.ctypes.data,
                 out.ctypes.data, o.efc.capacity, con_cap, cmode)
  res, off = {}, 0
  for f in fields.DATA_FIELDS:
    res[f.name] = out[off:off + B * sizes[f.name]].reshape(B, sizes[f.name])
    off += B * sizes[f.name]
  L.cg_set_full_blk(-1)
  elided = set()
  if full_blk >= 0:
    M = codegen._Model(m)
    elided = codegen.fd_elided(codegen._GEN[st](M, None) for st in codegen.STAGES)
    assert elided and not elided & codegen.FD_KEEP
  nefc = 0
  for i in range(B):
    o.inverse(q[i], v[i], a[i])
    nefc += o.d.nefc > 0
    sunk = full_blk >= 0 and i // 64 >= full_blk
    for f in fields.DATA_FIELDS:
      if f.stage > 0:
        if sunk and f.name in elided:
          assert not res[f.name][i].any(), f"{name}.{f.name} inst {i} stored"
          continue
        np.testing.assert_array_equal(res[f.name][i], getattr(o.d, f.name),
                                      err_msg=f"{name}.{f.name} inst {i}")
  if cmode == 1:
    assert nwl == nefc
  return nwl


def test_humanoid_generated_bitexact(humanoid):
  q, v, a = sample_states(humanoid, 96)
  assert run_and_compare(humanoid, "humanoid", q, v, a) == 0


def test_humanoid_generated_worklist(humanoid):
  q, v, a = sample_states(humanoid, 64, first=5000, margin=-0.1, resample_tendons=False)
  assert run_and_compare(humanoid, "humanoid", q, v, a) > 10


def test_fd_store_elision_bitexact(humanoid):
  """mjd_inverseFD's perturbed instances (Mirror::fd_elide, from block 1 on): the fields a later
  kernel reads -- FD_KEEP and every field a stage re-loads -- equal the oracle's bit for bit,
  limit rows (the work-list's generic constraint part) included, and the elided ones are
  never written to the instance's slot; block 0 (the centres) keeps every field."""
  q, v, a = sample_states(humanoid, 128, first=5000, margin=-0.1, resample_tendons=False)
  assert run_and_compare(humanoid, "humanoid", q, v, a, full_blk=1) > 10


def test_fluid_model_generated_bitexact():
  """Fluid forces after the generated kernels (csrc/post_pass.h): inertia-box and ellipsoid
  models with wind and gravity compensation; every output equals the oracle's bit for bit."""
  from mujoco_inversedynamicstest_amd import mjcf
  m = mjcf.load_xml_string("""<mujoco><option density="1.2" viscosity=".3" wind=".4 -.2 .1">
    <flag contact="disable"/></option><worldbody>
    <body pos="0 0 1" gravcomp=".5"><freejoint/><geom type="box" size=".2 .1 .05"
      fluidshape="ellipsoid" fluidcoef=".4 .3 1.2 .9 1.1"/>
      <body pos="0 .3 0"><joint axis="1 0 0" damping=".2" stiffness="3"/>
        <geom type="capsule" size=".05 .2"/>
        <body pos="0 .3 0"><joint axis="0 1 1"/><geom type="ellipsoid" size=".1 .05 .2"
          fluidshape="ellipsoid"/></body></body></body>
    <body pos="1 0 1"><freejoint/><geom type="box" size=".1 .2 .3"/></body>
    </worldbody></mujoco>""")
  assert codegen.fast_path_supported(m) is None and codegen.constraint_mode(m) == "all"
  q, v, a = sample_states(m, 48, first=2)
  run_and_compare(m, "fluid", q, v, a)


@pytest.mark.parametrize("name", ["inverse_test", "linear", "inertia"])
def test_small_models_generated_bitexact(name):
  # linear.xml has sensors: they run in the sensor pass after the generated kernels
  m = models.load(name, disable_contact=True)
  q, v, a = sample_states(m, 40, first=3)
  run_and_compare(m, name, q, v, a)


def test_generated_all_branches():
  """gravcomp, ball/slide/free joints, tendon spring-damper, cameras/lights of all modes."""
  xml = """<mujoco><option><flag contact="disable"/></option><worldbody>
    <light mode="targetbody" target="b1" pos="1 0 2"/><light mode="track" pos="0 1 2"/>
    <camera mode="targetbodycom" target="b1" pos="2 0 1"/>
    <body name="b1" pos="0 0 1" gravcomp="0.7"><freejoint/><geom size=".1"/>
      <camera mode="track" pos="0 -1 0"/><site pos=".1 0 0" euler="0 30 0"/>
      <body pos=".2 0 0" gravcomp="1"><joint name="a" axis="0 1 0" damping=".3"
          range="-90 90"/>
        <geom type="capsule" fromto="0 0 0 .3 0 0" size=".05"/>
        <body pos=".3 0 0"><joint name="b" type="ball" stiffness="2" pos="0 0 .01"/>
          <geom type="box" size=".05 .1 .02" pos=".1 0 0" euler="10 20 30"/>
          <geom type="sphere" size=".03" pos="0 .05 0"/></body>
        <body pos=".3 0 0"><joint name="c" type="slide" axis="1 1 0" stiffness="3"/>
          <geom size=".04"/></body>
      </body></body></worldbody>
    <tendon><fixed stiffness="5" damping=".2" springlength=".1" range="-1 1">
      <joint joint="a" coef="1"/><joint joint="c" coef="-.5"/></fixed></tendon></mujoco>"""
  m = mjcf.load_xml_string(xml)
  q, v, a = sample_states(m, 40)
  run_and_compare(m, "allbranches", q, v, a)


def test_humanoid_contacts_generated_bitexact():
  """Config 4 (contacts on): the generated kernels run the constraint-free stages of every
  instance and the constraint part (collision, rows, assembly) follows for all of them."""
  m = models.load("humanoid", disable_contact=False)
  assert codegen.constraint_mode(m) == "all"
  q, v, a = sample_contact_states(m, 48, first=9)
  assert run_and_compare(m, "humanoid_contact", q, v, a) == 48


def test_friction_loss_generated_bitexact():
  """Always-active dof friction-loss rows: 'all' mode without contacts."""
  m = models.load("humanoid", disable_contact=True)
  m.dof_frictionloss[6:] = 0.3
  assert codegen.constraint_mode(m) == "all"
  q, v, a = sample_states(m, 32, first=17)
  run_and_compare(m, "humanoid_friction", q, v, a)


def test_generated_with_equality_constraints():
  """Active equality constraints put every instance through the constraint kernel
  (constraint_mode 'all'): connect, weld (body and site semantics), joint and tendon."""
  xml = """<mujoco><option><flag contact="disable"/></option><worldbody>
    <site name="w" pos=".3 .1 1" euler="10 0 0"/>
    <body name="a" pos="0 0 1"><freejoint/><geom type="box" size=".1 .2 .05"/>
      <site name="as" pos=".1 0 0"/>
      <body name="b" pos=".2 0 0"><joint name="h1" axis="0 1 0"/>
        <geom type="capsule" fromto="0 0 0 .3 0 0" size=".04"/>
        <body name="c" pos=".3 0 0"><joint name="h2" axis="0 0 1"/>
          <geom type="sphere" size=".05"/></body></body></body>
    <body name="d" pos="1 0 1"><joint name="s" type="slide" axis="0 0 1"/>
      <geom size=".1"/></body></worldbody>
    <tendon><fixed name="t"><joint joint="h1" coef="1"/><joint joint="s" coef="-1"/></fixed>
    </tendon>
    <equality><connect body1="c" body2="d" anchor=".05 0 0"/>
      <weld body1="a" torquescale=".3"/><weld site1="w" site2="as" solref=".03 1"/>
      <joint joint1="h1" joint2="h2" polycoef="0 .5 0 0 0"/>
      <tendon tendon1="t" polycoef=".01"/></equality></mujoco>"""
  m = mjcf.load_xml_string(xml)
  assert codegen.constraint_mode(m) == "all"
  q, v, a = sample_states(m, 16, first=3)
  run_and_compare(m, "equality", q, v, a)


def test_generated_tendon_transmissions():
  """Fixed-tendon transmissions on the straight-line path: length gear*ten_length, the
  model-constant moment row gear*coef, actuator_velocity by mju_dotSparse over the row;
  a zero coefficient drops its column."""
  xml = """<mujoco><option><flag contact="disable"/></option><worldbody>
    <body pos="0 0 1"><joint name="a" axis="0 1 0" range="-60 60"/>
      <geom type="capsule" fromto="0 0 0 .3 0 0" size=".05"/>
      <body pos=".3 0 0"><joint name="b" axis="0 0 1"/><geom size=".05"/>
        <body pos=".1 0 0"><joint name="c" type="slide" axis="1 0 0"/><geom size=".03"/>
        </body></body></body></worldbody>
    <tendon><fixed name="t1" limited="true" range="-.5 .6"><joint joint="a" coef="1.5"/>
      <joint joint="c" coef="-.25"/></fixed>
      <fixed name="t2"><joint joint="b" coef="0"/><joint joint="c" coef="2"/>
      <joint joint="a" coef=".5"/></fixed></tendon>
    <actuator><motor tendon="t1" gear="3"/><motor joint="b"/><motor tendon="t2" gear="-.7"/>
    </actuator></mujoco>"""
  m = mjcf.load_xml_string(xml)
  assert codegen.fast_path_supported(m) is None
  q, v, a = sample_states(m, 48, margin=-0.2)
  run_and_compare(m, "tendontrn", q, v, a)


MIXED_TENDONS = """<mujoco><option density="1.1" viscosity=".2"/><worldbody>
  <geom type="plane" size="3 3 .1" pos="0 0 1"/><site name="top" pos="0 0 2"/>
  <body pos="0 0 1" gravcomp=".4"><freejoint/><geom type="box" size=".1 .1 .05"/>
    <site name="s0" pos=".1 0 .05"/>
    <body pos=".1 0 0"><joint name="h1" axis="0 1 0" range="-80 80"/>
      <geom name="ball" type="sphere" size=".06"/><site name="side" pos="0 0 .1"/>
      <geom type="capsule" fromto="0 0 0 .3 0 0" size=".03"/><site name="s1" pos=".25 0 .06"/>
      <body pos=".3 0 0"><joint name="h2" axis="0 0 1" damping=".1"/>
        <geom type="capsule" fromto="0 0 0 .3 0 0" size=".03"/>
        <site name="s2" pos=".3 0 -.04"/></body></body></body>
  </worldbody>
  <tendon>
    <fixed name="fx" stiffness="4" damping=".2" limited="true" range="-.6 .6">
      <joint joint="h1" coef="1"/><joint joint="h2" coef="-.5"/></fixed>
    <spatial name="sp" limited="true" range=".2 .9" stiffness="3" damping=".3"
        frictionloss=".05">
      <site site="top"/><site site="s0"/><geom geom="ball" sidesite="side"/>
      <site site="s1"/><pulley divisor="2"/><site site="s1"/><site site="s2"/></spatial>
  </tendon>
  <actuator><motor tendon="fx" gear="2"/><motor name="asp" tendon="sp" gear="-1.5"/>
    <motor joint="h2"/></actuator>
  <sensor><tendonpos tendon="sp"/><tendonvel tendon="sp"/><actuatorpos actuator="asp"/>
    <actuatorvel actuator="asp"/><tendonpos tendon="fx"/></sensor></mujoco>"""


@pytest.mark.parametrize("which", ["arm", "wrap", "mixed"])
def test_spatial_tendons_generated_bitexact(which):
  """Spatial tendons on the straight-line path: the generated kernel leaves their length,
  Jacobian, velocity, transmissions and mj_passive to the tendon pass (csrc/post_pass.h),
  which runs before the constraint kernel serves every instance. Sites and pulleys (ARM),
  sphere and cylinder wrapping (WRAP), and a model mixing a fixed and a spatial tendon with
  limits, friction loss, contacts, fluid, gravity compensation and tendon sensors: every
  output equals the oracle's bit for bit."""
  from test_tendon_cpu import ARM, WRAP
  m = mjcf.load_xml_string({"arm": ARM, "wrap": WRAP, "mixed": MIXED_TENDONS}[which])
  assert codegen.fast_path_supported(m) is None and codegen.constraint_mode(m) == "all"
  assert codegen.spatial_tendons(m)
  q, v, a = sample_states(m, 48, first=3, margin=-0.1)
  assert run_and_compare(m, f"spatial_{which}", q, v, a) == 48


@pytest.mark.parametrize("integrator", [0, 2, 3])
def test_invdiscrete_generated_bitexact(integrator):
  """mjENBL_INVDISCRETE on the straight-line path: the generated kernel, then the discrete
  pass (mj_discreteAcc and mj_rne over its qacc, csrc/post_pass.h), the unfused constraint
  kernel for every instance, the sensor pass on the discrete qacc, and qacc restored.
  Euler (implicit damping), implicit and implicitfast on the humanoid with dof damping,
  contacts and acceleration sensors: every output equals the oracle's bit for bit."""
  m = models.load("humanoid", disable_contact=False)
  m.opt["enableflags"] |= 1 << 3
  m.opt["integrator"] = integrator
  assert codegen.fast_path_supported(m) is None and codegen.constraint_mode(m) == "all"
  q, v, a = sample_contact_states(m, 24, first=5)
  run_and_compare(m, f"invdiscrete{integrator}", q, v, a)


def test_invdiscrete_generated_sensors_tendons():
  """INVDISCRETE (implicitfast: actuator, dof and tendon damping derivatives) with a spatial
  tendon pass before it and acceleration sensors after it."""
  xml = MIXED_TENDONS.replace('<option density="1.1" viscosity=".2"/>',
                              '<option timestep=".01" integrator="implicitfast">'
                              '<flag invdiscrete="enable"/></option>')
  xml = xml.replace('<tendonpos tendon="fx"/>', '<tendonpos tendon="fx"/>'
                    '<accelerometer site="s1"/><framelinacc objtype="site" objname="s2"/>')
  xml = xml.replace('<motor joint="h2"/>', '<velocity joint="h2" kv="2"/>')
  m = mjcf.load_xml_string(xml)
  assert codegen.fast_path_supported(m) is None
  q, v, a = sample_states(m, 32, first=7, margin=-0.1)
  run_and_compare(m, "invdiscrete_tendons", q, v, a)


def test_generated_then_sensor_pass():
  """Sensor models on the straight-line path: every supported sensor type (limit and
  contact rows active) computed by the sensor pass after the generated kernels and the
  constraint part equals the oracle bit for bit."""
  import sys
  sys.path.insert(0, HERE)
  from test_sensors_cpu import _all_model
  m = _all_model()
  assert codegen.fast_path_supported(m) is None
  q, v, a = sample_states(m, 32, first=11, margin=-0.3, resample_tendons=False)
  run_and_compare(m, "allsensors", q, v, a)


def test_generated_ball_free_transmissions():
  """Ball and free-joint transmissions, in the joint and the parent frame, on the
  straight-line path (the model of tests/test_transmission_cpu.py)."""
  import sys
  sys.path.insert(0, HERE)
  import re
  from test_transmission_cpu import XML
  m = mjcf.load_xml_string(re.sub(r'<general site="tip"[^>]*/>', "", XML))   # site: generic
  assert codegen.fast_path_supported(m) is None
  assert set(int(t) for t in m.actuator_trntype) >= {0, 1}
  q, v, a = sample_states(m, 40, first=5)
  run_and_compare(m, "ballfree", q, v, a)


def test_generated_with_energy():
  """mjENBL_ENERGY on the straight-line path: mj_energyPos/Vel in the pass after the
  generated kernels (the humanoid, limits active on some instances); every mirror output
  here, the energy values themselves on the GPU (test_gpu.py::test_energy_parity)."""
  m = models.load("humanoid", disable_contact=True)
  m.opt["enableflags"] |= 1 << 1
  assert codegen.fast_path_supported(m) is None
  q, v, a = sample_states(m, 32, first=500, margin=-0.1, resample_tendons=False)
  run_and_compare(m, "humanoid_energy", q, v, a)


def test_generated_site_slidercrank_body_transmissions():
  """Slider-crank, site (with and without a reference site) and body (adhesion)
  transmissions on the straight-line path: the generated kernels skip them and
  mjh::transmissionAfter computes them (and their actuator_velocity) after the constraint
  part, the body ones from the instance's contacts. Every output equals the oracle's; the
  slider-crank model (BASELINE.json config 1) also exercises its capsule-cylinder pair."""
  import sys
  sys.path.insert(0, HERE)
  from test_transmission_cpu import ADHESION, REFSITE, XML
  m = mjcf.load_xml_string(XML)
  assert codegen.fast_path_supported(m) is None and 4 in set(int(t) for t in m.actuator_trntype)
  q, v, a = sample_states(m, 40, first=9)
  run_and_compare(m, "sitetrn", q, v, a)
  m = mjcf.load_xml_string(REFSITE)
  rng = np.random.default_rng(8)
  q, v, a = rng.uniform(-1, 1, (24, m.nq)), rng.normal(size=(24, m.nv)), rng.normal(size=(24, m.nv))
  run_and_compare(m, "refsite", q, v, a)
  m = models.load("slider_crank")
  assert codegen.fast_path_supported(m) is None and codegen.constraint_mode(m) == "all"
  rng = np.random.default_rng(11)
  q = rng.uniform(-np.pi, np.pi, (64, m.nq))
  run_and_compare(m, "slider_crank", q, rng.normal(size=(64, m.nv)), rng.normal(size=(64, m.nv)))
  m = mjcf.load_xml_string(ADHESION.format(cone="pyramidal", condim=3, margin=0.01, gap=0.005,
                                           z=0.1))
  q = np.tile(m.qpos0, (32, 1))
  q[:, 2] = 0.1 + 0.03 * rng.normal(size=32)
  q[:, 7:9] = q[:, 0:2] + rng.uniform(-0.4, 0.4, (32, 2))
  q[:, 9] = 0.1 + 0.05 * rng.normal(size=32)
  run_and_compare(m, "adhesion", q, rng.normal(size=(32, m.nv)), rng.normal(size=(32, m.nv)))


# slider-crank and site transmissions (left by the generated kernels to the pass after the
# constraint kernel), damped so that mj_discreteAcc's implicit integrators read their moments
TRN_AFTER_XML = """<mujoco><option integrator="{integ}"><flag invdiscrete="enable" contact="disable"/>
  </option><worldbody>
  <body name="crank"><joint name="c" axis="0 1 0" damping=".1"/>
    <geom type="capsule" fromto="0 0 0 .2 0 0" size=".02"/><site name="pin" pos=".2 0 0"/></body>
  <body name="slider" pos=".5 0 0"><joint name="s" type="slide" axis="1 0 0" damping=".2"/>
    <geom type="box" size=".05 .05 .05"/><site name="slide" zaxis="1 0 0"/></body>
  <body name="arm" pos="0 0 .5"><joint name="a" axis="1 0 0" damping=".05"/>
    <geom type="capsule" fromto="0 0 0 0 .2 0" size=".03"/>
    <site name="tip" pos="0 .2 0"/><site name="ref" pos="0 0 .1"/></body>
  </worldbody><actuator>
  <general cranksite="pin" slidersite="slide" cranklength=".45" biastype="affine"
           biasprm="0 0 -0.5"/>
  <velocity site="tip" gear="0 0 1 0 0 0" kv="0.7"/>
  <general site="tip" refsite="ref" gear="0 1 0 0 0 0" gaintype="affine" gainprm="1 0 0.3"/>
  </actuator></mujoco>"""


@pytest.mark.parametrize("integ", ["Euler", "implicit", "implicitfast"])
def test_invdiscrete_trn_after_generated_bitexact(integ):
  """INVDISCRETE with slider-crank and site transmissions on the straight-line path: the
  discrete pass forms those transmissions first (k_discrete_before; the reference has them
  from mj_fwdPosition before mj_discreteAcc), so the implicit damping reads their moments;
  every output equals the oracle's bit for bit."""
  m = mjcf.load_xml_string(TRN_AFTER_XML.format(integ=integ))
  assert codegen.fast_path_supported(m) is None
  assert any(int(t) in codegen.TRN_AFTER for t in m.actuator_trntype[:m.nu])
  rng = np.random.default_rng(12)
  B = 48
  q = rng.uniform(-1, 1, (B, m.nq)) * 0.5
  v, a = rng.normal(size=(B, m.nv)), rng.normal(size=(B, m.nv))
  run_and_compare(m, f"trn_after_{integ}", q, v, a)
