""".mjb model files (mjb.py): the reference's binary layout, read and written.

  * round trip: every bundled model -> mjb.write -> mjb.read equals the model field for field
    (and by model signature, so the engine selects the same kernel)
  * header and consistency checks with mj_loadModelBuffer's messages (engine_io.c:776-890)
  * models outside the device subset are refused
  * the layout table and struct sizes against the reference headers (only where
    /root/reference exists: this container, never the GPU box)
"""
import os
import re
import struct
import subprocess

import numpy as np
import pytest

from mujoco_inversedynamicstest_amd import engine, fields, mjb, mjcf, models

REF = "/root/reference"
BUNDLED = ["humanoid", "slider_crank", "inverse_test", "inertia", "linear", "weld", "connect",
           "equality_site", "equality_compare"]


@pytest.mark.parametrize("name", BUNDLED)
def test_round_trip(name, tmp_path):
  m = models.load(name)
  path = tmp_path / f"{name}.mjb"
  mjb.save(m, str(path))
  r = mjb.load(str(path))
  for f in fields.MODEL_FIELDS:
    a, b = getattr(m, f.name), getattr(r, f.name)
    assert a.shape == b.shape and a.dtype == b.dtype, f.name
    np.testing.assert_array_equal(a, b, err_msg=f.name)
  assert r.sizes == m.sizes
  assert r.names == m.names
  for k, v in m.opt.items():
    assert r.opt[k] == v, k
  assert fields.model_signature(r) == fields.model_signature(m)


def test_header_and_sizes(humanoid):
  buf = mjb.write(humanoid)
  hdr = struct.unpack_from("<5i", buf, 0)
  assert hdr == (54321, 8, 83, 2, 399)
  ints = dict(zip(mjb.INTS, struct.unpack_from("<83i", buf, 20)))
  narena, nbuffer = struct.unpack_from("<2Q", buf, 20 + 4 * 83)
  assert nbuffer == mjb.buffer_size(ints)
  assert ints["nq"] == 28 and ints["nv"] == 27 and ints["nM"] == 243 and ints["nbody"] == 17
  assert len(buf) == mjb.offsets(ints)["__end__"]


def _patch(buf, offset, fmt, *vals):
  b = bytearray(buf)
  struct.pack_into(fmt, b, offset, *vals)
  return bytes(b)


@pytest.mark.parametrize("idx,msg", [
    (0, "Model missing header ID"),
    (1, "different floating point precision"),
    (2, "different number of ints"),
    (3, "different number of size_t"),
    (4, "different number of pointers")])
def test_header_checks(humanoid, idx, msg):
  buf = mjb.write(humanoid)
  hdr = list(struct.unpack_from("<5i", buf, 0))
  hdr[idx] += 1
  with pytest.raises(mjb.MJBError, match=msg):
    mjb.read(_patch(buf, 0, "<5i", *hdr))


def test_truncation_and_size_checks(humanoid):
  buf = mjb.write(humanoid)
  with pytest.raises(mjb.MJBError, match="incomplete header"):
    mjb.read(buf[:12])
  with pytest.raises(mjb.MJBError, match="while reading sizes"):
    mjb.read(buf[:40])
  with pytest.raises(mjb.MJBError, match="while reading structs"):
    mjb.read(buf[:20 + 4 * 83 + 16 + 100])
  ints = dict(zip(mjb.INTS, struct.unpack_from("<83i", buf, 20)))
  off = mjb.offsets(ints)
  with pytest.raises(mjb.MJBError, match="while reading body_mass"):
    mjb.read(buf[:off["body_mass"] + 8])
  with pytest.raises(mjb.MJBError, match="too large"):
    mjb.read(buf + b"\0")
  nb = struct.unpack_from("<Q", buf, 20 + 4 * 83 + 8)[0]
  with pytest.raises(mjb.MJBError, match="wrong size parameters"):
    mjb.read(_patch(buf, 20 + 4 * 83 + 8, "<Q", nb + 64))


def test_options_survive(humanoid):
  m = models.load("humanoid", disable_contact=True)
  r = mjb.read(mjb.write(m))
  assert r.opt["disableflags"] == m.opt["disableflags"] != 0
  assert r.opt["timestep"] == m.opt["timestep"]
  assert r.opt["iterations"] == 100          # mj_defaultOption for members the loader skips


def test_ellipsoid_fluid_survives():
  """geom_fluid (the ellipsoid fluid model's 12 coefficients per geom) round-trips."""
  m = mjcf.load_xml_string("""<mujoco><option density="1.2" viscosity=".1"/><worldbody>
    <body><freejoint/><geom type="box" size=".2 .1 .05" fluidshape="ellipsoid"/>
    <geom type="sphere" size=".1" pos=".3 0 0"/></body></worldbody></mujoco>""")
  r = mjb.read(mjb.write(m))
  assert m.geom_fluid[0, 0] == 1 and m.geom_fluid[1, 0] == 0
  np.testing.assert_array_equal(r.geom_fluid, m.geom_fluid)


@pytest.mark.parametrize("field,value,msg", [
    ("wrap_type", 7, "unknown tendon wrap object type")])
def test_unsupported_features_refused(humanoid, field, value, msg):
  buf = mjb.write(humanoid)
  ints = dict(zip(mjb.INTS, struct.unpack_from("<83i", buf, 20)))
  off = mjb.offsets(ints)[field]
  code = next(c for n, r, c, _ in mjb.LAYOUT if n == field)
  b = _patch(buf, off, "<d" if code == "d" else "<i", value)
  with pytest.raises(mjb.MJBError, match=msg):
    mjb.read(b)


def test_pairs_roundtrip():
  """npair > 0: the predefined-pair arrays go through the .mjb layout and back unchanged
  (they were refused before this round)."""
  import pair_models as P
  m = P.mixed()
  m2 = mjb.read(mjb.write(m))
  assert m2.sizes["npair"] == m.sizes["npair"] == 5
  for f in ("pair_dim", "pair_geom1", "pair_geom2", "pair_signature", "pair_solref",
            "pair_solreffriction", "pair_solimp", "pair_margin", "pair_gap", "pair_friction"):
    np.testing.assert_array_equal(getattr(m2, f), getattr(m, f), err_msg=f)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference headers not present")
def test_layout_matches_reference_headers(tmp_path):
  """The transcribed field table and struct sizes against include/mujoco (read as text, and
  sizeof from a probe compiled against the public headers; the reference is not built)."""
  text = open(os.path.join(REF, "include/mujoco/mjxmacro.h")).read()
  ints = re.findall(r"X(?:MJV)?\s*\(\s*(\w+)\s*\)",
                    text[text.index("#define MJMODEL_INTS"):text.index("#define MJMODEL_POINTERS_PREAMBLE")])
  assert ints == mjb.INTS + ["narena", "nbuffer"]
  body = text[text.index("#define MJMODEL_POINTERS "):text.index("#define MJDATA_POINTERS_PREAMBLE")]
  ref = re.findall(r"X(?:MJV|NV)?\s*\(\s*(\w+)\s*,\s*(\w+)\s*,\s*(\w+)\s*,\s*(.+?)\s*\)\s*\\",
                   body)
  consts = {"mjNREF": "2", "mjNIMP": "5", "mjNEQDATA": "11", "mjNDYN": "10", "mjNGAIN": "10",
            "mjNBIAS": "10", "mjNFLUID": "12", "mjNTEXROLE": "10"}
  tmap = {"mjtNum": "d", "float": "f", "int": "i", "mjtByte": "b", "char": "c"}
  got = []
  for t, n, r, c in ref:
    c = re.sub(r"MJ_M\((\w+)\)", r"\1", c).replace(" ", "")
    got.append((n, r, tmap[t], consts.get(c, c)))
  assert got == [tuple(x) for x in mjb.LAYOUT]
  probe = tmp_path / "probe.c"
  probe.write_text('#include <stdio.h>\n#include <mujoco/mjmodel.h>\n'
                   'int main(void){printf("%zu %zu %zu", sizeof(mjOption), sizeof(mjVisual),'
                   ' sizeof(mjStatistic)); return 0;}\n')
  exe = tmp_path / "probe"
  subprocess.run(["gcc", "-I", os.path.join(REF, "include"), "-o", str(exe), str(probe)],
                 check=True)
  sizes = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
  assert [int(x) for x in sizes] == [mjb.SIZEOF_OPTION, mjb.SIZEOF_VISUAL,
                                     mjb.SIZEOF_STATISTIC]


def _imported_cases():
  from mujoco_inversedynamicstest_amd.sampler import sample_contact_states, sample_states
  rng = np.random.default_rng(5)
  hc = models.load("humanoid")
  sc = models.load("slider_crank")
  return {
      # config 2: no contacts, limits inactive (the straight-line kernel)
      "humanoid": (models.load("humanoid", disable_contact=True),
                   lambda m: sample_states(m, 512, first=7), "humanoid"),
      # config 4: floor contacts and limits on keyframe poses
      "humanoid_contacts": (hc, lambda m: sample_contact_states(m, 256), "humanoid_contact"),
      # config 1's model: slider-crank transmissions and a capsule-cylinder (GJK/EPA) pair
      "slider_crank": (sc, lambda m: (rng.uniform(-np.pi, np.pi, (128, 3)),
                                      rng.normal(size=(128, 3)), rng.normal(size=(128, 3))),
                       "slider_crank"),
  }


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["humanoid", "humanoid_contacts", "slider_crank"])
def test_engine_on_imported_model(name):
  """The engine on a model imported from .mjb bytes (mjb.read) against the CPU oracle on the
  MJCF-compiled original: the same straight-line kernel is selected, counts are exact and
  qfrc_inverse and the efc rows agree to the north-star 1e-10."""
  from oracle.oracle import Oracle
  m, states, kernel = _imported_cases()[name]
  r = mjb.read(mjb.write(m))
  q, v, a = states(m)
  B = len(q)
  e = engine.InverseEngine(r, capacity=B)
  e0 = engine.InverseEngine(m, capacity=B)
  try:
    assert e.fast_kernel == kernel
    f, st = e.inverse(q, v, a, status=True)
    nefc = e.field_int("efc_count", 0, B)[:, 0]
    # the imported model is the same model: bit-identical on the device
    np.testing.assert_array_equal(f, e0.inverse(q, v, a))
    o = Oracle(m)
    ref, rnefc, rst = [], [], []
    for i in range(B):
      ref.append(o.inverse(q[i], v[i], a[i]).copy())
      rnefc.append(o.d.nefc)
      rst.append(o.d.status)
  finally:
    e.close()
    e0.close()
  np.testing.assert_array_equal(st, rst)
  np.testing.assert_array_equal(nefc, rnefc)
  ref = np.array(ref)
  scale = np.maximum(1.0, np.abs(ref).max(axis=1))
  err = np.abs(f - ref).max(axis=1) / scale
  # north-star 1e-10; the slider-crank's capsule-cylinder contacts come from the iterative
  # GJK/EPA solver, whose depth is defined to ccd_tolerance and moves under the device's FMA
  # contraction of its inputs (convex pairs): instances with a contact are held to
  # the solver's own bound instead
  convex = (np.array(rnefc) > 0) if name == "slider_crank" else np.zeros(B, bool)
  assert err[~convex].max(initial=0) <= 1e-10, f"{name}: error {err[~convex].max():.3e}"
  assert err[convex].max(initial=0) <= 1e-6, f"{name}: contact error {err[convex].max():.3e}"
  if name != "humanoid":
    assert np.array(rnefc).max() > 0      # rows were exercised


def _round2_models():
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  import test_tendon_cpu as T
  import test_transmission_cpu as R
  from mujoco_inversedynamicstest_amd import mjcf
  return {"wrap": mjcf.load_xml_string(T.WRAP), "refsite": mjcf.load_xml_string(R.REFSITE),
          "adhesion": R._adhesion()}


@pytest.mark.parametrize("name", ["wrap", "refsite", "adhesion"])
def test_round_trip_round2_features(name, tmp_path):
  """Wrapping spatial tendons (wrap_type 4/5 with side-site ids in wrap_prm), site-relative
  and body transmissions survive the .mjb layout, sparse moment structure included."""
  m = _round2_models()[name]
  path = tmp_path / f"{name}.mjb"
  mjb.save(m, str(path))
  r = mjb.load(str(path))
  for f in fields.MODEL_FIELDS:
    np.testing.assert_array_equal(getattr(m, f.name), getattr(r, f.name), err_msg=f.name)
  assert fields.model_signature(r) == fields.model_signature(m)


def test_round_trip_reference_model(tmp_path):
  """The reference's inverse-test model (mesh, height field, fluid, actuator dynamics):
  collision-mesh vertices, faces and hull graph and the height-field data survive the .mjb
  layout; a model with an SDF geom is refused."""
  import sys
  sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
  import reference_model_states as R
  m = R.model()
  path = tmp_path / "model.mjb"
  mjb.save(m, str(path))
  r = mjb.load(str(path))
  for f in fields.MODEL_FIELDS:
    np.testing.assert_array_equal(getattr(m, f.name), getattr(r, f.name), err_msg=f.name)
  assert r.sizes["nmeshgraph"] == m.sizes["nmeshgraph"] > 0
  assert r.sizes["nmeshpoly"] == m.sizes["nmeshpoly"] > 0       # the compiled mesh polygons
  assert fields.model_signature(r) == fields.model_signature(m)
  buf = bytearray(mjb.write(m))
  ints = dict(zip(mjb.INTS, struct.unpack_from("<83i", buf, 20)))
  off = mjb.offsets(ints)["geom_type"]
  struct.pack_into("<i", buf, off + 4 * 5, 8)
  with pytest.raises(mjb.MJBError, match="SDF"):
    mjb.read(bytes(buf))
