"""Binary model files (.mjb): read a model that MuJoCo's mj_saveModel wrote, and write one.

The format is the one of src/engine/engine_io.c (MuJoCo 3.3.1):

  mj_saveModel  :720-773     header, size ints, mjOption, mjVisual, mjStatistic, every
                             mjModel array in field-table order, packed
  mj_loadModelBuffer :776-890  the checks restated by `read` (header :789-816, truncation
                             :819-822 and :853-865, size consistency :838-842, trailing
                             bytes :869-873)
  mj_makeModel :560-616      the 64-byte aligned buffer whose size `nbuffer` must match

The field table below is the mjModel layout of include/mujoco/mjxmacro.h (MJMODEL_INTS,
MJMODEL_POINTERS) written as a compact list: the file is a byte-exact dump of the model
arrays in that order, so reading it needs every array's type and shape, including the ones
(textures, flexes, skins, mesh normals and polygons, ...) that the inverse-dynamics path never
reads. Collision meshes (vertices, faces, convex-hull graph) and height fields are read.

`read` returns the same compiled-model object the MJCF loader produces (mjcf.Model), with the
sparse structures the reference derives in mj_makeData (C, D, B, mapM2C, mapM2D, moment
pattern) rebuilt by mjcf.sparse_structures, and rejects models outside the device subset as
the drop-in adapter does (integration/engine_inverse_mjhip.c adapter_unsupported). This is
how the engine consumes a model compiled by real MuJoCo, byte for byte.
"""
from __future__ import annotations

import struct

import numpy as np

from . import fields

ID = 54321                   # engine_io.c:298
NHEADER = 5

# MJMODEL_INTS, in order (the trailing narena and nbuffer are size_t)
INTS = """
nq nv nu na nbody nbvh nbvhstatic nbvhdynamic njnt ngeom nsite ncam nlight nflex nflexnode
nflexvert nflexedge nflexelem nflexelemdata nflexelemedge nflexshelldata nflexevpair
nflextexcoord nmesh nmeshvert nmeshnormal nmeshtexcoord nmeshface nmeshgraph nmeshpoly
nmeshpolyvert nmeshpolymap nskin nskinvert nskintexvert nskinface nskinbone nskinbonevert
nhfield nhfielddata ntex ntexdata nmat npair nexclude neq ntendon nwrap nsensor nnumeric
nnumericdata ntext ntextdata ntuple ntupledata nkey nmocap nplugin npluginattr nuser_body
nuser_jnt nuser_geom nuser_site nuser_cam nuser_tendon nuser_actuator nuser_sensor nnames
npaths nnames_map nM nB nC nD nJmom ntree ngravcomp nemax njmax nconmax nuserdata
nsensordata npluginstate
""".split()
SIZES = ("narena", "nbuffer")

# MJMODEL_POINTERS: "<rows> <type> <cols>: names..." runs of consecutive arrays with the same
# row count, element type and column count. Types: d mjtNum, f float, i int, b mjtByte,
# c char. Columns: an integer, a size name, or size*k.
POINTERS = """
nq d 1: qpos0 qpos_spring
nbody i 1: body_parentid body_rootid body_weldid body_mocapid body_jntnum body_jntadr
  body_dofnum body_dofadr body_treeid body_geomnum body_geomadr
nbody b 1: body_simple body_sameframe
nbody d 3: body_pos
nbody d 4: body_quat
nbody d 3: body_ipos
nbody d 4: body_iquat
nbody d 1: body_mass body_subtreemass
nbody d 3: body_inertia
nbody d 2: body_invweight0
nbody d 1: body_gravcomp body_margin
nbody d nuser_body: body_user
nbody i 1: body_plugin body_contype body_conaffinity body_bvhadr body_bvhnum
nbvh i 1: bvh_depth
nbvh i 2: bvh_child
nbvh i 1: bvh_nodeid
nbvhstatic d 6: bvh_aabb
njnt i 1: jnt_type jnt_qposadr jnt_dofadr jnt_bodyid jnt_group
njnt b 1: jnt_limited jnt_actfrclimited jnt_actgravcomp
njnt d 2: jnt_solref
njnt d 5: jnt_solimp
njnt d 3: jnt_pos jnt_axis
njnt d 1: jnt_stiffness
njnt d 2: jnt_range jnt_actfrcrange
njnt d 1: jnt_margin
njnt d nuser_jnt: jnt_user
nv i 1: dof_bodyid dof_jntid dof_parentid dof_treeid dof_Madr dof_simplenum
nv d 2: dof_solref
nv d 5: dof_solimp
nv d 1: dof_frictionloss dof_armature dof_damping dof_invweight0 dof_M0
ngeom i 1: geom_type geom_contype geom_conaffinity geom_condim geom_bodyid geom_dataid
  geom_matid geom_group geom_priority geom_plugin
ngeom b 1: geom_sameframe
ngeom d 1: geom_solmix
ngeom d 2: geom_solref
ngeom d 5: geom_solimp
ngeom d 3: geom_size
ngeom d 6: geom_aabb
ngeom d 1: geom_rbound
ngeom d 3: geom_pos
ngeom d 4: geom_quat
ngeom d 3: geom_friction
ngeom d 1: geom_margin geom_gap
ngeom d 12: geom_fluid
ngeom d nuser_geom: geom_user
ngeom f 4: geom_rgba
nsite i 1: site_type site_bodyid site_matid site_group
nsite b 1: site_sameframe
nsite d 3: site_size site_pos
nsite d 4: site_quat
nsite d nuser_site: site_user
nsite f 4: site_rgba
ncam i 1: cam_mode cam_bodyid cam_targetbodyid
ncam d 3: cam_pos
ncam d 4: cam_quat
ncam d 3: cam_poscom0 cam_pos0
ncam d 9: cam_mat0
ncam i 1: cam_orthographic
ncam d 1: cam_fovy cam_ipd
ncam i 2: cam_resolution
ncam f 2: cam_sensorsize
ncam f 4: cam_intrinsic
ncam d nuser_cam: cam_user
nlight i 1: light_mode light_bodyid light_targetbodyid
nlight b 1: light_directional light_castshadow
nlight f 1: light_bulbradius
nlight b 1: light_active
nlight d 3: light_pos light_dir light_poscom0 light_pos0 light_dir0
nlight f 3: light_attenuation
nlight f 1: light_cutoff light_exponent
nlight f 3: light_ambient light_diffuse light_specular
nflex i 1: flex_contype flex_conaffinity flex_condim flex_priority
nflex d 1: flex_solmix
nflex d 2: flex_solref
nflex d 5: flex_solimp
nflex d 3: flex_friction
nflex d 1: flex_margin flex_gap
nflex b 1: flex_internal
nflex i 1: flex_selfcollide flex_activelayers flex_dim flex_matid flex_group flex_interp
  flex_nodeadr flex_nodenum flex_vertadr flex_vertnum flex_edgeadr flex_edgenum flex_elemadr
  flex_elemnum flex_elemdataadr flex_elemedgeadr flex_shellnum flex_shelldataadr
  flex_evpairadr flex_evpairnum flex_texcoordadr
nflexnode i 1: flex_nodebodyid
nflexvert i 1: flex_vertbodyid
nflexedge i 2: flex_edge
nflexelemdata i 1: flex_elem flex_elemtexcoord
nflexelemedge i 1: flex_elemedge
nflexelem i 1: flex_elemlayer
nflexshelldata i 1: flex_shell
nflexevpair i 2: flex_evpair
nflexvert d 3: flex_vert flex_vert0
nflexnode d 3: flex_node flex_node0
nflexedge d 1: flexedge_length0 flexedge_invweight0
nflex d 1: flex_radius
nflexelem d 21: flex_stiffness
nflex d 1: flex_damping flex_edgestiffness flex_edgedamping
nflex b 1: flex_edgeequality flex_rigid
nflexedge b 1: flexedge_rigid
nflex b 1: flex_centered flex_flatskin
nflex i 1: flex_bvhadr flex_bvhnum
nflex f 4: flex_rgba
nflextexcoord f 2: flex_texcoord
nmesh i 1: mesh_vertadr mesh_vertnum mesh_normaladr mesh_normalnum mesh_texcoordadr
  mesh_texcoordnum mesh_faceadr mesh_facenum mesh_bvhadr mesh_bvhnum mesh_graphadr
nmesh d 3: mesh_scale mesh_pos
nmesh d 4: mesh_quat
nmeshvert f 3: mesh_vert
nmeshnormal f 3: mesh_normal
nmeshtexcoord f 2: mesh_texcoord
nmeshface i 3: mesh_face mesh_facenormal mesh_facetexcoord
nmeshgraph i 1: mesh_graph
nmesh i 1: mesh_pathadr mesh_polynum mesh_polyadr
nmeshpoly d 3: mesh_polynormal
nmeshpoly i 1: mesh_polyvertadr mesh_polyvertnum
nmeshpolyvert i 1: mesh_polyvert
nmeshvert i 1: mesh_polymapadr mesh_polymapnum
nmeshpolymap i 1: mesh_polymap
nskin i 1: skin_matid skin_group
nskin f 4: skin_rgba
nskin f 1: skin_inflate
nskin i 1: skin_vertadr skin_vertnum skin_texcoordadr skin_faceadr skin_facenum skin_boneadr
  skin_bonenum
nskinvert f 3: skin_vert
nskintexvert f 2: skin_texcoord
nskinface i 3: skin_face
nskinbone i 1: skin_bonevertadr skin_bonevertnum
nskinbone f 3: skin_bonebindpos
nskinbone f 4: skin_bonebindquat
nskinbone i 1: skin_bonebodyid
nskinbonevert i 1: skin_bonevertid
nskinbonevert f 1: skin_bonevertweight
nskin i 1: skin_pathadr
nhfield d 4: hfield_size
nhfield i 1: hfield_nrow hfield_ncol hfield_adr
nhfielddata f 1: hfield_data
nhfield i 1: hfield_pathadr
ntex i 1: tex_type tex_height tex_width tex_nchannel tex_adr
ntexdata b 1: tex_data
ntex i 1: tex_pathadr
nmat i 10: mat_texid
nmat b 1: mat_texuniform
nmat f 2: mat_texrepeat
nmat f 1: mat_emission mat_specular mat_shininess mat_reflectance mat_metallic mat_roughness
nmat f 4: mat_rgba
npair i 1: pair_dim pair_geom1 pair_geom2 pair_signature
npair d 2: pair_solref pair_solreffriction
npair d 5: pair_solimp
npair d 1: pair_margin pair_gap
npair d 5: pair_friction
nexclude i 1: exclude_signature
neq i 1: eq_type eq_obj1id eq_obj2id eq_objtype
neq b 1: eq_active0
neq d 2: eq_solref
neq d 5: eq_solimp
neq d 11: eq_data
ntendon i 1: tendon_adr tendon_num tendon_matid tendon_group
ntendon b 1: tendon_limited
ntendon d 1: tendon_width
ntendon d 2: tendon_solref_lim
ntendon d 5: tendon_solimp_lim
ntendon d 2: tendon_solref_fri
ntendon d 5: tendon_solimp_fri
ntendon d 2: tendon_range
ntendon d 1: tendon_margin tendon_stiffness tendon_damping tendon_frictionloss
ntendon d 2: tendon_lengthspring
ntendon d 1: tendon_length0 tendon_invweight0
ntendon d nuser_tendon: tendon_user
ntendon f 4: tendon_rgba
nwrap i 1: wrap_type wrap_objid
nwrap d 1: wrap_prm
nu i 1: actuator_trntype actuator_dyntype actuator_gaintype actuator_biastype
nu i 2: actuator_trnid
nu i 1: actuator_actadr actuator_actnum actuator_group
nu b 1: actuator_ctrllimited actuator_forcelimited actuator_actlimited
nu d 10: actuator_dynprm actuator_gainprm actuator_biasprm
nu b 1: actuator_actearly
nu d 2: actuator_ctrlrange actuator_forcerange actuator_actrange
nu d 6: actuator_gear
nu d 1: actuator_cranklength actuator_acc0 actuator_length0
nu d 2: actuator_lengthrange
nu d nuser_actuator: actuator_user
nu i 1: actuator_plugin
nsensor i 1: sensor_type sensor_datatype sensor_needstage sensor_objtype sensor_objid
  sensor_reftype sensor_refid sensor_dim sensor_adr
nsensor d 1: sensor_cutoff sensor_noise
nsensor d nuser_sensor: sensor_user
nsensor i 1: sensor_plugin
nplugin i 1: plugin plugin_stateadr plugin_statenum
npluginattr c 1: plugin_attr
nplugin i 1: plugin_attradr
nnumeric i 1: numeric_adr numeric_size
nnumericdata d 1: numeric_data
ntext i 1: text_adr text_size
ntextdata c 1: text_data
ntuple i 1: tuple_adr tuple_size
ntupledata i 1: tuple_objtype tuple_objid
ntupledata d 1: tuple_objprm
nkey d 1: key_time
nkey d nq: key_qpos
nkey d nv: key_qvel
nkey d na: key_act
nkey d nmocap*3: key_mpos
nkey d nmocap*4: key_mquat
nkey d nu: key_ctrl
nbody i 1: name_bodyadr
njnt i 1: name_jntadr
ngeom i 1: name_geomadr
nsite i 1: name_siteadr
ncam i 1: name_camadr
nlight i 1: name_lightadr
nflex i 1: name_flexadr
nmesh i 1: name_meshadr
nskin i 1: name_skinadr
nhfield i 1: name_hfieldadr
ntex i 1: name_texadr
nmat i 1: name_matadr
npair i 1: name_pairadr
nexclude i 1: name_excludeadr
neq i 1: name_eqadr
ntendon i 1: name_tendonadr
nu i 1: name_actuatoradr
nsensor i 1: name_sensoradr
nnumeric i 1: name_numericadr
ntext i 1: name_textadr
ntuple i 1: name_tupleadr
nkey i 1: name_keyadr
nplugin i 1: name_pluginadr
nnames c 1: names
nnames_map i 1: names_map
npaths c 1: paths
"""

DTYPE = {"d": np.float64, "f": np.float32, "i": np.int32, "b": np.uint8, "c": np.uint8}

# mjOption in declaration order (include/mujoco/mjmodel.h): 31 mjtNum then 13 int, padded to
# the struct's 8-byte alignment; mjVisual is 157 4-byte members; mjStatistic 7 mjtNum
OPTION_DOUBLES = [("timestep", 1), ("apirate", 1), ("impratio", 1), ("tolerance", 1),
                  ("ls_tolerance", 1), ("noslip_tolerance", 1), ("ccd_tolerance", 1),
                  ("gravity", 3), ("wind", 3), ("magnetic", 3), ("density", 1),
                  ("viscosity", 1), ("o_margin", 1), ("o_solref", 2), ("o_solimp", 5),
                  ("o_friction", 5)]
OPTION_INTS = ["integrator", "cone", "jacobian", "solver", "iterations", "ls_iterations",
               "noslip_iterations", "ccd_iterations", "disableflags", "enableflags",
               "disableactuator", "sdf_initpoints", "sdf_iterations"]
SIZEOF_OPTION = 304
SIZEOF_VISUAL = 157 * 4
SIZEOF_STATISTIC = 7 * 8
# mj_defaultOption (engine_io.c) values for the members the compiled subset does not set
OPTION_DEFAULTS = {"timestep": 0.002, "apirate": 100.0, "impratio": 1.0, "tolerance": 1e-8,
                   "ls_tolerance": 0.01, "noslip_tolerance": 1e-6, "ccd_tolerance": 1e-6,
                   "gravity": [0.0, 0.0, -9.81], "wind": [0.0, 0.0, 0.0],
                   "magnetic": [0.0, -0.5, 0.0], "density": 0.0, "viscosity": 0.0,
                   "o_margin": 0.0, "o_solref": [0.02, 1.0],
                   "o_solimp": [0.9, 0.95, 0.001, 0.5, 2.0],
                   "o_friction": [1.0, 1.0, 0.005, 0.0001, 0.0001], "integrator": 0,
                   "cone": 0, "jacobian": 2, "solver": 2, "iterations": 100,
                   "ls_iterations": 50, "noslip_iterations": 0, "ccd_iterations": 50,
                   "disableflags": 0, "enableflags": 0, "disableactuator": 0,
                   "sdf_initpoints": 40, "sdf_iterations": 10}

# object kind -> (name_*adr array, size) for the names buffer
NAME_ADR = {"body": ("name_bodyadr", "nbody"), "jnt": ("name_jntadr", "njnt"),
            "geom": ("name_geomadr", "ngeom"), "site": ("name_siteadr", "nsite"),
            "cam": ("name_camadr", "ncam"), "light": ("name_lightadr", "nlight"),
            "tendon": ("name_tendonadr", "ntendon"), "actuator": ("name_actuatoradr", "nu"),
            "sensor": ("name_sensoradr", "nsensor"), "key": ("name_keyadr", "nkey"),
            "eq": ("name_eqadr", "neq"), "exclude": ("name_excludeadr", "nexclude")}


class MJBError(ValueError):
  """A buffer mj_loadModelBuffer would refuse (its warning text), or a model outside the
  device subset."""


def _parse_pointers():
  out = []
  for run in POINTERS.replace("\n  ", " ").strip().split("\n"):
    head, names = run.split(":")
    rows, code, cols = head.split()
    for name in names.split():
      out.append((name, rows, code, cols))
  return out


LAYOUT = _parse_pointers()


def _cols(expr, ints):
  if expr.isdigit():
    return int(expr)
  if "*" in expr:
    a, k = expr.split("*")
    return ints[a] * int(k)
  return ints[expr]


def _skip(offset):                       # SKIP (engine_io.c:387-391): 64-byte alignment
  return (64 - offset % 64) % 64


def buffer_size(ints: dict) -> int:
  """nbuffer as mj_makeModel computes it: every array 64-byte aligned, in table order."""
  off = 0
  for name, rows, code, cols in LAYOUT:
    off += _skip(off) + np.dtype(DTYPE[code]).itemsize * ints[rows] * _cols(cols, ints)
  return off


def header() -> list:
  return [ID, 8, len(INTS), len(SIZES), len(LAYOUT)]


def offsets(ints: dict) -> dict:
  """Byte offset of every array in an .mjb file with these sizes (arrays are packed)."""
  p = NHEADER*4 + 4*len(INTS) + 8*len(SIZES) + SIZEOF_OPTION + SIZEOF_VISUAL + SIZEOF_STATISTIC
  out = {}
  for name, rows, code, cols in LAYOUT:
    out[name] = p
    p += np.dtype(DTYPE[code]).itemsize * ints[rows] * _cols(cols, ints)
  out["__end__"] = p
  return out


#----------------------------------------- read -------------------------------------------

def read_raw(buf: bytes):
  """Parse an .mjb buffer: (ints, sizes, option dict, {field: array}). The checks and
  messages are mj_loadModelBuffer's."""
  buf = memoryview(bytes(buf))
  n = len(buf)
  if n < NHEADER * 4:
    raise MJBError("Model file has an incomplete header")
  hdr = struct.unpack_from(f"<{NHEADER}i", buf, 0)
  msgs = ["Model missing header ID",
          "Model and executable have different floating point precision",
          "Model and executable have different number of ints in mjModel",
          "Model and executable have different number of size_t members in mjModel",
          "Model and executable have different number of pointers in mjModel"]
  for i, (got, want) in enumerate(zip(hdr, header())):
    if got != want:
      raise MJBError(msgs[i])
  p = NHEADER * 4
  if p + 4 * len(INTS) + 8 * len(SIZES) > n:
    raise MJBError("Truncated model file - ran out of data while reading sizes")
  ints = dict(zip(INTS, struct.unpack_from(f"<{len(INTS)}i", buf, p)))
  p += 4 * len(INTS)
  sizes = dict(zip(SIZES, struct.unpack_from(f"<{len(SIZES)}Q", buf, p)))
  p += 8 * len(SIZES)
  if any(v < 0 for k, v in ints.items() if k not in ("njmax", "nconmax")) or \
     sizes["nbuffer"] != buffer_size(ints):
    raise MJBError("Corrupted model, wrong size parameters")
  if p + SIZEOF_OPTION + SIZEOF_VISUAL + SIZEOF_STATISTIC > n:
    raise MJBError("Truncated model file - ran out of data while reading structs")
  opt = {}
  q = p
  for k, cnt in OPTION_DOUBLES:
    v = struct.unpack_from(f"<{cnt}d", buf, q)
    opt[k] = float(v[0]) if cnt == 1 else [float(x) for x in v]
    q += 8 * cnt
  for k in OPTION_INTS:
    opt[k] = struct.unpack_from("<i", buf, q)[0]
    q += 4
  p += SIZEOF_OPTION + SIZEOF_VISUAL + SIZEOF_STATISTIC
  arrays = {}
  for name, rows, code, cols in LAYOUT:
    nr, nc = ints[rows], _cols(cols, ints)
    dt = np.dtype(DTYPE[code]).newbyteorder("<")
    nbytes = dt.itemsize * nr * nc
    if p + nbytes > n:
      raise MJBError(f"Truncated model file - ran out of data while reading {name}")
    arrays[name] = np.frombuffer(buf, dtype=dt, count=nr * nc, offset=p).reshape(nr, nc).copy()
    p += nbytes
  if p != n:
    raise MJBError("Model file is too large")
  return ints, sizes, opt, arrays


def _names(ints, arrays):
  raw = bytes(arrays["names"].reshape(-1))

  def at(adr):
    end = raw.find(b"\0", adr)
    return raw[adr:end if end >= 0 else len(raw)].decode()

  out = {kind: [at(int(a)) for a in arrays[adr].reshape(-1)]
         for kind, (adr, size) in NAME_ADR.items()}
  return out, (at(0) if raw else "")


def unsupported(ints, arrays) -> str | None:
  """Features outside the device subset that the compiled-model arrays cannot express
  (the adapter's adapter_unsupported list plus the loader's subset)."""
  if ints["nflex"]:
    return "flexes"
  if ints["nplugin"]:
    return "plugins"
  if ints["nwrap"] and not np.isin(arrays["wrap_type"], (1, 2, 3, 4, 5)).all():
    return "unknown tendon wrap object type"
  if ints["nu"]:
    dyn = np.asarray(arrays["actuator_dyntype"]).reshape(-1)
    gain = np.asarray(arrays["actuator_gaintype"]).reshape(-1)
    kv = np.asarray(arrays["actuator_gainprm"]).reshape(ints["nu"], -1)[:, 2]
    if np.any((dyn != 0) & (gain == 1) & (kv != 0)):
      return "an affine velocity gain with activation dynamics (reads mjData.act)"
    if np.any(gain >= 2) or np.any(np.asarray(arrays["actuator_biastype"]) >= 2):
      return "muscle or user actuator gain/bias"
  if ints["ngeom"] and np.any(np.asarray(arrays["geom_type"]) == 8):
    return "SDF geoms"
  return None


def read(buf: bytes):
  """mj_loadModelBuffer for the engine: an .mjb buffer -> mjcf.Model."""
  from . import mjcf
  ints, sizes, opt, arrays = read_raw(buf)
  why = unsupported(ints, arrays)
  if why:
    raise MJBError(f"model uses {why}, which the MI355X inverse path does not implement")
  m = mjcf.Model()
  m.sizes = {k: int(ints[k]) for k in fields.MODEL_SIZES if k in ints}
  m.opt = opt
  A = {k: v for k, v in arrays.items()}
  try:
    derived = mjcf.sparse_structures(dict(m.sizes), A, jacobian=int(opt["jacobian"]))
  except mjcf.MJCFError as e:
    raise MJBError(f"inconsistent model: {e}") from e
  A.update(derived)
  for f in fields.MODEL_FIELDS:
    if f.name not in A:
      raise MJBError(f"field {f.name} missing from the layout")   # SHOULD NOT OCCUR
    want = f.shape(m.sizes)
    a = np.asarray(A[f.name]).astype(fields.NPTYPE[f.ctype])
    if a.size != want[0] * want[1]:
      raise MJBError(f"{f.name}: {a.size} values, expected {want[0]}x{want[1]}")
    setattr(m, f.name, np.ascontiguousarray(a.reshape(want if want[1] != 1 else want[:1])))
  m.names, m.model_name = _names(ints, arrays)
  m.names = {k: v for k, v in m.names.items() if k in mjcf._NAME_SIZE}
  m.mjb_ints = ints
  return m


def load(path: str):
  with open(path, "rb") as f:
    return read(f.read())


#----------------------------------------- write ------------------------------------------

_MINUS_ONE = ("_plugin", "_matid", "_dataid", "_pathadr", "_bvhadr", "_actadr")


def _model_ints(m) -> dict:
  ints = {k: 0 for k in INTS}
  for k, v in m.sizes.items():
    if k in ints:
      ints[k] = int(v)
  ints["nuser_body"] = ints["nuser_jnt"] = ints["nuser_geom"] = ints["nuser_site"] = 0
  ints["nuser_cam"] = ints["nuser_tendon"] = ints["nuser_actuator"] = 0
  ints["nuser_sensor"] = 0
  ints["njmax"] = ints["nconmax"] = -1          # mjCModel defaults: arena sized at runtime
  eqt = np.asarray(getattr(m, "eq_type", np.zeros(0))).reshape(-1)
  ints["nemax"] = int(sum(3 if t == 0 else (6 if t == 1 else 1) for t in eqt))
  return ints


def _name_buffer(m, ints):
  buf = bytearray((getattr(m, "model_name", "") or "").encode() + b"\0")
  adrs = {}
  for kind, (adr, size) in NAME_ADR.items():
    lst = list(m.names.get(kind, [])) if hasattr(m, "names") else []
    a = np.zeros(ints[size], dtype=np.int32)
    for i in range(ints[size]):
      nm = lst[i] if i < len(lst) else ""
      a[i] = len(buf)
      buf += nm.encode() + b"\0"
    adrs[adr] = a
  return bytes(buf), adrs


def write(m) -> bytes:
  """mj_saveModel of a compiled model: arrays the model does not carry are written as the
  reference's empty values (0, or -1 for object ids)."""
  ints = _model_ints(m)
  names, adrs = _name_buffer(m, ints)
  ints["nnames"] = len(names)
  ints["npaths"] = 0
  ints["nnames_map"] = 0
  nu = ints["nu"]
  dyn = np.asarray(getattr(m, "actuator_dyntype")).reshape(-1) if nu else np.zeros(0)
  actadr = np.full(nu, -1, np.int32)
  actnum = np.zeros(nu, np.int32)
  k = 0
  for i in range(nu):
    if dyn[i]:
      actadr[i], actnum[i] = k, 1
      k += 1
  extra = {"names": np.frombuffer(names, dtype=np.uint8), "actuator_actadr": actadr,
           "actuator_actnum": actnum, **adrs}
  out = [struct.pack(f"<{NHEADER}i", *header()),
         struct.pack(f"<{len(INTS)}i", *[ints[k] for k in INTS]),
         struct.pack("<QQ", 1 << 24, buffer_size(ints))]
  opt = dict(OPTION_DEFAULTS)
  opt.update(m.opt)
  ob = b"".join(struct.pack(f"<{cnt}d", *(opt[k] if cnt > 1 else [opt[k]]))
                for k, cnt in OPTION_DOUBLES)
  ob += b"".join(struct.pack("<i", int(opt[k])) for k in OPTION_INTS)
  out.append(ob + b"\0" * (SIZEOF_OPTION - len(ob)))
  out.append(b"\0" * (SIZEOF_VISUAL + SIZEOF_STATISTIC))
  have = {f.name for f in fields.MODEL_FIELDS}
  for name, rows, code, cols in LAYOUT:
    nr, nc = ints[rows], _cols(cols, ints)
    dt = np.dtype(DTYPE[code]).newbyteorder("<")
    if name in extra:
      a = np.asarray(extra[name])
    elif name in have:
      a = np.asarray(getattr(m, name))
    else:
      fill = -1 if name.endswith(_MINUS_ONE) else 0
      a = np.full(nr * nc, fill)
    if a.size != nr * nc:
      raise MJBError(f"{name}: {a.size} values, expected {nr}x{nc}")
    out.append(np.ascontiguousarray(a.reshape(-1).astype(dt)).tobytes())
  return b"".join(out)


def save(m, path: str):
  with open(path, "wb") as f:
    f.write(write(m))
