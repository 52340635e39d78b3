"""Model-specialized HIP kernel generator: the fast path of mj_inverse for one model.

The generic kernel (csrc/engine_device.h) walks the model's arrays at run time and keeps
every intermediate in the device mirror. This generator instead unrolls the reference's
loops over the model's bodies, joints and dofs at build time. Model constants become exact
literals, and every mjData output is stored to the mirror exactly once. Arithmetic goes
through the same helper templates as the generic kernel (mjh::mulQuat, mjh::inertCom,
mjh::dot6, ...) in the same order, so the outputs are bit-identical to the generic kernel's
and the oracle's (tests/test_codegen_cpu.py).

Schedule (why it is not one fused kernel): one lane owns one instance and a 65,536 batch is
one wave per SIMD, so nothing hides a stall. Every load on CDNA waits for all of the wave's
older stores (one vmcnt counter). Any value that spills to scratch and is reloaded after
mirror stores therefore waits for those stores to reach memory. The generator keeps the live
set small enough for the register file and puts all of a kernel's loads ahead of its stores:

  k_pos  qpos -> tree pass 1 (kinematics, subtree COM), tree pass 2 (kinematics again, stores,
         cinert, cdof, crb, qM). Pass 2 recomputes instead of keeping pass 1's frames live.
  k_fac  qM -> mj_factorM (qLD, qLDiagInv)
  k_vel  qvel, cinert, cdof -> fwdVelocity, passive, comVel + mj_rne(flg_acc=0)
  k_acc  qvel, qacc, cinert, cdof, cvel, cdof_dot -> mj_rne(flg_acc=1) + mj_inverse assembly

The tree passes are depth-first, with children in DESCENDING body index. The post-order of
that traversal is exactly the descending body order of the reference's backward loops
(subtree_com, crb, cfrc accumulation), so every sum is formed in the reference's order while
only the current root-to-body path is live.

Constraint rows are left to the generic constraint kernel (k_constraint, mjhip.hip:
collision, mj_makeConstraint and its velocity/acceleration-stage parts, final assembly),
which reads the constraint-free stages from the mirror. constraint_mode(m) says which
instances it serves: 'list' -- joint/tendon limits only; k_pos evaluates the predicates of
mj_instantiateLimit (engine_core_constraint.c:824-959) and appends limit-active instances to
a device work-list, marked in efc_count[0] (-1); 'all' -- contacts or always-active friction
loss, every instance; 'none' -- no rows possible. For a served instance k_va stores the raw
mj_rne(flg_acc = 1) result as qfrc_inverse, so the assembly rne + ((armature*qacc - passive)
- constraint) happens once, in the reference's order, in k_constraint.

Reference functions restated (engine_core_smooth.c unless noted): mj_kinematics :38-178,
mj_comPos :183-270, mj_camlight :275-392, mj_tendon :651-723 (fixed), mj_transmission
:865-916 (joint), mj_crb :1353-1401, mj_factorM/mj_factorI :1470-1511, mj_fwdVelocity
engine_forward.c:193-231, mj_comVel :1833-1896, mj_passive engine_passive.c:436-493,
mj_rne :1969-2023, mj_inverseSkip engine_inverse.c:197-261.
"""
from __future__ import annotations

import hashlib
import re

import numpy as np

from . import fields

FREE, BALL, SLIDE, HINGE = 0, 1, 2, 3
STAGES = ("pos", "fac", "va")
FRAMES_IN_PASS1 = True   # k_pos: pass 1 stores the frames, pass 2 cinert/cdof/crb/qM
MAX_LDS_HINGES = 32
PREFETCH = 1      # tree-pass events between a body's mirror loads and their first use
FUSE = True       # one launch running the three stage bodies back to back per wave
# k_va recomputes each body's frame, cinert and pre-visit cdof along its tree pass (from
# qpos, the root's subtree_com and k_pos's hinge sin/cos in LDS) instead of re-reading them
# from the mirror (332 fewer doubles read per humanoid instance; needs the fused kernel's LDS
# trig). Off: the frames kept along the path make k_all spill 844 B/lane (1,228 B when cdof
# is kept for the projections too), far worse than the reads it saves
# (tools/kernel_resources.py). Bit-exact either way (tests/test_codegen_cpu.py).
VA_RECOMPUTE = False
# lanes per workgroup of each stage kernel: 64 = one instance block per wave; 32 = a block
# split over two half-filled waves (twice the waves per SIMD, same mirror layout)
# Experiment (round 2, off): k_all hands qM from the pos stage to the fac stage in a
# kernel-local array the compiler promotes to registers, instead of fac re-reading it from
# the mirror (the staged kernels pass nullptr and keep the re-read). Exact, but the 243 qM
# values live across pos's post-order push k_all from 20 B to 1,968 B of scratch per lane
# (tools/kernel_resources.py), and every spill reload waits for the store stream.
QM_FORWARD = False
LANES = {"pos": 64, "fac": 64, "va": 64}
# k_all's workgroup: ALL_LANES lanes (64 = one instance block per wave; 32 = each block split
# over two half-filled waves, so batch 65,536 is 2,048 waves) and the waves per SIMD it is
# compiled for (__launch_bounds__'s second argument: 2 caps the kernel at 256 registers so
# two waves share a SIMD)
ALL_LANES = 64
ALL_WAVES = 1
# stores of mirror fields go out as streaming (non-temporal) stores, MJH_NT_STORE in
# engine_device.h, except those the fac stage re-reads right after the pos stage stored them
# (qM): those stay in L2 for it. The va stage's re-reads (cinert, cdof) come long after their
# stores, by which time 32 waves per XCD have written far more than its 4 MB L2 holds, so
# keeping them temporal only displaced qM (round 4 A/B, tools/exp_variants.py: 347.6 us with
# every re-read field temporal, 317.4 us with qM alone, 338.4 us with none; bit-identical
# outputs). -DMJHIP_NO_NT compiles them as plain stores (the A/B build)
NT_STORES = True
# experiment knobs (tools/exp_variants.py): NT_TEMPORAL None = the rule above, else the set
# of fields whose stores stay temporal (all others stream); NT_STAGES: the stages whose
# stores may stream
NT_TEMPORAL = None
NT_STAGES = ("pos", "fac", "va")
# batches from which k_all also streams the stores the va stage re-reads (SV = true): below
# it, L2 is not oversubscribed and keeping them pays (mjd_inverseFD's position-stage launch,
# whose centres' fields k_vaskip re-reads)
NT_SV_MIN_B = 49152
# experiment knob: stages whose re-reads of the mirror load as streaming (non-temporal)
# loads (MJH_NT_LOAD), so they do not displace the lines a later stage re-reads
NT_LOAD_STAGES = ()
# stages whose mirror loads stream in the SV instantiation only (batches >= NT_SV_MIN_B, where
# the va stage's re-read fields stream as well): 319.7 against 324.2 us per 65,536 in the A/B
# (profiles/r04/experiments/nt_variants_3.log); below it, and in k_vaskip (whose loads of the
# centre's fields are shared by 54 perturbations), they stay temporal
NT_LOAD_SV_STAGES = ("va",)
# k_fdall: polls of a centre block's flag before a skip wave gives up (each poll sleeps
# 8 x 64 cycles; 2^22 polls is about a second -- the flag is raised within the launch's
# first hundred microseconds, as every centre block is dispatched before any waiting one)
FD_WAIT_ITERS = 1 << 22


# mjd_inverseFD's perturbed instances (mjhip_inverseFDBatch with a stage-skip layout, whose
# centres come first): a mirror field the straight-line stages store but never load is read
# by no later kernel of that call either -- the finite differences read qfrc_inverse (and qM
# for DmDq), a work-list model's limit rows the fields below -- so in instance blocks at or
# past Mirror::full_blk (Mirror::fd_elide set) its stores are compiled out: the FD = true
# instantiation of the stage bodies drops them (if constexpr), and the k_all kernel launched
# when Mirror::fd_elide is set runs it on those blocks and the plain bodies on the centres'
# (one wave-uniform branch at the top); k_vaskip has the FD bodies only. Every other launch is
# the plain kernel. The arithmetic is the plain kernel's, so every result is the full
# pipeline's bit for bit (test_inverse_fd_stage_skip_bit_exact). Measured (28,672 instances of
# the humanoid, mjd_inverseFD's position stage): 134.6 us storing everything, 126.6 us with
# streaming stores into a shared sink (a streaming store reaches memory wherever it points),
# 125.4 us with temporal stores into it, 148 us skipping each store behind a wave-uniform
# branch (which also moved results by an ulp: the branches split the blocks the
# multiply-adds are formed in); selecting the sink in every instantiation cost the headline
# kernel 4%.
FD_KEEP = frozenset({"qpos", "qvel", "qacc", "qfrc_inverse", "qfrc_passive", "qfrc_constraint",
                     "qfrc_actuator", "ten_length", "ten_J", "ten_velocity", "actuator_length",
                     "actuator_moment", "actuator_velocity", "qM", "sensordata"})


def fd_elided(bodies) -> set:
  """The mirror fields the stage bodies store and never load, less FD_KEEP."""
  import re
  text = re.sub(r"double\* __restrict__ P_\w+ = [^;]*;", "", "\n".join(bodies))
  store_nt = re.compile(r"MJH_NT_STORE(?:_IF)?\((?:\w+, )?P_(\w+)\[")
  store_eq = re.compile(r"^\s*P_(\w+)\[[^\]]+\] = ", re.M)
  stores = set(store_nt.findall(text)) | set(store_eq.findall(text))
  loads = set(re.findall(r"P_(\w+)\[", store_eq.sub("", store_nt.sub("", text))))
  return stores - loads - FD_KEEP


def _elide_stores(body: str, elided) -> str:
  """FD instantiation: the elided fields' stores are compiled out (if constexpr); k_all runs
  it on the instance blocks past Mirror::full_blk and the plain body on the others."""
  import re
  store = re.compile(r"^(\s*)((?:MJH_NT_STORE(?:_IF)?\((?:\w+, )?P_(\w+)\[|P_(\w+)\[[^\]]+\] = ).*;)$")

  def one(line):
    mt = store.match(line)
    if not mt or (mt.group(3) or mt.group(4)) not in elided:
      return line
    return f"{mt.group(1)}if constexpr (!FD) {{ {mt.group(2)} }}"
  return "\n".join(one(x) for x in body.split("\n"))


def fdall_ok(m) -> bool:
  """The model gets k_fdall (mjd_inverseFD layout 1 in one launch): it has k_vaskip and the
  stage bodies index their LDS by a 64-lane block."""
  return constraint_mode(m) in ("none", "list") and ALL_LANES == 64 and \
      all(n == 64 for n in LANES.values())


def _ll(st):
  """LDS lane index and stride of stage st (LDS arrays are per workgroup)."""
  n = LANES[st]
  return ("lane", 64) if n == 64 else (f"(lane & {n - 1})", n)


def lit(x) -> str:
  """Exact C literal for a double (hex float keeps every bit)."""
  x = float(x)
  if x == 0:
    return "-0.0" if np.signbit(x) else "0.0"
  if x == int(x) and abs(x) < 2**53:
    return f"{int(x)}.0"
  return x.hex()


def arr_lit(vals) -> str:
  return "{" + ", ".join(lit(v) for v in np.ravel(vals)) + "}"


class _Emitter:
  def __init__(self):
    self.lines = []
    self.ind = 1

  def __call__(self, s=""):
    self.lines.append("  " * self.ind + s if s else "")

  def open(self, s="{"):
    self(s)
    self.ind += 1

  def close(self, s="}"):
    self.ind -= 1
    self(s)

  def text(self):
    return "\n".join(self.lines)


def fast_path_supported(m) -> str | None:
  """Return why the model cannot use the straight-line kernels, or None."""
  if m.nv == 0:
    # nothing to unroll (and zero-length arrays are not valid device code)
    return "no degrees of freedom"
  if m.nv >= 60:
    # straight-line code grows with the tree; large models (the reference's sparse-Jacobian
    # range) run the generic kernel
    return "large model (nv >= 60)"
  if fields.is_sparse(m):
    # compressed constraint rows (mj_isSparse) are built by the generic kernel only
    return "sparse-Jacobian model (jacobian=\"sparse\")"
  if m.opt["enableflags"] & (1 << 3):
    if int(m.opt["integrator"]) == 1:
      return "INVDISCRETE with RK4 (an error in the reference)"
    if any(int(t) == 5 for t in m.actuator_trntype[:m.nu]):
      # mj_discreteAcc's implicit damping reads actuator_moment before the constraint kernel
      # (k_discrete_before forms the slider-crank and site ones first), but a body
      # transmission needs the contacts that kernel makes
      return "INVDISCRETE with body (adhesion) transmissions"
  for a in range(m.nu):
    if m.actuator_trntype[a] not in (0, 1, 2, 3, 4, 5):
      return "unknown transmission"
  return None


# transmissions the generated kernels leave to the pass after the constraint kernel
# (mjh::transmissionAfter in k_sensors): slider-crank, site and body. Inverse dynamics does not
# read actuators, so their actuator_length/moment/velocity can come last; a body transmission
# needs the instance's contacts, which only the constraint kernel makes.
TRN_AFTER = (2, 4, 5)


def _pair_uses_ccd(t1, t2) -> bool:
  """mjhip_pairUsesCcd (include/mjhip_contact.h) for type-ordered t1 <= t2: the pair runs
  the iterative native solver (mjc_Convex, mjc_ConvexHField)."""
  if t1 == 1:                                           # height field
    return 2 <= t2 <= 7
  if t1 == 0:
    return False
  if t2 in (4, 7):                                      # ellipsoid, mesh
    return True
  if t2 == 5:                                           # cylinder
    return t1 in (3, 4, 5)
  if t2 == 6:                                           # box
    return t1 in (4, 5)
  return False


def exact_fp(m) -> bool:
  """True when some collidable geom pair runs the iterative native solver. Its result moves
  by up to ccd_tolerance under a last-bit change of the geom frames, so the generated
  kernels of such a model compute the frames without multiply-add contraction, rounding
  each operation as the reference does (the solver itself is compiled that way too,
  csrc/engine_device.h)."""
  if int(m.opt["disableflags"]) & ((1 << 4) | 1):       # contact or constraint disabled
    return False
  ng = m.sizes["ngeom"]
  t = np.asarray(m.geom_type)[:ng]
  ct = np.asarray(m.geom_contype)[:ng]
  ca = np.asarray(m.geom_conaffinity)[:ng]
  wb = np.asarray(m.body_weldid)[np.asarray(m.geom_bodyid)[:ng]]
  for i in range(ng):
    for j in range(i + 1, ng):
      if wb[i] == wb[j] or not ((ct[i] & ca[j]) or (ct[j] & ca[i])):
        continue
      if _pair_uses_ccd(min(t[i], t[j]), max(t[i], t[j])):
        return True
  return False


def spatial_tendons(m) -> list:
  """Tendons whose path is spatial (their first wrap is not a joint, engine_core_smooth.c
  mj_tendon): their length, Jacobian and velocity, the tendon transmissions on them and
  mj_passive are left to the pass before the constraint kernel (csrc/post_pass.h)."""
  return [t for t in range(m.ntendon) if int(m.wrap_type[int(m.tendon_adr[t])]) != 1]


def constraint_mode(m) -> str:
  """Which instances the constraint kernel serves: 'all', 'list' or 'none' (module doc)."""
  dsbl = int(m.opt["disableflags"])
  if spatial_tendons(m):
    return "all"          # the tendon pass (csrc/post_pass.h) forms ten_J and qfrc_passive
  if int(m.opt["enableflags"]) & (1 << 3):
    return "all"          # the discrete pass (csrc/post_pass.h) changes qacc before the
                          # constraint kernel, which assembles qfrc_inverse from it
  if (m.opt["density"] > 0 or m.opt["viscosity"] > 0) and not dsbl & (1 << 5):
    return "all"          # fluid: the post pass (csrc/post_pass.h) updates qfrc_passive, and
                          # the constraint kernel assembles qfrc_inverse for every instance
  if dsbl & 1:                                             # mjDSBL_CONSTRAINT
    return "none"
  contacts = not (dsbl & (1 << 4)) and m.nbody >= 2 and \
      bool(np.any((m.geom_contype != 0) | (m.geom_conaffinity != 0)))
  friction = (bool(np.any(m.dof_frictionloss > 0)) or
              bool(np.any(np.asarray(m.tendon_frictionloss)[:m.ntendon] > 0))) and \
      not (dsbl & (1 << 2))
  equality = m.sizes.get("neq", 0) > 0 and bool(np.any(m.eq_active0)) and not (dsbl & (1 << 1))
  if contacts or friction or equality:
    return "all"
  limits = not (dsbl & (1 << 3)) and (bool(np.any(m.jnt_limited)) or
                                      bool(np.any(m.tendon_limited[:m.ntendon])))
  return "list" if limits else "none"


CONSTRAINT_MODES = {"none": 0, "list": 1, "all": 2}


class _Model:
  """Model constants the emitters share."""

  def __init__(self, m):
    self.m = m
    self.nbody, self.nv, self.nq, self.njnt = m.nbody, m.nv, m.nq, m.njnt
    self.parent = [int(x) for x in m.body_parentid]
    self.rootid = [int(x) for x in m.body_rootid]
    self.children = {b: [] for b in range(m.nbody)}
    for b in range(1, m.nbody):
      self.children[self.parent[b]].append(b)
    for b in self.children:
      self.children[b].sort(reverse=True)
    self.mass = [float(x) for x in m.body_mass]
    self.dsbl = int(m.opt["disableflags"])
    self.cmode = constraint_mode(m)
    self.bdofadr = [int(x) for x in m.body_dofadr]
    self.bdofnum = [int(x) for x in m.body_dofnum]
    self.djnt = [int(x) for x in m.dof_jntid]
    self.dbody = [int(x) for x in m.dof_bodyid]
    self.Madr = [int(x) for x in m.dof_Madr]
    self.dparent = [int(x) for x in m.dof_parentid]
    self.simplenum = [int(x) for x in m.dof_simplenum]
    S = {f.name: f.size(m.sizes) for f in fields.DATA_FIELDS}
    self.S = S
    # subtree masses are model constants (mj_comPos accumulates them in descending order)
    ms = [0.0] * m.nbody
    for i in range(m.nbody - 1, -1, -1):
      ms[i] = ms[i] + self.mass[i]
      if i:
        ms[self.parent[i]] = ms[self.parent[i]] + ms[i]
    self.subtree_mass = ms
    # hinge joints whose sin/cos k_pos evaluates once, into LDS (2 doubles per lane each;
    # 4 waves per CU must fit in 160 KB)
    hinges = [j for j in range(m.njnt) if int(m.jnt_type[j]) == HINGE]
    self.trig = {j: h for h, j in enumerate(hinges)} if 0 < len(hinges) <= MAX_LDS_HINGES else {}
    self.spatial = set(spatial_tendons(m))
    self.ten_terms = []
    for t in range(m.ntendon):
      adr, num = int(m.tendon_adr[t]), int(m.tendon_num[t])
      if t in self.spatial:
        self.ten_terms.append(None)      # formed by the tendon pass, never emitted here
        continue
      self.ten_terms.append([(float(m.wrap_prm[w]), int(m.jnt_qposadr[m.wrap_objid[w]]),
                              int(m.jnt_dofadr[m.wrap_objid[w]]))
                             for w in range(adr, adr + num)])

  def ten_row(self, t):
    assert t not in self.spatial, "spatial tendon rows are formed at run time"
    J = np.zeros(self.nv)
    for prm, _, da in self.ten_terms[t]:
      J[da] = prm
    return J

  def jnt_ndof(self, j):
    return {FREE: 6, BALL: 3}.get(int(self.m.jnt_type[j]), 1)

  def preorder(self):
    out = []
    self.dfs(lambda b: out.append(b) if b else None, lambda b: None)
    return out

  def dfs(self, pre, post, root=0):
    """Depth-first over the tree, children in descending index (post-order = descending)."""
    pre(root)
    for c in self.children[root]:
      self.dfs(pre, post, c)
    post(root)


class _Stage:
  """Code of one stage body: pointer setup + emission helpers."""

  def __init__(self, M: _Model, store_fields=None):
    self.M = M
    self.E = _Emitter()
    self.store_fields = store_fields
    self.stored = set()      # mirror fields this stage stores through (k_vaskip's own set)

  def st(self, field, k, expr):
    self.stored.add(field)
    if field == "qM" and QM_FORWARD:
      self.E(f"{{ const double v_ = {expr}; if (qmr) qmr[{k}] = v_;")
      if self.store_fields is None or field in self.store_fields:
        self.E(f"  P_qM[{k}*64] = v_;")
      self.E("}")
      return
    if self.store_fields is None or field in self.store_fields:
      self.E(f"P_{field}[{k}*64] = {expr};")

  def stv(self, field, k0, arr, n):
    for c in range(n):
      self.st(field, k0 + c, f"{arr}[{c}]")

  def pointers(self, names):
    for nm in names:
      n = self.M.S[nm]
      if n:
        self.E(f"double* __restrict__ P_{nm} = mr.{nm} + ((long)blk*{n})*64 + lane;")

  def prologue(self):
    E = self.E
    E("const long inst = (long)blk*64 + lane;")
    E("if (inst >= B) return;")
    E("int* __restrict__ ec = efc_count + (long)blk*4*64 + lane;")

  def load(self, arr, field, n, off=0):
    self.E(f"double {arr}[{max(n, 1)}];")
    for k in range(n):
      self.E(f"{arr}[{k}] = P_{field}[{off + k}*64];")


def _prefetched_dfs(G: _Stage, loads, pre, post, dist):
  """Tree pass whose mirror loads are issued `dist` visit events ahead of their use.

  The events are the pre- and post-visits of the depth-first pass (world excluded).
  loads(kind, i) -> (decls, [(dst, field, idx)]): declarations (emitted at function scope)
  and scalar loads `dst = P_field[idx]` the event needs. A scheduling fence at each event
  keeps the loads where they are emitted, so at most `dist` events' worth is in flight.
  """
  M, E = G.M, G.E
  events = []
  M.dfs(lambda b: events.append(("pre", b)) if b else None,
        lambda b: events.append(("post", b)) if b else None)
  for ev in events:
    for d in loads(*ev)[0]:
      E(d)

  def emit_loads(ev):
    for dst, field, idx in loads(*ev)[1]:
      E(f"{dst} = P_{field}[{idx}*64];")

  for ev in events[:dist]:
    emit_loads(ev)
  pos = {ev: k for k, ev in enumerate(events)}

  def visit(kind, fn):
    def f(i):
      if i:
        E("MJH_SCHED_FENCE();")
        k = pos[(kind, i)] + dist
        if k < len(events):
          emit_loads(events[k])
      fn(i)
    return f

  M.dfs(visit("pre", pre), visit("post", post))


def _vec_loads(name, field, first, n):
  return [(f"{name}[{c}]", field, first + c) for c in range(n)]


# ------------------------------------------------------------------------------ kinematics
def _emit_frame(G: _Stage, i, store):
  """Frame of body i from its parent's frame (mj_kinematics, engine_core_smooth.c:56-160).

  Declares xpos_i, xquat_i, xmat_i and xanchor_j, xaxis_j for the body's joints.
  """
  M, E, m = G.M, G.E, G.M.m
  ja, jn = int(m.body_jntadr[i]), int(m.body_jntnum[i])
  E(f"double xpos_{i}[3], xquat_{i}[4], xmat_{i}[9];")
  if jn == 1 and m.jnt_type[ja] == FREE:
    qa = int(m.jnt_qposadr[ja])
    E(f"mjh::copy3(xpos_{i}, qpos + {qa});")
    E(f"mjh::copy4(xquat_{i}, qpos + {qa + 3});")
    E(f"mjh::normalize4s(xquat_{i});")
    E(f"double xanchor_{ja}[3], xaxis_{ja}[3] = {arr_lit(m.jnt_axis[ja])};")
    E(f"mjh::copy3(xanchor_{ja}, xpos_{i});")
  else:
    pid = M.parent[i]
    E.open()
    mid = int(m.body_mocapid[i]) if m.nmocap else -1
    if mid >= 0:                       # :72-82 mocap body: the per-instance input pose
      E(f"double bpos[3], bquat[4];")
      E(f"for (int k = 0; k < 3; k++) bpos[k] = P_mocap_pos[({3 * mid} + k)*64];")
      E(f"for (int k = 0; k < 4; k++) bquat[k] = P_mocap_quat[({4 * mid} + k)*64];")
      E("mjh::normalize4s(bquat);")
    else:
      E(f"const double bpos[3] = {arr_lit(m.body_pos[i])};")
      E(f"const double bquat[4] = {arr_lit(m.body_quat[i])};")
    if pid:
      E(f"mjh::mulMatVec3(xpos_{i}, xmat_{pid}, bpos);")
      E(f"mjh::addTo3(xpos_{i}, xpos_{pid});")
      E(f"mjh::mulQuat(xquat_{i}, xquat_{pid}, bquat);")
    else:
      E(f"mjh::copy3(xpos_{i}, bpos);")
      E(f"mjh::copy4(xquat_{i}, bquat);")
    E.close()
    for j in range(ja, ja + jn):
      t = int(m.jnt_type[j])
      qa = int(m.jnt_qposadr[j])
      E(f"double xanchor_{j}[3], xaxis_{j}[3];")
      E.open()
      E(f"const double jaxis[3] = {arr_lit(m.jnt_axis[j])};")
      E(f"const double jpos[3] = {arr_lit(m.jnt_pos[j])};")
      E(f"mjh::rotVecQuat(xaxis_{j}, jaxis, xquat_{i});")
      E(f"mjh::rotVecQuat(xanchor_{j}, jpos, xquat_{i});")
      E(f"mjh::addTo3(xanchor_{j}, xpos_{i});")
      if t == SLIDE:
        E(f"mjh::addToScl3(xpos_{i}, xaxis_{j}, qpos[{qa}] - {lit(m.qpos0[qa])});")
      else:
        E("double qloc[4];")
        if t == BALL:
          E(f"mjh::copy4(qloc, qpos + {qa});")
          E("mjh::normalize4s(qloc);")
        else:
          if j in M.trig:
            h = M.trig[j]
            E(f"mjh::axisAngle2QuatSC(qloc, jaxis, qpos[{qa}] - {lit(m.qpos0[qa])}, "
              f"trig[{2 * h}*{_ll('pos')[1]} + {_ll('pos')[0]}], "
              f"trig[{2 * h + 1}*{_ll('pos')[1]} + {_ll('pos')[0]}]);")
          else:
            E(f"mjh::axisAngle2Quat(qloc, jaxis, qpos[{qa}] - {lit(m.qpos0[qa])});")
        E(f"mjh::mulQuat(xquat_{i}, xquat_{i}, qloc);")
        E("double vec[3];")
        E(f"mjh::rotVecQuat(vec, jpos, xquat_{i});")
        E(f"mjh::sub3(xpos_{i}, xanchor_{j}, vec);")
      E.close()
  E(f"mjh::normalize4s(xquat_{i});")
  E(f"mjh::quat2Mats(xmat_{i}, xquat_{i});")
  if store:
    G.stv("xquat", 4 * i, f"xquat_{i}", 4)
    G.stv("xpos", 3 * i, f"xpos_{i}", 3)
    G.stv("xmat", 9 * i, f"xmat_{i}", 9)
    for j in range(ja, ja + jn):
      G.stv("xanchor", 3 * j, f"xanchor_{j}", 3)
      G.stv("xaxis", 3 * j, f"xaxis_{j}", 3)


def _emit_local2global(G: _Stage, dst_pos, dst_mat, pos, quat, body, sf, with_mat=True):
  """mj_local2Global (engine_support.c:1565-1606) into local arrays."""
  E = G.E
  E(f"double {dst_pos}[3]" + (f", {dst_mat}[9];" if with_mat else ";"))
  E.open()
  E(f"const double lp[3] = {arr_lit(pos)};")
  if sf in (0, 3, 4):
    E(f"mjh::mulMatVec3({dst_pos}, xmat_{body}, lp);")
    E(f"mjh::addTo3({dst_pos}, xpos_{body});")
  elif sf == 1:
    E(f"mjh::copy3({dst_pos}, xpos_{body});")
  else:
    E(f"mjh::copy3({dst_pos}, xipos_{body});")
  if with_mat:
    if sf == 0:
      E(f"const double lq[4] = {arr_lit(quat)};")
      E("double tmp[4];")
      E(f"mjh::mulQuat(tmp, xquat_{body}, lq);")
      E(f"mjh::quat2Mats({dst_mat}, tmp);")
    elif sf in (1, 3):
      E(f"mjh::copy({dst_mat}, xmat_{body}, 9);")
    else:
      E(f"mjh::copy({dst_mat}, ximat_{body}, 9);")
  E.close()


def _world_frame(E):
  E("double xpos_0[3] = {0.0, 0.0, 0.0}, xquat_0[4] = {1.0, 0.0, 0.0, 0.0};")
  E("double xmat_0[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};")
  E("double xipos_0[3] = {0.0, 0.0, 0.0};")
  E("double ximat_0[9] = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0};")


def _camlight_needs(m):
  """Bodies whose subtree COM / position the camera and light modes need in pass 2."""
  stc, xpos = set(), set()
  for mode, b, tgt in ([(int(m.cam_mode[c]), int(m.cam_bodyid[c]), int(m.cam_targetbodyid[c]))
                        for c in range(m.ncam)] +
                       [(int(m.light_mode[l]), int(m.light_bodyid[l]),
                         int(m.light_targetbodyid[l])) for l in range(m.nlight)]):
    if mode == 2:
      stc.add(b)
    elif mode == 4 and tgt >= 0:
      stc.add(tgt)
    elif mode == 3 and tgt >= 0:
      xpos.add(tgt)
  return stc, xpos


# ------------------------------------------------------------------------------ k_pos
def _gen_pos(M: _Model, store_fields=None) -> str:
  G = _Stage(M, store_fields)
  E, m = G.E, M.m
  nq, nv, dsbl = M.nq, M.nv, M.dsbl
  # the next call's work-list counter (two alternate; stream order makes this safe)
  E("if (worklist_next && blk == 0 && lane == 0) *worklist_next = 0;")
  G.prologue()
  G.pointers([f.name for f in fields.DATA_FIELDS if f.stage <= 1])
  E(f"double qpos[{max(nq, 1)}];")
  E("if (qpos_in) {")
  E(f"  for (int k = 0; k < {nq}; k++) {{ qpos[k] = qpos_in[inst*{nq} + k]; "
    f"P_qpos[k*64] = qpos[k]; }}")
  E(f"  for (int k = 0; k < {nv}; k++) P_qvel[k*64] = qvel_in[inst*{nv} + k];")
  E(f"  for (int k = 0; k < {nv}; k++) P_qacc[k*64] = qacc_in[inst*{nv} + k];")
  E("} else {")
  E(f"  for (int k = 0; k < {nq}; k++) qpos[k] = P_qpos[k*64];")
  E("}")

  # limits predicate: mj_instantiateLimit (engine_core_constraint.c:824-959)
  E("// ---- constraint detection (mj_instantiateLimit predicates)")
  E("bool active = false;")
  limits_on = M.cmode == "list"
  if limits_on:
    for j in range(M.njnt):
      if not m.jnt_limited[j]:
        continue
      t = int(m.jnt_type[j])
      qa = int(m.jnt_qposadr[j])
      mg = lit(m.jnt_margin[j])
      if t in (SLIDE, HINGE):
        lo, hi = m.jnt_range[j]
        E(f"active |= (-1.0*({lit(lo)} - qpos[{qa}]) < {mg}) | "
          f"(1.0*({lit(hi)} - qpos[{qa}]) < {mg});")
      elif t == BALL:
        E.open()
        E(f"double q4[4] = {{qpos[{qa}], qpos[{qa+1}], qpos[{qa+2}], qpos[{qa+3}]}}, aa[3];")
        E("mjh::normalize4s(q4); mjh::quat2Vel(aa, q4, 1);")
        E("double val = mjh::normalize3s(aa);")
        E(f"active |= (mjh::dmax({lit(m.jnt_range[j][0])}, {lit(m.jnt_range[j][1])}) - val"
          f" < {mg});")
        E.close()
  if m.ntendon:
    E(f"double ten_length[{m.ntendon}];")
    for t, terms in enumerate(M.ten_terms):
      if terms is None:
        continue
      E(f"ten_length[{t}] = 0.0;")
      for prm, qa, _ in terms:
        E(f"ten_length[{t}] += {lit(prm)} * qpos[{qa}];")
    if limits_on:
      for t in range(m.ntendon):
        if m.tendon_limited[t] and t not in M.spatial:
          lo, hi = m.tendon_range[t]
          mg = lit(m.tendon_margin[t])
          E(f"active |= (-1.0*({lit(lo)} - ten_length[{t}]) < {mg}) | "
            f"(1.0*({lit(hi)} - ten_length[{t}]) < {mg});")
  if M.cmode == "list":
    E("if (active) {   // k_constraint's work-list; the stages below still run")
    E("  int slot = MJH_ATOMIC_ADD(worklist_count, 1);")
    E("  worklist[slot] = (int)inst;")
    E("}")
    E("ec[0] = active ? -1 : 0;")
  else:
    E("(void)active;")

  # tendons and transmission depend on qpos only
  if m.ntendon:
    E("// ---- mj_tendon (fixed, dense ten_J)")   # spatial ones: the tendon pass
    for t in range(m.ntendon):
      if t in M.spatial:
        continue
      G.st("ten_length", t, f"ten_length[{t}]")
      J = M.ten_row(t)
      for k in range(nv):
        G.st("ten_J", t * nv + k, lit(J[k]))
  if m.nu:
    E("// ---- mj_transmission (hinge/slide/ball/free joint, fixed tendon)")
    for a in range(m.nu):
      if int(m.actuator_trntype[a]) in TRN_AFTER:
        continue                       # k_sensors' mjh::transmissionAfter
      jid = int(m.actuator_trnid[a, 0])
      if m.actuator_trntype[a] == 3 and jid in M.spatial:
        continue                       # the tendon pass (csrc/post_pass.h)
      g = float(m.actuator_gear[a, 0])
      adr = int(m.moment_rowadr[a])
      if m.actuator_trntype[a] == 3:   # :1053-1081: gear * ten_J over the row's nonzeros
        G.st("actuator_length", a, f"ten_length[{jid}]*{lit(g)}")
        J = M.ten_row(jid)
        for k in range(int(m.moment_rownnz[a])):
          G.st("actuator_moment", adr + k, lit(float(J[int(m.moment_colind[adr + k])]) * g))
        continue
      jt, qa = int(m.jnt_type[jid]), int(m.jnt_qposadr[jid])
      inparent = m.actuator_trntype[a] == 1
      gear = [float(x) for x in m.actuator_gear[a]]
      if jt == BALL:                   # :912-942 expmap axis . gear axis
        E.open()
        E("double axis[3], quat[4], ga[3];")
        E(f"mjh::copy4(quat, qpos + {qa});")
        E("mjh::normalize4(quat);")
        E("mjh::quat2Vel(axis, quat, 1);")
        E(f"const double g3[3] = {arr_lit(gear[:3])};")
        if inparent:
          E("quat[1] = -quat[1]; quat[2] = -quat[2]; quat[3] = -quat[3];")
          E("mjh::rotVecQuat(ga, g3, quat);")
        else:
          E("mjh::copy3(ga, g3);")
        G.st("actuator_length", a, "axis[0]*ga[0] + axis[1]*ga[1] + axis[2]*ga[2]")
        G.stv("actuator_moment", adr, "ga", 3)
        E.close()
        continue
      if jt == FREE:                   # :944-971 length 0, moment = (gear, gear axis)
        E.open()
        E("double ga[3];")
        E(f"const double g3[3] = {arr_lit(gear[3:6])};")
        if inparent:
          E("double quat[4];")
          E(f"mjh::copy4(quat, qpos + {qa + 3});")
          E("mjh::normalize4(quat);")
          E("quat[1] = -quat[1]; quat[2] = -quat[2]; quat[3] = -quat[3];")
          E("mjh::rotVecQuat(ga, g3, quat);")
        else:
          E("mjh::copy3(ga, g3);")
        G.st("actuator_length", a, "0.0")
        for k in range(3):
          G.st("actuator_moment", adr + k, lit(gear[k]))
        G.stv("actuator_moment", adr + 3, "ga", 3)
        E.close()
        continue
      G.st("actuator_length", a, f"qpos[{qa}]*{lit(g)}")
      G.st("actuator_moment", adr, lit(g))

  cams = {}
  for c in range(m.ncam):
    cams.setdefault(int(m.cam_bodyid[c]), []).append(("cam", c))
  for l in range(m.nlight):
    cams.setdefault(int(m.light_bodyid[l]), []).append(("light", l))
  geoms, sites = {}, {}
  for g in range(m.ngeom):
    geoms.setdefault(int(m.geom_bodyid[g]), []).append(g)
  for s in range(m.nsite):
    sites.setdefault(int(m.site_bodyid[s]), []).append(s)
  if M.trig:
    # every hinge's sin/cos once, into LDS: both tree passes read them, so neither carries
    # the branches of the trig functions' argument reduction
    E("// ---- hinge half-angle sin/cos (mju_axisAngle2Quat, engine_util_spatial.c:78-90)")
    for j, h in M.trig.items():
      qa = int(m.jnt_qposadr[j])
      E.open()
      E(f"double s, c, a = (qpos[{qa}] - {lit(m.qpos0[qa])})*0.5;")
      E("MJH_SINCOS(a, s, c);")
      li, ls = _ll("pos")
      E(f"trig[{2 * h}*{ls} + {li}] = s; trig[{2 * h + 1}*{ls} + {li}] = c;")
      E.close()
    E("MJH_MEM_BARRIER();")
  # ---- pass 1: kinematics -> subtree centers of mass (mj_comPos :183-208)
  E("// ---- tree pass 1: mj_kinematics -> mj_comPos subtree_com (post-order = descending)")
  need_stc, need_xpos = _camlight_needs(m)
  roots = sorted(set(M.rootid[1:]))
  need_stc |= set(roots)
  for b in sorted(need_stc):
    E(f"double keep_stc_{b}[3];")
  for b in sorted(need_xpos):
    E(f"double keep_xpos_{b}[3];")
  _world_frame(E)

  def frame_outputs(i):
    """xipos/ximat, geom and site frames of body i (stored by whichever pass owns them)."""
    G.stv("xipos", 3 * i, f"xipos_{i}", 3)
    G.stv("ximat", 9 * i, f"ximat_{i}", 9)
    for g in geoms.get(i, []):
      E.open()
      _emit_local2global(G, "gp", "gm", m.geom_pos[g], m.geom_quat[g], i,
                         int(m.geom_sameframe[g]))
      G.stv("geom_xpos", 3 * g, "gp", 3)
      G.stv("geom_xmat", 9 * g, "gm", 9)
      E.close()
    for s in sites.get(i, []):
      E.open()
      _emit_local2global(G, "sp", "sm", m.site_pos[s], m.site_quat[s], i,
                         int(m.site_sameframe[s]))
      G.stv("site_xpos", 3 * s, "sp", 3)
      G.stv("site_xmat", 9 * s, "sm", 9)
      E.close()

  def pre1(i):
    E.open(f"{{  // body {i}")
    if i:
      _emit_frame(G, i, store=FRAMES_IN_PASS1)
      _emit_local2global(G, f"xipos_{i}", f"ximat_{i}", m.body_ipos[i], m.body_iquat[i], i,
                         int(m.body_sameframe[i]), with_mat=FRAMES_IN_PASS1)
    elif FRAMES_IN_PASS1:
      G.stv("xpos", 0, "xpos_0", 3)
      G.stv("xquat", 0, "xquat_0", 4)
      G.stv("xmat", 0, "xmat_0", 9)
    if FRAMES_IN_PASS1:
      frame_outputs(i)
    if i in need_xpos:
      E(f"mjh::copy3(keep_xpos_{i}, xpos_{i});")
    E(f"double stc_{i}[3] = {{0.0, 0.0, 0.0}};")

  def post1(i):
    E(f"mjh::addToScl3(stc_{i}, xipos_{i}, {lit(M.mass[i])});")
    if i:
      E(f"mjh::addTo3(stc_{M.parent[i]}, stc_{i});")
    if M.subtree_mass[i] < 1e-15:
      E(f"mjh::copy3(stc_{i}, xipos_{i});")
    else:
      E(f"mjh::scl3(stc_{i}, stc_{i}, 1.0/{lit(max(1e-15, M.subtree_mass[i]))});")
    G.stv("subtree_com", 3 * i, f"stc_{i}", 3)
    if i in need_stc:
      E(f"mjh::copy3(keep_stc_{i}, stc_{i});")
    E.close()

  M.dfs(pre1, post1)

  # pass 2 recomputes the frames: make qpos opaque so the compiler cannot reuse pass 1's
  # (which would keep every frame live across the passes)
  E("// ---- tree pass 2: kinematics (stored), cinert, cdof, camlight, crb, qM")
  E(f"for (int k = 0; k < {nq}; k++) MJH_OPAQUE(qpos[k]);")
  if M.trig:
    E("MJH_MEM_BARRIER();")


  def pre2(i):
    E.open(f"{{  // body {i}")
    if i:
      _emit_frame(G, i, store=not FRAMES_IN_PASS1)
      _emit_local2global(G, f"xipos_{i}", f"ximat_{i}", m.body_ipos[i], m.body_iquat[i], i,
                         int(m.body_sameframe[i]))
    else:
      _world_frame(E)
      if not FRAMES_IN_PASS1:
        G.stv("xpos", 0, "xpos_0", 3)
        G.stv("xquat", 0, "xquat_0", 4)
        G.stv("xmat", 0, "xmat_0", 9)
    if not FRAMES_IN_PASS1:
      frame_outputs(i)
    for kind, c in cams.get(i, []):
      _emit_camlight(G, kind, c)
    # cinert (mj_comPos :211-222), crb starts as a copy (mj_crb :1360)
    if i:
      E(f"double crb_{i}[10];")
      E.open()
      E("double off[3];")
      E(f"mjh::sub3(off, xipos_{i}, keep_stc_{M.rootid[i]});")
      E(f"const double inert[3] = {arr_lit(m.body_inertia[i])};")
      E(f"mjh::inertCom(crb_{i}, inert, ximat_{i}, off, {lit(M.mass[i])});")
      E.close()
      G.stv("cinert", 10 * i, f"crb_{i}", 10)
    else:
      E("double crb_0[10] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};")
      G.stv("cinert", 0, "crb_0", 10)
    # cdof (mj_comPos :225-268)
    ja, jn = int(m.body_jntadr[i]), int(m.body_jntnum[i])
    for j in range(ja, ja + jn):
      da = int(m.jnt_dofadr[j])
      t = int(m.jnt_type[j])
      ndof = M.jnt_ndof(j)
      for k in range(ndof):
        E(f"double cdof_{da + k}[6];")
      E.open()
      E("double off[3], axis[3];")
      E(f"mjh::sub3(off, keep_stc_{M.rootid[i]}, xanchor_{j});")
      skip = 0
      if t == FREE:
        for k in range(3):
          E(f"mjh::zero(cdof_{da + k}, 6); cdof_{da + k}[{3 + k}] = 1.0;")
        skip = 3
      if t in (FREE, BALL):
        for k in range(3):
          E(f"axis[0] = xmat_{i}[{k}]; axis[1] = xmat_{i}[{k + 3}]; axis[2] = xmat_{i}[{k + 6}];")
          E(f"mjh::dofComHinge(cdof_{da + skip + k}, axis, off);")
      elif t == SLIDE:
        E(f"mjh::zero3(cdof_{da}); mjh::copy3(cdof_{da} + 3, xaxis_{j});")
      else:
        E(f"mjh::dofComHinge(cdof_{da}, xaxis_{j}, off);")
      E.close()
      for k in range(ndof):
        G.stv("cdof", 6 * (da + k), f"cdof_{da + k}", 6)

  def post2(i):
    # crb_i is final: every child (higher index) has been added, in descending order
    G.stv("crb", 10 * i, f"crb_{i}", 10)
    # qM rows of this body's dofs (mj_crb :1370-1399); qM starts zeroed (mju_zero)
    for k in range(M.bdofadr[i], M.bdofadr[i] + M.bdofnum[i]):
      adr = M.Madr[k]
      rowlen = 0
      j = k
      while j >= 0:
        rowlen += 1
        j = M.dparent[j]
      if M.simplenum[k]:
        G.st("qM", adr, lit(m.dof_M0[k]))
        for a in range(adr + 1, adr + rowlen):
          G.st("qM", a, "0.0")
        continue
      E.open()
      E("double buf[6];")
      E(f"mjh::mulInertVec(buf, crb_{i}, cdof_{k});")
      j, a, first = k, adr, True
      while j >= 0:
        expr = (f"{lit(m.dof_armature[k])} + mjh::dot6(cdof_{j}, buf)" if first
                else f"0.0 + mjh::dot6(cdof_{j}, buf)")
        G.st("qM", a, expr)
        first = False
        a += 1
        j = M.dparent[j]
      E.close()
    if i and M.parent[i] > 0:
      E(f"mjh::addTo(crb_{M.parent[i]}, crb_{i}, 10);")
    E.close()

  M.dfs(pre2, post2)
  return E.text()


def _emit_camlight(G: _Stage, kind, c):
  """mj_camlight (engine_core_smooth.c:275-392) for one camera or light on the current body."""
  E, m = G.E, G.M.m
  E.open()
  if kind == "cam":
    b = int(m.cam_bodyid[c])
    mode = int(m.cam_mode[c])
    tgt = int(m.cam_targetbodyid[c])
    _emit_local2global(G, "cp", "cm", m.cam_pos[c], m.cam_quat[c], b, 0)
    if mode in (1, 2):
      E(f"const double mat0[9] = {arr_lit(m.cam_mat0[c])};")
      E("mjh::copy(cm, mat0, 9);")
      if mode == 1:
        E(f"const double p0[3] = {arr_lit(m.cam_pos0[c])};")
        E(f"mjh::add3(cp, xpos_{b}, p0);")
      else:
        E(f"const double p0[3] = {arr_lit(m.cam_poscom0[c])};")
        E(f"mjh::add3(cp, keep_stc_{b}, p0);")
    elif mode in (3, 4) and tgt >= 0:
      src = f"keep_xpos_{tgt}" if mode == 3 else f"keep_stc_{tgt}"
      E("double matT[9];")
      E(f"mjh::sub3(matT + 6, cp, {src});")
      E("mjh::normalize3s(matT + 6);")
      E("matT[3] = 0; matT[4] = 0; matT[5] = 1;")
      E("mjh::cross(matT, matT + 3, matT + 6);")
      E("mjh::normalize3s(matT);")
      E("mjh::cross(matT + 3, matT + 6, matT);")
      E("mjh::normalize3s(matT + 3);")
      E("for (int r = 0; r < 3; r++) for (int q = 0; q < 3; q++) cm[3*q + r] = matT[3*r + q];")
    G.stv("cam_xpos", 3 * c, "cp", 3)
    G.stv("cam_xmat", 9 * c, "cm", 9)
  else:
    l = c
    b = int(m.light_bodyid[l])
    mode = int(m.light_mode[l])
    tgt = int(m.light_targetbodyid[l])
    E(f"const double lp[3] = {arr_lit(m.light_pos[l])};")
    E(f"const double ld[3] = {arr_lit(m.light_dir[l])};")
    E("double lx[3], dx[3];")
    E(f"mjh::mulMatVec3(lx, xmat_{b}, lp);")
    E(f"mjh::addTo3(lx, xpos_{b});")
    E(f"mjh::rotVecQuat(dx, ld, xquat_{b});")
    if mode in (1, 2):
      E(f"const double d0[3] = {arr_lit(m.light_dir0[l])};")
      E("mjh::copy3(dx, d0);")
      if mode == 1:
        E(f"const double p0[3] = {arr_lit(m.light_pos0[l])};")
        E(f"mjh::add3(lx, xpos_{b}, p0);")
      else:
        E(f"const double p0[3] = {arr_lit(m.light_poscom0[l])};")
        E(f"mjh::add3(lx, keep_stc_{b}, p0);")
    elif mode in (3, 4) and tgt >= 0:
      src = f"keep_xpos_{tgt}" if mode == 3 else f"keep_stc_{tgt}"
      E(f"mjh::sub3(dx, {src}, lx);")
    E("mjh::normalize3s(dx);")
    G.stv("light_xpos", 3 * l, "lx", 3)
    G.stv("light_xdir", 3 * l, "dx", 3)
  E.close()


# ------------------------------------------------------------------------------ k_fac
def _gen_fac(M: _Model, store_fields=None) -> str:
  """mj_factorM / mj_factorI (engine_core_smooth.c:1470-1511) on qM loaded from the mirror."""
  G = _Stage(M, store_fields)
  E, m = G.E, M.m
  nv = M.nv
  G.prologue()
  G.pointers(["qM", "qLD", "qLDiagInv"])
  for a in range(m.nM):
    E(f"const double M_{a} = qmr ? qmr[{a}] : P_qM[{a}*64];" if QM_FORWARD
      else f"const double M_{a} = P_qM[{a}*64];")
  rownnz = [int(x) for x in m.C_rownnz]
  rowadr = [int(x) for x in m.C_rowadr]
  colind = [int(x) for x in m.C_colind]
  mapM2C = [int(x) for x in m.mapM2C]
  E(f"double {', '.join(f'L_{c} = M_{mapM2C[c]}' for c in range(m.nC))};")
  for k in range(nv - 1, -1, -1):
    ra = rowadr[k]
    dk = ra + rownnz[k] - 1
    E(f"const double diaginv_{k} = 1 / L_{dk};")
    G.st("qLDiagInv", k, f"diaginv_{k}")
    if not M.simplenum[k]:
      for a in range(dk - 1, ra - 1, -1):
        ii = colind[a]
        E.open()
        E(f"double tmp = L_{a} * diaginv_{k};")
        for t in range(rownnz[ii]):
          E(f"L_{rowadr[ii] + t} += L_{ra + t} * -tmp;")
        E(f"L_{a} = tmp;")
        E.close()
    # row k is final once its own update is done (later rows only update rows < k)
    for c in range(ra, ra + rownnz[k]):
      G.st("qLD", c, f"L_{c}")
  return E.text()


# ------------------------------------------------------------------------------ k_vel / k_acc
def _emit_muldofvec(E, res, arrname, bda, n, vec):
  """mju_mulDofVec (engine_util_spatial.c:481-489) with dof arrays named arrname_<k>."""
  if n == 1:
    E(f"mjh::scl({res}, {arrname}_{bda}, {vec}[{bda}], 6);")
  elif n <= 0:
    E(f"mjh::zero({res}, 6);")
  else:
    E(f"mjh::zero({res}, 6);")
    for r in range(n):
      E(f"mjh::addToSclIf({res}, {arrname}_{bda + r}, {vec}[{bda + r}], 6);")


def _gravity_acc(M, E):
  m = M.m
  E("double cacc_0[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};")
  if not (M.dsbl & (1 << 6)):
    g = m.opt["gravity"]
    E(f"cacc_0[3] = {lit(g[0])}*-1; cacc_0[4] = {lit(g[1])}*-1; cacc_0[5] = {lit(g[2])}*-1;")


def _gen_va(M: _Model, store_fields=None) -> str:
  """Velocity and acceleration stages in one kernel: fwdVelocity, passive, then one tree
  pass with mj_comVel and both mj_rne calls (flg_acc = 0 -> qfrc_bias, 1 -> qfrc_inverse).
  The two RNE recursions share cdof_dot*qvel and the gyroscopic term cvel x (cinert*cvel),
  which the reference computes identically in each call."""
  G = _Stage(M, store_fields)
  M.va_stored = G.stored     # filled as the body is emitted; read by generate (k_vaskip)
  E, m = G.E, M.m
  nv, nq, dsbl = M.nv, M.nq, M.dsbl
  recompute = VA_RECOMPUTE and FUSE
  G.prologue()
  if M.cmode == "list":   # k_pos's work-list flag: k_constraint assembles this instance
    E("const bool cflag = ec[0] != 0;")
  G.pointers(["qpos", "qvel", "qacc", "cinert", "cdof", "xipos", "subtree_com", "ten_length",
              "ten_velocity", "actuator_velocity", "actuator_moment", "cvel", "cdof_dot",
              "qfrc_spring",
              "qfrc_damper", "qfrc_gravcomp", "qfrc_fluid", "qfrc_passive", "qfrc_bias",
              "qfrc_constraint", "qfrc_inverse"])
  G.load("qpos", "qpos", nq)
  G.load("qvel", "qvel", nv)
  if m.ntendon:
    G.load("ten_length", "ten_length", m.ntendon)
  E(f"double qfg[{nv}];")
  E(f"mjh::zero(qfg, {nv});")
  g = np.asarray(m.opt["gravity"], dtype=float)
  has_gravcomp = bool(m.ngravcomp and not (dsbl & (1 << 5)) and not (dsbl & (1 << 6)) and
                      np.sqrt(g @ g) != 0)
  if has_gravcomp:
    E("// ---- mj_gravcomp (engine_passive.c:381-399), bodies in ascending order")
    for b in range(1, M.nbody):
      if m.body_gravcomp[b]:
        _emit_applyforce(E, M, b)

  E("// ---- mj_fwdVelocity (engine_forward.c:193-231)")
  for t in range(m.ntendon):
    if t in M.spatial:
      continue
    E(f"double ten_velocity_{t};")
    E.open()
    E(f"const double J[{nv}] = {arr_lit(M.ten_row(t))};")
    E(f"ten_velocity_{t} = mjh::dot(J, qvel, {nv});")
    E.close()
    G.st("ten_velocity", t, f"ten_velocity_{t}")
  if m.nu and not (dsbl & (1 << 10)):
    for a in range(m.nu):
      adr, n = int(m.moment_rowadr[a]), int(m.moment_rownnz[a])
      g = float(m.actuator_gear[a, 0])
      if int(m.actuator_trntype[a]) in TRN_AFTER:
        continue                       # with its transmission, after the constraint kernel
      if m.actuator_trntype[a] == 3 and int(m.actuator_trnid[a, 0]) in M.spatial:
        continue                       # the tendon pass (csrc/post_pass.h)
      if m.actuator_trntype[a] == 3:   # mju_dotSparse over the tendon row's nonzeros
        if not n:
          G.st("actuator_velocity", a, "0.0")
          continue
        J = M.ten_row(int(m.actuator_trnid[a, 0]))
        cols = [int(c) for c in m.moment_colind[adr:adr + n]]
        E.open()
        E(f"const double mom[{n}] = {arr_lit([float(J[c]) * g for c in cols])};")
        E(f"const int ind[{n}] = {{{', '.join(str(c) for c in cols)}}};")
        G.st("actuator_velocity", a, f"mjh::dotSparse(mom, qvel, {n}, ind)")
        E.close()
        continue
      if int(m.jnt_type[int(m.actuator_trnid[a, 0])]) in (BALL, FREE):
        cols = [int(c) for c in m.moment_colind[adr:adr + n]]
        E.open()                       # the row k_pos stored, over its 3 or 6 columns
        E(f"double mom[{n}];")
        for k in range(n):
          E(f"mom[{k}] = P_actuator_moment[{adr + k}*64];")
        E(f"const int ind[{n}] = {{{', '.join(str(c) for c in cols)}}};")
        G.st("actuator_velocity", a, f"mjh::dotSparse(mom, qvel, {n}, ind)")
        E.close()
        continue
      col = int(m.moment_colind[adr])
      G.st("actuator_velocity", a, f"((0.0 + 0.0) + (0.0 + 0.0)) + {lit(g)}*qvel[{col}]")

  # mj_passive: springs, dampers, tendon spring-dampers (engine_passive.c:436-493)
  E("// ---- mj_passive (engine_passive.c:436-493)")
  E(f"double qfs[{nv}], qfd[{nv}];")
  E(f"mjh::zero(qfs, {nv}); mjh::zero(qfd, {nv});")
  if not (dsbl & (1 << 5)):
    for j in range(M.njnt):
      k = float(m.jnt_stiffness[j])
      if k == 0:
        continue
      pa, da, t = int(m.jnt_qposadr[j]), int(m.jnt_dofadr[j]), int(m.jnt_type[j])
      if t == FREE:
        for c in range(3):
          E(f"qfs[{da + c}] = -{lit(k)}*(qpos[{pa + c}] - {lit(m.qpos_spring[pa + c])});")
        pa += 3
        da += 3
        t = BALL
      if t == BALL:
        E.open()
        E(f"double dif[3], quat[4]; mjh::copy4(quat, qpos + {pa}); mjh::normalize4s(quat);")
        E(f"const double qs[4] = {arr_lit(m.qpos_spring[pa:pa + 4])};")
        E("mjh::subQuat(dif, quat, qs);")
        for c in range(3):
          E(f"qfs[{da + c}] = -{lit(k)}*dif[{c}];")
        E.close()
      else:
        E(f"qfs[{da}] = -{lit(k)}*(qpos[{pa}] - {lit(m.qpos_spring[pa])});")
    for dof in range(nv):
      b = float(m.dof_damping[dof])
      if b != 0:
        E(f"qfd[{dof}] = -{lit(b)}*qvel[{dof}];")
    for t in range(m.ntendon):
      k, b = float(m.tendon_stiffness[t]), float(m.tendon_damping[t])
      if (k == 0 and b == 0) or t in M.spatial:
        continue                       # spatial: the tendon pass re-forms mj_passive
      lo, hi = m.tendon_lengthspring[t]
      E.open()
      E(f"const double J[{nv}] = {arr_lit(M.ten_row(t))};")
      E(f"double L = ten_length[{t}], fs = 0;")
      E(f"if (L > {lit(hi)}) fs = {lit(k)} * ({lit(hi)} - L);")
      E(f"else if (L < {lit(lo)}) fs = {lit(k)} * ({lit(lo)} - L);")
      E(f"double fd = -{lit(b)} * ten_velocity_{t};")
      E(f"if (fs) mjh::addToScl(qfs, J, fs, {nv});")
      E(f"if (fd) mjh::addToScl(qfd, J, fd, {nv});")
      E.close()
  actgc = set()
  for j in range(M.njnt):
    if m.jnt_actgravcomp[j]:
      actgc.update(range(int(m.jnt_dofadr[j]), int(m.jnt_dofadr[j]) + M.jnt_ndof(j)))
  for dof in range(nv):
    G.st("qfrc_spring", dof, f"qfs[{dof}]")
    G.st("qfrc_damper", dof, f"qfd[{dof}]")
    G.st("qfrc_gravcomp", dof, f"qfg[{dof}]")
    G.st("qfrc_fluid", dof, "0.0")
    if dsbl & (1 << 5):
      G.st("qfrc_passive", dof, "0.0")
    elif has_gravcomp and dof not in actgc:
      G.st("qfrc_passive", dof, f"(qfs[{dof}] + qfd[{dof}]) + qfg[{dof}]")
    else:
      G.st("qfrc_passive", dof, f"qfs[{dof}] + qfd[{dof}]")

  # mj_comVel (:1833-1896) and both mj_rne calls (:1969-2023) in one tree pass
  E("// ---- tree pass: mj_comVel + mj_rne(flg_acc=0) + mj_rne(flg_acc=1)")
  if recompute:
    # frames, cinert and cdof recomputed along the pass as k_pos's pass 2 computes them (the
    # same operations on the same inputs: bit-identical values)
    roots = sorted(set(M.rootid[1:]))
    for r in roots:
      E(f"double keep_stc_{r}[3];")
      for c in range(3):
        E(f"keep_stc_{r}[{c}] = P_subtree_com[{3 * r + c}*64];")
    _world_frame(E)
  E("double cvel_0[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};")
  G.stv("cvel", 0, "cvel_0", 6)
  _gravity_acc(M, E)
  E("double acca_0[6]; mjh::copy(acca_0, cacc_0, 6);")
  E(f"double qacc[{nv}];")
  # row-major qfrc_inverse copy, or (no output array) a harmless second write of the mirror
  # slot: a select instead of a branch keeps the pass one scheduling region
  # the row-major qfrc_inverse copy goes through LDS (qo_lds[lane][k]); the kernel wrapper
  # writes the block's rows out coalesced after the body (an in-place row-major store per
  # dof would scatter 64 lanes over 64 rows)

  def recompute_body(i):
    """Body i's frame, cinert_i and cdof of its dofs (mj_kinematics, mj_comPos :211-268)."""
    _emit_frame(G, i, store=False)
    _emit_local2global(G, f"xipos_{i}", f"ximat_{i}", m.body_ipos[i], m.body_iquat[i], i,
                       int(m.body_sameframe[i]))
    E(f"double cinert_{i}[10];")
    E.open()
    E("double off[3];")
    E(f"mjh::sub3(off, xipos_{i}, keep_stc_{M.rootid[i]});")
    E(f"const double inert[3] = {arr_lit(m.body_inertia[i])};")
    E(f"mjh::inertCom(cinert_{i}, inert, ximat_{i}, off, {lit(M.mass[i])});")
    E.close()
    ja, jn = int(m.body_jntadr[i]), int(m.body_jntnum[i])
    for j in range(ja, ja + jn):
      da, t = int(m.jnt_dofadr[j]), int(m.jnt_type[j])
      for k in range(M.jnt_ndof(j)):
        E(f"double cdof_{da + k}[6];")
      E.open()
      E("double off[3], axis[3];")
      E(f"mjh::sub3(off, keep_stc_{M.rootid[i]}, xanchor_{j});")
      skip = 0
      if t == FREE:
        for k in range(3):
          E(f"mjh::zero(cdof_{da + k}, 6); cdof_{da + k}[{3 + k}] = 1.0;")
        skip = 3
      if t in (FREE, BALL):
        for k in range(3):
          E(f"axis[0] = xmat_{i}[{k}]; axis[1] = xmat_{i}[{k + 3}]; axis[2] = xmat_{i}[{k + 6}];")
          E(f"mjh::dofComHinge(cdof_{da + skip + k}, axis, off);")
      elif t == SLIDE:
        E(f"mjh::zero3(cdof_{da}); mjh::copy3(cdof_{da} + 3, xaxis_{j});")
      else:
        E(f"mjh::dofComHinge(cdof_{da}, xaxis_{j}, off);")
      E.close()

  def pre(i):
    if not i:
      return
    bda, dn = M.bdofadr[i], M.bdofnum[i]
    p = M.parent[i]
    E.open(f"{{  // body {i}")
    if recompute:
      recompute_body(i)
    E(f"double cvel_{i}[6];")
    E(f"mjh::copy(cvel_{i}, cvel_{p}, 6);")
    j = 0
    while j < dn:
      t = int(m.jnt_type[M.djnt[bda + j]])
      if t == FREE:
        for k in range(3):
          E(f"double cdofdot_{bda + k}[6] = {{0.0, 0.0, 0.0, 0.0, 0.0, 0.0}};")
        E.open()
        E("double tmp[6];")
        E("mjh::zero(tmp, 6);")
        for r in range(3):
          E(f"mjh::addToSclIf(tmp, cdof_{bda + r}, qvel[{bda + r}], 6);")
        E(f"mjh::addTo(cvel_{i}, tmp, 6);")
        E.close()
        j += 3
        t = BALL
      if t == BALL:
        for k in range(3):
          E(f"double cdofdot_{bda + j + k}[6];")
          E(f"mjh::crossMotion(cdofdot_{bda + j + k}, cvel_{i}, cdof_{bda + j + k});")
        E.open()
        E("double tmp[6];")
        E("mjh::zero(tmp, 6);")
        for r in range(3):
          E(f"mjh::addToSclIf(tmp, cdof_{bda + j + r}, qvel[{bda + j + r}], 6);")
        E(f"mjh::addTo(cvel_{i}, tmp, 6);")
        E.close()
        j += 3
      else:
        E(f"double cdofdot_{bda + j}[6];")
        E(f"mjh::crossMotion(cdofdot_{bda + j}, cvel_{i}, cdof_{bda + j});")
        E.open()
        E("double tmp[6];")
        E(f"mjh::scl(tmp, cdof_{bda + j}, qvel[{bda + j}], 6);")
        E(f"mjh::addTo(cvel_{i}, tmp, 6);")
        E.close()
        j += 1
    G.stv("cvel", 6 * i, f"cvel_{i}", 6)
    for k in range(bda, bda + dn):
      G.stv("cdof_dot", 6 * k, f"cdofdot_{k}", 6)
    # forward step of both recursions (engine_core_smooth.c:1986-2006)
    E(f"double cacc_{i}[6], cfrc_{i}[6], acca_{i}[6], frca_{i}[6];")
    E.open()
    E("double tmp[6], tmp1[6];")
    _emit_muldofvec(E, "tmp", "cdofdot", bda, dn, "qvel")
    E("mjh::pin(tmp, 6);")       # shared with _gen_acc: both round these terms alike
    E(f"mjh::add(cacc_{i}, cacc_{p}, tmp, 6);")
    E(f"mjh::add(acca_{i}, acca_{p}, tmp, 6);")
    _emit_muldofvec(E, "tmp", "cdof", bda, dn, "qacc")
    E(f"mjh::addTo(acca_{i}, tmp, 6);")
    E(f"mjh::mulInertVec(cfrc_{i}, cinert_{i}, cacc_{i});")
    E(f"mjh::mulInertVec(frca_{i}, cinert_{i}, acca_{i});")
    E(f"mjh::mulInertVec(tmp, cinert_{i}, cvel_{i});")
    E(f"mjh::crossForce(tmp1, cvel_{i}, tmp);")
    E("mjh::pin(tmp1, 6);")
    E(f"mjh::addTo(cfrc_{i}, tmp1, 6);")
    E(f"mjh::addTo(frca_{i}, tmp1, 6);")
    E.close()

  def post(i):
    if not i:
      return
    # cfrc_i is final (children added in descending order): project, then add to the parent
    # (engine_core_smooth.c:2008-2022); qfrc_inverse += armature*qacc - passive - constraint
    cd = "cdofp"
    for k in range(M.bdofadr[i], M.bdofadr[i] + M.bdofnum[i]):
      G.st("qfrc_bias", k, f"mjh::dot6({cd}_{k}, cfrc_{i})")
      E.open()
      E(f"double qfi = mjh::dot6({cd}_{k}, frca_{i});")
      if M.cmode == "all":     # raw rne: k_constraint assembles every instance
        G.st("qfrc_inverse", k, "qfi")
      else:
        E(f"const double qfa = qfi + ({lit(m.dof_armature[k])} * qacc[{k}] - qfp_{k} - 0.0);")
        if M.cmode == "list":
          E("qfi = cflag ? qfi : qfa;")
        else:
          E("qfi = qfa;")
        G.st("qfrc_constraint", k, "0.0")
        G.st("qfrc_inverse", k, "qfi")
        E(f"qo_lds[{_ll('va')[0]}*{nv} + {k}] = qfi;")
      E.close()
    if M.parent[i]:
      E(f"mjh::addTo(cfrc_{M.parent[i]}, cfrc_{i}, 6);")
      E(f"mjh::addTo(frca_{M.parent[i]}, frca_{i}, 6);")
    E.close()

  def loads(kind, i):
    dofs = range(M.bdofadr[i], M.bdofadr[i] + M.bdofnum[i])
    if recompute and kind == "pre":     # cinert and cdof recomputed, qacc from the mirror
      return [], [(f"qacc[{k}]", "qacc", k) for k in dofs]
    if kind == "pre":
      decls = [f"double cinert_{i}[10];"] + [f"double cdof_{k}[6];" for k in dofs]
      ld = _vec_loads(f"cinert_{i}", "cinert", 10 * i, 10)
      for k in dofs:
        ld += _vec_loads(f"cdof_{k}", "cdof", 6 * k, 6) + [(f"qacc[{k}]", "qacc", k)]
    else:   # the projections reload cdof rather than keeping it live along the path
      decls = [f"double cdofp_{k}[6], qfp_{k};" for k in dofs]
      ld = []
      for k in dofs:
        ld += _vec_loads(f"cdofp_{k}", "cdof", 6 * k, 6) + [(f"qfp_{k}", "qfrc_passive", k)]
    return decls, ld

  _prefetched_dfs(G, loads, pre, post, PREFETCH)
  if M.cmode == "none":
    E("ec[0] = 0; ec[64] = 0; ec[128] = 0; ec[192] = 0;")
  elif M.cmode == "list":   # served instances get their counts from k_constraint
    E("if (!cflag) { ec[0] = 0; ec[64] = 0; ec[128] = 0; ec[192] = 0; }")
  E("if (status) status[inst] = 0;")
  return E.text()


def _perturb_loads(body: str, which: dict) -> str:
  """mjd_inverseFD's perturbation applied as an input lands: `arr[k] = <load>;` becomes
  `arr[k] = k == idx ? <load> + eps : <load>;` for arr in `which` (arr -> index variable), the
  sum k_fd_expand would have stored (engine_derivative_fd.c:646-699: x[i] + eps)."""
  import re

  def sub(mt):
    arr, k, rhs = mt.group(2), mt.group(3), mt.group(4)
    return (f"{mt.group(1)}{arr}[{k}] = ({which[arr]} == {k}) ? ({rhs}) + eps : ({rhs});")
  names = "|".join(which)
  out, n = re.subn(rf"^(\s*)({names})\[(\d+)\] = (.*P_(?:{names})\[\d+\*64\].*);$", sub,
                   body, flags=re.M)
  # every line that loads a perturbed input must have been rewritten: a load of another shape
  # would silently leave that Jacobian column unperturbed (zero)
  loads = len(re.findall(rf"^.*P_(?:{names})\[[^\]]+\](?!\)? ?=[^=]).*$", body, flags=re.M))
  assert n == loads, f"_perturb_loads: rewrote {n} of {loads} lines loading {sorted(which)}"
  return out


def _gen_acc(M: _Model, store_fields=None) -> str:
  """The acceleration stage alone: mj_inverseSkip(mjSTAGE_VEL) (engine_inverse.c:197-261)
  with the position and velocity stages' outputs read from the mirror. One tree pass of
  mj_rne(flg_acc = 1) (engine_core_smooth.c:1969-2023) over the stored cinert, cdof, cvel and
  cdof_dot, then the assembly qfrc_inverse += armature*qacc - passive - constraint, with the
  same operations as the va stage's second recursion, so the result is its bit for bit. An
  instance with rows (work-list models) stores the raw RNE for the rows pass (k_skip_rows)."""
  G = _Stage(M, store_fields)
  M.acc_stored = G.stored
  E, m = G.E, M.m
  nv = M.nv
  G.prologue()
  if M.cmode == "list":
    E("const bool cflag = ec[0] != 0;")
  G.pointers(["qvel", "qacc", "cinert", "cdof", "cvel", "cdof_dot", "qfrc_passive",
              "qfrc_constraint", "qfrc_inverse"])
  G.load("qvel", "qvel", nv)
  E(f"double qacc[{nv}];")
  E("// ---- tree pass: mj_rne(flg_acc=1) over the stored velocity-stage outputs")
  _gravity_acc(M, E)
  E("double acca_0[6]; mjh::copy(acca_0, cacc_0, 6);")

  def pre(i):
    if not i:
      return
    bda, dn = M.bdofadr[i], M.bdofnum[i]
    p = M.parent[i]
    E.open(f"{{  // body {i}")
    E(f"double acca_{i}[6], frca_{i}[6];")
    E.open()
    E("double tmp[6], tmp1[6];")
    _emit_muldofvec(E, "tmp", "cdofdot", bda, dn, "qvel")
    E("mjh::pin(tmp, 6);")       # as _gen_va pins them (there each has two uses)
    E(f"mjh::add(acca_{i}, acca_{p}, tmp, 6);")
    _emit_muldofvec(E, "tmp", "cdof", bda, dn, "qacc")
    E(f"mjh::addTo(acca_{i}, tmp, 6);")
    E(f"mjh::mulInertVec(frca_{i}, cinert_{i}, acca_{i});")
    E(f"mjh::mulInertVec(tmp, cinert_{i}, cvel_{i});")
    E(f"mjh::crossForce(tmp1, cvel_{i}, tmp);")
    E("mjh::pin(tmp1, 6);")
    E(f"mjh::addTo(frca_{i}, tmp1, 6);")
    E.close()

  def post(i):
    if not i:
      return
    for k in range(M.bdofadr[i], M.bdofadr[i] + M.bdofnum[i]):
      E.open()
      E(f"double qfi = mjh::dot6(cdofp_{k}, frca_{i});")
      if M.cmode == "all":
        G.st("qfrc_inverse", k, "qfi")
      else:
        E(f"const double qfa = qfi + ({lit(m.dof_armature[k])} * qacc[{k}] - qfp_{k} - 0.0);")
        E("qfi = cflag ? qfi : qfa;" if M.cmode == "list" else "qfi = qfa;")
        G.st("qfrc_constraint", k, "0.0")
        G.st("qfrc_inverse", k, "qfi")
        E(f"qo_lds[{_ll('va')[0]}*{nv} + {k}] = qfi;")
      E.close()
    if M.parent[i]:
      E(f"mjh::addTo(frca_{M.parent[i]}, frca_{i}, 6);")
    E.close()

  def loads(kind, i):
    dofs = range(M.bdofadr[i], M.bdofadr[i] + M.bdofnum[i])
    if kind == "pre":
      decls = [f"double cinert_{i}[10], cvel_{i}[6];"] + \
          [f"double cdof_{k}[6], cdofdot_{k}[6];" for k in dofs]
      ld = _vec_loads(f"cinert_{i}", "cinert", 10 * i, 10) + \
          _vec_loads(f"cvel_{i}", "cvel", 6 * i, 6)
      for k in dofs:
        ld += _vec_loads(f"cdof_{k}", "cdof", 6 * k, 6) + \
            _vec_loads(f"cdofdot_{k}", "cdof_dot", 6 * k, 6) + [(f"qacc[{k}]", "qacc", k)]
    else:
      decls = [f"double cdofp_{k}[6], qfp_{k};" for k in dofs]
      ld = []
      for k in dofs:
        ld += _vec_loads(f"cdofp_{k}", "cdof", 6 * k, 6) + [(f"qfp_{k}", "qfrc_passive", k)]
    return decls, ld

  _prefetched_dfs(G, loads, pre, post, PREFETCH)
  E("if (status) status[inst] = 0;")
  return E.text()


def _emit_applyforce(E, M, b):
  """mj_gravcomp -> mj_applyFT(force, torque = 0, xipos, body) (engine_passive.c:381-399,
  engine_support.c:1194-1251, mj_jac :389-441) accumulated into qfg. Reads xipos, subtree_com
  and cdof from the mirror (k_pos wrote them)."""
  m, nv = M.m, M.nv
  g = [float(x) for x in m.opt["gravity"]]
  s = -(float(m.body_mass[b]) * float(m.body_gravcomp[b]))
  r = M.rootid[b]
  E.open()
  E(f"double force[3] = {{{lit(g[0])}*{lit(s)}, {lit(g[1])}*{lit(s)}, {lit(g[2])}*{lit(s)}}};")
  E(f"double jacp[{3*nv}], jacr[{3*nv}], qforce[{nv}], off[3];")
  E(f"mjh::zero(jacp, {3*nv}); mjh::zero(jacr, {3*nv});")
  E(f"off[0] = P_xipos[{3*b}*64] - P_subtree_com[{3*r}*64];")
  E(f"off[1] = P_xipos[{3*b + 1}*64] - P_subtree_com[{3*r + 1}*64];")
  E(f"off[2] = P_xipos[{3*b + 2}*64] - P_subtree_com[{3*r + 2}*64];")
  body = b
  while body and not m.body_dofnum[body]:
    body = int(m.body_parentid[body])
  if body:
    i = int(m.body_dofadr[body] + m.body_dofnum[body] - 1)
    while i >= 0:
      E.open()
      E("double cd[6], tmp[3];")
      for c in range(6):
        E(f"cd[{c}] = P_cdof[{6*i + c}*64];")
      E(f"jacr[{i}] = cd[0]; jacr[{i + nv}] = cd[1]; jacr[{i + 2*nv}] = cd[2];")
      E("mjh::cross(tmp, cd, off);")
      E(f"jacp[{i}] = cd[3] + tmp[0]; jacp[{i + nv}] = cd[4] + tmp[1]; "
        f"jacp[{i + 2*nv}] = cd[5] + tmp[2];")
      E.close()
      i = int(m.dof_parentid[i])
  E(f"mjh::mulMatTVec(qforce, jacp, force, 3, {nv}); mjh::addTo(qfg, qforce, {nv});")
  E("double zt[3] = {0.0, 0.0, 0.0};")
  E(f"mjh::mulMatTVec(qforce, jacr, zt, 3, {nv}); mjh::addTo(qfg, qforce, {nv});")
  E.close()


# ------------------------------------------------------------------------------ assembly
def model_hash(m) -> str:
  h = hashlib.sha1()
  for f in fields.MODEL_FIELDS:
    h.update(np.ascontiguousarray(getattr(m, f.name)).tobytes())
  h.update(repr(sorted(m.opt.items())).encode())
  return h.hexdigest()[:12]


_SIG = {
    "pos": ("const double* __restrict__ qpos_in, const double* __restrict__ qvel_in, "
            "const double* __restrict__ qacc_in, int* __restrict__ worklist, "
            "int* __restrict__ worklist_count, int* __restrict__ worklist_next, "
            "int* __restrict__ efc_count, double* __restrict__ trig, double* __restrict__ qmr",
            "qpos_in, qvel_in, qacc_in, worklist, worklist_count, worklist_next, efc_count, trig, "
            "qmr"),
    "fac": ("int* __restrict__ efc_count, const double* __restrict__ qmr", "efc_count, qmr"),
    "va": ("double* __restrict__ qfrc_out, int* __restrict__ status, "
           "int* __restrict__ efc_count, double* __restrict__ qo_lds, "
           "double* __restrict__ trig",
           "qfrc_out, status, efc_count, qo_lds, trig"),
}
_GEN = {"pos": lambda M, sf: _gen_pos(M, sf), "fac": lambda M, sf: _gen_fac(M, sf),
        "va": lambda M, sf: _gen_va(M, sf)}


def generate(m, name: str, store_fields=None, extern_c: bool = False, shared: bool = False) -> str:
  """HIP source of the four stage kernels of model `m` (skipstage = mjSTAGE_NONE).

  Also emits `fast_body_<name>`, which runs the four stage bodies for one instance in
  order (the host harness's entry), and `launch_fast_<name>`, which launches the kernels.
  store_fields: optional set of mirror fields to store (default: all); used only by
  performance experiments (tools/exp_bounds.py) to separate compute from store costs.
  shared: the launch functions get external linkage (a model compiled in another
  translation unit than the registry, generate_registries).
  extern_c: give k_all_<name> C linkage (a run-time code object, specialize.py, whose
  kernel mjhip_contextLoadKernel looks up by name).
  """
  why = fast_path_supported(m)
  if why:
    raise ValueError(f"model '{name}' cannot use the straight-line kernels: {why}")
  M = _Model(m)
  bodies = {st: _GEN[st](M, store_fields) for st in STAGES}
  if NT_STORES:
    import re
    # the fac stage's re-reads stay temporal; the other stages' re-reads stream only in the
    # SV = true instantiation of k_all (a batch large enough to oversubscribe L2, NT_SV_MIN_B)
    reread = set(re.findall(r"= P_(\w+)\[", bodies["fac"]))
    later = set(re.findall(r"= P_(\w+)\[", "\n".join(bodies.values()))) - reread
    if NT_TEMPORAL is not None:
      reread, later = set(NT_TEMPORAL), set()
    store = re.compile(r"^(\s*)P_(\w+)\[(\d+)\*64\] = (.+);$")

    def nt(line):
      mt = store.match(line)
      if not mt or mt.group(2) in reread:
        return line
      if mt.group(2) in later:
        return (f"{mt.group(1)}MJH_NT_STORE_IF(SV, P_{mt.group(2)}[{mt.group(3)}*64], "
                f"{mt.group(4)});")
      return f"{mt.group(1)}MJH_NT_STORE(P_{mt.group(2)}[{mt.group(3)}*64], {mt.group(4)});"
    bodies = {st: ("\n".join(nt(x) for x in b.split("\n")) if st in NT_STAGES else b)
              for st, b in bodies.items()}
    load = re.compile(r"= P_(\w+)\[(\d+)\*64\];")
    bodies = {st: (load.sub(lambda mt: f"= MJH_NT_LOAD(P_{mt.group(1)}[{mt.group(2)}*64]);", b)
                   if st in NT_LOAD_STAGES else b) for st, b in bodies.items()}
    bodies = {st: (load.sub(lambda mt: f"= MJH_NT_LOAD_IF(SV, P_{mt.group(1)}[{mt.group(2)}*64]);",
                            b)
                   if st in NT_LOAD_SV_STAGES and st not in NT_LOAD_STAGES else b)
              for st, b in bodies.items()}
  if M.cmode in ("none", "list") and store_fields is None:
    elided = fd_elided(bodies.values())
    bodies = {st: _elide_stores(b, elided) for st, b in bodies.items()}
  out = [f"// GENERATED by mujoco_inversedynamicstest_amd/codegen.py -- do not edit.",
         f"// model '{name}' (nq={m.nq} nv={m.nv} nbody={m.nbody}), hash {model_hash(m)}"]
  exact = exact_fp(m)
  if exact:   # frames for the native solver: every operation rounded (exact_fp)
    out.append("#if defined(__clang__)\n#pragma clang fp contract(off)\n#endif")
  for st in STAGES:
    params, args = _SIG[st]
    out.append(f"template <bool SV = true, bool FD = false>\n"
               f"MJH_HD void fast_{st}_{name}(const Mirror& mr, int blk, int lane, int B, "
               f"{params}) {{\n{bodies[st]}\n}}\n")
  out.append(f"""MJH_HD void fast_body_{name}(
    const Mirror& mr, int blk, int lane, int B, const double* __restrict__ qpos_in,
    const double* __restrict__ qvel_in, const double* __restrict__ qacc_in,
    double* __restrict__ qfrc_out, int* __restrict__ status, int* __restrict__ worklist,
    int* __restrict__ worklist_count, int* __restrict__ worklist_next,
    int* __restrict__ efc_count) {{
  double trig[{max(1, 2 * len(M.trig) * 64)}];   // LDS on the device (k_pos)
  double qo_lds[{64 * max(M.nv, 1)}];             // LDS on the device (k_va)
  double qmr[{max(1, m.nM)}];                        // registers on the device (k_all)
  const bool fd = mr.fd_elide && blk >= mr.full_blk;   // mjd_inverseFD's perturbed blocks
""" + "".join(f"  if (fd) fast_{st}_{name}<true, true>(mr, blk, lane, B, {_SIG[st][1]});\n"
              f"  else fast_{st}_{name}<true, false>(mr, blk, lane, B, {_SIG[st][1]});\n"
              for st in STAGES)
             + (f"""  if (qfrc_out && (long)blk*64 + lane < B) {{
    for (int k = 0; k < {M.nv}; k++) qfrc_out[((long)blk*64 + lane)*{M.nv} + k] = qo_lds[lane*{M.nv} + k];
  }}
""" if M.cmode != "all" else "  (void)qo_lds;\n") + "}\n")
  out.append("#if defined(__HIPCC__)")
  for st in STAGES:
    params, args = _SIG[st]
    tail = ""
    nl = LANES[st]
    sub = 64 // nl    # workgroups per 64-instance block
    params = params.replace(", double* __restrict__ qmr", "").replace(
        ", const double* __restrict__ qmr", "")
    args = args.replace(", qmr", ", nullptr")      # staged: qM goes through the mirror
    if st == "pos":
      params = params.replace(", double* __restrict__ trig", "")
      decl = f"  __shared__ double trig[{max(1, 2 * len(M.trig) * nl)}];\n"
    elif st == "va":
      params = params.replace(", double* __restrict__ qo_lds", "")
      params = params.replace(", double* __restrict__ trig", "")
      args = args.replace(", trig", ", nullptr")   # staged k_va: no LDS trig (not fused)
      decl = f"  __shared__ double qo_lds[{nl * max(M.nv, 1)}];\n"
      if M.cmode != "all":   # coalesced row-major copy of the workgroup's qfrc_inverse rows
        tail = (f"  if (!qfrc_out) return;\n  __syncthreads();\n"
                f"  const long r0 = (long)blockIdx.x*{nl};\n"
                f"  const long n = ((long)B - r0 < {nl} ? (long)B - r0 : {nl}) * {M.nv};\n"
                f"  double* dst = qfrc_out + r0*{M.nv};\n"
                f"  for (long r = threadIdx.x; r < n; r += {nl}) dst[r] = qo_lds[r];\n")
    else:
      decl = ""
    if sub == 1:
      bl = "blockIdx.x, threadIdx.x"
    else:
      bl = f"blockIdx.x / {sub}, (blockIdx.x % {sub})*{nl} + threadIdx.x"
    out.append(f"__global__ __launch_bounds__({nl}, 1) void k_{st}_{name}(Mirror mr, int B, "
               f"{params}) {{\n{decl}  fast_{st}_{name}(mr, {bl}, B, {args});\n"
               f"{tail}}}")
  # k_all: the three stage bodies back to back in one launch. Each stage re-reads what the
  # previous one stored (a compiler memory barrier between them keeps the reloads), so the
  # live ranges stay those of the staged kernels; the reloads hit the wave's own freshly
  # written lines in L2, and no wave waits for the whole grid at a kernel boundary.
  nl = ALL_LANES
  if nl != 64:
    assert all(LANES[st] == nl for st in STAGES), "stage LDS indexing must match ALL_LANES"
  sub = 64 // nl
  ntrig = max(1, 2 * len(M.trig) * nl)
  nqo = nl * max(M.nv, 1)
  fuse_tail = ""
  if M.cmode != "all":
    fuse_tail = (f"  if (!qfrc_out) return;\n  __syncthreads();\n"
                 f"  const long r0 = (long)blockIdx.x*{nl};\n"
                 f"  const long n = ((long)B - r0 < {nl} ? (long)B - r0 : {nl}) * {M.nv};\n"
                 f"  double* dst = qfrc_out + r0*{M.nv};\n"
                 f"  for (long r = threadIdx.x; r < n; r += {nl}) dst[r] = qo_lds[r];\n")
  bl = "blk0 + blockIdx.x, threadIdx.x" if sub == 1 else \
      f"blk0 + blockIdx.x / {sub}, (blockIdx.x % {sub})*{nl} + threadIdx.x"
  fuse_tail = fuse_tail.replace("(long)blockIdx.x*", f"((long)blk0*{sub} + blockIdx.x)*")
  linkage = 'extern "C" ' if extern_c else ""
  # range: null, or a device-side instance range {first, end} (first a multiple of 64) read
  # at the start of the launch, so a launch's extent can be decided by an earlier kernel on
  # the stream (mjhip_inverseFDBatch's limit-centre fall-back) without a host round trip.
  # The next call's work-list counter is zeroed by the launch's first thread, before any
  # instance bound, so an empty range still hands the counters on.
  # SV: the va stage's re-read fields stream too (a batch that oversubscribes L2); a
  # run-time code object (C linkage, no template) has the SV = true kernel only
  tmpl = "" if extern_c else "template <bool SV, bool FD>\n"
  sv = "true" if extern_c else "SV"

  def stage_calls(fd, ind="  "):
    return "\n".join(f"{ind}fast_{st}_{name}<{sv}, {fd}>(mr, {bl}, B, "
                     f"{_SIG[st][1].replace('worklist_next', 'nullptr')});\n"
                     f"{ind}asm volatile(\"\" ::: \"memory\"); MJH_SCHED_FENCE(); MJH_PHASE({20 + k});"
                     for k, st in enumerate(STAGES))
  # the FD instantiation (mjd_inverseFD's stage-skip layout): the plain bodies on the centres'
  # blocks, the bodies without the elided stores on the blocks past them (Mirror::full_blk)
  blkexpr = "blk0 + (int)blockIdx.x" if sub == 1 else f"blk0 + (int)blockIdx.x / {sub}"
  all_calls = stage_calls("false") if extern_c else (
      f"  if (FD && mr.fd_elide && {blkexpr} >= mr.full_blk) {{\n{stage_calls('true', '    ')}\n"
      f"  }} else {{\n{stage_calls('false', '    ')}\n  }}")
  out.append(f"""{tmpl}{linkage}__global__ __launch_bounds__({nl}, {ALL_WAVES}) void k_all_{name}(Mirror mr, int B,
    const double* __restrict__ qpos_in, const double* __restrict__ qvel_in,
    const double* __restrict__ qacc_in, double* __restrict__ qfrc_out, int* __restrict__ status,
    int* __restrict__ worklist, int* __restrict__ worklist_count, int* __restrict__ worklist_next,
    int* __restrict__ efc_count, const int* __restrict__ range) {{
  __shared__ double trig[{ntrig}];
  __shared__ double qo_lds[{nqo}];
  double qmr[{max(1, m.nM)}];
  if (worklist_next && blockIdx.x == 0 && threadIdx.x == 0) *worklist_next = 0;
  int blk0 = 0;
  if (range) {{ blk0 = range[0] >> 6; B = range[1]; }}
  MJH_PHASE0(19, 27);
""" + all_calls + "\n" + fuse_tail + "}")
  # the split launch of a model whose constraint rows serve every instance (contacts): the
  # position stage alone (k_spos), then the fac and va stages (k_sfv), so that the
  # cooperative constraint kernel -- which reads only position-stage outputs and the inputs
  # -- runs on a second stream beside k_sfv, and the assembly kernel (mjhip.hip k_assemble)
  # joins them (mjhip.hip launch_inverse). Same stage bodies as k_all, so the same results.
  if M.cmode == "all" and not extern_c:
    pos_args = _SIG["pos"][1].replace("trig, qmr", "trig, nullptr")
    out.append(f"""template <bool SV>
__global__ __launch_bounds__(64, 1) void k_spos_{name}(Mirror mr, int B,
    const double* __restrict__ qpos_in, const double* __restrict__ qvel_in,
    const double* __restrict__ qacc_in, int* __restrict__ worklist,
    int* __restrict__ worklist_count, int* __restrict__ worklist_next,
    int* __restrict__ efc_count) {{
  __shared__ double trig[{ntrig}];
  MJH_PHASE0(19, 27);
  fast_pos_{name}<SV>(mr, blockIdx.x, threadIdx.x, B, {pos_args});
}}
template <bool SV>
__global__ __launch_bounds__(64, 1) void k_sfv_{name}(Mirror mr, int B,
    double* __restrict__ qfrc_out, int* __restrict__ status, int* __restrict__ efc_count) {{
  __shared__ double qo_lds[{nqo}];
  MJH_PHASE(20);     // the position span runs from k_spos's start to here (launch gap included)
  fast_fac_{name}<SV>(mr, blockIdx.x, threadIdx.x, B, efc_count, nullptr);
  asm volatile("" ::: "memory"); MJH_SCHED_FENCE(); MJH_PHASE(21);
  fast_va_{name}<SV>(mr, blockIdx.x, threadIdx.x, B, qfrc_out, status, efc_count, qo_lds,
                     nullptr);
  asm volatile("" ::: "memory"); MJH_SCHED_FENCE(); MJH_PHASE(22);
}}
{"" if shared else "static "}void launch_split_{name}(hipStream_t s, const Mirror& mr, int B, int part,
    const double* qpos_in, const double* qvel_in, const double* qacc_in, int* status,
    int* worklist_next, int* efc_count) {{
  const dim3 g((B + 63) / 64), b(64);
  if (part == 0) {{
    if (B >= {NT_SV_MIN_B}) {{
      hipLaunchKernelGGL(k_spos_{name}<true>, g, b, 0, s, mr, B, qpos_in, qvel_in, qacc_in,
                         nullptr, nullptr, worklist_next, efc_count);
    }} else {{
      hipLaunchKernelGGL(k_spos_{name}<false>, g, b, 0, s, mr, B, qpos_in, qvel_in, qacc_in,
                         nullptr, nullptr, worklist_next, efc_count);
    }}
  }} else if (B >= {NT_SV_MIN_B}) {{
    hipLaunchKernelGGL(k_sfv_{name}<true>, g, b, 0, s, mr, B, nullptr, status, efc_count);
  }} else {{
    hipLaunchKernelGGL(k_sfv_{name}<false>, g, b, 0, s, mr, B, nullptr, status, efc_count);
  }}
}}""")
  # batched mj_inverseSkip(POS / VEL) of a model whose rows serve every instance (contacts):
  # k_va (the staged va kernel) or k_acc store the raw RNE, and k_skip_rows (mjhip.hip)
  # finishes every instance -- the previous call's rows (referenceConstraint for POS,
  # invConstraint) and the assembly -- and writes the row-major output
  if M.cmode == "all" and not extern_c:
    import re
    ab = _gen_acc(M)
    if NT_STORES:
      ab = re.sub(r"^(\s*)P_(\w+)\[(\d+)\*64\] = (.+);$",
                  lambda mt: f"{mt.group(1)}MJH_NT_STORE(P_{mt.group(2)}[{mt.group(3)}*64], "
                             f"{mt.group(4)});", ab, flags=re.M)
    out.append(f"MJH_HD void fast_acc_{name}(const Mirror& mr, int blk, int lane, int B, "
               f"{_SIG['va'][0]}) {{\n{ab}\n}}\n")
    out.append(f"""__global__ __launch_bounds__(64, 1) void k_acc_{name}(Mirror mr, int B,
    double* __restrict__ qfrc_out, int* __restrict__ status, int* __restrict__ efc_count) {{
  fast_acc_{name}(mr, blockIdx.x, threadIdx.x, B, qfrc_out, status, efc_count, nullptr,
                  nullptr);
}}
{"" if shared else "static "}void launch_skip_{name}(hipStream_t s, const Mirror& mr, int B, int skipstage,
                              double* qfrc_out, int* status, int* efc_count) {{
  (void)qfrc_out;      // raw RNE only: k_skip_rows assembles and writes the output
  if (skipstage == 1) {{
    hipLaunchKernelGGL(k_va_{name}, dim3((B + 63) / 64), dim3(64), 0, s, mr, B, nullptr,
                       status, efc_count);
  }} else {{
    hipLaunchKernelGGL(k_acc_{name}, dim3((B + 63) / 64), dim3(64), 0, s, mr, B, nullptr,
                       status, efc_count);
  }}
}}""")
  # k_vaskip: the va stage of mj_inverseSkip(mjSTAGE_POS) for mjd_inverseFD's qvel and qacc
  # perturbations (engine_derivative_fd.c:646-699). Instance off + t reads every position-
  # stage output (the va pointers it never stores) from its centre instance
  # (t / per)*sstride, which ran the full kernel; its own qvel/qacc and every field the stage
  # stores stay its own. Skipped stages see unchanged inputs, so the result is the full
  # pipeline's bit for bit. Work-list models: a centre with limit rows sets *needfull, and
  # k_fd_gate (mjhip.hip) then opens the range of a second k_all over the qvel/qacc
  # perturbations, which runs their full pipeline.
  if M.cmode in ("none", "list"):
    import re
    vb = bodies["va"]
    # the fields the va stage stores, as recorded by _Stage.st while emitting it; a store the
    # record missed would leave that pointer based at the centre instance, and all 2nv
    # perturbations would write the centre's slot concurrently, so the text is checked too
    textual = set(re.findall(r"P_(\w+)\[[^\]]+\]\)? ?=[^=]", vb)) | \
        set(re.findall(r"MJH_NT_STORE\(P_(\w+)\[", vb))
    # qpos/qvel/qacc are based at the centre instance unless stored (then `own` keeps them)
    assert textual <= M.va_stored, \
        f"k_vaskip: va stores outside the record: {textual - M.va_stored}"
    # qpos, qvel and qacc are read from the centre too: k_fd_expand writes only the
    # position-stage block, and the perturbed component is added as the loads land (pa / pv:
    # the qacc / qvel dof this instance perturbs, -1 for none)
    own = set(M.va_stored)
    skip_body = re.sub(r"(double\* __restrict__ P_(\w+) = mr\.\w+ \+ \(\(long\))blk(\*\d+\)\*64 \+ )lane;",
                       lambda mt: mt.group(0) if mt.group(2) in own else
                       f"{mt.group(1)}sblk{mt.group(3)}slane;", vb)
    skip_body = skip_body.replace("const bool cflag = ec[0] != 0;",
                                  "const bool cflag = ecs[0] != 0;")
    skip_body = skip_body.replace("MJH_NT_STORE_IF(SV, ", "MJH_NT_STORE_IF(true, ")
    skip_body = skip_body.replace("if constexpr (!FD) {", "if constexpr (false) {")
    assert "FD" not in re.sub(r"\w*FD\w+|\w+FD\w*", "", skip_body), "k_vaskip: FD left"
    skip_body = skip_body.replace("MJH_NT_LOAD_IF(SV, ", "MJH_NT_LOAD_IF(false, ")
    skip_body = _perturb_loads(skip_body, {"qvel": "pv", "qacc": "pa"})
    out.append(f"MJH_HD void fast_vaskip_{name}(const Mirror& mr, int blk, int lane, int sblk, "
               f"int slane, int B, const int* __restrict__ ecs, int pa, int pv, double eps, "
               f"{_SIG['va'][0]}) {{\n{skip_body}\n}}\n")
  if M.cmode in ("none", "list"):
    # the acceleration stage alone (mj_inverseSkip(mjSTAGE_VEL)): k_acc for batched calls, and
    # in k_fdskip for mjd_inverseFD's qacc perturbations, whose velocity-stage inputs (cvel,
    # cdof_dot, qfrc_passive) and position-stage inputs are their centre's
    import re
    ab = _gen_acc(M)
    if NT_STORES:
      ab = re.sub(r"^(\s*)P_(\w+)\[(\d+)\*64\] = (.+);$",
                  lambda mt: f"{mt.group(1)}MJH_NT_STORE(P_{mt.group(2)}[{mt.group(3)}*64], "
                             f"{mt.group(4)});", ab, flags=re.M)
    out.append(f"MJH_HD void fast_acc_{name}(const Mirror& mr, int blk, int lane, int B, "
               f"{_SIG['va'][0]}) {{\n{ab}\n}}\n")
    own_acc = set(M.acc_stored)          # qacc from the centre, perturbed at pa
    acc_skip = re.sub(r"(double\* __restrict__ P_(\w+) = mr\.\w+ \+ \(\(long\))blk(\*\d+\)\*64 \+ )lane;",
                      lambda mt: mt.group(0) if mt.group(2) in own_acc else
                      f"{mt.group(1)}sblk{mt.group(3)}slane;", ab)
    acc_skip = acc_skip.replace("const bool cflag = ec[0] != 0;", "const bool cflag = ecs[0] != 0;")
    acc_skip = _perturb_loads(acc_skip, {"qacc": "pa"})
    out.append(f"MJH_HD void fast_accskip_{name}(const Mirror& mr, int blk, int lane, int sblk, "
               f"int slane, int B, const int* __restrict__ ecs, int pa, double eps, "
               f"{_SIG['va'][0]}) {{\n{acc_skip}\n}}\n")
  if M.cmode in ("none", "list"):
    flag = ("  if (ecs[0] != 0) needfull[0] = 1;\n" if M.cmode == "list" else "")
    pos_call = _SIG["pos"][1].replace("worklist_next", "nullptr")
    fac_call, va_call = _SIG["fac"][1], _SIG["va"][1]
    linkage_fd = "" if shared else "static "
    nv = M.nv
    out.append(f"""// layout 1 over [off, B): per = 2nv perturbations per centre, the first nv of qacc, the
// next nv of qvel (engine_derivative_fd.c:646-699 order)
__global__ __launch_bounds__(64, 1) void k_vaskip_{name}(Mirror mr, int B, int off,
    int per, int sstride, int* __restrict__ efc_count, int* __restrict__ needfull, double eps) {{
  __shared__ double qo_lds[{64 * max(M.nv, 1)}];
  const long gi = (long)off + (long)blockIdx.x*64 + threadIdx.x;
  if (gi >= B) return;
  const long si = (gi - off) / per * sstride;
  const int j = (int)((gi - off) % per);
  const int* ecs = efc_count + (si >> 6)*4*64 + (si & 63);
{flag}  fast_vaskip_{name}(mr, (int)(gi >> 6), (int)(gi & 63), (int)(si >> 6), (int)(si & 63), B,
                    ecs, j < {M.nv} ? j : -1, j < {M.nv} ? -1 : j - {M.nv}, eps, nullptr,
                    nullptr, efc_count, qo_lds, nullptr);
}}
{"" if shared else "static "}void launch_vaskip_{name}(hipStream_t s, const Mirror& mr, int B, int off, int per,
                                int sstride, int* efc_count, int* needfull, double eps) {{
  hipLaunchKernelGGL(k_vaskip_{name}, dim3((B - off + 63) / 64), dim3(64), 0, s, mr, B, off,
                     per, sstride, efc_count, needfull, eps);
}}
// mjd_inverseFD layout 1 in one launch (k_fdall, opt-in: MJHIP_FD_FUSED=1, measured slower
// than k_all then k_vaskip): the position-stage instances [0, B) -- the
// centres, then the qpos perturbations -- run the whole pipeline (FD: elided stores) on the
// first B/64 blocks, and the 2nv qvel/qacc perturbations per base state [B, ninst) run
// k_vaskip's va stage on the blocks after them, beside the qpos perturbations instead of
// after them. A skip lane reads its centre's position-stage outputs, so it first waits for
// the centre block's flag (flags[block] == epoch), which that block raises after its
// position stage behind a device-scope fence (its stores are visible on every XCD); the
// waiting side fences again before its loads. Blocks are dispatched in index order, so
// every centre block is running before any block that waits; the wait is bounded all the
// same, and a wave that gives up raises needfull[3] (the host reports it).
template <bool SV>
__global__ __launch_bounds__(64, 1) void k_fdall_{name}(Mirror mr, int B, int ninst, int per,
    double eps, int* __restrict__ worklist, int* __restrict__ worklist_count,
    int* __restrict__ worklist_next, int* __restrict__ efc_count, int* __restrict__ needfull,
    int* __restrict__ flags, int epoch) {{
  __shared__ double trig[{ntrig}];
  __shared__ double qo_lds[{nqo}];
  if (worklist_next && blockIdx.x == 0 && threadIdx.x == 0) *worklist_next = 0;
  const int nblk = B / 64;                  // B: a whole number of waves
  if ((int)blockIdx.x < nblk) {{
    double qmr[{max(1, m.nM)}];
    const double* qpos_in = nullptr;
    const double* qvel_in = nullptr;
    const double* qacc_in = nullptr;
    double* qfrc_out = nullptr;
    int* status = nullptr;
    const int blk = blockIdx.x, lane = threadIdx.x;
    if (blk < mr.full_blk) {{               // a centre block: every field, position stage out
      fast_pos_{name}<SV, false>(mr, blk, lane, B, {pos_call});
      asm volatile("" ::: "memory");
      __threadfence();
      if (lane == 0) __hip_atomic_store(flags + blk, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      MJH_SCHED_FENCE();
      fast_fac_{name}<SV, false>(mr, blk, lane, B, {fac_call});
      asm volatile("" ::: "memory"); MJH_SCHED_FENCE();
      fast_va_{name}<SV, false>(mr, blk, lane, B, {va_call});
    }} else {{
      fast_pos_{name}<SV, true>(mr, blk, lane, B, {pos_call});
      asm volatile("" ::: "memory"); MJH_SCHED_FENCE();
      fast_fac_{name}<SV, true>(mr, blk, lane, B, {fac_call});
      asm volatile("" ::: "memory"); MJH_SCHED_FENCE();
      fast_va_{name}<SV, true>(mr, blk, lane, B, {va_call});
    }}
    (void)qpos_in; (void)qvel_in; (void)qacc_in; (void)qfrc_out; (void)status;
    return;
  }}
  const long gi = (long)B + (long)(blockIdx.x - nblk)*64 + threadIdx.x;
  if (gi >= ninst) return;
  const long si = (gi - B) / per;
  const int j = (int)((gi - B) % per);
  for (int it = 0; __hip_atomic_load(flags + (si >> 6), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT) != epoch; it++) {{
    if (it >= {FD_WAIT_ITERS}) {{
      __hip_atomic_store(needfull + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }}
    __builtin_amdgcn_s_sleep(8);
  }}
  __threadfence();
  const int* ecs = efc_count + (si >> 6)*4*64 + (si & 63);
{flag}  fast_vaskip_{name}(mr, (int)(gi >> 6), (int)(gi & 63), (int)(si >> 6), (int)(si & 63), ninst,
                    ecs, j < {nv} ? j : -1, j < {nv} ? -1 : j - {nv}, eps, nullptr,
                    nullptr, efc_count, qo_lds, nullptr);
}}
{linkage_fd}void launch_fdall_{name}(hipStream_t s, const Mirror& mr, int B, int ninst, int per,
                               double eps, int* worklist, int* worklist_count,
                               int* worklist_next, int* efc_count, int* needfull, int* flags,
                               int epoch) {{
  const dim3 g((unsigned)((ninst + 63) / 64)), b(64);
  if (B >= {NT_SV_MIN_B}) {{
    hipLaunchKernelGGL((k_fdall_{name}<true>), g, b, 0, s, mr, B, ninst, per, eps, worklist,
                       worklist_count, worklist_next, efc_count, needfull, flags, epoch);
  }} else {{
    hipLaunchKernelGGL((k_fdall_{name}<false>), g, b, 0, s, mr, B, ninst, per, eps, worklist,
                       worklist_count, worklist_next, efc_count, needfull, flags, epoch);
  }}
}}
// mjd_inverseFD layout 2 in one launch over [off, B): the nq = (B - off)/2 qvel perturbations
// (mj_inverseSkip(mjSTAGE_POS): the va stage over the centre's position stage) on the first
// blocks, the longer waves, then the nq qacc perturbations (mjSTAGE_VEL: the acceleration
// stage over the centre's position and velocity stages). nq is a multiple of 64, so each wave
// has one role; the two run side by side instead of as two under-filled launches.
__global__ __launch_bounds__(64, 1) void k_fdskip_{name}(Mirror mr, int B, int off,
    int per, int sstride, int* __restrict__ efc_count, int* __restrict__ needfull, double eps) {{
  __shared__ double qo_lds[{64 * max(M.nv, 1)}];
  const long nq = ((long)B - off) / 2;
  const long t = (long)blockIdx.x*64 + threadIdx.x;
  if (t >= 2*nq) return;
  const bool vel = t < nq;
  const long gi = vel ? off + nq + t : off + (t - nq);
  const long si = (vel ? t : t - nq) / per * sstride;
  const int j = (int)((vel ? t : t - nq) % per);
  const int* ecs = efc_count + (si >> 6)*4*64 + (si & 63);
{flag}  if (vel) {{
    fast_vaskip_{name}(mr, (int)(gi >> 6), (int)(gi & 63), (int)(si >> 6), (int)(si & 63), B,
                      ecs, -1, j, eps, nullptr, nullptr, efc_count, qo_lds, nullptr);
  }} else {{
    fast_accskip_{name}(mr, (int)(gi >> 6), (int)(gi & 63), (int)(si >> 6), (int)(si & 63), B,
                       ecs, j, eps, nullptr, nullptr, efc_count, qo_lds, nullptr);
  }}
}}
{"" if shared else "static "}void launch_fdskip_{name}(hipStream_t s, const Mirror& mr, int B, int off, int per,
                                int sstride, int* efc_count, int* needfull, double eps) {{
  hipLaunchKernelGGL(k_fdskip_{name}, dim3((B - off + 63) / 64), dim3(64), 0, s, mr, B, off,
                     per, sstride, efc_count, needfull, eps);
}}
// batched mj_inverseSkip on the straight-line path: POS runs the va stage (k_va), VEL the
// acceleration stage (k_acc); rows of the previous call go through k_skip_rows (mjhip.hip)
__global__ __launch_bounds__(64, 1) void k_acc_{name}(Mirror mr, int B,
    double* __restrict__ qfrc_out, int* __restrict__ status, int* __restrict__ efc_count) {{
  __shared__ double qo_lds[{64 * max(M.nv, 1)}];
  fast_acc_{name}(mr, blockIdx.x, threadIdx.x, B, qfrc_out, status, efc_count, qo_lds, nullptr);
  if (!qfrc_out) return;
  __syncthreads();
  const long r0 = (long)blockIdx.x*64;
  const long n = ((long)B - r0 < 64 ? (long)B - r0 : 64) * {M.nv};
  double* dst = qfrc_out + r0*{M.nv};
  for (long r = threadIdx.x; r < n; r += 64) dst[r] = qo_lds[r];
}}
{"" if shared else "static "}void launch_skip_{name}(hipStream_t s, const Mirror& mr, int B, int skipstage,
                              double* qfrc_out, int* status, int* efc_count) {{
  if (skipstage == 1) {{
    hipLaunchKernelGGL(k_va_{name}, dim3((B + 63) / 64), dim3(64), 0, s, mr, B, qfrc_out,
                       status, efc_count);
  }} else {{
    hipLaunchKernelGGL(k_acc_{name}, dim3((B + 63) / 64), dim3(64), 0, s, mr, B, qfrc_out,
                       status, efc_count);
  }}
}}""")
  out.append(f"""{"" if shared else "static "}void launch_fast_{name}(dim3 g, dim3 b, hipStream_t s, const Mirror& mr,
    int B, const double* qpos_in, const double* qvel_in, const double* qacc_in, double* qfrc_out,
    int* status, int* worklist, int* worklist_count, int* worklist_next, int* efc_count,
    const int* range) {{""")
  if FUSE:
    gb = "g, b" if ALL_LANES == 64 else f"dim3(g.x*{64 // ALL_LANES}), dim3({ALL_LANES})"
    variants = ((f"B >= {NT_SV_MIN_B}", "<true, false>"), ("true", "<false, false>")) \
        if not extern_c else (("true", ""),)
    if not extern_c and M.cmode in ("none", "list"):   # mjd_inverseFD's perturbed instances
      variants = ((f"mr.fd_elide && B >= {NT_SV_MIN_B}", "<true, true>"),
                  ("mr.fd_elide", "<false, true>")) + variants
    for cond, v in variants:
      out.append(f"  if ({cond}) {{\n    hipLaunchKernelGGL((k_all_{name}{v}), {gb}, 0, s, mr, B, "
                 f"qpos_in, qvel_in, qacc_in, qfrc_out, status, worklist, worklist_count, "
                 f"worklist_next, efc_count, range);\n    return;\n  }}")
  else:   # staged kernels (experiments): the whole [0, B) range only
    out.append("  if (range) return;   // device-side ranges need k_all")
    for st in STAGES:
      args = _SIG[st][1].replace(", trig", "").replace(", qo_lds", "").replace(", qmr", ", nullptr")
      gb = "g, b" if LANES[st] == 64 else f"dim3(g.x*{64 // LANES[st]}), dim3({LANES[st]})"
      out.append(f"  hipLaunchKernelGGL(k_{st}_{name}, {gb}, 0, s, mr, B, {args});")
  out.append("}")
  out.append("#endif")
  if exact:
    out.append("#if defined(__clang__)\n#pragma clang fp contract(fast)\n#endif")
  return "\n".join(out) + "\n"


_TOKEN = re.compile(r'"(?:\\.|[^"\\\n])*"|\'(?:\\.|[^\'\\\n])*\'|//[^\n]*|/\*.*?\*/|\s+',
                    re.S)


def code_text(src: str) -> str:
  """C/C++ source with comments removed and every whitespace run collapsed to one space
  (string and character literals kept as written): what the compiler sees, so an edit to a
  comment or to indentation does not change it."""
  parts, pos = [], 0
  for mt in _TOKEN.finditer(src):
    if mt.start() > pos:
      parts.append(src[pos:mt.start()])
    t = mt.group(0)
    if t[0] in "\"'":
      parts.append(t)
    elif parts and parts[-1] != " ":
      parts.append(" ")
    pos = mt.end()
  parts.append(src[pos:])
  return "".join(parts).strip()


# the device sources a generated kernel's translation unit compiles besides its own text
HASHED_HEADERS = ("engine_device.h", "fast_kernels.h", "kernels.h", "post_pass.h",
                  "pair_program.h", "kern_constraint.hip")


def source_hash(m, name: str) -> str:
  """Identity of the code a kernel of model m named `name` is built from: its generated
  source, the device headers it includes and the constraint kernels launched beside it, each
  with comments and whitespace removed (code_text). Keys committed PMC and rocprof summaries
  to the kernels they measured, so a comment edit after the final profiles keeps them
  matched; a run-time kernel, rt_*, has C linkage."""
  import os
  h = hashlib.sha256(code_text(generate(m, name, extern_c=name.startswith("rt_"))).encode())
  csrc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")
  for f in HASHED_HEADERS:
    with open(os.path.join(csrc, f), encoding="utf-8") as fh:
      h.update(code_text(fh.read()).encode())
  return h.hexdigest()[:16]


def hot_kernels(name: str) -> list:
  """Names of the kernels one fast-path launch of model `name` runs (profiles, bench)."""
  return [f"k_all_{name}"] if FUSE else [f"k_{st}_{name}" for st in STAGES]


def generate_registries(entries) -> tuple:
  """entries: list of (name, model). Returns (gen_fast.inc, gen_fast_exact.inc): the models
  with native-solver pairs (exact_fp) go to a translation unit of their own, compiled without
  multiply-add contraction throughout (gen_fast_exact.hip) so they round every operation as
  the oracle does; the others, and the registry of all, to gen_fast.inc."""
  head = ["// GENERATED by mujoco_inversedynamicstest_amd/codegen.py (build()) -- do not edit."]
  main = head + ["// Straight-line mj_inverse kernels for the bundled models + their signatures.", ""]
  exact = head + ["// Straight-line kernels of the bundled models with native-solver pairs.", ""]
  reg = []
  for name, m in entries:
    vaskip = constraint_mode(m) in ("none", "list")
    if exact_fp(m):
      exact.append(generate(m, name, shared=True))
      main.append(f"void launch_fast_{name}(dim3, dim3, hipStream_t, const Mirror&, int, "
                  "const double*, const double*, const double*, double*, int*, int*, int*, "
                  "int*, int*, const int*);")
      if vaskip:
        for k in ("vaskip", "fdskip"):
          main.append(f"void launch_{k}_{name}(hipStream_t, const Mirror&, int, int, int, int, "
                      "int*, int*, double);")
      main.append(f"void launch_skip_{name}(hipStream_t, const Mirror&, int, int, double*, "
                  "int*, int*);")
      if constraint_mode(m) == "all":
        main.append(f"void launch_split_{name}(hipStream_t, const Mirror&, int, int, "
                    "const double*, const double*, const double*, int*, int*, int*);")
      if fdall_ok(m):
        main.append(f"void launch_fdall_{name}(hipStream_t, const Mirror&, int, int, int, double, "
                    "int*, int*, int*, int*, int*, int*, int);")
    else:
      main.append(generate(m, name))
    fns = ", ".join(f"launch_{k}_{name}" if vaskip else "nullptr" for k in ("vaskip", "fdskip"))
    split = f"launch_split_{name}" if constraint_mode(m) == "all" else "nullptr"
    fdall = f"launch_fdall_{name}" if fdall_ok(m) else "nullptr"
    reg.append(f'  {{0x{fields.model_signature(m):016x}ull, launch_fast_{name}, "{name}", '
               f'{CONSTRAINT_MODES[constraint_mode(m)]}, {fns}, launch_skip_{name}, {split}, '
               f'{fdall}}},')
  main.append("static const FastKernelEntry g_fast_kernels[] = {")
  main.extend(reg)
  main.append("  {0ull, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr}};")
  return "\n".join(main) + "\n", "\n".join(exact) + "\n"


def generate_registry(entries) -> str:
  """entries: list of (name, model). Returns the .inc compiled into libmjhip.so."""
  out = ["// GENERATED by mujoco_inversedynamicstest_amd/codegen.py (build()) -- do not edit.",
         "// Straight-line mj_inverse kernels for the bundled models + their signatures.", ""]
  reg = []
  for name, m in entries:
    out.append(generate(m, name))
    sk = constraint_mode(m) in ("none", "list")
    fns = ", ".join(f"launch_{k}_{name}" if sk else "nullptr" for k in ("vaskip", "fdskip"))
    split = f"launch_split_{name}" if constraint_mode(m) == "all" else "nullptr"
    fdall = f"launch_fdall_{name}" if fdall_ok(m) else "nullptr"
    reg.append(f'  {{0x{fields.model_signature(m):016x}ull, launch_fast_{name}, "{name}", '
               f'{CONSTRAINT_MODES[constraint_mode(m)]}, {fns}, launch_skip_{name}, {split}, '
               f'{fdall}}},')
  out.append("static const FastKernelEntry g_fast_kernels[] = {")
  out.extend(reg)
  out.append("  {0ull, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr}};")
  return "\n".join(out) + "\n"
