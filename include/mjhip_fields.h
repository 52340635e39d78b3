/* mjhip_fields.h — field tables (X-macros) shared by the C-ABI, the HIP kernels,
 * the CPU oracle and the Python host mirror (which parses this file).
 *
 * Names, element types and per-field shapes follow the reference's own tables:
 *   model fields : /root/reference/include/mujoco/mjxmacro.h:183- (MJMODEL_POINTERS)
 *   data fields  : /root/reference/include/mujoco/mjxmacro.h:594-699 (MJDATA_POINTERS)
 * Only the subset the inverse-dynamics path reads or writes is kept.
 * Row-major per field, exactly as in the reference (e.g. xmat is nbody x 9).
 *
 * The three sparse-structure arrays C_rownnz/C_rowadr/C_colind/mapM2C live in mjData in
 * the reference (engine_io.c:1977-1989) but are model constants; here they are model fields.
 *
 * Syntax (one entry per line, parsed by mujoco_inversedynamicstest_amd/fields.py):
 *   X(ctype, name, dim0, dim1)   dim0 is a size name, dim1 an integer or MJ_M(size)
 */
#ifndef MJHIP_FIELDS_H_
#define MJHIP_FIELDS_H_

/* integer sizes of the model (mjModel scalar ints, mjmodel.h) */
#define MJHIP_MODEL_SIZES \
  XS(nq)          \
  XS(nv)          \
  XS(nu)          \
  XS(na)          \
  XS(nbody)       \
  XS(njnt)        \
  XS(ngeom)       \
  XS(nsite)       \
  XS(ncam)        \
  XS(nlight)      \
  XS(ntendon)     \
  XS(nwrap)       \
  XS(nM)          \
  XS(nC)          \
  XS(nD)          \
  XS(nB)          \
  XS(nJmom)       \
  XS(nmocap)      \
  XS(ngravcomp)   \
  XS(nexclude)    \
  XS(npair)       \
  XS(nkey)        \
  XS(ntree)       \
  XS(nsensor)     \
  XS(nsensordata) \
  XS(neq)         \
  XS(nmat)        \
  XS(nmesh)       \
  XS(nmeshvert)   \
  XS(nmeshface)   \
  XS(nmeshgraph)  \
  XS(nmeshpoly)   \
  XS(nmeshpolyvert) \
  XS(nmeshpolymap) \
  XS(nhfield)     \
  XS(nhfielddata)

/* model arrays that live in mjModel in the reference (mjxmacro.h MJMODEL_POINTERS) */
#define MJHIP_MODEL_POINTERS_M \
  X(mjtNum,  qpos0,                nq,        1) \
  X(mjtNum,  qpos_spring,          nq,        1) \
  X(int,     body_parentid,        nbody,     1) \
  X(int,     body_rootid,          nbody,     1) \
  X(int,     body_weldid,          nbody,     1) \
  X(int,     body_mocapid,         nbody,     1) \
  X(int,     body_jntnum,          nbody,     1) \
  X(int,     body_jntadr,          nbody,     1) \
  X(int,     body_dofnum,          nbody,     1) \
  X(int,     body_dofadr,          nbody,     1) \
  X(int,     body_treeid,          nbody,     1) \
  X(int,     body_geomnum,         nbody,     1) \
  X(int,     body_geomadr,         nbody,     1) \
  X(mjtByte, body_simple,          nbody,     1) \
  X(mjtByte, body_sameframe,       nbody,     1) \
  X(mjtNum,  body_pos,             nbody,     3) \
  X(mjtNum,  body_quat,            nbody,     4) \
  X(mjtNum,  body_ipos,            nbody,     3) \
  X(mjtNum,  body_iquat,           nbody,     4) \
  X(mjtNum,  body_mass,            nbody,     1) \
  X(mjtNum,  body_subtreemass,     nbody,     1) \
  X(mjtNum,  body_inertia,         nbody,     3) \
  X(mjtNum,  body_invweight0,      nbody,     2) \
  X(mjtNum,  body_gravcomp,        nbody,     1) \
  X(mjtNum,  body_margin,          nbody,     1) \
  X(int,     body_contype,         nbody,     1) \
  X(int,     body_conaffinity,     nbody,     1) \
  X(int,     jnt_type,             njnt,      1) \
  X(int,     jnt_qposadr,          njnt,      1) \
  X(int,     jnt_dofadr,           njnt,      1) \
  X(int,     jnt_bodyid,           njnt,      1) \
  X(int,     jnt_group,            njnt,      1) \
  X(mjtByte, jnt_limited,          njnt,      1) \
  X(mjtByte, jnt_actgravcomp,      njnt,      1) \
  X(mjtNum,  jnt_solref,           njnt,      2) \
  X(mjtNum,  jnt_solimp,           njnt,      5) \
  X(mjtNum,  jnt_pos,              njnt,      3) \
  X(mjtNum,  jnt_axis,             njnt,      3) \
  X(mjtNum,  jnt_stiffness,        njnt,      1) \
  X(mjtNum,  jnt_range,            njnt,      2) \
  X(mjtNum,  jnt_margin,           njnt,      1) \
  X(int,     dof_bodyid,           nv,        1) \
  X(int,     dof_jntid,            nv,        1) \
  X(int,     dof_parentid,         nv,        1) \
  X(int,     dof_treeid,           nv,        1) \
  X(int,     dof_Madr,             nv,        1) \
  X(int,     dof_simplenum,        nv,        1) \
  X(mjtNum,  dof_solref,           nv,        2) \
  X(mjtNum,  dof_solimp,           nv,        5) \
  X(mjtNum,  dof_frictionloss,     nv,        1) \
  X(mjtNum,  dof_armature,         nv,        1) \
  X(mjtNum,  dof_damping,          nv,        1) \
  X(mjtNum,  dof_invweight0,       nv,        1) \
  X(mjtNum,  dof_M0,               nv,        1) \
  X(int,     geom_type,            ngeom,     1) \
  X(int,     geom_contype,         ngeom,     1) \
  X(int,     geom_conaffinity,     ngeom,     1) \
  X(int,     geom_condim,          ngeom,     1) \
  X(int,     geom_bodyid,          ngeom,     1) \
  X(int,     geom_group,           ngeom,     1) \
  X(int,     geom_priority,        ngeom,     1) \
  X(mjtByte, geom_sameframe,       ngeom,     1) \
  X(mjtNum,  geom_solmix,          ngeom,     1) \
  X(mjtNum,  geom_solref,          ngeom,     2) \
  X(mjtNum,  geom_solimp,          ngeom,     5) \
  X(mjtNum,  geom_size,            ngeom,     3) \
  X(mjtNum,  geom_rbound,          ngeom,     1) \
  X(mjtNum,  geom_pos,             ngeom,     3) \
  X(mjtNum,  geom_quat,            ngeom,     4) \
  X(mjtNum,  geom_friction,        ngeom,     3) \
  X(mjtNum,  geom_fluid,           ngeom,     12) \
  X(mjtNum,  geom_margin,          ngeom,     1) \
  X(mjtNum,  geom_gap,             ngeom,     1) \
  X(int,     geom_dataid,          ngeom,     1) \
  X(int,     geom_matid,           ngeom,     1) \
  X(float,   geom_rgba,            ngeom,     4) \
  X(int,     site_type,            nsite,     1) \
  X(int,     site_bodyid,          nsite,     1) \
  X(mjtByte, site_sameframe,       nsite,     1) \
  X(mjtNum,  site_size,            nsite,     3) \
  X(mjtNum,  site_pos,             nsite,     3) \
  X(mjtNum,  site_quat,            nsite,     4) \
  X(int,     cam_mode,             ncam,      1) \
  X(int,     cam_bodyid,           ncam,      1) \
  X(int,     cam_targetbodyid,     ncam,      1) \
  X(mjtNum,  cam_pos,              ncam,      3) \
  X(mjtNum,  cam_quat,             ncam,      4) \
  X(mjtNum,  cam_poscom0,          ncam,      3) \
  X(mjtNum,  cam_pos0,             ncam,      3) \
  X(mjtNum,  cam_mat0,             ncam,      9) \
  X(mjtNum,  cam_fovy,             ncam,      1) \
  X(int,     cam_resolution,       ncam,      2) \
  X(float,   cam_sensorsize,       ncam,      2) \
  X(float,   cam_intrinsic,        ncam,      4) \
  X(int,     light_mode,           nlight,    1) \
  X(int,     light_bodyid,         nlight,    1) \
  X(int,     light_targetbodyid,   nlight,    1) \
  X(mjtNum,  light_pos,            nlight,    3) \
  X(mjtNum,  light_dir,            nlight,    3) \
  X(mjtNum,  light_poscom0,        nlight,    3) \
  X(mjtNum,  light_pos0,           nlight,    3) \
  X(mjtNum,  light_dir0,           nlight,    3) \
  X(int,     tendon_adr,           ntendon,   1) \
  X(int,     tendon_num,           ntendon,   1) \
  X(mjtByte, tendon_limited,       ntendon,   1) \
  X(mjtNum,  tendon_solref_lim,    ntendon,   2) \
  X(mjtNum,  tendon_solimp_lim,    ntendon,   5) \
  X(mjtNum,  tendon_solref_fri,    ntendon,   2) \
  X(mjtNum,  tendon_solimp_fri,    ntendon,   5) \
  X(mjtNum,  tendon_range,         ntendon,   2) \
  X(mjtNum,  tendon_margin,        ntendon,   1) \
  X(mjtNum,  tendon_stiffness,     ntendon,   1) \
  X(mjtNum,  tendon_damping,       ntendon,   1) \
  X(mjtNum,  tendon_frictionloss,  ntendon,   1) \
  X(mjtNum,  tendon_lengthspring,  ntendon,   2) \
  X(mjtNum,  tendon_length0,       ntendon,   1) \
  X(mjtNum,  tendon_invweight0,    ntendon,   1) \
  X(int,     wrap_type,            nwrap,     1) \
  X(int,     wrap_objid,           nwrap,     1) \
  X(mjtNum,  wrap_prm,             nwrap,     1) \
  X(int,     actuator_trntype,     nu,        1) \
  X(int,     actuator_dyntype,     nu,        1) \
  X(int,     actuator_gaintype,    nu,        1) \
  X(int,     actuator_biastype,    nu,        1) \
  X(int,     actuator_trnid,       nu,        2) \
  X(mjtByte, actuator_ctrllimited, nu,        1) \
  X(mjtByte, actuator_forcelimited, nu,       1) \
  X(mjtNum,  actuator_dynprm,      nu,        10) \
  X(mjtNum,  actuator_gainprm,     nu,        10) \
  X(mjtNum,  actuator_biasprm,     nu,        10) \
  X(mjtNum,  actuator_ctrlrange,   nu,        2) \
  X(mjtNum,  actuator_forcerange,  nu,        2) \
  X(mjtNum,  actuator_gear,        nu,        6) \
  X(mjtNum,  actuator_cranklength, nu,        1) \
  X(mjtNum,  actuator_length0,     nu,        1) \
  X(mjtNum,  actuator_acc0,        nu,        1) \
  X(int,     exclude_signature,    nexclude,  1) \
  X(int,     pair_dim,             npair,     1) \
  X(int,     pair_geom1,           npair,     1) \
  X(int,     pair_geom2,           npair,     1) \
  X(int,     pair_signature,       npair,     1) \
  X(mjtNum,  pair_solref,          npair,     2) \
  X(mjtNum,  pair_solreffriction,  npair,     2) \
  X(mjtNum,  pair_solimp,          npair,     5) \
  X(mjtNum,  pair_margin,          npair,     1) \
  X(mjtNum,  pair_gap,             npair,     1) \
  X(mjtNum,  pair_friction,        npair,     5) \
  X(int,     eq_type,              neq,       1) \
  X(int,     eq_obj1id,            neq,       1) \
  X(int,     eq_obj2id,            neq,       1) \
  X(int,     eq_objtype,           neq,       1) \
  X(mjtByte, eq_active0,           neq,       1) \
  X(mjtNum,  eq_solref,            neq,       2) \
  X(mjtNum,  eq_solimp,            neq,       5) \
  X(mjtNum,  eq_data,              neq,       11) \
  X(int,     sensor_type,          nsensor,   1) \
  X(int,     sensor_datatype,      nsensor,   1) \
  X(int,     sensor_needstage,     nsensor,   1) \
  X(int,     sensor_objtype,       nsensor,   1) \
  X(int,     sensor_objid,         nsensor,   1) \
  X(int,     sensor_reftype,       nsensor,   1) \
  X(int,     sensor_refid,         nsensor,   1) \
  X(int,     sensor_dim,           nsensor,   1) \
  X(int,     sensor_adr,           nsensor,   1) \
  X(mjtNum,  sensor_cutoff,        nsensor,   1) \
  X(float,   mat_rgba,             nmat,      4) \
  X(int,     mesh_vertadr,         nmesh,     1) \
  X(int,     mesh_vertnum,         nmesh,     1) \
  X(int,     mesh_faceadr,         nmesh,     1) \
  X(int,     mesh_facenum,         nmesh,     1) \
  X(int,     mesh_graphadr,        nmesh,     1) \
  X(float,   mesh_vert,            nmeshvert, 3) \
  X(int,     mesh_face,            nmeshface, 3) \
  X(int,     mesh_graph,           nmeshgraph, 1) \
  X(int,     mesh_polynum,         nmesh,     1) \
  X(int,     mesh_polyadr,         nmesh,     1) \
  X(mjtNum,  mesh_polynormal,      nmeshpoly, 3) \
  X(int,     mesh_polyvertadr,     nmeshpoly, 1) \
  X(int,     mesh_polyvertnum,     nmeshpoly, 1) \
  X(int,     mesh_polyvert,        nmeshpolyvert, 1) \
  X(int,     mesh_polymapadr,      nmeshvert, 1) \
  X(int,     mesh_polymapnum,      nmeshvert, 1) \
  X(int,     mesh_polymap,         nmeshpolymap, 1) \
  X(mjtNum,  hfield_size,          nhfield,   4) \
  X(int,     hfield_nrow,          nhfield,   1) \
  X(int,     hfield_ncol,          nhfield,   1) \
  X(int,     hfield_adr,           nhfield,   1) \
  X(float,   hfield_data,          nhfielddata, 1) \
  X(mjtNum,  key_qpos,             nkey,      MJ_M(nq))

/* model-constant sparse structures that live in mjData in the reference
 * (engine_io.c:1977-1989 for C/mapM2C; mj_transmission writes moment_* each call,
 * engine_core_smooth.c:865-916, constant for joint transmissions) */
#define MJHIP_MODEL_POINTERS_D \
  X(int,     C_rownnz,             nv,        1) \
  X(int,     C_rowadr,             nv,        1) \
  X(int,     C_colind,             nC,        1) \
  X(int,     mapM2C,               nC,        1) \
  X(int,     moment_rownnz,        nu,        1) \
  X(int,     moment_rowadr,        nu,        1) \
  X(int,     moment_colind,        nJmom,     1) \
  X(int,     B_rownnz,             nbody,     1) \
  X(int,     B_rowadr,             nbody,     1) \
  X(int,     B_colind,             nB,        1) \
  X(int,     D_rownnz,             nv,        1) \
  X(int,     D_rowadr,             nv,        1) \
  X(int,     D_colind,             nD,        1) \
  X(int,     mapM2D,               nD,        1)

#define MJHIP_MODEL_POINTERS \
  MJHIP_MODEL_POINTERS_M      \
  MJHIP_MODEL_POINTERS_D

/* Per-instance fp64 mjData fields produced or consumed by mj_inverseSkip, in pipeline order.
 * XD(name, dim0, dim1, stage): stage 0 = input, 1 = position, 2 = velocity, 3 = acceleration.
 * The sum over stages 1..3 of dim0*dim1 is W in SURVEY.md §8d (2,563 for the humanoid). */
#define MJHIP_DATA_INPUTS \
  XD(qpos,              nq,      1,   0) \
  XD(qvel,              nv,      1,   0) \
  XD(qacc,              nv,      1,   0) \
  XD(mocap_pos,         nmocap,  3,   0) \
  XD(mocap_quat,        nmocap,  4,   0)

#define MJHIP_DATA_POSITION \
  XD(xpos,              nbody,   3,   1) \
  XD(xquat,             nbody,   4,   1) \
  XD(xmat,              nbody,   9,   1) \
  XD(xipos,             nbody,   3,   1) \
  XD(ximat,             nbody,   9,   1) \
  XD(xanchor,           njnt,    3,   1) \
  XD(xaxis,             njnt,    3,   1) \
  XD(geom_xpos,         ngeom,   3,   1) \
  XD(geom_xmat,         ngeom,   9,   1) \
  XD(site_xpos,         nsite,   3,   1) \
  XD(site_xmat,         nsite,   9,   1) \
  XD(cam_xpos,          ncam,    3,   1) \
  XD(cam_xmat,          ncam,    9,   1) \
  XD(light_xpos,        nlight,  3,   1) \
  XD(light_xdir,        nlight,  3,   1) \
  XD(subtree_com,       nbody,   3,   1) \
  XD(cdof,              nv,      6,   1) \
  XD(cinert,            nbody,   10,  1) \
  XD(ten_length,        ntendon, 1,   1) \
  XD(ten_J,             ntendon, MJ_M(nv), 1) \
  XD(actuator_length,   nu,      1,   1) \
  XD(actuator_moment,   nJmom,   1,   1) \
  XD(crb,               nbody,   10,  1) \
  XD(qM,                nM,      1,   1) \
  XD(qLD,               nC,      1,   1) \
  XD(qLDiagInv,         nv,      1,   1)

#define MJHIP_DATA_VELOCITY \
  XD(ten_velocity,      ntendon, 1,   2) \
  XD(actuator_velocity, nu,      1,   2) \
  XD(cvel,              nbody,   6,   2) \
  XD(cdof_dot,          nv,      6,   2) \
  XD(qfrc_spring,       nv,      1,   2) \
  XD(qfrc_damper,       nv,      1,   2) \
  XD(qfrc_gravcomp,     nv,      1,   2) \
  XD(qfrc_fluid,        nv,      1,   2) \
  XD(qfrc_passive,      nv,      1,   2) \
  XD(qfrc_bias,         nv,      1,   2)

/* sensordata is written by mj_sensorPos/Vel/Acc in the stage each sensor needs
 * (engine_inverse.c:203-242); listed with the acceleration stage for the W accounting */
#define MJHIP_DATA_ACCELERATION \
  XD(qfrc_constraint,   nv,      1,   3) \
  XD(qfrc_inverse,      nv,      1,   3) \
  XD(sensordata,        nsensordata, 1, 3)

#define MJHIP_DATA_FIELDS \
  MJHIP_DATA_INPUTS       \
  MJHIP_DATA_POSITION     \
  MJHIP_DATA_VELOCITY     \
  MJHIP_DATA_ACCELERATION

/* Forward dynamics (mj_forward, engine_forward.c: mj_fwdActuation :276-515,
 * mj_fwdAcceleration :520-531) and the fwd/inv comparison harness (mj_compareFwdInv
 * engine_inverse.c:275-316): applied inputs (stage 4) and forward outputs (stage 5).
 * Not part of mj_inverse's output contract (W), so kept out of MJHIP_DATA_FIELDS. */
#define MJHIP_DATA_FORWARD \
  XD(ctrl,              nu,      1,   4) \
  XD(qfrc_applied,      nv,      1,   4) \
  XD(xfrc_applied,      nbody,   6,   4) \
  XD(actuator_force,    nu,      1,   5) \
  XD(qfrc_actuator,     nv,      1,   5) \
  XD(qfrc_smooth,       nv,      1,   5) \
  XD(qacc_smooth,       nv,      1,   5)

/* mjData fields the sensor stages compute on demand (stage 6): mj_subtreeVel
 * (engine_core_smooth.c:1900-1958) for subtreelinvel/subtreeangmom sensors and
 * mj_rnePostConstraint (:2027-2181) for accelerometer/force/torque/framelin/angacc sensors
 * (engine_sensor.c:552-561, :712-723). Host data (mjhipData) only; on the device they are
 * scratch fields sized only for models whose sensors need them. */
#define MJHIP_DATA_SENSOR_AUX \
  XD(subtree_linvel,    nbody,   3,   6) \
  XD(subtree_angmom,    nbody,   3,   6) \
  XD(cacc,              nbody,   6,   6) \
  XD(cfrc_int,          nbody,   6,   6) \
  XD(cfrc_ext,          nbody,   6,   6)

/* Constraint rows of one instance: the reference's efc_* arena arrays of the dense path
 * (mjxmacro.h:707-732 MJDATA_ARENA_POINTERS_SOLVER; efc_J is nefc x nv, efc_KBIP nefc x 4).
 * XE(type, name, width, stage): `width` elements per row; `stage` is the inverse stage that
 * writes the field (1 mj_makeConstraint, 2 mj_referenceConstraint, 3 mj_invConstraint).
 * The host data (mjhipData) holds caller-owned buffers of efc_capacity rows. */
#define MJHIP_DATA_EFC \
  XE(int,    efc_type,          1,        1) \
  XE(int,    efc_id,            1,        1) \
  XE(mjtNum, efc_J,             MJ_M(nv), 1) \
  XE(mjtNum, efc_pos,           1,        1) \
  XE(mjtNum, efc_margin,        1,        1) \
  XE(mjtNum, efc_frictionloss,  1,        1) \
  XE(mjtNum, efc_diagApprox,    1,        1) \
  XE(mjtNum, efc_KBIP,          4,        1) \
  XE(mjtNum, efc_D,             1,        1) \
  XE(mjtNum, efc_R,             1,        1) \
  XE(mjtNum, efc_vel,           1,        2) \
  XE(mjtNum, efc_aref,          1,        2) \
  XE(mjtNum, efc_force,         1,        3) \
  XE(int,    efc_state,         1,        3)

/* Contacts of one instance (mjContact, mjdata.h, the fields this path reads or writes) as
 * parallel arrays of con_capacity entries: XC(type, name, width, stage) as above (stage 1
 * mj_collision / mj_makeConstraint; con_mu is set by mj_makeImpedance). */
#define MJHIP_DATA_CONTACT \
  XC(mjtNum, con_dist,          1, 1) \
  XC(mjtNum, con_pos,           3, 1) \
  XC(mjtNum, con_frame,         9, 1) \
  XC(mjtNum, con_includemargin, 1, 1) \
  XC(mjtNum, con_friction,      5, 1) \
  XC(mjtNum, con_solref,        2, 1) \
  XC(mjtNum, con_solreffriction, 2, 1) \
  XC(mjtNum, con_solimp,        5, 1) \
  XC(mjtNum, con_mu,            1, 1) \
  XC(int,    con_dim,           1, 1) \
  XC(int,    con_geom,          2, 1) \
  XC(int,    con_exclude,       1, 1) \
  XC(int,    con_efc_address,   1, 1)

/* Sparse structures of sparse-Jacobian models (mjData ten_J_*, efc_J_*, efc_JT*; mjxmacro.h
 * MJDATA_POINTERS and MJDATA_ARENA_POINTERS_SOLVER): XJ(type, name, dim) with dim one of
 * ntendon, ntendon_nv (ntendon x nv), efc (efc_capacity), efc_nv (efc_capacity x nv), nv. */
#define MJHIP_DATA_SPARSE \
  XJ(int,    ten_J_rownnz,      ntendon)    \
  XJ(int,    ten_J_rowadr,      ntendon)    \
  XJ(int,    ten_J_colind,      ntendon_nv) \
  XJ(int,    efc_J_rownnz,      efc)        \
  XJ(int,    efc_J_rowadr,      efc)        \
  XJ(int,    efc_J_colind,      efc_nv)     \
  XJ(mjtNum, efc_JT,            efc_nv)     \
  XJ(int,    efc_JT_rownnz,     nv)         \
  XJ(int,    efc_JT_rowadr,     nv)         \
  XJ(int,    efc_JT_colind,     efc_nv)

#endif  /* MJHIP_FIELDS_H_ */
