/* mjhip_contact.h — static contact rules and per-instance capacities.
 *
 * Shared by the HIP engine, its host harnesses and the CPU oracle, so all three size their
 * contact and constraint arrays identically.
 *
 * Reference (MuJoCo 3.3.1 fork, src/engine/engine_collision_driver.c):
 *   canCollide / canCollide2 / filterBitmask / filterBodyPair  :105-200
 *   mj_broadphase: always-colliding world pairs + weld-filtered SAP pairs  :1148-1286
 *   mj_collision: body bitmask, exclude signatures, geom pairs  :265-497
 *   mj_collideGeoms: type order, collision table, geom bitmask  :1440-1620
 *   mj_contactParam (condim)  :1289-1384
 *   predefined pairs: merged in signature order :316-327, :432-437; mj_collideGeomPair :499-523
 *
 * The broadphase's bounding boxes are inflated by each geom's rbound + margin, so they never
 * reject a pair the narrowphase would report. A body pair is therefore a candidate exactly
 * when it passes the static rules below. mj_collision processes candidates in signature
 * order ((b1 << 16) + b2, b1 < b2); mjhip_pairMaxContacts bounds each primitive pair.
 *
 * A candidate pair whose collision function is not implemented here (SDFs; mjc_Convex and
 * height fields with the libccd fallback; MULTICCD with a mesh) adds no capacity. At run
 * time it goes through the
 * same bitmask and bounding-sphere filters as the reference (mj_collideGeoms :1470-1497);
 * an instance where one survives them is flagged MJHIP_INST_UNSUPPORTED instead of getting
 * contacts, so every unflagged instance is exact.
 */
#ifndef MJHIP_CONTACT_H_
#define MJHIP_CONTACT_H_

#include "mjhip.h"

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__HIPCC__)
  #define MJHIP_CONTACT_HD __host__ __device__ static inline
#else
  #define MJHIP_CONTACT_HD static inline
#endif

/* geom-level bitmask filter (filterBitmask): 1 = cannot collide */
MJHIP_CONTACT_HD int mjhip_filterBitmask(int contype1, int conaffinity1, int contype2,
                                         int conaffinity2) {
  return !(contype1 & conaffinity2) && !(contype2 & conaffinity1);
}

/* weld filter (filterBodyPair): 1 = skip */
MJHIP_CONTACT_HD int mjhip_filterBodyPair(int weld1, int pweld1, int weld2, int pweld2,
                                          int dsbl_filterparent) {
  if (weld1 == weld2) return 1;
  if (!dsbl_filterparent && weld1 != 0 && weld2 != 0 && (weld1 == pweld2 || weld2 == pweld1)) {
    return 1;
  }
  return 0;
}

/* body pair b1 < b2 that mj_broadphase can return and mj_collision does not filter
 * (body bitmask, exclude list); the geom-level tests come after */
MJHIP_CONTACT_HD int mjhip_bodyPairCandidate(const mjhipModel* m, int b1, int b2) {
  const int can1 = m->body_contype[b1] || m->body_conaffinity[b1];
  const int can2 = m->body_contype[b2] || m->body_conaffinity[b2];
  if (!can1 || !can2) return 0;
  const int weld2 = m->body_weldid[b2];
  const int pweld2 = m->body_weldid[m->body_parentid[weld2]];
  if (b1 == 0) {
    /* always-colliding pairs of a world body with geoms (mj_broadphase :1154-1186) */
    if (m->body_geomnum[0] <= 0) return 0;
    if (mjhip_filterBodyPair(0, 0, weld2, pweld2, 0)) return 0;
  } else {
    const int weld1 = m->body_weldid[b1];
    const int pweld1 = m->body_weldid[m->body_parentid[weld1]];
    if (mjhip_filterBodyPair(weld1, pweld1, weld2, pweld2,
                             m->opt.disableflags & mjhipDSBL_FILTERPARENT)) {
      return 0;
    }
  }
  if (mjhip_filterBitmask(m->body_contype[b1], m->body_conaffinity[b1], m->body_contype[b2],
                          m->body_conaffinity[b2])) {
    return 0;
  }
  const int sig = (b1 << 16) + b2;
  for (int i = 0; i < m->nexclude; i++) {
    if (m->exclude_signature[i] == sig) return 0;
  }
  return 1;
}

/* 1 if geoms g1, g2 (either order) form a predefined <pair>: the body-pair sweep then leaves
 * them to it (mj_collideGeomPair's merged test, engine_collision_driver.c:499-523; the pair
 * shares the body pair's signature, so it is among those merged for it) */
MJHIP_CONTACT_HD int mjhip_isPredefinedPair(const mjhipModel* m, int g1, int g2) {
  for (int k = 0; k < m->npair; k++) {
    if ((m->pair_geom1[k] == g1 && m->pair_geom2[k] == g2) ||
        (m->pair_geom1[k] == g2 && m->pair_geom2[k] == g1)) {
      return 1;
    }
  }
  return 0;
}

/* pairs mjCOLLISIONFUNC serves with mjc_Convex (engine_collision_driver.c:41-52) among the
 * geom types built here: sphere-ellipsoid, capsule-ellipsoid/cylinder, ellipsoid and cylinder
 * pairs among themselves and with boxes, and every primitive or mesh with a mesh
 * (type-ordered t1 <= t2) */
MJHIP_CONTACT_HD int mjhip_isConvexPair(int t1, int t2) {
  if (t1 == mjhipGEOM_PLANE || t1 == mjhipGEOM_HFIELD) return 0;
  if (t2 == mjhipGEOM_ELLIPSOID || t2 == mjhipGEOM_MESH) return 1;
  if (t2 == mjhipGEOM_CYLINDER) {
    return t1 == mjhipGEOM_CAPSULE || t1 == mjhipGEOM_ELLIPSOID || t1 == mjhipGEOM_CYLINDER;
  }
  if (t2 == mjhipGEOM_BOX) return t1 == mjhipGEOM_ELLIPSOID || t1 == mjhipGEOM_CYLINDER;
  return 0;
}

/* contacts a (type-ordered t1 <= t2) geom pair can produce with the functions implemented
 * here: 0 = no collision function in the reference table, -1 = a reference collision
 * function that this engine does not implement. mjc_Convex runs the native GJK/EPA solver
 * for one contact (mjc_CCDIteration, engine_collision_convex.c:792-819); with MULTICCD, a
 * pair without a sphere or an ellipsoid adds up to four perturbed contacts (:933-999), 5 in
 * all (a box / mesh pair without margin: up to 4 from the multicontact polygon, :895-909);
 * the libccd MPR fallback (mjDSBL_NATIVECCD) is not built. mjc_PlaneConvex gives a mesh up to
 * maxplanemesh = 3 contacts (:1006), mjc_ConvexHField up to mjMAXCONPAIR = 50 (one per prism,
 * mjhip_geomPairMaxContacts bounds it by the field's grid). */
MJHIP_CONTACT_HD int mjhip_pairMaxContacts(const mjhipModel* m, int t1, int t2) {
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_MESH) return 3;
  if (t1 == mjhipGEOM_HFIELD && t2 >= mjhipGEOM_SPHERE && t2 <= mjhipGEOM_MESH) {
    return (m->opt.disableflags & mjhipDSBL_NATIVECCD) ? -1 : 50;
  }
  if (mjhip_isConvexPair(t1, t2)) {
    if (m->opt.disableflags & mjhipDSBL_NATIVECCD) return -1;
    if ((m->opt.enableflags & mjhipENBL_MULTICCD) && t1 != mjhipGEOM_SPHERE &&
        t1 != mjhipGEOM_ELLIPSOID && t2 != mjhipGEOM_ELLIPSOID) {
      return 5;
    }
    return 1;
  }
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_ELLIPSOID) return 1;   /* mjc_PlaneConvex */
  if (t1 == mjhipGEOM_PLANE && t2 <= mjhipGEOM_HFIELD) return 0;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_SPHERE) return 1;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_CAPSULE) return 2;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_CYLINDER) return 4;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_BOX) return 4;
  if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_SPHERE) return 1;
  if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_CAPSULE) return 1;
  if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_CYLINDER) return 1;
  if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_BOX) return 1;
  if (t1 == mjhipGEOM_CAPSULE && t2 == mjhipGEOM_CAPSULE) return 2;
  if (t1 == mjhipGEOM_CAPSULE && t2 == mjhipGEOM_BOX) return 2;
  if (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX) return 24;   /* mjc_BoxBox's most */
  if (t1 == mjhipGEOM_HFIELD && t2 <= mjhipGEOM_HFIELD) return 0;
  return -1;
}

/* pairs whose function runs the native GJK/EPA solver (mjc_Convex, mjc_ConvexHField) */
MJHIP_CONTACT_HD int mjhip_pairUsesCcd(int t1, int t2) {
  return mjhip_isConvexPair(t1, t2) ||
         (t1 == mjhipGEOM_HFIELD && t2 >= mjhipGEOM_SPHERE && t2 <= mjhipGEOM_MESH);
}

/* mjhip_pairMaxContacts for type-ordered geoms g1, g2: a height field's bound is one contact
 * per triangular prism of its grid, at most 50 */
MJHIP_CONTACT_HD int mjhip_geomPairMaxContacts(const mjhipModel* m, int g1, int g2) {
  const int k = mjhip_pairMaxContacts(m, m->geom_type[g1], m->geom_type[g2]);
  if (k > 0 && m->geom_type[g1] == mjhipGEOM_HFIELD) {
    const int h = m->geom_dataid[g1];
    const int n = 2*(m->hfield_nrow[h] - 1)*(m->hfield_ncol[h] - 1);
    return n < k ? n : k;
  }
  return k;
}

/* condim of a geom pair (mj_contactParam: higher priority wins, else the max) */
MJHIP_CONTACT_HD int mjhip_pairCondim(const mjhipModel* m, int g1, int g2) {
  const int p1 = m->geom_priority[g1], p2 = m->geom_priority[g2];
  if (p1 > p2) return m->geom_condim[g1];
  if (p1 < p2) return m->geom_condim[g2];
  return m->geom_condim[g1] > m->geom_condim[g2] ? m->geom_condim[g1] : m->geom_condim[g2];
}

/* constraint rows of one contact (mj_instantiateContact): 2(condim-1) for a pyramidal
 * cone, condim for an elliptic one */
MJHIP_CONTACT_HD int mjhip_contactRows(int condim, int elliptic) {
  return condim == 1 ? 1 : (elliptic ? condim : 2*(condim - 1));
}

/* 1 if contacts are generated at all (mj_collision :284-287) */
MJHIP_CONTACT_HD int mjhip_contactsEnabled(const mjhipModel* m) {
  return !(m->opt.disableflags & (mjhipDSBL_CONSTRAINT | mjhipDSBL_CONTACT)) && m->nbody >= 2;
}

/* Maximum contacts per instance (exact for the implemented primitives; pairs without an
 * implemented function add none, see above). *rows receives the maximum number of contact
 * constraint rows. */
MJHIP_CONTACT_HD int mjhip_contactCapacity(const mjhipModel* m, int* rows) {
  int ncon = 0, nrow = 0;
  if (rows) *rows = 0;
  if (!mjhip_contactsEnabled(m)) return 0;
  for (int b1 = 0; b1 < m->nbody; b1++) {
    for (int b2 = b1 + 1; b2 < m->nbody; b2++) {
      if (!mjhip_bodyPairCandidate(m, b1, b2)) continue;
      for (int i = 0; i < m->body_geomnum[b1]; i++) {
        for (int j = 0; j < m->body_geomnum[b2]; j++) {
          int g1 = m->body_geomadr[b1] + i, g2 = m->body_geomadr[b2] + j;
          if (mjhip_isPredefinedPair(m, g1, g2)) continue;   /* counted below */
          if (m->geom_type[g1] > m->geom_type[g2]) { int t = g1; g1 = g2; g2 = t; }
          int k = mjhip_geomPairMaxContacts(m, g1, g2);
          if (k == 0) continue;
          if (mjhip_filterBitmask(m->geom_contype[g1], m->geom_conaffinity[g1],
                                  m->geom_contype[g2], m->geom_conaffinity[g2])) {
            continue;
          }
          if (k < 0) continue;                 /* flagged per instance at run time */
          ncon += k;
          nrow += k * mjhip_contactRows(mjhip_pairCondim(m, g1, g2),
                                        m->opt.cone == mjhipCONE_ELLIPTIC);
        }
      }
    }
  }
  for (int k = 0; k < m->npair; k++) {     /* predefined pairs: no bitmask, their own condim */
    int g1 = m->pair_geom1[k], g2 = m->pair_geom2[k];
    if (m->geom_type[g1] > m->geom_type[g2]) { int t = g1; g1 = g2; g2 = t; }
    const int kk = mjhip_geomPairMaxContacts(m, g1, g2);
    if (kk <= 0) continue;
    ncon += kk;
    nrow += kk * mjhip_contactRows(m->pair_dim[k], m->opt.cone == mjhipCONE_ELLIPTIC);
  }
  if (rows) *rows = nrow;
  return ncon;
}

/* constraint rows per instance: dof/tendon friction, joint/tendon limits, contacts,
   equalities */
MJHIP_CONTACT_HD int mjhip_efcCapacity(const mjhipModel* m) {
  int n = 0, crow = 0;
  for (int i = 0; i < m->njnt; i++) {
    if (m->jnt_limited[i]) n += (m->jnt_type[i] == mjhipJNT_BALL) ? 1 : 2;
  }
  for (int i = 0; i < m->ntendon; i++) {
    if (m->tendon_limited[i]) n += 2;
  }
  for (int i = 0; i < m->nv; i++) {
    if (m->dof_frictionloss[i] > 0) n += 1;
  }
  for (int i = 0; i < m->ntendon; i++) {
    if (m->tendon_frictionloss[i] > 0) n += 1;
  }
  if (mjhip_contactCapacity(m, &crow) > 0) n += crow;
  for (int i = 0; i < m->neq; i++) {        /* nemax (user_model.cc): rows per equality */
    const int t = m->eq_type[i];
    n += t == mjhipEQ_CONNECT ? 3 : (t == mjhipEQ_WELD ? 6 : 1);
  }
  return n;
}

#ifdef __cplusplus
}
#endif

#endif  /* MJHIP_CONTACT_H_ */
