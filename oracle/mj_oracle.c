/* mj_oracle.c — TEST INFRASTRUCTURE ONLY (see mj_oracle.h).
 *
 * Line-by-line CPU restatement of the reference's mj_inverse path, each function citing
 * the reference file:line it follows (paths relative to the reference root,
 * /root/reference). Scalar (non-AVX) summation orders. Compiled with -O2
 * -ffp-contract=off so no FMA contraction changes rounding.
 */
#define _GNU_SOURCE
#include "mj_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define mjMINVAL mjhipMINVAL
#define mjMAX(a, b) (((a) > (b)) ? (a) : (b))
#define mjMIN(a, b) (((a) < (b)) ? (a) : (b))
#define mjDISABLED(x) (m->opt.disableflags & (x))
#define mjENABLED(x) (m->opt.enableflags & (x))

/* mjtObj values (mjmodel.h) */
enum { OBJ_BODY = 1, OBJ_XBODY = 2, OBJ_GEOM = 5, OBJ_SITE = 6, OBJ_CAMERA = 7 };

/*============================ engine_util_blas.c ==========================================*/

static void mju_zero3(mjtNum r[3]) { r[0] = r[1] = r[2] = 0; }
static void mju_copy3(mjtNum r[3], const mjtNum a[3]) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
static void mju_copy4(mjtNum r[4], const mjtNum a[4]) {
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
}
static void mju_scl3(mjtNum r[3], const mjtNum a[3], mjtNum s) {
  r[0] = a[0]*s; r[1] = a[1]*s; r[2] = a[2]*s;
}
static void mju_add3(mjtNum r[3], const mjtNum a[3], const mjtNum b[3]) {
  r[0] = a[0]+b[0]; r[1] = a[1]+b[1]; r[2] = a[2]+b[2];
}
static void mju_sub3(mjtNum r[3], const mjtNum a[3], const mjtNum b[3]) {
  r[0] = a[0]-b[0]; r[1] = a[1]-b[1]; r[2] = a[2]-b[2];
}
static void mju_addTo3(mjtNum r[3], const mjtNum a[3]) { r[0] += a[0]; r[1] += a[1]; r[2] += a[2]; }
static void mju_addToScl3(mjtNum r[3], const mjtNum a[3], mjtNum s) {
  r[0] += a[0]*s; r[1] += a[1]*s; r[2] += a[2]*s;
}
static void mju_cross(mjtNum r[3], const mjtNum a[3], const mjtNum b[3]) {   /* blas.c */
  mjtNum tmp[3] = {a[1]*b[2] - a[2]*b[1], a[2]*b[0] - a[0]*b[2], a[0]*b[1] - a[1]*b[0]};
  r[0] = tmp[0]; r[1] = tmp[1]; r[2] = tmp[2];
}

/* engine_util_blas.c:123-140 */
static mjtNum mju_normalize3(mjtNum v[3]) {
  mjtNum norm = sqrt(v[0]*v[0] + v[1]*v[1] + v[2]*v[2]);
  if (norm < mjMINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0;
  } else {
    mjtNum normInv = 1/norm;
    v[0] *= normInv; v[1] *= normInv; v[2] *= normInv;
  }
  return norm;
}

/* engine_util_blas.c:165-176 */
static void mju_mulMatVec3(mjtNum res[3], const mjtNum mat[9], const mjtNum vec[3]) {
  mjtNum tmp[3] = {
    mat[0]*vec[0] + mat[1]*vec[1] + mat[2]*vec[2],
    mat[3]*vec[0] + mat[4]*vec[1] + mat[5]*vec[2],
    mat[6]*vec[0] + mat[7]*vec[1] + mat[8]*vec[2]
  };
  res[0] = tmp[0]; res[1] = tmp[1]; res[2] = tmp[2];
}

/* engine_util_blas.c:269-285 */
static mjtNum mju_normalize4(mjtNum v[4]) {
  mjtNum norm = sqrt(v[0]*v[0] + v[1]*v[1] + v[2]*v[2] + v[3]*v[3]);
  if (norm < mjMINVAL) {
    v[0] = 1; v[1] = 0; v[2] = 0; v[3] = 0;
  } else if (fabs(norm - 1) > mjMINVAL) {
    mjtNum normInv = 1/norm;
    v[0] *= normInv; v[1] *= normInv; v[2] *= normInv; v[3] *= normInv;
  }
  return norm;
}

static void mju_zero(mjtNum* r, int n) { memset(r, 0, n*sizeof(mjtNum)); }
static void mju_copy(mjtNum* r, const mjtNum* a, int n) { memcpy(r, a, n*sizeof(mjtNum)); }
static void mju_scl(mjtNum* r, const mjtNum* a, mjtNum s, int n) {            /* :342-383 */
  for (int i = 0; i < n; i++) r[i] = a[i]*s;
}
static void mju_add(mjtNum* r, const mjtNum* a, const mjtNum* b, int n) {    /* :387 */
  for (int i = 0; i < n; i++) r[i] = a[i] + b[i];
}
static void mju_sub(mjtNum* r, const mjtNum* a, const mjtNum* b, int n) {    /* :430 */
  for (int i = 0; i < n; i++) r[i] = a[i] - b[i];
}
static void mju_addTo(mjtNum* r, const mjtNum* a, int n) {                    /* :473 */
  for (int i = 0; i < n; i++) r[i] += a[i];
}
static void mju_subFrom(mjtNum* r, const mjtNum* a, int n) {                  /* :516 */
  for (int i = 0; i < n; i++) r[i] -= a[i];
}
static void mju_addToScl(mjtNum* r, const mjtNum* a, mjtNum s, int n) {      /* :559-600 */
  for (int i = 0; i < n; i++) r[i] += a[i]*s;
}

/* engine_util_blas.c:680-741, scalar branch: four lanes, then (r0+r2)+(r1+r3), then tail */
static mjtNum mju_dot(const mjtNum* a, const mjtNum* b, int n) {
  mjtNum res = 0;
  int i = 0;
  int n_4 = n - 4;
  mjtNum r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  for (; i <= n_4; i += 4) {
    r0 += a[i]*b[i];
    r1 += a[i+1]*b[i+1];
    r2 += a[i+2]*b[i+2];
    r3 += a[i+3]*b[i+3];
  }
  res = (r0 + r2) + (r1 + r3);
  int n_i = n - i;
  if (n_i == 3) {
    res += a[i]*b[i] + a[i+1]*b[i+1] + a[i+2]*b[i+2];
  } else if (n_i == 2) {
    res += a[i]*b[i] + a[i+1]*b[i+1];
  } else if (n_i == 1) {
    res += a[i]*b[i];
  }
  return res;
}

static mjtNum mju_norm(const mjtNum* a, int n) { return sqrt(mju_dot(a, a, n)); }

/* engine_util_blas.c:747-752 */
static void mju_mulMatVec(mjtNum* res, const mjtNum* mat, const mjtNum* vec, int nr, int nc) {
  for (int r = 0; r < nr; r++) res[r] = mju_dot(mat + r*nc, vec, nc);
}

/* engine_util_blas.c:756-766 */
static void mju_mulMatTVec(mjtNum* res, const mjtNum* mat, const mjtNum* vec, int nr, int nc) {
  mjtNum tmp;
  mju_zero(res, nc);
  for (int r = 0; r < nr; r++) {
    if ((tmp = vec[r])) mju_addToScl(res, mat + r*nc, tmp, nc);
  }
}

static int mju_isZero(const mjtNum* v, int n) {
  for (int i = 0; i < n; i++) if (v[i] != 0) return 0;
  return 1;
}

/* engine_util_sparse.h:115-160 (scalar branch) */
static mjtNum mju_dotSparse(const mjtNum* v1, const mjtNum* v2, int nnz1, const int* ind1) {
  int i = 0;
  mjtNum res = 0;
  int n_4 = nnz1 - 4;
  mjtNum r0 = 0, r1 = 0, r2 = 0, r3 = 0;
  for (; i <= n_4; i += 4) {
    r0 += v1[i+0]*v2[ind1[i+0]];
    r1 += v1[i+1]*v2[ind1[i+1]];
    r2 += v1[i+2]*v2[ind1[i+2]];
    r3 += v1[i+3]*v2[ind1[i+3]];
  }
  res = (r0 + r2) + (r1 + r3);
  for (; i < nnz1; i++) res += v1[i]*v2[ind1[i]];
  return res;
}

/*============================ engine_util_spatial.c =======================================*/

/* :23-46 */
static void mju_rotVecQuat(mjtNum res[3], const mjtNum vec[3], const mjtNum quat[4]) {
  if (vec[0] == 0 && vec[1] == 0 && vec[2] == 0) {
    mju_zero3(res);
  } else if (quat[0] == 1 && quat[1] == 0 && quat[2] == 0 && quat[3] == 0) {
    mju_copy3(res, vec);
  } else {
    mjtNum tmp[3] = {
      quat[0]*vec[0] + quat[2]*vec[2] - quat[3]*vec[1],
      quat[0]*vec[1] + quat[3]*vec[0] - quat[1]*vec[2],
      quat[0]*vec[2] + quat[1]*vec[1] - quat[2]*vec[0]
    };
    res[0] = vec[0] + 2 * (quat[2]*tmp[2] - quat[3]*tmp[1]);
    res[1] = vec[1] + 2 * (quat[3]*tmp[0] - quat[1]*tmp[2]);
    res[2] = vec[2] + 2 * (quat[1]*tmp[1] - quat[2]*tmp[0]);
  }
}

/* :62-74 */
static void mju_mulQuat(mjtNum res[4], const mjtNum qa[4], const mjtNum qb[4]) {
  mjtNum tmp[4] = {
    qa[0]*qb[0] - qa[1]*qb[1] - qa[2]*qb[2] - qa[3]*qb[3],
    qa[0]*qb[1] + qa[1]*qb[0] + qa[2]*qb[3] - qa[3]*qb[2],
    qa[0]*qb[2] - qa[1]*qb[3] + qa[2]*qb[0] + qa[3]*qb[1],
    qa[0]*qb[3] + qa[1]*qb[2] - qa[2]*qb[1] + qa[3]*qb[0]
  };
  res[0] = tmp[0]; res[1] = tmp[1]; res[2] = tmp[2]; res[3] = tmp[3];
}

/* :97-114 */
static void mju_axisAngle2Quat(mjtNum res[4], const mjtNum axis[3], mjtNum angle) {
  if (angle == 0) {
    res[0] = 1; res[1] = 0; res[2] = 0; res[3] = 0;
  } else {
    mjtNum s = sin(angle*0.5);
    res[0] = cos(angle*0.5);
    res[1] = axis[0]*s;
    res[2] = axis[1]*s;
    res[3] = axis[2]*s;
  }
}

/* :119-133 */
static void mju_quat2Vel(mjtNum res[3], const mjtNum quat[4], mjtNum dt) {
  mjtNum axis[3] = {quat[1], quat[2], quat[3]};
  mjtNum sin_a_2 = mju_normalize3(axis);
  mjtNum speed = 2 * atan2(sin_a_2, quat[0]);
  if (speed > mjhipPI) speed -= 2*mjhipPI;
  speed /= dt;
  mju_scl3(res, axis, speed);
}

/* :138-146 */
static void mju_subQuat(mjtNum res[3], const mjtNum qa[4], const mjtNum qb[4]) {
  mjtNum qneg[4] = {qb[0], -qb[1], -qb[2], -qb[3]}, qdif[4];
  mju_mulQuat(qdif, qneg, qa);
  mju_quat2Vel(res, qdif, 1);
}

/* :151-187 */
static void mju_quat2Mat(mjtNum res[9], const mjtNum quat[4]) {
  if (quat[0] == 1 && quat[1] == 0 && quat[2] == 0 && quat[3] == 0) {
    res[0] = 1; res[1] = 0; res[2] = 0;
    res[3] = 0; res[4] = 1; res[5] = 0;
    res[6] = 0; res[7] = 0; res[8] = 1;
  } else {
    const mjtNum q00 = quat[0]*quat[0], q01 = quat[0]*quat[1], q02 = quat[0]*quat[2];
    const mjtNum q03 = quat[0]*quat[3], q11 = quat[1]*quat[1], q12 = quat[1]*quat[2];
    const mjtNum q13 = quat[1]*quat[3], q22 = quat[2]*quat[2], q23 = quat[2]*quat[3];
    const mjtNum q33 = quat[3]*quat[3];
    res[0] = q00 + q11 - q22 - q33;
    res[4] = q00 - q11 + q22 - q33;
    res[8] = q00 - q11 - q22 + q33;
    res[1] = 2*(q12 - q03);
    res[2] = 2*(q13 + q02);
    res[3] = 2*(q12 + q03);
    res[5] = 2*(q23 - q01);
    res[6] = 2*(q13 - q02);
    res[7] = 2*(q23 + q01);
  }
}

/* :241-250 */
static void mju_quatIntegrate(mjtNum quat[4], const mjtNum vel[3], mjtNum scale) {
  mjtNum angle, tmp[4], qrot[4];
  mju_copy3(tmp, vel);
  angle = scale * mju_normalize3(tmp);
  mju_axisAngle2Quat(qrot, tmp, angle);
  mju_normalize4(quat);
  mju_mulQuat(quat, quat, qrot);
}

/* :385-396 */
static void mju_crossMotion(mjtNum res[6], const mjtNum vel[6], const mjtNum v[6]) {
  res[0] = -vel[2]*v[1] + vel[1]*v[2];
  res[1] =  vel[2]*v[0] - vel[0]*v[2];
  res[2] = -vel[1]*v[0] + vel[0]*v[1];
  res[3] = -vel[2]*v[4] + vel[1]*v[5];
  res[4] =  vel[2]*v[3] - vel[0]*v[5];
  res[5] = -vel[1]*v[3] + vel[0]*v[4];
  res[3] += -vel[5]*v[1] + vel[4]*v[2];
  res[4] +=  vel[5]*v[0] - vel[3]*v[2];
  res[5] += -vel[4]*v[0] + vel[3]*v[1];
}

/* :401-412 */
static void mju_crossForce(mjtNum res[6], const mjtNum vel[6], const mjtNum f[6]) {
  res[0] = -vel[2]*f[1] + vel[1]*f[2];
  res[1] =  vel[2]*f[0] - vel[0]*f[2];
  res[2] = -vel[1]*f[0] + vel[0]*f[1];
  res[3] = -vel[2]*f[4] + vel[1]*f[5];
  res[4] =  vel[2]*f[3] - vel[0]*f[5];
  res[5] = -vel[1]*f[3] + vel[0]*f[4];
  res[0] += -vel[5]*f[4] + vel[4]*f[5];
  res[1] +=  vel[5]*f[3] - vel[3]*f[5];
  res[2] += -vel[4]*f[3] + vel[3]*f[4];
}

/* :417-447 */
static void mju_inertCom(mjtNum res[10], const mjtNum inert[3], const mjtNum mat[9],
                         const mjtNum dif[3], mjtNum mass) {
  mjtNum tmp[9] = {mat[0]*inert[0], mat[3]*inert[0], mat[6]*inert[0],
                   mat[1]*inert[1], mat[4]*inert[1], mat[7]*inert[1],
                   mat[2]*inert[2], mat[5]*inert[2], mat[8]*inert[2]};
  res[0] = mat[0]*tmp[0] + mat[1]*tmp[3] + mat[2]*tmp[6];
  res[1] = mat[3]*tmp[1] + mat[4]*tmp[4] + mat[5]*tmp[7];
  res[2] = mat[6]*tmp[2] + mat[7]*tmp[5] + mat[8]*tmp[8];
  res[3] = mat[0]*tmp[1] + mat[1]*tmp[4] + mat[2]*tmp[7];
  res[4] = mat[0]*tmp[2] + mat[1]*tmp[5] + mat[2]*tmp[8];
  res[5] = mat[3]*tmp[2] + mat[4]*tmp[5] + mat[5]*tmp[8];
  res[0] += mass*(dif[1]*dif[1] + dif[2]*dif[2]);
  res[1] += mass*(dif[0]*dif[0] + dif[2]*dif[2]);
  res[2] += mass*(dif[0]*dif[0] + dif[1]*dif[1]);
  res[3] -= mass*dif[0]*dif[1];
  res[4] -= mass*dif[0]*dif[2];
  res[5] -= mass*dif[1]*dif[2];
  res[6] = mass*dif[0];
  res[7] = mass*dif[1];
  res[8] = mass*dif[2];
  res[9] = mass;
}

/* :452-459 */
static void mju_mulInertVec(mjtNum res[6], const mjtNum i[10], const mjtNum v[6]) {
  res[0] = i[0]*v[0] + i[3]*v[1] + i[4]*v[2] - i[8]*v[4] + i[7]*v[5];
  res[1] = i[3]*v[0] + i[1]*v[1] + i[5]*v[2] + i[8]*v[3] - i[6]*v[5];
  res[2] = i[4]*v[0] + i[5]*v[1] + i[2]*v[2] - i[7]*v[3] + i[6]*v[4];
  res[3] = i[8]*v[1] - i[7]*v[2] + i[9]*v[3];
  res[4] = i[6]*v[2] - i[8]*v[0] + i[9]*v[4];
  res[5] = i[7]*v[0] - i[6]*v[1] + i[9]*v[5];
}

/* :464-476 */
static void mju_dofCom(mjtNum res[6], const mjtNum axis[3], const mjtNum offset[3]) {
  if (offset) {
    mju_copy3(res, axis);
    mju_cross(res+3, axis, offset);
  } else {
    mju_zero3(res);
    mju_copy3(res+3, axis);
  }
}

/* :481-489 */
static void mju_mulDofVec(mjtNum* res, const mjtNum* dof, const mjtNum* vec, int n) {
  if (n == 1) {
    mju_scl(res, dof, vec[0], 6);
  } else if (n <= 0) {
    mju_zero(res, 6);
  } else {
    mju_mulMatTVec(res, dof, vec, n, 6);
  }
}

/*============================ engine_support.c ============================================*/

/* :1565-1606 */
static void mj_local2Global(mjhipData* d, mjtNum xpos[3], mjtNum xmat[9], const mjtNum pos[3],
                            const mjtNum quat[4], int body, mjtByte sameframe) {
  if (xpos && pos) {
    switch (sameframe) {
    case mjhipSAMEFRAME_NONE:
    case mjhipSAMEFRAME_BODYROT:
    case mjhipSAMEFRAME_INERTIAROT:
      mju_mulMatVec3(xpos, d->xmat+9*body, pos);
      mju_addTo3(xpos, d->xpos+3*body);
      break;
    case mjhipSAMEFRAME_BODY:
      mju_copy3(xpos, d->xpos+3*body);
      break;
    case mjhipSAMEFRAME_INERTIA:
      mju_copy3(xpos, d->xipos+3*body);
      break;
    }
  }
  if (xmat && quat) {
    mjtNum tmp[4];
    switch (sameframe) {
    case mjhipSAMEFRAME_NONE:
      mju_mulQuat(tmp, d->xquat+4*body, quat);
      mju_quat2Mat(xmat, tmp);
      break;
    case mjhipSAMEFRAME_BODY:
    case mjhipSAMEFRAME_BODYROT:
      mju_copy(xmat, d->xmat+9*body, 9);
      break;
    case mjhipSAMEFRAME_INERTIA:
    case mjhipSAMEFRAME_INERTIAROT:
      mju_copy(xmat, d->ximat+9*body, 9);
      break;
    }
  }
}

/* :389-441, dense */
static void mj_jac(const mjhipModel* m, const mjhipData* d, mjtNum* jacp, mjtNum* jacr,
                   const mjtNum point[3], int body) {
  int nv = m->nv;
  mjtNum offset[3];
  if (jacp) {
    mju_zero(jacp, 3*nv);
    mju_sub3(offset, point, d->subtree_com+3*m->body_rootid[body]);
  }
  if (jacr) mju_zero(jacr, 3*nv);
  while (body && !m->body_dofnum[body]) body = m->body_parentid[body];
  if (!body) return;
  int i = m->body_dofadr[body] + m->body_dofnum[body] - 1;
  while (i >= 0) {
    mjtNum* cdof = d->cdof+6*i;
    if (jacr) {
      jacr[i+0*nv] = cdof[0];
      jacr[i+1*nv] = cdof[1];
      jacr[i+2*nv] = cdof[2];
    }
    if (jacp) {
      mjtNum tmp[3];
      mju_cross(tmp, cdof, offset);
      jacp[i+0*nv] = cdof[3] + tmp[0];
      jacp[i+1*nv] = cdof[4] + tmp[1];
      jacp[i+2*nv] = cdof[5] + tmp[2];
    }
    i = m->dof_parentid[i];
  }
}

/*---------------------------- sparse Jacobians (mj_isSparse models) -----------------------*/

/* mj_isSparse, engine_core_constraint.c:99-106 */
static int mj_isSparse(const mjhipModel* m) {
  return m->opt.jacobian == mjhipJAC_SPARSE || (m->opt.jacobian == mjhipJAC_AUTO && m->nv >= 60);
}

/* mj_mergeChain :264-304: the union of two bodies' dof ancestor chains, increasing */
static int mj_mergeChain(const mjhipModel* m, int* chain, int b1, int b2) {
  int da1, da2, NV = 0;
  while (b1 && !m->body_dofnum[b1]) b1 = m->body_parentid[b1];
  while (b2 && !m->body_dofnum[b2]) b2 = m->body_parentid[b2];
  if (b1 == 0 && b2 == 0) return 0;
  da1 = m->body_dofadr[b1] + m->body_dofnum[b1] - 1;
  da2 = m->body_dofadr[b2] + m->body_dofnum[b2] - 1;
  while (da1 >= 0 || da2 >= 0) {
    chain[NV] = mjMAX(da1, da2);
    if (da1 == chain[NV]) da1 = m->dof_parentid[da1];
    if (da2 == chain[NV]) da2 = m->dof_parentid[da2];
    NV++;
  }
  for (int i = 0; i < NV/2; i++) {
    int tmp = chain[i];
    chain[i] = chain[NV-i-1];
    chain[NV-i-1] = tmp;
  }
  return NV;
}

/* mj_mergeChainSimple :309-336 */
static int mj_mergeChainSimple(const mjhipModel* m, int* chain, int b1, int b2) {
  if (b1 > b2) {
    int tmp = b1;
    b1 = b2;
    b2 = tmp;
  }
  int n1 = m->body_dofnum[b1], n2 = m->body_dofnum[b2];
  if (n1 == 0 && n2 == 0) return 0;
  for (int i = 0; i < n1; i++) chain[i] = m->body_dofadr[b1] + i;
  for (int i = 0; i < n2; i++) chain[n1+i] = m->body_dofadr[b2] + i;
  return n1 + n2;
}

/* mj_jacSparse :526-591: the 3 x NV Jacobians over `chain` */
static void mj_jacSparse(const mjhipModel* m, const mjhipData* d, mjtNum* jacp, mjtNum* jacr,
                         const mjtNum* point, int body, int NV, const int* chain) {
  if (jacp) mju_zero(jacp, 3*NV);
  if (jacr) mju_zero(jacr, 3*NV);
  mjtNum offset[3];
  mju_sub3(offset, point, d->subtree_com+3*m->body_rootid[body]);
  while (body && !m->body_dofnum[body]) body = m->body_parentid[body];
  if (!body) return;
  int da = m->body_dofadr[body] + m->body_dofnum[body] - 1;
  int ci = NV-1;
  while (da >= 0) {
    while (ci >= 0 && chain[ci] > da) ci--;
    /* chain[ci] == da: the chain holds every ancestral dof (SHOULD NOT OCCUR otherwise) */
    const mjtNum* cdof = d->cdof + 6*da;
    if (jacr) {
      jacr[ci+0*NV] = cdof[0];
      jacr[ci+1*NV] = cdof[1];
      jacr[ci+2*NV] = cdof[2];
    }
    if (jacp) {
      mjtNum tmp[3];
      mju_cross(tmp, cdof, offset);
      jacp[ci+0*NV] = cdof[3] + tmp[0];
      jacp[ci+1*NV] = cdof[4] + tmp[1];
      jacp[ci+2*NV] = cdof[5] + tmp[2];
    }
    da = m->dof_parentid[da];
  }
}

/* mj_jacSparseSimple :596-654: the signed Jacobian of a simple body straight into the
 * difference, at chain positions start.. */
static void mj_jacSparseSimple(const mjhipModel* m, const mjhipData* d, mjtNum* jacdifp,
                               mjtNum* jacdifr, const mjtNum* point, int body, int flg_second,
                               int NV, int start) {
  mjtNum offset[3];
  mju_sub3(offset, point, d->subtree_com+3*m->body_rootid[body]);
  if (!m->body_dofnum[body]) return;
  int ci = start;
  int end = m->body_dofadr[body] + m->body_dofnum[body];
  for (int da = m->body_dofadr[body]; da < end; da++) {
    const mjtNum* cdof = d->cdof+6*da;
    if (jacdifr) {
      if (flg_second) {
        jacdifr[ci+0*NV] = cdof[0];
        jacdifr[ci+1*NV] = cdof[1];
        jacdifr[ci+2*NV] = cdof[2];
      } else {
        jacdifr[ci+0*NV] = -cdof[0];
        jacdifr[ci+1*NV] = -cdof[1];
        jacdifr[ci+2*NV] = -cdof[2];
      }
    }
    if (jacdifp) {
      mjtNum tmp[3];
      mju_cross(tmp, cdof, offset);
      if (flg_second) {
        jacdifp[ci+0*NV] = (cdof[3] + tmp[0]);
        jacdifp[ci+1*NV] = (cdof[4] + tmp[1]);
        jacdifp[ci+2*NV] = (cdof[5] + tmp[2]);
      } else {
        jacdifp[ci+0*NV] = -(cdof[3] + tmp[0]);
        jacdifp[ci+1*NV] = -(cdof[4] + tmp[1]);
        jacdifp[ci+2*NV] = -(cdof[5] + tmp[2]);
      }
    }
    ci++;
  }
}

/* mj_jacDifPair :659-731: pos2 - pos1 Jacobians, dense (NV = nv) or over the merged chain */
static int mj_jacDifPair(const mjhipModel* m, const mjhipData* d, int* chain, int b1, int b2,
                         const mjtNum pos1[3], const mjtNum pos2[3], mjtNum* jac1p,
                         mjtNum* jac2p, mjtNum* jacdifp, mjtNum* jac1r, mjtNum* jac2r,
                         mjtNum* jacdifr) {
  int issimple = (m->body_simple[b1] && m->body_simple[b2]);
  int issparse = mj_isSparse(m);
  int NV = m->nv;
  if (!NV) return 0;
  if (issparse) {
    NV = issimple ? mj_mergeChainSimple(m, chain, b1, b2) : mj_mergeChain(m, chain, b1, b2);
  }
  if (!NV) return 0;
  if (issparse) {
    if (issimple) {
      mj_jacSparseSimple(m, d, jacdifp, jacdifr, pos1, b1, 0, NV,
                         b1 < b2 ? 0 : m->body_dofnum[b2]);
      mj_jacSparseSimple(m, d, jacdifp, jacdifr, pos2, b2, 1, NV,
                         b2 < b1 ? 0 : m->body_dofnum[b1]);
    } else {
      mj_jacSparse(m, d, jac1p, jac1r, pos1, b1, NV, chain);
      mj_jacSparse(m, d, jac2p, jac2r, pos2, b2, NV, chain);
      if (jacdifp) mju_sub(jacdifp, jac2p, jac1p, 3*NV);
      if (jacdifr) mju_sub(jacdifr, jac2r, jac1r, 3*NV);
    }
  } else {
    mj_jac(m, d, jac1p, jac1r, pos1, b1);
    mj_jac(m, d, jac2p, jac2r, pos2, b2);
    if (jacdifp) mju_sub(jacdifp, jac2p, jac1p, 3*NV);
    if (jacdifr) mju_sub(jacdifr, jac2r, jac1r, 3*NV);
  }
  return NV;
}

/* mju_combineSparse engine_util_sparse.h:244-303: dst = a*dst + b*src over the union of the
 * two index sets (buf/buf_ind: scratch of the result's size) */
static int mju_combineSparse(mjtNum* dst, const mjtNum* src, mjtNum a, mjtNum b, int dst_nnz,
                             int src_nnz, int* dst_ind, const int* src_ind, mjtNum* buf,
                             int* buf_ind) {
  if (dst_nnz == src_nnz && !memcmp(dst_ind, src_ind, dst_nnz*sizeof(int))) {
    for (int i = 0; i < dst_nnz; i++) dst[i] = dst[i]*a + src[i]*b;   /* mju_addToSclScl */
    return dst_nnz;
  }
  if (dst_nnz) {
    memcpy(buf, dst, dst_nnz*sizeof(mjtNum));
    memcpy(buf_ind, dst_ind, dst_nnz*sizeof(int));
  }
  int bi = 0, si = 0, nnz = 0, buf_nnz = dst_nnz;
  while (bi < buf_nnz && si < src_nnz) {
    int badr = buf_ind[bi], sadr = src_ind[si];
    if (badr == sadr) {
      dst[nnz] = a*buf[bi++] + b*src[si++];
      dst_ind[nnz++] = badr;
    } else if (badr < sadr) {
      dst[nnz] = a*buf[bi++];
      dst_ind[nnz++] = badr;
    } else {
      dst[nnz] = b*src[si++];
      dst_ind[nnz++] = sadr;
    }
  }
  while (si < src_nnz) {
    dst[nnz] = b*src[si];
    dst_ind[nnz++] = src_ind[si++];
  }
  while (bi < buf_nnz) {
    dst[nnz] = a*buf[bi];
    dst_ind[nnz++] = buf_ind[bi++];
  }
  return nnz;
}

/* mju_mulMatVecSparse engine_util_sparse.c:156-167 (the AVX build's supernode path groups
 * each row's products the same way, engine_util_sparse_avx.h:116-249) */
static void mju_mulMatVecSparse(mjtNum* res, const mjtNum* mat, const mjtNum* vec, int nr,
                                const int* rownnz, const int* rowadr, const int* colind) {
  for (int r = 0; r < nr; r++) {
    res[r] = mju_dotSparse(mat+rowadr[r], vec, rownnz[r], colind+rowadr[r]);
  }
}

/* mju_transposeSparse engine_util_sparse.c:474-515 */
static void mju_transposeSparse(mjtNum* res, const mjtNum* mat, int nr, int nc, int* res_rownnz,
                                int* res_rowadr, int* res_colind, const int* rownnz,
                                const int* rowadr, const int* colind) {
  memset(res_rownnz, 0, nc*sizeof(int));
  for (int r = 0; r < nr; r++) {
    for (int j = rowadr[r]; j < rowadr[r] + rownnz[r]; j++) res_rownnz[colind[j]]++;
  }
  res_rowadr[0] = 0;
  for (int i = 1; i < nc; i++) res_rowadr[i] = res_rowadr[i-1] + res_rownnz[i-1];
  for (int r = 0; r < nr; r++) {
    for (int i = rowadr[r]; i < rowadr[r] + rownnz[r]; i++) {
      int c = res_rowadr[colind[i]]++;
      res_colind[c] = r;
      res[c] = mat[i];
    }
  }
  for (int i = nc-1; i > 0; i--) res_rowadr[i] = res_rowadr[i-1];
  res_rowadr[0] = 0;
}

/* value of tendon t's Jacobian at dof col: dense row, or the compressed row of a sparse
 * model (the derivative code reads single entries) */
static mjtNum ten_J_at(const mjhipModel* m, const mjhipData* d, int t, int col) {
  if (!mj_isSparse(m)) return d->ten_J[t*m->nv + col];
  for (int k = 0; k < d->ten_J_rownnz[t]; k++) {
    if (d->ten_J_colind[d->ten_J_rowadr[t]+k] == col) return d->ten_J[d->ten_J_rowadr[t]+k];
  }
  return 0;
}

/* :1194-1251, dense case. The sparse case (:1211-1230) forms the same column values over
 * the body's chain and adds only those, so qfrc_target gets the same values. */
static void mj_applyFT(const mjhipModel* m, mjhipData* d, const mjtNum force[3],
                       const mjtNum torque[3], const mjtNum point[3], int body,
                       mjtNum* qfrc_target) {
  int nv = m->nv;
  mjtNum* jacp = force ? (mjtNum*)malloc(3*nv*sizeof(mjtNum)) : NULL;
  mjtNum* jacr = torque ? (mjtNum*)malloc(3*nv*sizeof(mjtNum)) : NULL;
  mjtNum* qforce = (mjtNum*)malloc(nv*sizeof(mjtNum));
  mj_jac(m, d, jacp, jacr, point, body);
  if (force) {
    mju_mulMatTVec(qforce, jacp, force, 3, nv);
    mju_addTo(qfrc_target, qforce, nv);
  }
  if (torque) {
    mju_mulMatTVec(qforce, jacr, torque, 3, nv);
    mju_addTo(qfrc_target, qforce, nv);
  }
  free(jacp); free(jacr); free(qforce);
}

/* :1254-1261 */
void or_xfrcAccumulate(const mjhipModel* m, mjhipData* d, mjtNum* qfrc) {
  for (int i = 1; i < m->nbody; i++) {
    if (!mju_isZero(d->xfrc_applied+6*i, 6)) {
      mj_applyFT(m, d, d->xfrc_applied+6*i, d->xfrc_applied+6*i+3, d->xipos+3*i, i, qfrc);
    }
  }
}

/* :1518-1550 */
static void mj_integratePos(const mjhipModel* m, mjtNum* qpos, const mjtNum* qvel, mjtNum dt) {
  for (int j = 0; j < m->njnt; j++) {
    int padr = m->jnt_qposadr[j];
    int vadr = m->jnt_dofadr[j];
    switch (m->jnt_type[j]) {
    case mjhipJNT_FREE:
      for (int i = 0; i < 3; i++) qpos[padr+i] += dt * qvel[vadr+i];
      padr += 3;
      vadr += 3;
      /* fallthrough */
    case mjhipJNT_BALL:
      mju_quatIntegrate(qpos+padr, qvel+vadr, dt);
      break;
    case mjhipJNT_HINGE:
    case mjhipJNT_SLIDE:
      qpos[padr] += dt * qvel[vadr];
    }
  }
}

/*============================ engine_core_smooth.c ========================================*/

/* :38-178 */
void or_kinematics(const mjhipModel* m, mjhipData* d) {
  int nbody = m->nbody, nsite = m->nsite, ngeom = m->ngeom;
  mju_zero3(d->xpos);
  d->xquat[0] = 1; d->xquat[1] = d->xquat[2] = d->xquat[3] = 0;
  mju_zero3(d->xipos);
  mju_zero(d->xmat, 9);
  mju_zero(d->ximat, 9);
  d->xmat[0] = d->xmat[4] = d->xmat[8] = 1;
  d->ximat[0] = d->ximat[4] = d->ximat[8] = 1;

  for (int i = 1; i < nbody; i++) {
    mjtNum xpos[3], xquat[4];
    int jntadr = m->body_jntadr[i];
    int jntnum = m->body_jntnum[i];

    if (jntnum == 1 && m->jnt_type[jntadr] == mjhipJNT_FREE) {
      int qadr = m->jnt_qposadr[jntadr];
      mju_copy3(xpos, d->qpos+qadr);
      mju_copy4(xquat, d->qpos+qadr+3);
      mju_normalize4(xquat);
      mju_copy3(d->xanchor+3*jntadr, xpos);
      mju_copy3(d->xaxis+3*jntadr, m->jnt_axis+3*jntadr);
    } else {
      int pid = m->body_parentid[i];
      mjtNum *bodypos, *bodyquat, quat[4];
      if (m->body_mocapid[i] >= 0) {
        bodypos = d->mocap_pos + 3*m->body_mocapid[i];
        mju_copy4(quat, d->mocap_quat + 4*m->body_mocapid[i]);
        mju_normalize4(quat);
        bodyquat = quat;
      } else {
        bodypos = m->body_pos+3*i;
        bodyquat = m->body_quat+4*i;
      }
      if (pid) {
        mju_mulMatVec3(xpos, d->xmat+9*pid, bodypos);
        mju_addTo3(xpos, d->xpos+3*pid);
        mju_mulQuat(xquat, d->xquat+4*pid, bodyquat);
      } else {
        mju_copy3(xpos, bodypos);
        mju_copy4(xquat, bodyquat);
      }
      mjtNum xanchor[3], xaxis[3];
      for (int j = 0; j < jntnum; j++) {
        int jid = jntadr + j;
        int qadr = m->jnt_qposadr[jid];
        int jtype = m->jnt_type[jid];
        mju_rotVecQuat(xaxis, m->jnt_axis+3*jid, xquat);
        mju_rotVecQuat(xanchor, m->jnt_pos+3*jid, xquat);
        mju_addTo3(xanchor, xpos);
        switch (jtype) {
        case mjhipJNT_SLIDE:
          mju_addToScl3(xpos, xaxis, d->qpos[qadr] - m->qpos0[qadr]);
          break;
        case mjhipJNT_BALL:
        case mjhipJNT_HINGE:
          {
            mjtNum qloc[4];
            if (jtype == mjhipJNT_BALL) {
              mju_copy4(qloc, d->qpos+qadr);
              mju_normalize4(qloc);
            } else {
              mju_axisAngle2Quat(qloc, m->jnt_axis+3*jid, d->qpos[qadr] - m->qpos0[qadr]);
            }
            mju_mulQuat(xquat, xquat, qloc);
            mjtNum vec[3];
            mju_rotVecQuat(vec, m->jnt_pos+3*jid, xquat);
            mju_sub3(xpos, xanchor, vec);
          }
          break;
        }
        mju_copy3(d->xanchor+3*jid, xanchor);
        mju_copy3(d->xaxis+3*jid, xaxis);
      }
    }
    mju_normalize4(xquat);
    mju_copy4(d->xquat+4*i, xquat);
    mju_copy3(d->xpos+3*i, xpos);
    mju_quat2Mat(d->xmat+9*i, xquat);
  }

  for (int i = 1; i < nbody; i++) {
    mj_local2Global(d, d->xipos+3*i, d->ximat+9*i, m->body_ipos+3*i, m->body_iquat+4*i,
                    i, m->body_sameframe[i]);
  }
  for (int i = 0; i < ngeom; i++) {
    mj_local2Global(d, d->geom_xpos+3*i, d->geom_xmat+9*i, m->geom_pos+3*i,
                    m->geom_quat+4*i, m->geom_bodyid[i], m->geom_sameframe[i]);
  }
  for (int i = 0; i < nsite; i++) {
    mj_local2Global(d, d->site_xpos+3*i, d->site_xmat+9*i, m->site_pos+3*i,
                    m->site_quat+4*i, m->site_bodyid[i], m->site_sameframe[i]);
  }
}

/* :183-270 */
void or_comPos(const mjhipModel* m, mjhipData* d) {
  int nbody = m->nbody, njnt = m->njnt;
  mjtNum offset[3], axis[3];
  mjtNum* mass_subtree = (mjtNum*)calloc(nbody, sizeof(mjtNum));
  mju_zero(d->subtree_com, nbody*3);
  for (int i = nbody-1; i >= 0; i--) {
    mju_addToScl3(d->subtree_com+3*i, d->xipos+3*i, m->body_mass[i]);
    mass_subtree[i] += m->body_mass[i];
    if (i) {
      int j = m->body_parentid[i];
      mju_addTo3(d->subtree_com+3*j, d->subtree_com+3*i);
      mass_subtree[j] += mass_subtree[i];
    }
    if (mass_subtree[i] < mjMINVAL) {
      mju_copy3(d->subtree_com+3*i, d->xipos+3*i);
    } else {
      mju_scl3(d->subtree_com+3*i, d->subtree_com+3*i, 1.0/mjMAX(mjMINVAL, mass_subtree[i]));
    }
  }
  mju_zero(d->cinert, 10);
  for (int i = 1; i < nbody; i++) {
    mju_sub3(offset, d->xipos+3*i, d->subtree_com+3*m->body_rootid[i]);
    mju_inertCom(d->cinert+10*i, m->body_inertia+3*i, d->ximat+9*i, offset, m->body_mass[i]);
  }
  for (int j = 0; j < njnt; j++) {
    int da = 6*m->jnt_dofadr[j];
    int bi = m->jnt_bodyid[j];
    mju_sub3(offset, d->subtree_com+3*m->body_rootid[bi], d->xanchor+3*j);
    int skip = 0;
    switch (m->jnt_type[j]) {
    case mjhipJNT_FREE:
      mju_zero(d->cdof+da, 18);
      for (int i = 0; i < 3; i++) d->cdof[da+3+7*i] = 1;
      skip = 18;
      /* fallthrough */
    case mjhipJNT_BALL:
      for (int i = 0; i < 3; i++) {
        axis[0] = d->xmat[9*bi+i+0];
        axis[1] = d->xmat[9*bi+i+3];
        axis[2] = d->xmat[9*bi+i+6];
        mju_dofCom(d->cdof+da+skip+6*i, axis, offset);
      }
      break;
    case mjhipJNT_SLIDE:
      mju_dofCom(d->cdof+da, d->xaxis+3*j, 0);
      break;
    case mjhipJNT_HINGE:
      mju_dofCom(d->cdof+da, d->xaxis+3*j, offset);
      break;
    }
  }
  free(mass_subtree);
}

/* :275-392 */
static void or_camlight(const mjhipModel* m, mjhipData* d) {
  mjtNum pos[3], matT[9];
  for (int i = 0; i < m->ncam; i++) {
    mj_local2Global(d, d->cam_xpos+3*i, d->cam_xmat+9*i, m->cam_pos+3*i, m->cam_quat+4*i,
                    m->cam_bodyid[i], 0);
    int id = m->cam_bodyid[i];
    int id1 = m->cam_targetbodyid[i];
    switch (m->cam_mode[i]) {
    case mjhipCAMLIGHT_FIXED:
      break;
    case mjhipCAMLIGHT_TRACK:
    case mjhipCAMLIGHT_TRACKCOM:
      mju_copy(d->cam_xmat+9*i, m->cam_mat0+9*i, 9);
      if (m->cam_mode[i] == mjhipCAMLIGHT_TRACK) {
        mju_add3(d->cam_xpos+3*i, d->xpos+3*id, m->cam_pos0+3*i);
      } else {
        mju_add3(d->cam_xpos+3*i, d->subtree_com+3*id, m->cam_poscom0+3*i);
      }
      break;
    case mjhipCAMLIGHT_TARGETBODY:
    case mjhipCAMLIGHT_TARGETBODYCOM:
      if (id1 >= 0) {
        if (m->cam_mode[i] == mjhipCAMLIGHT_TARGETBODY) {
          mju_copy3(pos, d->xpos+3*id1);
        } else {
          mju_copy3(pos, d->subtree_com+3*id1);
        }
        mju_sub3(matT+6, d->cam_xpos+3*i, pos);
        mju_normalize3(matT+6);
        matT[3] = 0; matT[4] = 0; matT[5] = 1;
        mju_cross(matT, matT+3, matT+6);
        mju_normalize3(matT);
        mju_cross(matT+3, matT+6, matT);
        mju_normalize3(matT+3);
        /* mju_transpose(cam_xmat, matT, 3, 3) */
        for (int r = 0; r < 3; r++)
          for (int c = 0; c < 3; c++) d->cam_xmat[9*i + 3*c + r] = matT[3*r + c];
      }
    }
  }
  for (int i = 0; i < m->nlight; i++) {
    mj_local2Global(d, d->light_xpos+3*i, 0, m->light_pos+3*i, 0, m->light_bodyid[i], 0);
    mju_rotVecQuat(d->light_xdir+3*i, m->light_dir+3*i, d->xquat+4*m->light_bodyid[i]);
    int id = m->light_bodyid[i];
    int id1 = m->light_targetbodyid[i];
    switch (m->light_mode[i]) {
    case mjhipCAMLIGHT_FIXED:
      break;
    case mjhipCAMLIGHT_TRACK:
    case mjhipCAMLIGHT_TRACKCOM:
      mju_copy3(d->light_xdir+3*i, m->light_dir0+3*i);
      if (m->light_mode[i] == mjhipCAMLIGHT_TRACK) {
        mju_add3(d->light_xpos+3*i, d->xpos+3*id, m->light_pos0+3*i);
      } else {
        mju_add3(d->light_xpos+3*i, d->subtree_com+3*id, m->light_poscom0+3*i);
      }
      break;
    case mjhipCAMLIGHT_TARGETBODY:
    case mjhipCAMLIGHT_TARGETBODYCOM:
      if (id1 >= 0) {
        if (m->light_mode[i] == mjhipCAMLIGHT_TARGETBODY) {
          mju_copy3(pos, d->xpos+3*id1);
        } else {
          mju_copy3(pos, d->subtree_com+3*id1);
        }
        mju_sub3(d->light_xdir+3*i, pos, d->light_xpos+3*i);
      }
    }
    mju_normalize3(d->light_xdir+3*i);
  }
}

/* ---- tendon wrapping around spheres and cylinders (engine_util_misc.c:33-418) ---- */
static mjtNum mju_dot3(const mjtNum* a, const mjtNum* b);
static mjtNum mju_norm3(const mjtNum* a);
static void mju_mulMatTVec3(mjtNum res[3], const mjtNum mat[9], const mjtNum vec[3]);

/* mju_normalize for n = 2 (engine_util_blas.c:651-668) */
static mjtNum or_normalize2(mjtNum* v) {
  mjtNum norm = sqrt(mju_dot(v, v, 2));
  if (norm < mjMINVAL) {
    v[0] = 1; v[1] = 0;
  } else {
    mjtNum inv = 1/norm;
    v[0] *= inv; v[1] *= inv;
  }
  return norm;
}

/* :33-50 do segments p1-p2 and p3-p4 intersect */
static int or_isIntersect(const mjtNum* p1, const mjtNum* p2, const mjtNum* p3,
                          const mjtNum* p4) {
  mjtNum det = (p4[1]-p3[1])*(p2[0]-p1[0]) - (p4[0]-p3[0])*(p2[1]-p1[1]);
  if (fabs(det) < mjMINVAL) return 0;
  mjtNum a = ((p4[0]-p3[0])*(p1[1]-p3[1]) - (p4[1]-p3[1])*(p1[0]-p3[0])) / det;
  mjtNum b = ((p2[0]-p1[0])*(p1[1]-p3[1]) - (p2[1]-p1[1])*(p1[0]-p3[0])) / det;
  return a >= 0 && a <= 1 && b >= 0 && b <= 1;
}

/* :55-71 arc length from p0 to p1 on the circle, the long way for the flipped solution */
static mjtNum or_lengthCircle(const mjtNum* p0, const mjtNum* p1, int ind, mjtNum radius) {
  mjtNum a[2] = {p0[0], p0[1]}, b[2] = {p1[0], p1[1]};
  or_normalize2(a);
  or_normalize2(b);
  mjtNum angle = acos(mju_dot(a, b, 2));
  mjtNum cross = p0[1]*p1[0] - p0[0]*p1[1];
  if ((cross > 0 && ind) || (cross < 0 && !ind)) angle = 2*mjhipPI - angle;
  return radius*angle;
}

/* :77-151 wrap a 2D segment around the circle of the given radius: tangent points in
 * pnt[4], the arc length, or -1 when the segment clears the circle */
static mjtNum or_wrapCircle(mjtNum pnt[4], const mjtNum end[4], const mjtNum* side,
                            mjtNum radius) {
  mjtNum sqlen0 = end[0]*end[0] + end[1]*end[1];
  mjtNum sqlen1 = end[2]*end[2] + end[3]*end[3];
  mjtNum sqrad = radius*radius;
  if (sqlen0 < sqrad || sqlen1 < sqrad || radius < mjMINVAL) return -1;
  mjtNum dif[2] = {end[2]-end[0], end[3]-end[1]};
  mjtNum dd = dif[0]*dif[0] + dif[1]*dif[1];
  if (dd < mjMINVAL) return -1;
  mjtNum a = -(dif[0]*end[0] + dif[1]*end[1])/dd;
  if (a < 0) a = 0;
  else if (a > 1) a = 1;
  mjtNum tmp[2] = {a*dif[0] + end[0], a*dif[1] + end[1]};
  if (tmp[0]*tmp[0] + tmp[1]*tmp[1] > sqrad && (!side || mju_dot(side, tmp, 2) >= 0)) {
    return -1;
  }
  mjtNum sol[2][2][2], good[2];
  for (int i = 0; i < 2; i++) {
    mjtNum sqrt0 = sqrt(sqlen0 - sqrad);
    mjtNum sqrt1 = sqrt(sqlen1 - sqrad);
    int sgn = i == 0 ? 1 : -1;
    sol[i][0][0] = (end[0]*sqrad + sgn*radius*end[1]*sqrt0)/sqlen0;
    sol[i][0][1] = (end[1]*sqrad - sgn*radius*end[0]*sqrt0)/sqlen0;
    sol[i][1][0] = (end[2]*sqrad - sgn*radius*end[3]*sqrt1)/sqlen1;
    sol[i][1][1] = (end[3]*sqrad + sgn*radius*end[2]*sqrt1)/sqlen1;
    if (side) {
      mju_add(tmp, sol[i][0], sol[i][1], 2);
      or_normalize2(tmp);
      good[i] = mju_dot(tmp, side, 2);
    } else {
      mju_sub(tmp, sol[i][0], sol[i][1], 2);
      good[i] = -mju_dot(tmp, tmp, 2);
    }
    if (or_isIntersect(end, sol[i][0], end+2, sol[i][1])) good[i] = -10000;
  }
  int i = good[0] > good[1] ? 0 : 1;
  pnt[0] = sol[i][0][0];
  pnt[1] = sol[i][0][1];
  pnt[2] = sol[i][1][0];
  pnt[3] = sol[i][1][1];
  if (or_isIntersect(end, pnt, end+2, pnt+2)) return -1;
  return or_lengthCircle(sol[i][0], sol[i][1], i, radius);
}

/* :157-272 wrap with the side site inside the circle: one contact point found by Newton
 * iterations on asin(A z) + asin(B z) - 2 asin(z) + G = 0; length 0, or -1 */
static mjtNum or_wrapInside(mjtNum pnt[4], const mjtNum end[4], mjtNum radius) {
  const int maxiter = 20;
  const mjtNum zinit = 1 - 1e-7, tolerance = 1e-6;
  mjtNum len0 = mju_norm(end, 2);
  mjtNum len1 = mju_norm(end+2, 2);
  mjtNum dif[2] = {end[2]-end[0], end[3]-end[1]};
  mjtNum dd = dif[0]*dif[0] + dif[1]*dif[1];
  if (len0 <= radius || len1 <= radius || radius < mjMINVAL || len0 < mjMINVAL ||
      len1 < mjMINVAL) {
    return -1;
  }
  if (dd > mjMINVAL) {
    mjtNum a = -(dif[0]*end[0] + dif[1]*end[1]) / dd;
    if (a > 0 && a < 1) {
      mjtNum tmp[2] = {end[0] + a*dif[0], end[1] + a*dif[1]};
      if (mju_norm(tmp, 2) <= radius) return -1;
    }
  }
  pnt[0] = 0.5*(end[0] + end[2]);
  pnt[1] = 0.5*(end[1] + end[3]);
  or_normalize2(pnt);
  pnt[0] *= radius;
  pnt[1] *= radius;
  pnt[2] = pnt[0];
  pnt[3] = pnt[1];
  mjtNum A = radius/len0, B = radius/len1;
  mjtNum cosG = (len0*len0 + len1*len1 - dd) / (2*len0*len1);
  if (cosG < -1+mjMINVAL) return -1;
  if (cosG > 1-mjMINVAL) return 0;
  mjtNum G = acos(cosG);
  mjtNum z = zinit;
  mjtNum f = asin(A*z) + asin(B*z) - 2*asin(z) + G;
  if (f > 0) return 0;
  int iter;
  for (iter = 0; iter < maxiter && fabs(f) > tolerance; iter++) {
    mjtNum df = A/fmax(mjMINVAL, sqrt(1-z*z*A*A)) + B/fmax(mjMINVAL, sqrt(1-z*z*B*B)) -
                2/fmax(mjMINVAL, sqrt(1-z*z));
    if (df > -mjMINVAL) return 0;
    mjtNum z1 = z - f/df;
    if (z1 > z) return 0;
    z = z1;
    f = asin(A*z) + asin(B*z) - 2*asin(z) + G;
    if (f > tolerance) return 0;
  }
  if (iter >= maxiter) return 0;
  mjtNum vec[2], ang;
  if (end[0]*end[3] - end[1]*end[2] > 0) {
    vec[0] = end[0]; vec[1] = end[1];
    ang = asin(z) - asin(A*z);
  } else {
    vec[0] = end[2]; vec[1] = end[3];
    ang = asin(z) - asin(B*z);
  }
  or_normalize2(vec);
  pnt[0] = radius*(cos(ang)*vec[0] - sin(ang)*vec[1]);
  pnt[1] = radius*(sin(ang)*vec[0] + cos(ang)*vec[1]);
  pnt[2] = pnt[0];
  pnt[3] = pnt[1];
  return 0;
}

/* :282-418 mju_wrap: the segment x0-x1 around a sphere or cylinder at xpos/xmat; the two
 * tangent points in wpnt[6] (global frame) and the wrapped length, or -1 for no wrap */
static mjtNum or_wrap(mjtNum wpnt[6], const mjtNum x0[3], const mjtNum x1[3],
                      const mjtNum xpos[3], const mjtNum xmat[9], mjtNum radius, int type,
                      const mjtNum* side) {
  mjtNum tmp[3], p[2][3];
  mju_sub3(tmp, x0, xpos);
  mju_mulMatTVec3(p[0], xmat, tmp);
  mju_sub3(tmp, x1, xpos);
  mju_mulMatTVec3(p[1], xmat, tmp);
  if (mju_norm3(p[0]) < mjMINVAL || mju_norm3(p[1]) < mjMINVAL) return -1;
  mjtNum axis[2][3];
  if (type == mjhipWRAP_SPHERE) {
    mju_copy3(axis[0], p[0]);
    mju_normalize3(axis[0]);
    mjtNum normal[3];
    mju_cross(normal, p[0], p[1]);
    mjtNum nrm = mju_normalize3(normal);
    if (nrm < mjMINVAL) {
      int i = 0;
      if (fabs(axis[0][1]) > fabs(axis[0][0]) && fabs(axis[0][1]) > fabs(axis[0][2])) i = 1;
      if (fabs(axis[0][2]) > fabs(axis[0][0]) && fabs(axis[0][2]) > fabs(axis[0][1])) i = 2;
      axis[1][0] = 1; axis[1][1] = 1; axis[1][2] = 1;
      axis[1][i] = 0;
      mju_cross(normal, axis[0], axis[1]);
      mju_normalize3(normal);
    }
    mju_cross(axis[1], normal, axis[0]);
    mju_normalize3(axis[1]);
  } else {
    axis[0][0] = 1; axis[0][1] = 0; axis[0][2] = 0;
    axis[1][0] = 0; axis[1][1] = 1; axis[1][2] = 0;
  }
  mjtNum s[3], dd[4], sd[2];
  dd[0] = mju_dot3(p[0], axis[0]);
  dd[1] = mju_dot3(p[0], axis[1]);
  dd[2] = mju_dot3(p[1], axis[0]);
  dd[3] = mju_dot3(p[1], axis[1]);
  if (side) {
    mju_sub3(tmp, side, xpos);
    mju_mulMatTVec3(s, xmat, tmp);
    sd[0] = mju_dot3(s, axis[0]);
    sd[1] = mju_dot3(s, axis[1]);
    or_normalize2(sd);
    sd[0] *= radius;
    sd[1] *= radius;
  }
  mjtNum wlen, pnt[4];
  if (side && mju_norm3(s) < radius) {
    wlen = or_wrapInside(pnt, dd, radius);
  } else {
    wlen = or_wrapCircle(pnt, dd, side ? sd : NULL, radius);
  }
  if (wlen < 0) return -1;
  mjtNum res[6];
  for (int i = 0; i < 2; i++) {
    mju_scl3(res+3*i, axis[0], pnt[2*i]);
    mju_scl3(tmp, axis[1], pnt[2*i+1]);
    mju_addTo3(res+3*i, tmp);
  }
  if (type == mjhipWRAP_CYLINDER) {
    mjtNum L0 = sqrt((p[0][0]-res[0])*(p[0][0]-res[0]) + (p[0][1]-res[1])*(p[0][1]-res[1]));
    mjtNum L1 = sqrt((p[1][0]-res[3])*(p[1][0]-res[3]) + (p[1][1]-res[4])*(p[1][1]-res[4]));
    res[2] = p[0][2] + (p[1][2] - p[0][2])*L0 / (L0+wlen+L1);
    res[5] = p[0][2] + (p[1][2] - p[0][2])*(L0+wlen) / (L0+wlen+L1);
    mjtNum height = fabs(res[5] - res[2]);
    wlen = sqrt(wlen*wlen + height*height);
  }
  mju_mulMatVec3(wpnt, xmat, res);
  mju_mulMatVec3(wpnt+3, xmat, res+3);
  mju_addTo3(wpnt, xpos);
  mju_addTo3(wpnt+3, xpos);
  return wlen;
}

/* :651-860, fixed tendons and spatial tendons through sites, pulleys and wrapping spheres
 * and cylinders, dense Jacobian (the wrap visualization outputs ten_wrapadr/ten_wrapnum/
 * wrap_obj/wrap_xpos are not kept) */
static void mju_mulMatTVec(mjtNum* res, const mjtNum* mat, const mjtNum* vec, int nr, int nc);

static void or_tendon(const mjhipModel* m, mjhipData* d) {
  int nv = m->nv, nten = m->ntendon, issparse = mj_isSparse(m);
  mjtNum *L = d->ten_length, *J = d->ten_J;
  int *rownnz = d->ten_J_rownnz, *rowadr = d->ten_J_rowadr, *colind = d->ten_J_colind;
  if (!nten) return;
  mju_zero(L, nten);
  /* clear the Jacobian: sparse or dense (:677-682) */
  if (issparse) {
    memset(rownnz, 0, nten*sizeof(int));
  } else {
    mju_zero(J, nten*nv);
  }
  mjtNum* jac1 = (mjtNum*)malloc(sizeof(mjtNum)*3*(nv ? nv : 1));
  mjtNum* jac2 = (mjtNum*)malloc(sizeof(mjtNum)*3*(nv ? nv : 1));
  mjtNum* jacdif = (mjtNum*)malloc(sizeof(mjtNum)*3*(nv ? nv : 1));
  mjtNum* tmp = (mjtNum*)malloc(sizeof(mjtNum)*(nv ? nv : 1));
  mjtNum* sparse_buf = (mjtNum*)malloc(sizeof(mjtNum)*(nv ? nv : 1));
  int* chain = (int*)malloc(sizeof(int)*(nv ? nv : 1));
  int* buf_ind = (int*)malloc(sizeof(int)*(nv ? nv : 1));
  for (int i = 0; i < nten; i++) {
    int adr = m->tendon_adr[i];
    int tendon_num = m->tendon_num[i];
    if (issparse) rowadr[i] = (i > 0 ? rowadr[i-1] + rownnz[i-1] : 0);
    if (m->wrap_type[adr] == mjhipWRAP_JOINT) {
      for (int j = 0; j < tendon_num; j++) {
        int k = m->wrap_objid[adr+j];
        L[i] += m->wrap_prm[adr+j] * d->qpos[m->jnt_qposadr[k]];
        if (issparse) {
          /* :709-714: combine the joint's coefficient into the row (a repeated joint adds) */
          rownnz[i] = mju_combineSparse(J+rowadr[i], &m->wrap_prm[adr+j], 1, 1, rownnz[i], 1,
                                        colind+rowadr[i], &m->jnt_dofadr[k], sparse_buf,
                                        buf_ind);
        } else {
          J[i*nv + m->jnt_dofadr[k]] = m->wrap_prm[adr+j];
        }
      }
      continue;
    }
    /* spatial: site-site or site-geom-site sequences, a pulley divides what follows
     * (:725-855) */
    mjtNum divisor = 1;
    int j = 0;
    while (j < tendon_num - 1) {
      int type0 = m->wrap_type[adr+j], type1 = m->wrap_type[adr+j+1];
      if (type0 == mjhipWRAP_PULLEY || type1 == mjhipWRAP_PULLEY) {
        if (type0 == mjhipWRAP_PULLEY) divisor = m->wrap_prm[adr+j];
        j++;
        continue;
      }
      int id0 = m->wrap_objid[adr+j], id1 = m->wrap_objid[adr+j+1];
      mjtNum wlen = -1, wpnt[12];
      int wrapid = -1, wrapped = 0, wbody[4];
      mju_copy3(wpnt, d->site_xpos + 3*id0);
      wbody[0] = m->site_bodyid[id0];
      if (type1 == mjhipWRAP_SPHERE || type1 == mjhipWRAP_CYLINDER) {
        wrapped = 1;
        wrapid = id1;
        id1 = m->wrap_objid[adr+j+2];
        int sideid = (int)lround(m->wrap_prm[adr+j+1]);
        wlen = or_wrap(wpnt+3, d->site_xpos + 3*id0, d->site_xpos + 3*id1,
                       d->geom_xpos + 3*wrapid, d->geom_xmat + 9*wrapid,
                       m->geom_size[3*wrapid], type1,
                       sideid >= 0 ? d->site_xpos + 3*sideid : NULL);
      }
      if (wlen < 0) {
        mju_copy3(wpnt+3, d->site_xpos + 3*id1);
        wbody[1] = m->site_bodyid[id1];
        mjtNum dif[3];
        mju_sub3(dif, wpnt, wpnt+3);
        L[i] += mju_norm3(dif) / divisor;
      } else {
        mju_copy3(wpnt+9, d->site_xpos + 3*id1);
        wbody[1] = wbody[2] = m->geom_bodyid[wrapid];
        wbody[3] = m->site_bodyid[id1];
        mjtNum d0[3], d2[3];
        mju_sub3(d0, wpnt, wpnt+3);
        mju_sub3(d2, wpnt+6, wpnt+9);
        L[i] += (mju_norm3(d0) + wlen + mju_norm3(d2)) / divisor;
      }
      for (int k = 0; k < (wlen < 0 ? 1 : 3); k++) {
        if (wbody[k] == wbody[k+1]) continue;
        mjtNum dif[3];
        mju_sub3(dif, wpnt+3*k+3, wpnt+3*k);
        mju_normalize3(dif);
        if (issparse) {
          /* :801-819: the chain rule over the merged chain, combined into the row */
          int NV = mj_jacDifPair(m, d, chain, wbody[k], wbody[k+1], wpnt+3*k, wpnt+3*k+3,
                                 jac1, jac2, jacdif, NULL, NULL, NULL);
          if (!NV) continue;
          mju_mulMatTVec(tmp, jacdif, dif, 3, NV);
          rownnz[i] = mju_combineSparse(J+rowadr[i], tmp, 1, 1/divisor, rownnz[i], NV,
                                        colind+rowadr[i], chain, sparse_buf, buf_ind);
        } else {
          mj_jac(m, d, jac1, NULL, wpnt+3*k, wbody[k]);
          mj_jac(m, d, jac2, NULL, wpnt+3*k+3, wbody[k+1]);
          for (int c = 0; c < 3*nv; c++) jac2[c] = jac2[c] - jac1[c];
          mju_mulMatTVec(tmp, jac2, dif, 3, nv);
          mju_addToScl(J + i*nv, tmp, 1/divisor, nv);
        }
      }
      j += wrapped ? 2 : 1;
    }
  }
  free(jac1);
  free(jac2);
  free(jacdif);
  free(tmp);
  free(sparse_buf);
  free(chain);
  free(buf_ind);
}

/* :865-916, joint transmission (slide/hinge) */
static mjtNum mju_dot3(const mjtNum* a, const mjtNum* b);

static void or_mulJacTVec(const mjhipModel* m, const orEfc* e, mjtNum* res,
                          const mjtNum* vec);

/* engine_core_smooth.c:862-1100 mj_transmission: joint (slide/hinge/ball/free, in the
 * joint or the parent frame) and tendon transmissions (fixed tendons: their sparsity is a
 * model constant, moment_* model fields) */
static void or_transmission(const mjhipModel* m, mjhipData* d, const orEfc* e) {
  int nu = m->nu, nv = m->nv;
  int* rowadr = m->moment_rowadr;
  for (int i = 0; i < nu; i++) {
    int adr = rowadr[i];
    int id = m->actuator_trnid[2*i];
    mjtNum* gear = m->actuator_gear+6*i;
    mjtNum* length = d->actuator_length + i;
    mjtNum* moment = d->actuator_moment + adr;
    int trn = m->actuator_trntype[i];
    if (trn == mjhipTRN_JOINT || trn == mjhipTRN_JOINTINPARENT) {
      int t = m->jnt_type[id];
      if (t == mjhipJNT_SLIDE || t == mjhipJNT_HINGE) {
        *length = d->qpos[m->jnt_qposadr[id]]*gear[0];
        moment[0] = gear[0];
      } else if (t == mjhipJNT_BALL) {
        mjtNum axis[3], quat[4], gearAxis[3];
        mju_copy4(quat, d->qpos+m->jnt_qposadr[id]);
        mju_normalize4(quat);
        mju_quat2Vel(axis, quat, 1);
        if (trn == mjhipTRN_JOINT) {
          mju_copy3(gearAxis, gear);
        } else {
          quat[1] = -quat[1]; quat[2] = -quat[2]; quat[3] = -quat[3];
          mju_rotVecQuat(gearAxis, gear, quat);
        }
        *length = mju_dot3(axis, gearAxis);
        mju_copy3(moment, gearAxis);
      } else {
        mjtNum gearAxis[3];
        *length = 0;
        if (trn == mjhipTRN_JOINT) {
          mju_copy3(gearAxis, gear+3);
        } else {
          mjtNum quat[4];
          mju_copy4(quat, d->qpos+m->jnt_qposadr[id]+3);
          mju_normalize4(quat);
          quat[1] = -quat[1]; quat[2] = -quat[2]; quat[3] = -quat[3];
          mju_rotVecQuat(gearAxis, gear+3, quat);
        }
        mju_copy3(moment, gear);
        mju_copy3(moment+3, gearAxis);
      }
    } else if (trn == mjhipTRN_SLIDERCRANK) {   /* :1000-1052 */
      int idslider = m->actuator_trnid[2*i+1];
      mjtNum rod = m->actuator_cranklength[i];
      mjtNum axis[3] = {d->site_xmat[9*idslider+2], d->site_xmat[9*idslider+5],
                        d->site_xmat[9*idslider+8]};
      mjtNum vec[3], dlda[3], dldv[3];
      mju_sub3(vec, d->site_xpos+3*id, d->site_xpos+3*idslider);
      mjtNum av = mju_dot3(vec, axis);
      mjtNum sdet, det = av*av + rod*rod - mju_dot3(vec, vec);
      int ok = 1;
      if (det <= 0) {
        ok = 0;
        sdet = 0;
        *length = av;
      } else {
        sdet = sqrt(det);
        *length = av - sdet;
      }
      if (ok) {
        mju_scl3(dldv, axis, 1-av/sdet);
        mju_scl3(dlda, vec, 1/sdet);
        mju_addTo3(dldv, dlda);
        mju_scl3(dlda, vec, 1-av/sdet);
      } else {
        mju_copy3(dlda, vec);
        mju_copy3(dldv, axis);
      }
      /* mj_jacPointAxis (engine_support.c:501-521) and mj_jacSite */
      mjtNum* jacS = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mjtNum* jacr = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mjtNum* jacA = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mjtNum* jac = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mj_jac(m, d, jacS, jacr, d->site_xpos+3*idslider, m->site_bodyid[idslider]);
      for (int j = 0; j < nv; j++) {
        jacA[j]      = jacr[nv+j]*axis[2] - jacr[2*nv+j]*axis[1];
        jacA[nv+j]   = jacr[2*nv+j]*axis[0] - jacr[j]*axis[2];
        jacA[2*nv+j] = jacr[j]*axis[1] - jacr[nv+j]*axis[0];
      }
      mj_jac(m, d, jac, NULL, d->site_xpos+3*id, m->site_bodyid[id]);
      for (int j = 0; j < 3*nv; j++) jac[j] -= jacS[j];
      mju_zero(moment, nv);
      for (int j = 0; j < nv; j++) {
        for (int k = 0; k < 3; k++) {
          moment[j] += dlda[k]*jacA[k*nv+j] + dldv[k]*jac[k*nv+j];
        }
      }
      *length *= gear[0];
      for (int j = 0; j < nv; j++) moment[j] *= gear[0];
      /* compress to the structural nonzeros (the reference drops entries that evaluate
       * to exactly 0; the structure here is the two sites' dof chains) */
      for (int k = 0; k < m->moment_rownnz[i]; k++) moment[k] = moment[m->moment_colind[adr+k]];
      free(jacS); free(jacr); free(jacA); free(jac);
    } else if (trn == mjhipTRN_SITE) {   /* :1084-1225 */
      mjtNum wrench[6];
      mjtNum* jac = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mjtNum* jacS = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mj_jac(m, d, jac, jacS, d->site_xpos+3*id, m->site_bodyid[id]);
      *length = 0;
      const int refid = m->actuator_trnid[2*i+1];
      if (refid == -1) {                 /* :1092-1102 gear in the site frame */
        mju_mulMatVec3(wrench, d->site_xmat+9*id, gear);
        mju_mulMatVec3(wrench+3, d->site_xmat+9*id, gear+3);
        mju_mulMatTVec(moment, jac, wrench, 3, nv);
        mju_mulMatTVec(jac, jacS, wrench+3, 3, nv);
        mju_addTo(moment, jac, nv);
      } else {                           /* :1105-1212 relative to the reference site */
        mjtNum* jacref = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
        mjtNum* jtmp = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
        int b0 = m->body_weldid[m->site_bodyid[id]];
        int b1 = m->body_weldid[m->site_bodyid[refid]];
        int dofadr0 = m->body_dofadr[b0] + m->body_dofnum[b0] - 1;
        int dofadr1 = m->body_dofadr[b1] + m->body_dofnum[b1] - 1;
        int common = -1;
        if (dofadr0 >= 0 && dofadr1 >= 0) {
          while (dofadr0 != dofadr1) {
            if (dofadr0 < dofadr1) dofadr1 = m->dof_parentid[dofadr1];
            else dofadr0 = m->dof_parentid[dofadr0];
            if (dofadr0 == -1 || dofadr1 == -1) break;
          }
          if (dofadr0 == dofadr1) common = dofadr0;
        }
        mju_zero(moment, nv);
        if (!mju_isZero(gear, 3)) {      /* translation: site position in the refsite frame */
          mjtNum vec[3];
          mju_sub3(vec, d->site_xpos+3*id, d->site_xpos+3*refid);
          mju_mulMatTVec3(vec, d->site_xmat+9*refid, vec);
          *length += mju_dot3(vec, gear);
          mj_jac(m, d, jacref, jtmp, d->site_xpos+3*refid, m->site_bodyid[refid]);
          mju_subFrom(jac, jacref, 3*nv);
          for (int da = common; da >= 0; da = m->dof_parentid[da]) {
            jac[da] = 0; jac[nv+da] = 0; jac[2*nv+da] = 0;
          }
          mju_mulMatVec3(wrench, d->site_xmat+9*refid, gear);
          mju_mulMatTVec(moment, jac, wrench, 3, nv);
        }
        if (!mju_isZero(gear+3, 3)) {    /* rotation: expmap of the relative orientation */
          mjtNum quat[4], refquat[4], vec[3];
          mju_mulQuat(quat, m->site_quat+4*id, d->xquat+4*m->site_bodyid[id]);
          mju_mulQuat(refquat, m->site_quat+4*refid, d->xquat+4*m->site_bodyid[refid]);
          mju_subQuat(vec, quat, refquat);
          *length += mju_dot3(vec, gear+3);
          mj_jac(m, d, jtmp, jacref, d->site_xpos+3*refid, m->site_bodyid[refid]);
          mju_subFrom(jacS, jacref, 3*nv);
          for (int da = common; da >= 0; da = m->dof_parentid[da]) {
            jacS[da] = 0; jacS[nv+da] = 0; jacS[2*nv+da] = 0;
          }
          mju_mulMatVec3(wrench, d->site_xmat+9*refid, gear+3);
          mju_mulMatTVec(jtmp, jacS, wrench, 3, nv);
          mju_addTo(moment, jtmp, nv);
        }
        free(jacref); free(jtmp);
      }
      for (int k = 0; k < m->moment_rownnz[i]; k++) moment[k] = moment[m->moment_colind[adr+k]];
      free(jac); free(jacS);
    } else if (trn == mjhipTRN_BODY) {   /* :1228-1318 adhesion: the contacts' normals */
      *length = 0;
      mju_zero(moment, nv);
      mjtNum* force = (mjtNum*)calloc(e->nefc ? e->nefc : 1, sizeof(mjtNum));
      mjtNum* mexcl = (mjtNum*)calloc(nv ? nv : 1, sizeof(mjtNum));
      mjtNum* jac1 = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mjtNum* jac2 = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
      mjtNum* jrow = (mjtNum*)malloc(nv*sizeof(mjtNum));
      int counter = 0;
      for (int j = 0; j < e->ncon; j++) {
        int g1 = e->con_geom[2*j], g2 = e->con_geom[2*j+1];
        if (g1 < 0 || g2 < 0) continue;
        int b1 = m->geom_bodyid[g1], b2 = m->geom_bodyid[g2];
        if (b1 != id && b2 != id) continue;
        if (!e->con_exclude[j]) {          /* normal rows get weight in efc_force */
          counter++;
          int dim = e->con_dim[j], adrj = e->con_efc_address[j];
          if (dim == 1 || m->opt.cone == mjhipCONE_ELLIPTIC) {
            force[adrj] = 1;
          } else {
            int npyramid = dim - 1;
            for (int k = 0; k < 2*npyramid; k++) force[adrj + k] = 0.5/npyramid;
          }
        } else if (e->con_exclude[j] == 1) {   /* in the gap: the normal's Jacobian */
          counter++;
          const mjtNum* pos = e->con_pos + 3*j;
          const mjtNum* frame = e->con_frame + 9*j;
          int* chain = (int*)malloc(sizeof(int)*(nv ? nv : 1));
          mjtNum* jacd = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
          int NV = mj_jacDifPair(m, d, chain, b1, b2, pos, pos, jac1, jac2, jacd, NULL, NULL,
                                 NULL);
          mju_zero(jrow, nv);              /* mju_mulMatMat(jac, frame, jacdif, 1, 3, NV) */
          for (int k = 0; k < 3; k++) {
            if (frame[k]) mju_addToScl(jrow, jacd + k*NV, frame[k], NV);
          }
          if (mj_isSparse(m)) {            /* :1304-1307 */
            for (int k = 0; k < NV; k++) mexcl[chain[k]] += jrow[k];
          } else {
            mju_addTo(mexcl, jrow, nv);
          }
          free(chain);
          free(jacd);
        }
      }
      if (counter) {
        or_mulJacTVec(m, e, moment, force);   /* mj_mulJacTVec :426-442 */
        mju_addTo(moment, mexcl, nv);
        mju_scl(moment, moment, -1.0/counter, nv);
      }
      for (int k = 0; k < m->moment_rownnz[i]; k++) moment[k] = moment[m->moment_colind[adr+k]];
      free(force); free(mexcl); free(jac1); free(jac2); free(jrow);
    } else if (mj_isSparse(m)) {   /* mjTRN_TENDON, sparse (:1060-1067): gear*ten_J over
                                       the tendon's row, whose pattern the model's must be */
      *length = d->ten_length[id]*gear[0];
      int nnz = d->ten_J_rownnz[id], tadr = d->ten_J_rowadr[id];
      if (nnz != m->moment_rownnz[i] ||
          memcmp(d->ten_J_colind + tadr, m->moment_colind + adr, nnz*sizeof(int))) {
        d->status |= MJHIP_INST_UNSUPPORTED;   /* a state-dependent pattern (spatial tendon) */
      }
      for (int k = 0; k < m->moment_rownnz[i] && k < nnz; k++) {
        moment[k] = d->ten_J[tadr + k]*gear[0];
      }
    } else {   /* mjTRN_TENDON, dense: gear*ten_J compressed to its nonzeros */
      *length = d->ten_length[id]*gear[0];
      for (int k = 0; k < m->moment_rownnz[i]; k++) {
        moment[k] = d->ten_J[id*nv + m->moment_colind[adr+k]]*gear[0];
      }
    }
  }
}

/* :1353-1401 */
void or_crb(const mjhipModel* m, mjhipData* d) {
  mjtNum buf[6];
  mjtNum* crb = d->crb;
  int last_body = m->nbody - 1, nv = m->nv;
  mju_copy(crb, d->cinert, 10*m->nbody);
  for (int i = last_body; i > 0; i--) {
    if (m->body_parentid[i] > 0) mju_addTo(crb+10*m->body_parentid[i], crb+10*i, 10);
  }
  mju_zero(d->qM, m->nM);
  for (int i = 0; i < nv; i++) {
    if (m->dof_simplenum[i]) {
      int n = i + m->dof_simplenum[i];
      for (; i < n; i++) d->qM[m->dof_Madr[i]] = m->dof_M0[i];
      if (i == nv) break;
    }
    int Madr_ij = m->dof_Madr[i];
    d->qM[Madr_ij] = m->dof_armature[i];
    mju_mulInertVec(buf, crb+10*m->dof_bodyid[i], d->cdof+6*i);
    for (int j = i; j >= 0; j = m->dof_parentid[j]) {
      d->qM[Madr_ij++] += mju_dot(d->cdof+6*j, buf, 6);
    }
  }
}

/* :1483-1511 */
static void mj_factorI(mjtNum* mat, mjtNum* diaginv, int nv, const int* rownnz,
                       const int* rowadr, const int* diagnum, const int* colind) {
  for (int k = nv-1; k >= 0; k--) {
    int rowadr_k = rowadr[k];
    int diag_k = rowadr_k + rownnz[k] - 1;
    mjtNum invD = 1 / mat[diag_k];
    if (diaginv) diaginv[k] = invD;
    if (diagnum[k]) continue;
    for (int adr = diag_k - 1; adr >= rowadr_k; adr--) {
      mjtNum tmp = mat[adr] * invD;
      int i = colind[adr];
      mju_addToScl(mat + rowadr[i], mat + rowadr_k, -tmp, rownnz[i]);
      mat[adr] = tmp;
    }
  }
}

/* :1470-1478 */
void or_factorM(const mjhipModel* m, mjhipData* d) {
  for (int i = 0; i < m->nC; i++) d->qLD[i] = d->qM[m->mapM2C[i]];
  mj_factorI(d->qLD, d->qLDiagInv, m->nv, m->C_rownnz, m->C_rowadr, m->dof_simplenum,
             m->C_colind);
  /* the engine's status word: a pivot D(k) below mjMINVAL, the condition the legacy
   * factorization reports as mjWARN_INERTIA (:1426-1430); no clamping on this path */
  for (int k = 0; k < m->nv; k++) {
    if (!(d->qLD[m->C_rowadr[k] + m->C_rownnz[k] - 1] >= mjMINVAL)) {
      d->status |= MJHIP_INST_INERTIA;
    }
  }
}

/* mju_isBad (engine_util_misc.c:1315-1317) */
static int mju_isBad(mjtNum x) { return x != x || x > mjhipMAXVAL || x < -mjhipMAXVAL; }

/* mj_checkPos/Vel/Acc (engine_forward.c:53-102) as the engine's per-instance status bits:
 * on the inputs a call reads; no reset, no change to any result */
static int or_checkInputs(const mjhipModel* m, const mjhipData* d, int pos, int vel, int acc) {
  int st = 0;
  for (int i = 0; pos && i < m->nq; i++) if (mju_isBad(d->qpos[i])) st |= MJHIP_INST_BADQPOS;
  for (int i = 0; vel && i < m->nv; i++) if (mju_isBad(d->qvel[i])) st |= MJHIP_INST_BADQVEL;
  for (int i = 0; acc && i < m->nv; i++) if (mju_isBad(d->qacc[i])) st |= MJHIP_INST_BADQACC;
  return st;
}

/* :1629-1707 */
static void mj_solveLD(mjtNum* x, const mjtNum* qLDs, const mjtNum* qLDiagInv, int nv, int n,
                       const int* rownnz, const int* rowadr, const int* diagnum,
                       const int* colind) {
  for (int i = nv-1; i > 0; i--) {
    if (diagnum[i]) continue;
    int start = rowadr[i];
    int end = start + rownnz[i] - 1;
    for (int offset = 0; offset < n*nv; offset += nv) {
      mjtNum x_i;
      if ((x_i = x[i+offset])) {
        for (int adr = start; adr < end; adr++) x[offset + colind[adr]] -= qLDs[adr] * x_i;
      }
    }
  }
  for (int i = 0; i < nv; i++) {
    mjtNum invD_i = qLDiagInv[i];
    for (int offset = 0; offset < n*nv; offset += nv) x[i+offset] *= invD_i;
  }
  for (int i = 1; i < nv; i++) {
    if (diagnum[i]) {
      i += diagnum[i] - 1;
      continue;
    }
    int dd;
    if ((dd = rownnz[i] - 1) > 0) {
      int adr = rowadr[i];
      for (int offset = 0; offset < n*nv; offset += nv) {
        x[i+offset] -= mju_dotSparse(qLDs+adr, x+offset, dd, colind+adr);
      }
    }
  }
}

/* :1713-1719 */
void or_solveM(const mjhipModel* m, const mjhipData* d, mjtNum* x, const mjtNum* y, int n) {
  if (x != y) mju_copy(x, y, n*m->nv);
  mj_solveLD(x, d->qLD, d->qLDiagInv, m->nv, n, m->C_rownnz, m->C_rowadr, m->dof_simplenum,
             m->C_colind);
}

/* mj_fullM, engine_support.c (dense symmetric M from qM) */
void or_fullM(const mjhipModel* m, mjtNum* dst, const mjtNum* M) {
  int nv = m->nv, adr = 0;
  mju_zero(dst, nv*nv);
  for (int i = 0; i < nv; i++) {
    int j = i;
    while (j >= 0) {
      dst[i*nv+j] = M[adr];
      dst[j*nv+i] = M[adr];
      j = m->dof_parentid[j];
      adr++;
    }
  }
}

/* :1833-1896 */
static void or_comVel(const mjhipModel* m, mjhipData* d) {
  int nbody = m->nbody;
  mju_zero(d->cvel, 6);
  for (int i = 1; i < nbody; i++) {
    int bda = m->body_dofadr[i];
    mjtNum cvel[6];
    mju_copy(cvel, d->cvel + 6*m->body_parentid[i], 6);
    int dofnum = m->body_dofnum[i];
    mjtNum cdofdot[36];
    for (int j = 0; j < dofnum; j++) {
      mjtNum tmp[6];
      switch (m->jnt_type[m->dof_jntid[bda + j]]) {
      case mjhipJNT_FREE:
        mju_zero(cdofdot, 18);
        mju_mulDofVec(tmp, d->cdof + 6*bda, d->qvel + bda, 3);
        mju_addTo(cvel, tmp, 6);
        j += 3;
        /* fallthrough */
      case mjhipJNT_BALL:
        for (int k = 0; k < 3; k++) {
          mju_crossMotion(cdofdot + 6*(j + k), cvel, d->cdof + 6*(bda + j + k));
        }
        mju_mulDofVec(tmp, d->cdof + 6*(bda + j), d->qvel + bda + j, 3);
        mju_addTo(cvel, tmp, 6);
        j += 2;
        break;
      default:
        mju_crossMotion(cdofdot + 6*j, cvel, d->cdof + 6*(bda + j));
        mju_mulDofVec(tmp, d->cdof + 6*(bda + j), d->qvel + bda + j, 1);
        mju_addTo(cvel, tmp, 6);
      }
    }
    mju_copy(d->cvel + 6*i, cvel, 6);
    if (dofnum) mju_copy(d->cdof_dot + 6*bda, cdofdot, 6*dofnum);
  }
}

/* :1969-2023 */
void or_rne(const mjhipModel* m, mjhipData* d, int flg_acc, mjtNum* result) {
  int nbody = m->nbody, nv = m->nv;
  mjtNum tmp[6], tmp1[6];
  mjtNum* loc_cacc = (mjtNum*)malloc(nbody*6*sizeof(mjtNum));
  mjtNum* loc_cfrc_body = (mjtNum*)malloc(nbody*6*sizeof(mjtNum));
  mju_zero(loc_cacc, 6);
  if (!mjDISABLED(mjhipDSBL_GRAVITY)) mju_scl3(loc_cacc + 3, m->opt.gravity, -1);
  for (int i = 1; i < nbody; i++) {
    int bda = m->body_dofadr[i];
    mju_mulDofVec(tmp, d->cdof_dot + 6*bda, d->qvel + bda, m->body_dofnum[i]);
    mju_add(loc_cacc + 6*i, loc_cacc + 6*m->body_parentid[i], tmp, 6);
    if (flg_acc) {
      mju_mulDofVec(tmp, d->cdof + 6*bda, d->qacc + bda, m->body_dofnum[i]);
      mju_addTo(loc_cacc + 6*i, tmp, 6);
    }
    mju_mulInertVec(loc_cfrc_body + 6*i, d->cinert + 10*i, loc_cacc + 6*i);
    mju_mulInertVec(tmp, d->cinert + 10*i, d->cvel + 6*i);
    mju_crossForce(tmp1, d->cvel + 6*i, tmp);
    mju_addTo(loc_cfrc_body + 6*i, tmp1, 6);
  }
  mju_zero(loc_cfrc_body, 6);
  for (int i = nbody - 1; i > 0; i--) {
    if (m->body_parentid[i]) {
      mju_addTo(loc_cfrc_body + 6*m->body_parentid[i], loc_cfrc_body + 6*i, 6);
    }
  }
  for (int i = 0; i < nv; i++) {
    result[i] = mju_dot(d->cdof + 6*i, loc_cfrc_body + 6*m->dof_bodyid[i], 6);
  }
  free(loc_cacc);
  free(loc_cfrc_body);
}

/*============================ engine_passive.c ============================================*/

/* :57-378 (joint springs, dof dampers, tendon spring-dampers) */
static void or_springdamper(const mjhipModel* m, mjhipData* d) {
  int nv = m->nv, njnt = m->njnt, ntendon = m->ntendon;
  for (int i = 0; i < njnt; i++) {
    mjtNum stiffness = m->jnt_stiffness[i];
    if (stiffness == 0) continue;
    int padr = m->jnt_qposadr[i];
    int dadr = m->jnt_dofadr[i];
    switch (m->jnt_type[i]) {
    case mjhipJNT_FREE:
      d->qfrc_spring[dadr+0] = -stiffness*(d->qpos[padr+0] - m->qpos_spring[padr+0]);
      d->qfrc_spring[dadr+1] = -stiffness*(d->qpos[padr+1] - m->qpos_spring[padr+1]);
      d->qfrc_spring[dadr+2] = -stiffness*(d->qpos[padr+2] - m->qpos_spring[padr+2]);
      dadr += 3;
      padr += 3;
      /* fallthrough */
    case mjhipJNT_BALL:
      {
        mjtNum dif[3], quat[4];
        mju_copy4(quat, d->qpos+padr);
        mju_normalize4(quat);
        mju_subQuat(dif, quat, m->qpos_spring + padr);
        d->qfrc_spring[dadr+0] = -stiffness*dif[0];
        d->qfrc_spring[dadr+1] = -stiffness*dif[1];
        d->qfrc_spring[dadr+2] = -stiffness*dif[2];
      }
      break;
    case mjhipJNT_SLIDE:
    case mjhipJNT_HINGE:
      d->qfrc_spring[dadr] = -stiffness*(d->qpos[padr] - m->qpos_spring[padr]);
      break;
    }
  }
  for (int i = 0; i < nv; i++) {
    mjtNum damping = m->dof_damping[i];
    if (damping != 0) d->qfrc_damper[i] = -damping*d->qvel[i];
  }
  for (int i = 0; i < ntendon; i++) {
    mjtNum stiffness = m->tendon_stiffness[i];
    mjtNum damping = m->tendon_damping[i];
    if (stiffness == 0 && damping == 0) continue;
    mjtNum length = d->ten_length[i];
    mjtNum lower = m->tendon_lengthspring[2*i];
    mjtNum upper = m->tendon_lengthspring[2*i+1];
    mjtNum frc_spring = 0;
    if (length > upper) {
      frc_spring = stiffness * (upper - length);
    } else if (length < lower) {
      frc_spring = stiffness * (lower - length);
    }
    mjtNum frc_damper = -damping * d->ten_velocity[i];
    if (mj_isSparse(m)) {                  /* :361-370 */
      if (frc_spring || frc_damper) {
        int end = d->ten_J_rowadr[i] + d->ten_J_rownnz[i];
        for (int j = d->ten_J_rowadr[i]; j < end; j++) {
          int k = d->ten_J_colind[j];
          mjtNum J = d->ten_J[j];
          d->qfrc_spring[k] += J * frc_spring;
          d->qfrc_damper[k] += J * frc_damper;
        }
      }
    } else {
      if (frc_spring) mju_addToScl(d->qfrc_spring, d->ten_J+i*nv, frc_spring, nv);
      if (frc_damper) mju_addToScl(d->qfrc_damper, d->ten_J+i*nv, frc_damper, nv);
    }
  }
}

/* :381-399 */
static int or_gravcomp(const mjhipModel* m, mjhipData* d) {
  if (!m->ngravcomp || mjDISABLED(mjhipDSBL_GRAVITY) ||
      sqrt(m->opt.gravity[0]*m->opt.gravity[0] + m->opt.gravity[1]*m->opt.gravity[1] +
           m->opt.gravity[2]*m->opt.gravity[2]) == 0) {
    return 0;
  }
  int has_gravcomp = 0;
  mjtNum force[3], torque[3] = {0};
  for (int i = 1; i < m->nbody; i++) {
    if (m->body_gravcomp[i]) {
      has_gravcomp = 1;
      mju_scl3(force, m->opt.gravity, -(m->body_mass[i]*m->body_gravcomp[i]));
      mj_applyFT(m, d, force, torque, d->xipos+3*i, i, d->qfrc_gravcomp);
    }
  }
  return has_gravcomp;
}

static int or_fluid(const mjhipModel* m, mjhipData* d);

/* :436-493 */
static void or_passive(const mjhipModel* m, mjhipData* d) {
  int nv = m->nv;
  mju_zero(d->qfrc_spring, nv);
  mju_zero(d->qfrc_damper, nv);
  mju_zero(d->qfrc_gravcomp, nv);
  mju_zero(d->qfrc_fluid, nv);
  mju_zero(d->qfrc_passive, nv);
  if (mjDISABLED(mjhipDSBL_PASSIVE)) return;
  or_springdamper(m, d);
  int has_gravcomp = or_gravcomp(m, d);
  int has_fluid = or_fluid(m, d);
  mju_add(d->qfrc_passive, d->qfrc_spring, d->qfrc_damper, nv);
  if (has_fluid) mju_addTo(d->qfrc_passive, d->qfrc_fluid, nv);
  if (has_gravcomp) {
    for (int i = 0; i < m->njnt; i++) {
      if (m->jnt_actgravcomp[i]) continue;
      int dofnum = m->jnt_type[i] == mjhipJNT_FREE ? 6 : (m->jnt_type[i] == mjhipJNT_BALL ? 3 : 1);
      int dofadr = m->jnt_dofadr[i];
      for (int j = 0; j < dofnum; j++) d->qfrc_passive[dofadr+j] += d->qfrc_gravcomp[dofadr+j];
    }
  }
}

/*============================ engine_core_constraint.c ====================================*/



/*============================ engine_collision_*.c =========================================*/

static mjtNum mju_dot3(const mjtNum* a, const mjtNum* b) { return a[0]*b[0] + a[1]*b[1] + a[2]*b[2]; }
static mjtNum mju_norm3(const mjtNum* a) { return sqrt(a[0]*a[0] + a[1]*a[1] + a[2]*a[2]); }
static mjtNum mju_clip(mjtNum x, mjtNum lo, mjtNum hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* one narrowphase result before the contact parameters are attached */
typedef struct { mjtNum dist, pos[3], frame[9]; } orRaw;

/* engine_collision_primitive.c:95-195 mjc_PlaneCylinder */
static int col_planeCylinder(orRaw* con, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                             const mjtNum* pos2, const mjtNum* mat2, const mjtNum* size2) {
  mjtNum normal[3] = {mat1[2], mat1[5], mat1[8]};
  mjtNum axis[3] = {mat2[2], mat2[5], mat2[8]};
  mjtNum prjaxis = mju_dot3(normal, axis);
  if (prjaxis > 0) {
    mju_scl3(axis, axis, -1);
    prjaxis = -prjaxis;
  }
  mjtNum vec[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  mjtNum dist0 = mju_dot3(vec, normal);
  mju_scl3(vec, axis, prjaxis);
  vec[0] -= normal[0]; vec[1] -= normal[1]; vec[2] -= normal[2];
  mjtNum len_sqr = mju_dot3(vec, vec);
  if (len_sqr >= mjMINVAL*mjMINVAL) {
    mjtNum scl = size2[0]/sqrt(len_sqr);
    vec[0] *= scl; vec[1] *= scl; vec[2] *= scl;
  } else {
    vec[0] = mat2[0]*size2[0];
    vec[1] = mat2[3]*size2[0];
    vec[2] = mat2[6]*size2[0];
  }
  mjtNum prjvec = mju_dot3(vec, normal);
  mju_scl3(axis, axis, size2[1]);
  prjaxis *= size2[1];
  int cnt = 0;
  if (dist0 + prjaxis + prjvec <= margin) {
    con[cnt].dist = dist0 + prjaxis + prjvec;
    mju_add3(con[cnt].pos, pos2, vec);
    mju_addTo3(con[cnt].pos, axis);
    mju_addToScl3(con[cnt].pos, normal, -con[cnt].dist*0.5);
    mju_copy3(con[cnt].frame, normal);
    mju_zero3(con[cnt].frame+3);
    cnt++;
  } else {
    return 0;
  }
  if (dist0 - prjaxis + prjvec <= margin) {
    con[cnt].dist = dist0 - prjaxis + prjvec;
    mju_add3(con[cnt].pos, pos2, vec);
    con[cnt].pos[0] -= axis[0]; con[cnt].pos[1] -= axis[1]; con[cnt].pos[2] -= axis[2];
    mju_addToScl3(con[cnt].pos, normal, -con[cnt].dist*0.5);
    mju_copy3(con[cnt].frame, normal);
    mju_zero3(con[cnt].frame+3);
    cnt++;
  }
  mjtNum prjvec1 = -prjvec*0.5;
  if (dist0 + prjaxis + prjvec1 <= margin) {
    mjtNum vec1[3];
    mju_cross(vec1, vec, axis);
    mju_normalize3(vec1);
    mju_scl3(vec1, vec1, size2[0]*sqrt(3.0)/2);
    con[cnt].dist = dist0 + prjaxis + prjvec1;
    mju_add3(con[cnt].pos, pos2, vec1);
    mju_addTo3(con[cnt].pos, axis);
    mju_addToScl3(con[cnt].pos, vec, -0.5);
    mju_addToScl3(con[cnt].pos, normal, -con[cnt].dist*0.5);
    mju_copy3(con[cnt].frame, normal);
    mju_zero3(con[cnt].frame+3);
    cnt++;
    con[cnt].dist = dist0 + prjaxis + prjvec1;
    mju_sub3(con[cnt].pos, pos2, vec1);
    mju_addTo3(con[cnt].pos, axis);
    mju_addToScl3(con[cnt].pos, vec, -0.5);
    mju_addToScl3(con[cnt].pos, normal, -con[cnt].dist*0.5);
    mju_copy3(con[cnt].frame, normal);
    mju_zero3(con[cnt].frame+3);
    cnt++;
  }
  return cnt;
}

/* engine_collision_primitive.c:200-243 mjc_PlaneBox */
static int col_planeBox(orRaw* con, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                        const mjtNum* pos2, const mjtNum* mat2, const mjtNum* size2) {
  mjtNum norm[3] = {mat1[2], mat1[5], mat1[8]};
  mjtNum dif[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  mjtNum dist = mju_dot3(dif, norm);
  int cnt = 0;
  for (int i = 0; i < 8; i++) {
    mjtNum vec[3];
    vec[0] = (i&1 ? size2[0] : -size2[0]);
    vec[1] = (i&2 ? size2[1] : -size2[1]);
    vec[2] = (i&4 ? size2[2] : -size2[2]);
    mjtNum corner[3];
    mju_mulMatVec3(corner, mat2, vec);
    mjtNum ldist = mju_dot3(norm, corner);
    if (dist + ldist > margin || ldist > 0) continue;
    con[cnt].dist = dist + ldist;
    mju_copy3(con[cnt].frame, norm);
    mju_zero3(con[cnt].frame+3);
    mju_addTo3(corner, pos2);
    mju_scl3(vec, norm, -con[cnt].dist/2);
    mju_add3(con[cnt].pos, corner, vec);
    if (++cnt >= 4) return 4;
  }
  return cnt;
}

/* engine_collision_primitive.c mjraw_PlaneSphere */
static int raw_planeSphere(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                           const mjtNum* pos2, mjtNum r2) {
  c->frame[0] = mat1[2];
  c->frame[1] = mat1[5];
  c->frame[2] = mat1[8];
  mjtNum tmp[3] = {pos2[0] - pos1[0], pos2[1] - pos1[1], pos2[2] - pos1[2]};
  mjtNum cdist = mju_dot3(tmp, c->frame);
  if (cdist > margin + r2) return 0;
  c->dist = cdist - r2;
  mju_scl3(tmp, c->frame, -c->dist/2 - r2);
  mju_add3(c->pos, pos2, tmp);
  mju_zero3(c->frame + 3);
  return 1;
}

/* mjc_PlaneCapsule */
static int col_planeCapsule(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                            const mjtNum* pos2, const mjtNum* mat2, const mjtNum* size2) {
  mjtNum axis[3] = {mat2[2], mat2[5], mat2[8]};
  mjtNum seg[3] = {size2[1]*axis[0], size2[1]*axis[1], size2[1]*axis[2]};
  mjtNum p[3];
  mju_add3(p, pos2, seg);
  int n1 = raw_planeSphere(c, margin, pos1, mat1, p, size2[0]);
  mju_sub3(p, pos2, seg);
  int n2 = raw_planeSphere(c + n1, margin, pos1, mat1, p, size2[0]);
  if (n1) mju_copy3(c->frame + 3, axis);
  if (n2) mju_copy3((c + n1)->frame + 3, axis);
  return n1 + n2;
}

/* mjraw_SphereSphere */
static void mju_mulMatTVec3(mjtNum res[3], const mjtNum mat[9], const mjtNum vec[3]);

/* engine_collision_box.c:21-92 mju_clampVec + mjraw_SphereBox */
static int raw_sphereBox(orRaw* c, mjtNum margin, const mjtNum* pos1, mjtNum r1,
                         const mjtNum* pos2, const mjtNum* mat2, const mjtNum* size2) {
  mjtNum tmp[3], center[3], clamped[3], deepest[3], pos[3], dist, closest;
  int k = 0;
  mju_sub3(tmp, pos1, pos2);
  mju_mulMatTVec3(center, mat2, tmp);
  mju_copy3(clamped, center);
  for (int i = 0; i < 3; i++) {
    if (size2[i] > 0) {
      if (clamped[i] < -size2[i]) clamped[i] = -size2[i];
      else if (clamped[i] > size2[i]) clamped[i] = size2[i];
    }
  }
  mju_copy3(deepest, center);
  mju_sub3(tmp, clamped, center);
  dist = mju_normalize3(tmp);
  if (dist - r1 > margin) return 0;
  if (dist <= mjMINVAL) {
    closest = (size2[0] + size2[1] + size2[2]) * 2;
    for (int i = 0; i < 6; i++) {
      if (closest > fabs((i % 2 ? 1 : -1)*size2[i/2] - center[i/2])) {
        closest = fabs((i % 2 ? 1 : -1)*size2[i/2] - center[i/2]);
        k = i;
      }
    }
    mjtNum nearest[3] = {0, 0, 0};
    nearest[k/2] = (k % 2 ? -1 : 1);
    mju_copy3(pos, center);
    mju_addToScl3(pos, nearest, (r1 - closest) / 2);
    mju_mulMatVec3(c->frame, mat2, nearest);
    dist = -closest;
  } else {
    mju_addToScl3(deepest, tmp, r1);
    mju_zero3(pos);
    mju_addToScl3(pos, clamped, 0.5);
    mju_addToScl3(pos, deepest, 0.5);
    mju_mulMatVec3(c->frame, mat2, tmp);
  }
  mju_mulMatVec3(tmp, mat2, pos);
  mju_add3(c->pos, tmp, pos2);
  c->dist = dist - r1;
  mju_zero3(c->frame + 3);
  return 1;
}

static int raw_sphereSphere(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                            mjtNum r1, const mjtNum* pos2, const mjtNum* mat2, mjtNum r2) {
  mjtNum dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  mjtNum cdist_sqr = mju_dot3(dif, dif);
  mjtNum min_dist = margin + r1 + r2;
  if (cdist_sqr > min_dist*min_dist) return 0;
  c->dist = sqrt(cdist_sqr) - r1 - r2;
  mju_sub3(c->frame, pos2, pos1);
  mjtNum len = mju_normalize3(c->frame);
  if (len < mjMINVAL) {
    mjtNum a1[3] = {mat1[2], mat1[5], mat1[8]}, a2[3] = {mat2[2], mat2[5], mat2[8]};
    mju_cross(c->frame, a1, a2);
    mju_normalize3(c->frame);
  }
  mju_scl3(c->pos, c->frame, r1 + c->dist/2);
  mju_addTo3(c->pos, pos1);
  mju_zero3(c->frame + 3);
  return 1;
}

/* mjraw_SphereCapsule */
static int col_sphereCapsule(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                             mjtNum r1, const mjtNum* pos2, const mjtNum* mat2,
                             const mjtNum* size2) {
  mjtNum len = size2[1];
  mjtNum axis[3] = {mat2[2], mat2[5], mat2[8]};
  mjtNum vec[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  mjtNum x = mju_clip(mju_dot3(axis, vec), -len, len);
  mju_scl3(vec, axis, x);
  mju_addTo3(vec, pos2);
  return raw_sphereSphere(c, margin, pos1, mat1, r1, vec, mat2, size2[0]);
}

/* mju_addScl3 (engine_util_blas.c): res = vec1 + scl*vec2 */
static void mju_addScl3(mjtNum res[3], const mjtNum vec1[3], const mjtNum vec2[3], mjtNum scl) {
  res[0] = vec1[0] + scl*vec2[0];
  res[1] = vec1[1] + scl*vec2[1];
  res[2] = vec1[2] + scl*vec2[2];
}

/* mjc_SphereCylinder (engine_collision_primitive.c:323-391): side (sphere-sphere with the
 * axis point), cap (plane-sphere on the cap plane, normal flipped) or rim corner (sphere-
 * sphere with a point sphere at the corner) */
static int col_sphereCylinder(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                              mjtNum r1, const mjtNum* pos2, const mjtNum* mat2,
                              const mjtNum* size2) {
  mjtNum radius = size2[0], height = size2[1];
  mjtNum axis[3] = {mat2[2], mat2[5], mat2[8]};
  mjtNum vec[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  mjtNum x = mju_dot3(axis, vec);
  mjtNum a_proj[3], p_proj[3];
  mju_scl3(a_proj, axis, x);
  mju_sub3(p_proj, vec, a_proj);
  mjtNum p_proj_sqr = mju_dot3(p_proj, p_proj);
  int collide_side = fabs(x) < height;
  int collide_cap = p_proj_sqr < radius*radius;
  if (collide_side && collide_cap) {
    mjtNum dist_cap = height - fabs(x);
    mjtNum dist_radius = radius - sqrt(p_proj_sqr);
    if (dist_cap < dist_radius) {
      collide_side = 0;
    } else {
      collide_cap = 0;
    }
  }
  if (collide_side) {
    mju_addTo3(a_proj, pos2);
    return raw_sphereSphere(c, margin, pos1, mat1, r1, a_proj, mat2, size2[0]);
  }
  if (collide_cap) {
    const mjtNum flipmat[9] = {-mat2[0], mat2[1], -mat2[2], -mat2[3], mat2[4], -mat2[5],
                               -mat2[6], mat2[7], -mat2[8]};
    const mjtNum* mat_cap;
    mjtNum pos_cap[3];
    if (x > 0) {
      mju_addScl3(pos_cap, pos2, axis, height);
      mat_cap = mat2;
    } else {
      mju_addScl3(pos_cap, pos2, axis, -height);
      mat_cap = flipmat;
    }
    int ncon = raw_planeSphere(c, margin, pos_cap, mat_cap, pos1, r1);
    if (ncon) mju_scl3(c->frame, c->frame, -1);
    return ncon;
  }
  mju_scl3(p_proj, p_proj, size2[0] / sqrt(p_proj_sqr));
  mju_scl3(vec, axis, x > 0 ? height : -height);
  mju_addTo3(vec, p_proj);
  mju_addTo3(vec, pos2);
  return raw_sphereSphere(c, margin, pos1, mat1, r1, vec, mat2, 0);
}

/* mjraw_CapsuleBox (engine_collision_box.c:121-594): the box feature closest to the capsule
 * segment (an end point against a face, or the segment against one of the 12 edges, in the
 * box frame), the second point along the segment that can still touch the box, then one
 * sphere-box contact of the capsule's radius at each point (at most 2). The reference's
 * j == 2 block inside the edge loop computes nothing that is used later; it is omitted. */
static int col_capsuleBox(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                          const mjtNum* size1, const mjtNum* pos2, const mjtNum* mat2,
                          const mjtNum* size2) {
  mjtNum tmp[3], pos[3], axis[3], halfaxis[3];
  const mjtNum hl = size1[1];
  mju_sub3(tmp, pos1, pos2);
  mju_mulMatTVec3(pos, mat2, tmp);
  const mjtNum a1[3] = {mat1[2], mat1[5], mat1[8]};
  mju_mulMatTVec3(axis, mat2, a1);
  mju_scl3(halfaxis, axis, hl);
  const int axisdir = (halfaxis[0] > 0) + 2*(halfaxis[1] > 0) + 4*(halfaxis[2] > 0);
  mjtNum bestdist = margin + 2*(size1[0] + hl + size2[0] + size2[1] + size2[2]);
  mjtNum bestseg = 0, bestbox = 0, secondpos = -4;
  int cltype = -4, clface = -1, clcorner = 0, cledge = 0;

  /* a segment end against a face: the end clamped onto the box along at most one axis */
  for (int e = -1; e <= 1; e += 2) {
    mjtNum p[3], q[3];
    int nclamp = 0, face = -1;
    for (int k = 0; k < 3; k++) {
      p[k] = pos[k] + halfaxis[k]*e;
      q[k] = p[k];
      if (p[k] < -size2[k]) {
        nclamp++;
        face = k;
        p[k] = -size2[k];
      } else if (p[k] > size2[k]) {
        nclamp++;
        face = k;
        p[k] = size2[k];
      }
    }
    if (nclamp > 1) continue;
    for (int k = 0; k < 3; k++) p[k] -= q[k];
    const mjtNum dist = mju_dot3(p, p);
    if (dist < bestdist) {
      bestdist = dist;
      bestseg = e;
      cltype = -2 + e;
      clface = face;
    }
  }

  /* the segment against each edge: closest points of two segments, clamped */
  for (int j = 0; j < 3; j++) {
    for (int i = 0; i < 8; i++) {
      if (i & (1 << j)) continue;
      mjtNum corner[3] = {((i & 1) ? 1 : -1)*size2[0], ((i & 2) ? 1 : -1)*size2[1],
                          ((i & 4) ? 1 : -1)*size2[2]};
      corner[j] = 0;
      mjtNum dif[3];
      mju_sub3(dif, corner, pos);
      const mjtNum ma = size2[j]*size2[j], mb = -size2[j]*halfaxis[j], mc = size1[1]*size1[1];
      const mjtNum u = -size2[j]*dif[j], v = mju_dot3(halfaxis, dif);
      const mjtNum det = ma*mc - mb*mb;
      if (fabs(det) < mjMINVAL) continue;
      const mjtNum idet = 1/det;
      mjtNum x1 = (mc*u - mb*v)*idet, x2 = (ma*v - mb*u)*idet;
      int s1 = 1, s2 = 1;
      if (x1 > 1) {
        x1 = 1;
        s1 = 2;
        x2 = (v - mb)*(1/mc);
      } else if (x1 < -1) {
        x1 = -1;
        s1 = 0;
        x2 = (v + mb)*(1/mc);
      }
      if (x2 > 1 || x2 < -1) {
        const int hi = x2 > 1;
        x2 = hi ? 1 : -1;
        s2 = hi ? 2 : 0;
        x1 = (hi ? u - mb : u + mb)*(1/ma);
        if (x1 > 1) {
          x1 = 1;
          s1 = 2;
        } else if (x1 < -1) {
          x1 = -1;
          s1 = 0;
        }
      }
      mju_sub3(dif, corner, pos);
      mju_addToScl3(dif, halfaxis, -x2);
      dif[j] += size2[j]*x1;
      const mjtNum d2 = mju_dot3(dif, dif);
      const int t = s1*3 + s2;
      if (d2 < bestdist - mjMINVAL) {
        bestdist = d2;
        bestseg = x2;
        bestbox = x1;
        clcorner = i + (1 << j)*(t / 6);
        cledge = j;
        cltype = t;
      }
    }
  }
  if (cltype == -4) return 0;

  /* the second point along the segment (:392-559) */
  mjtNum mul = 0, e1, e2;
  if (cltype >= 0 && cltype / 3 != 1) {           /* a box corner is closest */
    int c1 = axisdir ^ clcorner, ax = 0, ax1 = 0, ax2 = 0;
    if (c1 != 0 && c1 != 7) {                     /* not pointing at or away from it */
      mjtNum de, dp;
      if (c1 == 1 || c1 == 2 || c1 == 4) {
        mul = 1;
        de = 1 - bestseg;
        dp = 1 + bestseg;
      } else {
        mul = -1;
        c1 = 7 - c1;
        dp = 1 - bestseg;
        de = 1 + bestseg;
      }
      if (c1 == 1) { ax = 0; ax1 = 1; ax2 = 2; }
      if (c1 == 2) { ax = 1; ax1 = 2; ax2 = 0; }
      if (c1 == 4) { ax = 2; ax1 = 0; ax2 = 1; }
      if (axis[ax]*axis[ax] > 0.5) {              /* along the box edge */
        secondpos = de;
        e1 = 2*size2[ax]/fabs(halfaxis[ax]);
        if (e1 < secondpos) secondpos = e1;
        secondpos *= mul;
      } else {                                    /* along a box face */
        secondpos = dp;
        e1 = 2*size2[ax1]/fabs(halfaxis[ax1]);
        if (e1 < secondpos) secondpos = e1;
        e1 = 2*size2[ax2]/fabs(halfaxis[ax2]);
        if (e1 < secondpos) secondpos = e1;
        secondpos *= -mul;
      }
    }
  } else if (cltype >= 0) {                       /* the middle of a box edge is closest */
    const int c1 = (axisdir ^ clcorner) & (7 - (1 << cledge));
    if (c1 == 1 || c1 == 2 || c1 == 4) {         /* crossing the edge, not a T */
      int ax = cledge, ax1 = (cledge + 1) % 3, ax2 = (cledge + 2) % 3;
      if (fabs(axis[ax1]) > fabs(axis[ax2])) ax1 = ax2;
      ax2 = 3 - ax - ax1;
      if (c1 & (1 << ax2)) {
        mul = 1;
        secondpos = 1 - bestseg;
      } else {
        mul = -1;
        secondpos = 1 + bestseg;
      }
      e1 = 2*size2[ax2]/fabs(halfaxis[ax2]);
      if (e1 < secondpos) secondpos = e1;
      e2 = (((axisdir & (1 << ax)) != 0) == ((c1 & (1 << ax2)) != 0)) ? 1 - bestbox : 1 + bestbox;
      e1 = size2[ax]*e2/fabs(halfaxis[ax]);
      if (e1 < secondpos) secondpos = e1;
      secondpos *= mul;
    }
  } else if (clface != -1) {                      /* an end against a face, outside the box */
    mul = cltype == -3 ? 1 : -1;
    secondpos = 2;
    mjtNum p[3];
    for (int k = 0; k < 3; k++) p[k] = pos[k] + halfaxis[k]*-mul;
    for (int k = 0; k < 3; k++) {
      if (k == clface) continue;
      e1 = (size2[k] - p[k]) / halfaxis[k] * mul;
      if (e1 > 0 && e1 < secondpos) secondpos = e1;
      e1 = (-size2[k] - p[k]) / halfaxis[k] * mul;
      if (e1 > 0 && e1 < secondpos) secondpos = e1;
    }
    secondpos *= mul;
  }

  /* spheres of the capsule's radius at the two points, collided with the box */
  mjtNum sp[3], w[3];
  for (int k = 0; k < 3; k++) sp[k] = pos[k] + halfaxis[k]*bestseg;
  mju_mulMatVec3(w, mat2, sp);
  mju_addTo3(w, pos2);
  int n = raw_sphereBox(c, margin, w, size1[0], pos2, mat2, size2);
  if (secondpos > -3) {
    for (int k = 0; k < 3; k++) sp[k] = pos[k] + halfaxis[k]*(secondpos + bestseg);
    mju_mulMatVec3(w, mat2, sp);
    mju_addTo3(w, pos2);
    n += raw_sphereBox(c + n, margin, w, size1[0], pos2, mat2, size2);
  }
  return n;
}

/* mjraw_CapsuleCapsule */
static int col_capsuleCapsule(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                              const mjtNum* size1, const mjtNum* pos2, const mjtNum* mat2,
                              const mjtNum* size2) {
  mjtNum axis1[3] = {mat1[2]*size1[1], mat1[5]*size1[1], mat1[8]*size1[1]};
  mjtNum axis2[3] = {mat2[2]*size2[1], mat2[5]*size2[1], mat2[8]*size2[1]};
  mjtNum dif[3] = {pos1[0] - pos2[0], pos1[1] - pos2[1], pos1[2] - pos2[2]};
  mjtNum ma = mju_dot3(axis1, axis1);
  mjtNum mb = -mju_dot3(axis1, axis2);
  mjtNum mc = mju_dot3(axis2, axis2);
  mjtNum u = -mju_dot3(axis1, dif);
  mjtNum v = mju_dot3(axis2, dif);
  mjtNum det = ma*mc - mb*mb;
  mjtNum vec1[3], vec2[3];
  if (fabs(det) >= mjMINVAL) {
    mjtNum x1 = (mc*u - mb*v) / det;
    mjtNum x2 = (ma*v - mb*u) / det;
    if (x1 > 1) {
      x1 = 1;
      x2 = (v - mb) / mc;
    } else if (x1 < -1) {
      x1 = -1;
      x2 = (v + mb) / mc;
    }
    if (x2 > 1) {
      x2 = 1;
      x1 = mju_clip((u - mb) / ma, -1, 1);
    } else if (x2 < -1) {
      x2 = -1;
      x1 = mju_clip((u + mb) / ma, -1, 1);
    }
    mju_scl3(vec1, axis1, x1);
    mju_addTo3(vec1, pos1);
    mju_scl3(vec2, axis2, x2);
    mju_addTo3(vec2, pos2);
    return raw_sphereSphere(c, margin, vec1, mat1, size1[0], vec2, mat2, size2[0]);
  }
  /* parallel axes: up to two contacts from the four segment ends */
  mju_add3(vec1, pos1, axis1);
  mjtNum x2 = mju_clip((v - mb) / mc, -1, 1);
  mju_scl3(vec2, axis2, x2);
  mju_addTo3(vec2, pos2);
  int n1 = raw_sphereSphere(c, margin, vec1, mat1, size1[0], vec2, mat2, size2[0]);
  mju_sub3(vec1, pos1, axis1);
  x2 = mju_clip((v + mb) / mc, -1, 1);
  mju_scl3(vec2, axis2, x2);
  mju_addTo3(vec2, pos2);
  int n2 = raw_sphereSphere(c + n1, margin, vec1, mat1, size1[0], vec2, mat2, size2[0]);
  if (n1 + n2 >= 2) return n1 + n2;
  mju_add3(vec2, pos2, axis2);
  mjtNum x1 = mju_clip((u - mb) / ma, -1, 1);
  mju_scl3(vec1, axis1, x1);
  mju_addTo3(vec1, pos1);
  int n3 = raw_sphereSphere(c + n1 + n2, margin, vec1, mat1, size1[0], vec2, mat2, size2[0]);
  if (n1 + n2 + n3 >= 2) return n1 + n2 + n3;
  mju_sub3(vec2, pos2, axis2);
  x1 = mju_clip((u + mb) / ma, -1, 1);
  mju_scl3(vec1, axis1, x1);
  mju_addTo3(vec1, pos1);
  int n4 = raw_sphereSphere(c + n1 + n2 + n3, margin, vec1, mat1, size1[0], vec2, mat2,
                            size2[0]);
  return n1 + n2 + n3 + n4;
}

/* engine_util_spatial.c mju_makeFrame (xaxis given, yaxis optional) */
static void mju_makeFrame(mjtNum* frame) {
  mjtNum tmp[3];
  mju_normalize3(frame);
  if (mju_norm3(frame + 3) < 0.5) {
    mju_zero3(frame + 3);
    if (frame[1] < 0.5 && frame[1] > -0.5) frame[4] = 1;
    else frame[5] = 1;
  }
  mju_scl3(tmp, frame, mju_dot3(frame, frame + 3));
  mju_sub3(frame + 3, frame + 3, tmp);
  mju_normalize3(frame + 3);
  mju_cross(frame + 6, frame, frame + 3);
}

/* engine_collision_driver.c mj_contactParam (geom : geom) */
static void or_contactParam(const mjhipModel* m, int g1, int g2, int* condim, mjtNum* gap,
                            mjtNum* solref, mjtNum* solimp, mjtNum* friction) {
  mjtNum fri[3];
  int p1 = m->geom_priority[g1], p2 = m->geom_priority[g2];
  *gap = mjMAX(m->geom_gap[g1], m->geom_gap[g2]);
  if (p1 != p2) {
    int g = p1 > p2 ? g1 : g2;
    *condim = m->geom_condim[g];
    mju_copy(solref, m->geom_solref + 2*g, 2);
    mju_copy(solimp, m->geom_solimp + 5*g, 5);
    mju_copy(fri, m->geom_friction + 3*g, 3);
  } else {
    *condim = mjMAX(m->geom_condim[g1], m->geom_condim[g2]);
    mjtNum s1 = m->geom_solmix[g1], s2 = m->geom_solmix[g2], mix;
    if (s1 >= mjMINVAL && s2 >= mjMINVAL) mix = s1 / (s1 + s2);
    else if (s1 < mjMINVAL && s2 < mjMINVAL) mix = 0.5;
    else if (s1 < mjMINVAL) mix = 0.0;
    else mix = 1.0;
    const mjtNum *r1 = m->geom_solref + 2*g1, *r2 = m->geom_solref + 2*g2;
    if (r1[0] > 0 && r2[0] > 0) {
      for (int i = 0; i < 2; i++) solref[i] = mix*r1[i] + (1-mix)*r2[i];
    } else {
      for (int i = 0; i < 2; i++) solref[i] = mjMIN(r1[i], r2[i]);
    }
    for (int i = 0; i < 5; i++) {
      solimp[i] = mix*m->geom_solimp[5*g1+i] + (1-mix)*m->geom_solimp[5*g2+i];
    }
    for (int i = 0; i < 3; i++) {
      fri[i] = mjMAX(m->geom_friction[3*g1+i], m->geom_friction[3*g2+i]);
    }
  }
  friction[0] = fri[0];
  friction[1] = fri[0];
  friction[2] = fri[1];
  friction[3] = fri[2];
  friction[4] = fri[2];
}

/* mj_filterSphere: 1 = the bounding spheres (or plane distance) rule the pair out */
static int or_filterSphere(const mjhipModel* m, const mjhipData* d, int g1, int g2,
                           mjtNum margin) {
  const mjtNum *p1 = d->geom_xpos + 3*g1, *p2 = d->geom_xpos + 3*g2;
  mjtNum rb1 = m->geom_rbound[g1], rb2 = m->geom_rbound[g2];
  if (rb1 > 0 && rb2 > 0) {
    mjtNum dif[3] = {p1[0]-p2[0], p1[1]-p2[1], p1[2]-p2[2]};
    mjtNum bound = rb1 + rb2 + margin;
    return dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2] > bound*bound;
  }
  for (int side = 0; side < 2; side++) {
    int gp = side ? g2 : g1, go = side ? g1 : g2;
    if (m->geom_type[gp] == mjhipGEOM_PLANE && m->geom_rbound[go] > 0) {
      const mjtNum* mat = d->geom_xmat + 9*gp;
      mjtNum norm[3] = {mat[2], mat[5], mat[8]}, dif[3];
      mju_sub3(dif, d->geom_xpos + 3*go, d->geom_xpos + 3*gp);
      if (mju_dot3(dif, norm) > margin + m->geom_rbound[go]) return 1;
    }
  }
  return 0;
}

/*---------------- collision driver rules (engine_collision_driver.c), restated here ----------
 * The oracle keeps its own copy of the driver's static rules and of its broadphase (sweep and
 * prune in the covariance frame) so that the HIP engine's candidate-pair program
 * (include/mjhip_contact.h: every statically admissible body pair, brute force) is checked
 * against the reference's algorithm, not against itself. */

/* filterBitmask :101-105 */
static int or_filterBitmask(int contype1, int conaffinity1, int contype2, int conaffinity2) {
  return !(contype1 & conaffinity2) && !(contype2 & conaffinity1);
}

/* filterBodyPair :165-182 */
static int or_filterBodyPair(int weldbody1, int weldparent1, int weldbody2, int weldparent2,
                             int dsbl_filterparent) {
  if (weldbody1 == weldbody2) return 1;
  if ((!dsbl_filterparent && weldbody1 != 0 && weldbody2 != 0) &&
      (weldbody1 == weldparent2 || weldbody2 == weldparent1)) {
    return 1;
  }
  return 0;
}

/* canCollide :187-195 and canCollide2 :200-210 (bodies only: flex is outside the subset) */
static int or_canCollide(const mjhipModel* m, int b) {
  return m->body_contype[b] || m->body_conaffinity[b];
}

static int or_canCollide2(const mjhipModel* m, int b1, int b2) {
  return !or_filterBitmask(m->body_contype[b1], m->body_conaffinity[b1], m->body_contype[b2],
                           m->body_conaffinity[b2]);
}

/* hasPlane :84-97 */
static int or_hasPlane(const mjhipModel* m, int b) {
  for (int g = m->body_geomadr[b]; g < m->body_geomadr[b] + m->body_geomnum[b]; g++) {
    if (m->geom_type[g] == mjhipGEOM_PLANE) return 1;
  }
  return 0;
}

/* ---- mjc_BoxBox (engine_collision_box.c:607-1343) ---- */
static void bb_mulMatTMat3(mjtNum r[9], const mjtNum a[9], const mjtNum b[9]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[3*i+j] = a[i]*b[j] + a[3+i]*b[3+j] + a[6+i]*b[6+j];
}
static void bb_mulMatMatT3(mjtNum r[9], const mjtNum a[9], const mjtNum b[9]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[3*i+j] = a[3*i]*b[3*j] + a[3*i+1]*b[3*j+1] + a[3*i+2]*b[3*j+2];
}
static void bb_transpose3(mjtNum r[9], const mjtNum a[9]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[3*j+i] = a[3*i+j];
}

/* the axis permutation and signs that turn face `f` (0-2: -x,-y,-z side... as the reference
 * numbers them, 3-5 the opposite) into +z: rotmore and its (index, sign) form */
static void bb_faceFrame(int f, mjtNum rotmore[9], int idx[3], mjtNum sgn[3]) {
  mju_zero(rotmore, 9);
  idx[0] = 0; idx[1] = 1; idx[2] = 2;
  sgn[0] = sgn[1] = sgn[2] = 1;
  switch (f) {
  case 0: rotmore[2] = -1; rotmore[4] = 1; rotmore[6] = 1; idx[0] = 2; sgn[0] = -1; idx[2] = 0; break;
  case 1: rotmore[0] = 1; rotmore[5] = -1; rotmore[7] = 1; idx[1] = 2; sgn[1] = -1; idx[2] = 1; break;
  case 2: rotmore[0] = 1; rotmore[4] = 1; rotmore[8] = 1; break;
  case 3: rotmore[2] = 1; rotmore[4] = 1; rotmore[6] = -1; idx[0] = 2; idx[2] = 0; sgn[2] = -1; break;
  case 4: rotmore[0] = 1; rotmore[5] = 1; rotmore[7] = -1; idx[1] = 2; idx[2] = 1; sgn[2] = -1; break;
  default: rotmore[0] = -1; rotmore[4] = 1; rotmore[8] = -1; sgn[0] = -1; sgn[2] = -1; break;
  }
}

/* Separating-axis test over the 6 face normals and 9 edge-edge cross products, then contact
 * points either by clipping the incident box's face/edges against the reference face
 * (face code < 12) or by clipping the two closest edges' quadrilateral (edge-edge). Raw
 * contacts in c (at most 24), normal in frame[0:3]; returns the count. */
static int col_boxBox(orRaw* c, mjtNum margin, const mjtNum* pos1, const mjtNum* mat1,
                      const mjtNum* size1, const mjtNum* pos2, const mjtNum* mat2,
                      const mjtNum* size2) {
  mjtNum pos12[3], pos21[3], rot[9], rott[9], rotabs[9], rottabs[9], tmp1[3], tmp2[3];
  mjtNum plen1[3], plen2[3], rotmore[9], p[3], r[9], s[3], ss[3], lp[3], rt[9];
  mjtNum points[24][3], depth[24], pts[6][3], ppts2[4][2], pu[4][3], axi[3][3];
  mjtNum linesu[4][6], lines[4][6], clnorm[3] = {0, 0, 0}, rnorm[3], sg[3];
  int idx[3];
  int code = -1, cle1 = 0, cle2 = 0, in = 0, n = 0;
  const mjtNum margin2 = margin*margin;

  mju_sub3(tmp1, pos2, pos1);
  mju_mulMatTVec3(pos21, mat1, tmp1);
  mju_sub3(tmp1, pos1, pos2);
  mju_mulMatTVec3(pos12, mat2, tmp1);
  bb_mulMatTMat3(rot, mat1, mat2);
  bb_transpose3(rott, rot);
  for (int i = 0; i < 9; i++) rotabs[i] = fabs(rot[i]);
  for (int i = 0; i < 9; i++) rottabs[i] = fabs(rott[i]);
  mju_mulMatVec3(plen2, rotabs, size2);
  mju_mulMatTVec3(plen1, rotabs, size1);

  /* face axes */
  mjtNum penetration = margin;
  for (int i = 0; i < 3; i++) penetration += size1[i]*3 + size2[i]*3;
  for (int i = 0; i < 3; i++) {
    mjtNum c1 = -fabs(pos21[i]) + size1[i] + plen2[i];
    mjtNum c2 = -fabs(pos12[i]) + size2[i] + plen1[i];
    if (c1 < -margin || c2 < -margin) return 0;
    if (c1 < penetration) { penetration = c1; code = i + 3*(pos21[i] < 0); }
    if (c2 < penetration) { penetration = c2; code = i + 3*(pos12[i] < 0) + 6; }
  }
  /* edge-edge axes: cross(e1_i, e2_j) in box 1's frame */
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      mju_zero3(tmp2);
      if (i == 0) { tmp2[1] = -rott[3*j+2]; tmp2[2] = rott[3*j+1]; }
      else if (i == 1) { tmp2[0] = rott[3*j+2]; tmp2[2] = -rott[3*j]; }
      else { tmp2[0] = -rott[3*j+1]; tmp2[1] = rott[3*j]; }
      mjtNum c1 = mju_normalize3(tmp2);
      if (c1 < mjMINVAL) continue;
      mjtNum c2 = mju_dot3(pos21, tmp2);
      mjtNum c3 = 0;
      for (int k = 0; k < 3; k++) if (k != i) c3 += size1[k]*fabs(tmp2[k]);
      for (int k = 0; k < 3; k++) if (k != j) c3 += size2[k]*rotabs[3*i + 3 - k - j] / c1;
      c3 -= fabs(c2);
      if (c3 < -margin) return 0;
      if (c3 < penetration*(1 - 1e-12)) {
        penetration = c3;
        cle1 = 0;
        for (int k = 0; k < 3; k++) if (k != i && ((tmp2[k] > 0) ^ (c2 < 0))) cle1 += 1 << k;
        cle2 = 0;
        for (int k = 0; k < 3; k++) {
          if (k != j && ((rot[3*i + 3 - k - j] > 0) ^ (c2 < 0) ^ ((k - j + 3) % 3 == 1))) {
            cle2 += 1 << k;
          }
        }
        code = 12 + 3*i + j;
        mju_copy3(clnorm, tmp2);
        in = c2 < 0;
      }
    }
  }
  if (code == -1) return 0;

  if (code < 12) {
    /* ---- face of one box against the other box */
    const int q1 = code % 6, q2 = code / 6;
    bb_faceFrame(q1, rotmore, idx, sg);
    if (q2) {
      bb_mulMatMatT3(r, rotmore, rot);
      for (int k = 0; k < 3; k++) { p[k] = pos12[idx[k]]*sg[k]; tmp1[k] = size2[idx[k]]*sg[k]; }
      mju_copy3(s, size1);
    } else {
      for (int k = 0; k < 3; k++) mju_scl3(r + 3*k, rot + 3*idx[k], sg[k]);
      for (int k = 0; k < 3; k++) { p[k] = pos21[idx[k]]*sg[k]; tmp1[k] = size1[idx[k]]*sg[k]; }
      mju_copy3(s, size2);
    }
    bb_transpose3(rt, r);
    for (int i = 0; i < 3; i++) ss[i] = fabs(tmp1[i]);
    const mjtNum lx = ss[0], ly = ss[1], hz = ss[2];
    p[2] -= hz;
    mju_copy3(lp, p);
    int clcorner = 0;
    for (int i = 0; i < 3; i++) if (r[6+i] < 0) clcorner += 1 << i;
    mju_addToScl3(lp, rt, s[0]*((clcorner & 1) ? 1 : -1));
    mju_addToScl3(lp, rt + 3, s[1]*((clcorner & 2) ? 1 : -1));
    mju_addToScl3(lp, rt + 6, s[2]*((clcorner & 4) ? 1 : -1));
    int m = 0, k = 0;
    mju_copy3(pts[m++], lp);
    for (int i = 0; i < 3; i++) {
      if (fabs(r[6+i]) < 0.5) mju_scl3(pts[m++], rt + 3*i, s[i]*((clcorner & (1 << i)) ? -2 : 2));
    }
    mju_add3(pts[3], pts[0], pts[1]);
    mju_add3(pts[4], pts[0], pts[2]);
    mju_add3(pts[5], pts[3], pts[2]);
    if (m > 1) { mju_copy3(lines[k], pts[0]); mju_copy3(lines[k++] + 3, pts[1]); }
    if (m > 2) {
      mju_copy3(lines[k], pts[0]); mju_copy3(lines[k++] + 3, pts[2]);
      mju_copy3(lines[k], pts[3]); mju_copy3(lines[k++] + 3, pts[2]);
      mju_copy3(lines[k], pts[4]); mju_copy3(lines[k++] + 3, pts[1]);
    }
    for (int i = 0; i < k; i++) {        /* incident edges against the face's rectangle */
      for (int q = 0; q < 2; q++) {
        mjtNum a = lines[i][q], b = lines[i][3+q], cc = lines[i][1-q], dd = lines[i][4-q];
        if (fabs(b) > mjMINVAL) {
          for (int j = -1; j <= 1; j += 2) {
            mjtNum l = ss[q]*j;
            mjtNum c1 = (l - a)*(1/b);
            if (c1 < 0 || c1 > 1) continue;
            mjtNum c2 = cc + dd*c1;
            if (fabs(c2) > ss[1-q]) continue;
            mju_copy3(points[n], lines[i]);
            mju_addToScl3(points[n++], lines[i] + 3, c1);
          }
        }
      }
    }
    mjtNum a = pts[1][0], b = pts[2][0], cc = pts[1][1], dd = pts[2][1];
    mjtNum c1 = a*dd - b*cc;
    if (m > 2) {                         /* face corners inside the incident face */
      for (int i = 0; i < 4; i++) {
        mjtNum llx = i/2 ? lx : -lx, lly = i % 2 ? ly : -ly;
        mjtNum x = llx - pts[0][0], y = lly - pts[0][1];
        mjtNum u = (x*dd - y*b)*(1/c1), v = (y*a - x*cc)*(1/c1);
        if (u <= 0 || v <= 0 || u >= 1 || v >= 1) continue;
        points[n][0] = llx;
        points[n][1] = lly;
        points[n][2] = pts[0][2] + u*pts[1][2] + v*pts[2][2];
        n++;
      }
    }
    for (int i = 0; i < (1 << (m - 1)); i++) {   /* incident corners inside the face */
      mju_copy3(tmp1, pts[i == 0 ? 0 : i + 2]);
      if (i && (tmp1[0] <= -lx || tmp1[0] >= lx)) continue;
      if (i && (tmp1[1] <= -ly || tmp1[1] >= ly)) continue;
      mju_copy3(points[n++], tmp1);
    }
    m = n;
    n = 0;
    for (int i = 0; i < m; i++) {
      if (points[i][2] > margin) continue;
      mju_copy3(points[n], points[i]);
      depth[n] = points[n][2];
      points[n][2] *= 0.5;
      n++;
    }
    bb_mulMatMatT3(r, q2 ? mat2 : mat1, rotmore);
    mju_copy3(p, q2 ? pos2 : pos1);
    const mjtNum f = q2 ? -1 : 1;
    tmp2[0] = f*r[2]; tmp2[1] = f*r[5]; tmp2[2] = f*r[8];
    for (int i = 0; i < n; i++) {
      c[i].dist = points[i][2];            /* the reference reports half the face depth */
      points[i][2] += hz;
      mju_mulMatVec3(tmp1, r, points[i]);
      mju_add3(c[i].pos, tmp1, p);
      mju_copy3(c[i].frame, tmp2);
      mju_zero(c[i].frame + 3, 6);
    }
    (void)depth;
    return n;
  }

  /* ---- edge against edge */
  code -= 12;
  const int q1 = code / 3, q2 = code % 3;
  int ax1 = q2 == 0 ? 1 : (q2 == 1 ? 0 : 1), ax2 = q2 == 2 ? 0 : 2;
  int pax1 = q1 == 0 ? 1 : (q1 == 1 ? 0 : 1), pax2 = q1 == 2 ? 0 : 2;
  if (rotabs[3*q1 + ax1] < rotabs[3*q1 + ax2]) { ax1 = ax2; ax2 = 3 - q2 - ax1; }
  if (rottabs[3*q2 + pax1] < rottabs[3*q2 + pax2]) { pax1 = pax2; pax2 = 3 - q1 - pax1; }
  const int clface = (cle1 & (1 << pax2)) ? pax2 : pax2 + 3;
  bb_faceFrame(clface, rotmore, idx, sg);
  for (int k = 0; k < 3; k++) { p[k] = pos21[idx[k]]*sg[k]; rnorm[k] = clnorm[idx[k]]*sg[k]; }
  for (int k = 0; k < 3; k++) mju_scl3(r + 3*k, rot + 3*idx[k], sg[k]);
  mju_mulMatTVec3(tmp1, rotmore, size1);
  for (int i = 0; i < 3; i++) s[i] = fabs(tmp1[i]);
  bb_transpose3(rt, r);
  const mjtNum lx = s[0], ly = s[1], hz = s[2];
  p[2] -= hz;
  /* the incident edge's two end points, and the parallel edge's */
  for (int e = 0; e < 2; e++) {
    mjtNum* p0 = points[2*e];
    mju_copy3(p0, p);
    mju_addToScl3(p0, rt + 3*ax1, size2[ax1]*(((cle2 & (1 << ax1)) ? 1 : -1)*(e ? -1 : 1)));
    mju_addToScl3(p0, rt + 3*ax2, size2[ax2]*((cle2 & (1 << ax2)) ? 1 : -1));
    mju_copy3(points[2*e + 1], p0);
    mju_addToScl3(p0, rt + 3*q2, size2[q2]);
    mju_addToScl3(points[2*e + 1], rt + 3*q2, -size2[q2]);
  }
  mju_copy3(axi[0], points[0]);
  mju_sub3(axi[1], points[1], points[0]);
  mju_sub3(axi[2], points[2], points[0]);
  if (fabs(rnorm[2]) < mjMINVAL) return 0;
  const mjtNum innorm = (1/rnorm[2])*(in ? -1 : 1);
  for (int i = 0; i < 4; i++) {          /* project onto the reference face along the normal */
    mjtNum c1 = -points[i][2]*(1/rnorm[2]);
    mju_copy3(pu[i], points[i]);
    mju_addToScl3(points[i], rnorm, c1);
    ppts2[i][0] = points[i][0];
    ppts2[i][1] = points[i][1];
  }
  mju_copy3(pts[0], points[0]);
  mju_sub3(pts[1], points[1], points[0]);
  mju_sub3(pts[2], points[2], points[0]);
  int k = 0;
  mju_copy3(lines[k], pts[0]); mju_copy3(lines[k] + 3, pts[1]);
  mju_copy3(linesu[k], axi[0]); mju_copy3(linesu[k++] + 3, axi[1]);
  mju_copy3(lines[k], pts[0]); mju_copy3(lines[k] + 3, pts[2]);
  mju_copy3(linesu[k], axi[0]); mju_copy3(linesu[k++] + 3, axi[2]);
  mju_add3(lines[k], pts[0], pts[1]); mju_copy3(lines[k] + 3, pts[2]);
  mju_add3(linesu[k], axi[0], axi[1]); mju_copy3(linesu[k++] + 3, axi[2]);
  mju_add3(lines[k], pts[0], pts[2]); mju_copy3(lines[k] + 3, pts[1]);
  mju_add3(linesu[k], axi[0], axi[2]); mju_copy3(linesu[k++] + 3, axi[1]);
  n = 0;
  for (int i = 0; i < k; i++) {          /* quadrilateral edges against the face rectangle */
    for (int q = 0; q < 2; q++) {
      mjtNum a = lines[i][q], b = lines[i][3+q], cc = lines[i][1-q], dd = lines[i][4-q];
      if (fabs(b) > mjMINVAL) {
        for (int j = -1; j <= 1; j += 2) {
          mjtNum l = s[q]*j;
          mjtNum c1 = (l - a)*(1/b);
          if (c1 < 0 || c1 > 1) continue;
          mjtNum c2 = cc + dd*c1;
          if (fabs(c2) > s[1-q]) continue;
          if ((linesu[i][2] + linesu[i][5]*c1)*innorm > margin) continue;
          mju_scl3(points[n], linesu[i], 0.5);
          mju_addToScl3(points[n], linesu[i] + 3, 0.5*c1);
          points[n][q] += 0.5*l;
          points[n][1-q] += 0.5*c2;
          depth[n] = points[n][2]*innorm*2;
          n++;
        }
      }
    }
  }
  const int nl = n;
  mjtNum a = pts[1][0], b = pts[2][0], cc = pts[1][1], dd = pts[2][1];
  mjtNum c1 = a*dd - b*cc;
  for (int i = 0; i < 4; i++) {          /* face corners against the quadrilateral */
    mjtNum llx = i/2 ? lx : -lx, lly = i % 2 ? ly : -ly;
    mjtNum x = llx - pts[0][0], y = lly - pts[0][1];
    mjtNum u = (x*dd - y*b)*(1/c1), v = (y*a - x*cc)*(1/c1);
    if (nl == 0) {
      if ((u < 0 || u > 1) && (v < 0 || v > 1)) continue;
    } else if (u < 0 || u > 1 || v < 0 || v > 1) {
      continue;
    }
    u = u < 0 ? 0 : (u > 1 ? 1 : u);
    v = v < 0 ? 0 : (v > 1 ? 1 : v);
    mju_scl3(tmp1, pu[0], 1 - u - v);
    mju_addToScl3(tmp1, pu[1], u);
    mju_addToScl3(tmp1, pu[2], v);
    points[n][0] = llx;
    points[n][1] = lly;
    points[n][2] = 0;
    mju_sub3(tmp2, points[n], tmp1);
    /* the reference reuses c1 here: later corners divide by this squared distance */
    c1 = mju_dot3(tmp2, tmp2);
    if (tmp1[2] > 0 && c1 > margin2) continue;
    mju_add3(points[n], points[n], tmp1);
    mju_scl3(points[n], points[n], 0.5);
    depth[n] = sqrt(c1)*(tmp1[2] < 0 ? -1 : 1);
    n++;
  }
  const int nf = n;
  for (int i = 0; i < 4; i++) {          /* quadrilateral corners over the face */
    mjtNum x = ppts2[i][0], y = ppts2[i][1];
    if (nl == 0) {
      if (nf != 0 && (x < -lx || x > lx) && (y < -ly || y > ly)) continue;
    } else if (x < -lx || x > lx || y < -ly || y > ly) {
      continue;
    }
    mjtNum d2 = 0;
    for (int j = 0; j < 2; j++) {
      if (ppts2[i][j] < -s[j]) d2 += (ppts2[i][j] + s[j])*(ppts2[i][j] + s[j]);
      else if (ppts2[i][j] > s[j]) d2 += (ppts2[i][j] - s[j])*(ppts2[i][j] - s[j]);
    }
    d2 += pu[i][2]*innorm*pu[i][2]*innorm;
    if (pu[i][2] > 0 && d2 > margin2) continue;
    tmp1[0] = ppts2[i][0]*0.5;
    tmp1[1] = ppts2[i][1]*0.5;
    tmp1[2] = 0;
    for (int j = 0; j < 2; j++) {
      if (ppts2[i][j] < -s[j]) tmp1[j] = -s[j]*0.5;
      else if (ppts2[i][j] > s[j]) tmp1[j] = s[j]*0.5;
    }
    mju_addToScl3(tmp1, pu[i], 0.5);
    mju_copy3(points[n], tmp1);
    depth[n] = sqrt(d2)*(pu[i][2] < 0 ? -1 : 1);
    n++;
  }
  bb_mulMatMatT3(r, mat1, rotmore);
  mju_mulMatVec3(tmp1, r, rnorm);
  mju_scl3(tmp2, tmp1, in ? -1 : 1);
  for (int i = 0; i < n; i++) {
    c[i].dist = depth[i];
    points[i][2] += hz;
    mju_mulMatVec3(tmp1, r, points[i]);
    mju_add3(c[i].pos, tmp1, pos1);
    mju_copy3(c[i].frame, tmp2);
    mju_zero(c[i].frame + 3, 6);
  }
  return n;
}

/* mju_outsideBox (engine_util_misc.c:911-950): 1 outside the inflated box, -1 inside the
 * deflated one, 0 between */
static int or_outsideBox(const mjtNum point[3], const mjtNum pos[3], const mjtNum mat[9],
                         const mjtNum size[3], mjtNum inflate) {
  mjtNum vec[3] = {point[0]-pos[0], point[1]-pos[1], point[2]-pos[2]};
  mju_mulMatTVec3(vec, mat, vec);
  mjtNum big[3] = {size[0]*inflate, size[1]*inflate, size[2]*inflate};
  if (vec[0] > big[0] || vec[0] < -big[0] || vec[1] > big[1] || vec[1] < -big[1] ||
      vec[2] > big[2] || vec[2] < -big[2]) {
    return 1;
  }
  mjtNum small[3] = {size[0]/inflate, size[1]/inflate, size[2]/inflate};
  if (vec[0] < small[0] && vec[0] > -small[0] && vec[1] < small[1] && vec[1] > -small[1] &&
      vec[2] < small[2] && vec[2] > -small[2]) {
    return -1;
  }
  return 0;
}

/* mj_collideGeoms' box-box clean-up (engine_collision_driver.c:1522-1588): drop contacts
 * outside one box (by 1%) and not inside the other, and earlier copies of repeated
 * positions; the survivors keep their order */
static int or_boxBoxFilter(orRaw* c, int num, mjtNum margin, const mjtNum* pos1,
                           const mjtNum* mat1, const mjtNum* size1, const mjtNum* pos2,
                           const mjtNum* mat2, const mjtNum* size2) {
  int bad[24];
  const mjtNum sz1[3] = {size1[0] + margin, size1[1] + margin, size1[2] + margin};
  const mjtNum sz2[3] = {size2[0] + margin, size2[1] + margin, size2[2] + margin};
  for (int i = 0; i < num; i++) {
    int out1 = or_outsideBox(c[i].pos, pos1, mat1, sz1, 1.01);
    int out2 = or_outsideBox(c[i].pos, pos2, mat2, sz2, 1.01);
    bad[i] = (out1 == 1 && out2 != -1) || (out2 == 1 && out1 != -1);
  }
  for (int i = 0; i < num - 1; i++) {
    if (bad[i]) continue;
    for (int j = i + 1; j < num; j++) {
      if (bad[j]) continue;
      if (c[i].pos[0] == c[j].pos[0] && c[i].pos[1] == c[j].pos[1] && c[i].pos[2] == c[j].pos[2]) {
        bad[i] = 1;
        break;
      }
    }
  }
  int n = 0;
  for (int j = 0; j < num; j++) {
    if (!bad[j]) {
      if (n < j) c[n] = c[j];
      n++;
    }
  }
  return n;
}

/* test entry: mjc_BoxBox alone (before mj_collideGeoms' clean-up) on the current geom
 * poses, as the reference's BadContacts/DuplicateContacts tests call it; out holds
 * (dist, pos[3], normal[3]) per contact */
int or_boxBoxRaw(const mjhipModel* m, const mjhipData* d, int g1, int g2, mjtNum margin,
                 mjtNum* out) {
  orRaw raw[24];
  int num = col_boxBox(raw, margin, d->geom_xpos + 3*g1, d->geom_xmat + 9*g1,
                       m->geom_size + 3*g1, d->geom_xpos + 3*g2, d->geom_xmat + 9*g2,
                       m->geom_size + 3*g2);
  for (int i = 0; i < num; i++) {
    out[7*i] = raw[i].dist;
    mju_copy3(out + 7*i + 1, raw[i].pos);
    mju_copy3(out + 7*i + 4, raw[i].frame);
  }
  return num;
}

/*============== native convex collision: mjc_Convex / mjc_PlaneConvex on mjc_ccd ==============
 * engine_collision_convex.c (supports :146-327, mjc_initCCDObj :716-768, mjc_CCDIteration
 * :792-819, mjc_Convex :915-1001 with mjENBL_MULTICCD off, mjc_PlaneConvex :1045-1080 for a
 * geom without mesh data) and engine_collision_gjk.c (gjk :163-272, supports :277-370,
 * gjkIntersect :393-448, the subdistance algorithm :482-814, polytope2/3/4 :892-1156, the EPA
 * :1161-1459, inflate and mjc_ccd :2195-2343). Only the native solver (mjDSBL_NATIVECCD
 * clear) with one contact per pair is restated; mesh, height-field and SDF geoms are not. */

enum { CCD_POINT = 100, CCD_LINE = 101 };      /* shrunken sphere / capsule supports */

/* Minkowski vertex, both witnesses, and the box corner / mesh vertex each support returned
   (Vertex.index1 / index2, gjk.h:51-57: the shape's vertindex after the support call) */
typedef struct { mjtNum v[3], p1[3], p2[3]; int i1, i2; } orVtx;

typedef struct {
  int kind;                /* mjtGeom of the geom, or CCD_POINT / CCD_LINE */
  int gtype;               /* the geom's own type (geom_type) */
  const mjtNum* pos;       /* geom_xpos, geom_xmat, geom_size of the geom */
  const mjtNum* mat;
  const mjtNum* size;
  mjtNum margin;
  /* mesh geoms: the mesh's float vertices and convex-hull graph (NULL: none), and the
     warm starts the supports keep between calls (mjCCDObj.vertindex / meshindex) */
  const float* vert;
  int nvert;
  const int* graph;
  int vertindex, meshindex;
  /* mesh geoms: the model and the mesh (the polygon data multicontact reads) */
  const mjhipModel* model;
  int meshid;
  /* height-field prism (mjCCDObj.prism) and its centre (mjc_prism_center) */
  mjtNum prism[6][3];
  mjtNum pcenter[3];
} orShape;

/* mulMatTVec3 / localToGlobal of engine_collision_convex.c:122-141 */
static void ccd_toLocal(mjtNum r[3], const mjtNum* mat, const mjtNum d[3]) {
  r[0] = mat[0]*d[0] + mat[3]*d[1] + mat[6]*d[2];
  r[1] = mat[1]*d[0] + mat[4]*d[1] + mat[7]*d[2];
  r[2] = mat[2]*d[0] + mat[5]*d[1] + mat[8]*d[2];
}

static void ccd_toGlobal(mjtNum r[3], const mjtNum* mat, const mjtNum t[3], const mjtNum* pos) {
  r[0] = mat[0]*t[0] + mat[1]*t[1] + mat[2]*t[2];
  r[1] = mat[3]*t[0] + mat[4]*t[1] + mat[5]*t[2];
  r[2] = mat[6]*t[0] + mat[7]*t[1] + mat[8]*t[2];
  r[0] += pos[0];
  r[1] += pos[1];
  r[2] += pos[2];
}

static mjtNum ccd_sign(mjtNum x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }

/* the native support functions (convex.c:146-327) */
/* dot product between mjtNum and float (convex.c:332-334) */
static mjtNum ccd_dot3f(const mjtNum a[3], const float b[3]) {
  return a[0]*(mjtNum)b[0] + a[1]*(mjtNum)b[1] + a[2]*(mjtNum)b[2];
}

/* mjc_meshSupport (:339-382, exhaustive) and mjc_hillclimbSupport (:387-433), as
   mjc_initCCDObj (:735-743) picks them: hill climbing on the hull graph from mjMESH_HILLCLIMB_MIN
   (10) vertices */
static void ccd_meshSupport(mjtNum r[3], orShape* s, const mjtNum dir[3]) {
  mjtNum ld[3], t[3];
  ccd_toLocal(ld, s->mat, dir);
  const float* V = s->vert;
  int imax;
  if (!s->graph || s->nvert < 10) {
    mjtNum max = -FLT_MAX;
    imax = 0;
    if (s->vertindex >= 0) {
      imax = s->vertindex;
      max = ccd_dot3f(ld, V + 3*imax);
    }
    for (int i = 0; i < s->nvert; i++) {
      mjtNum vdot = ccd_dot3f(ld, V + 3*i);
      if (vdot > max) {
        max = vdot;
        imax = i;
      }
    }
    s->vertindex = imax;
  } else {
    const int numvert = s->graph[0];
    const int* edgeadr = s->graph + 2;
    const int* globalid = s->graph + 2 + numvert;
    const int* localid = s->graph + 2 + 2*numvert;
    mjtNum max = -FLT_MAX;
    int prev;
    imax = s->meshindex < 0 ? 0 : s->meshindex;
    do {
      prev = imax;
      for (int i = edgeadr[imax]; localid[i] >= 0; i++) {
        mjtNum vdot = ccd_dot3f(ld, V + 3*globalid[localid[i]]);
        if (vdot > max) {
          max = vdot;
          imax = localid[i];
        }
      }
    } while (imax != prev);
    s->meshindex = imax;
    imax = globalid[imax];
    s->vertindex = imax;
  }
  t[0] = (mjtNum)V[3*imax];
  t[1] = (mjtNum)V[3*imax + 1];
  t[2] = (mjtNum)V[3*imax + 2];
  ccd_toGlobal(r, s->mat, t, s->pos);
}

static void ccd_support1(mjtNum r[3], orShape* s, const mjtNum dir[3]) {
  mjtNum ld[3], t[3];
  switch (s->kind) {
  case mjhipGEOM_MESH:
    ccd_meshSupport(r, s, dir);
    return;
  case mjhipGEOM_HFIELD: {             /* mjc_prism_support (:438-455) */
    int istart = dir[2] < 0 ? 0 : 3, ibest = istart;
    mjtNum best = mju_dot3(s->prism[istart], dir), tmp;
    for (int i = istart + 1; i < istart + 3; i++) {
      if ((tmp = mju_dot3(s->prism[i], dir)) > best) {
        ibest = i;
        best = tmp;
      }
    }
    mju_copy3(r, s->prism[ibest]);
    return;
  }
  case CCD_POINT:
    mju_copy3(r, s->pos);
    return;
  case mjhipGEOM_SPHERE:
    r[0] = s->size[0]*dir[0] + s->pos[0];
    r[1] = s->size[0]*dir[1] + s->pos[1];
    r[2] = s->size[0]*dir[2] + s->pos[2];
    return;
  case CCD_LINE:
    ccd_toLocal(ld, s->mat, dir);
    t[0] = 0;
    t[1] = 0;
    t[2] = ld[2] >= 0 ? s->size[1] : -s->size[1];
    break;
  case mjhipGEOM_CAPSULE:
    ccd_toLocal(ld, s->mat, dir);
    t[0] = ld[0]*s->size[0];
    t[1] = ld[1]*s->size[0];
    t[2] = ld[2]*s->size[0];
    t[2] += ld[2] >= 0 ? s->size[1] : -s->size[1];
    break;
  case mjhipGEOM_ELLIPSOID: {
    ccd_toLocal(ld, s->mat, dir);
    t[0] = ld[0]*s->size[0];
    t[1] = ld[1]*s->size[1];
    t[2] = ld[2]*s->size[2];
    mjtNum nrm = sqrt(t[0]*t[0] + t[1]*t[1] + t[2]*t[2]);
    if (nrm < mjMINVAL) {
      t[0] = s->size[0];
      t[1] = 0;
      t[2] = 0;
    } else {
      mjtNum inv = 1/nrm;
      t[0] *= inv*s->size[0];
      t[1] *= inv*s->size[1];
      t[2] *= inv*s->size[2];
    }
    break;
  }
  case mjhipGEOM_CYLINDER: {
    ccd_toLocal(ld, s->mat, dir);
    mjtNum n = ld[0]*ld[0] + ld[1]*ld[1];
    if (n > mjMINVAL*mjMINVAL) {
      n = s->size[0] / sqrt(n);
      t[0] = ld[0]*n;
      t[1] = ld[1]*n;
    } else {
      t[0] = t[1] = 0;
    }
    t[2] = ccd_sign(ld[2])*s->size[1];
    break;
  }
  default:   /* box; the corner's index for multicontact (mjc_boxSupport :314-323) */
    ccd_toLocal(ld, s->mat, dir);
    t[0] = (ld[0] >= 0 ? 1 : -1)*s->size[0];
    t[1] = (ld[1] >= 0 ? 1 : -1)*s->size[1];
    t[2] = (ld[2] >= 0 ? 1 : -1)*s->size[2];
    s->vertindex = (t[0] > 0 ? 1 : 0) | (t[1] > 0 ? 2 : 0) | (t[2] > 0 ? 4 : 0);
    break;
  }
  ccd_toGlobal(r, s->mat, t, s->pos);
}

/* support (gjk.c:277-296): each shape inflated by half its margin */
static void ccd_support(orVtx* v, orShape* a, orShape* b, const mjtNum dir[3],
                        const mjtNum ndir[3]) {
  ccd_support1(v->p1, a, dir);
  if (a->margin > 0) {
    mjtNum h = 0.5*a->margin;
    v->p1[0] += dir[0]*h;
    v->p1[1] += dir[1]*h;
    v->p1[2] += dir[2]*h;
  }
  ccd_support1(v->p2, b, ndir);
  if (b->margin > 0) {
    mjtNum h = 0.5*b->margin;
    v->p2[0] += ndir[0]*h;
    v->p2[1] += ndir[1]*h;
    v->p2[2] += ndir[2]*h;
  }
  mju_sub3(v->v, v->p1, v->p2);
  v->i1 = a->vertindex;       /* gjkSupport / epaSupport (:316-322, :346-351) */
  v->i2 = b->vertindex;
}

static mjtNum ccd_det3(const mjtNum a[3], const mjtNum b[3], const mjtNum c[3]) {
  return a[0]*(b[1]*c[2] - b[2]*c[1]) + a[1]*(b[2]*c[0] - b[0]*c[2])
       + a[2]*(b[0]*c[1] - b[1]*c[0]);
}

static int ccd_sameSign(mjtNum a, mjtNum b) {
  if (a > 0 && b > 0) return 1;
  if (a < 0 && b < 0) return -1;
  return 0;
}

/* lincomb (gjk.c:453-477): sum of the first n coef[i]*v[i], left to right */
static void ccd_lincomb(mjtNum r[3], const mjtNum* c, int n, const mjtNum* v1, const mjtNum* v2,
                        const mjtNum* v3, const mjtNum* v4) {
  for (int k = 0; k < 3; k++) {
    mjtNum s = c[0]*v1[k];
    if (n > 1) s = s + c[1]*v2[k];
    if (n > 2) s = s + c[2]*v3[k];
    if (n > 3) s = s + c[3]*v4[k];
    r[k] = s;
  }
}

/* projectOriginPlane (gjk.c:482-515): 1 if the plane is degenerate */
static int ccd_projPlane(mjtNum r[3], const mjtNum a[3], const mjtNum b[3], const mjtNum c[3]) {
  mjtNum ba[3], ca[3], cb[3], n[3], nv, nn;
  mju_sub3(ba, b, a);
  mju_sub3(ca, c, a);
  mju_sub3(cb, c, b);
  mju_cross(n, cb, ba);
  nv = mju_dot3(n, b);
  nn = mju_dot3(n, n);
  if (nn == 0) return 1;
  if (nv != 0 && nn > mjMINVAL) {
    mju_scl3(r, n, nv / nn);
    return 0;
  }
  mju_cross(n, ba, ca);
  nv = mju_dot3(n, a);
  nn = mju_dot3(n, n);
  if (nn == 0) return 1;
  if (nv != 0 && nn > mjMINVAL) {
    mju_scl3(r, n, nv / nn);
    return 0;
  }
  mju_cross(n, ca, cb);
  nv = mju_dot3(n, c);
  nn = mju_dot3(n, n);
  mju_scl3(r, n, nv / nn);
  return 0;
}

/* S1D (gjk.c:787-814) */
static void ccd_S1D(mjtNum lam[2], const mjtNum a[3], const mjtNum b[3]) {
  mjtNum d[3], p[3];
  mju_sub3(d, b, a);
  mjtNum s = -(mju_dot3(b, d) / mju_dot3(d, d));
  p[0] = b[0] + s*d[0];
  p[1] = b[1] + s*d[1];
  p[2] = b[2] + s*d[2];
  mjtNum mu = 0;
  int ix = 0;
  for (int i = 0; i < 3; i++) {
    mjtNum t = a[i] - b[i];
    if (fabs(t) >= fabs(mu)) {
      mu = t;
      ix = i;
    }
  }
  mjtNum c1 = p[ix] - b[ix], c2 = a[ix] - p[ix];
  if (ccd_sameSign(mu, c1) && ccd_sameSign(mu, c2)) {
    lam[0] = c1 / mu;
    lam[1] = c2 / mu;
  } else {
    lam[0] = 0;
    lam[1] = 1;
  }
}

/* the minors M_14, M_24, M_34 of S2D / triAffineCoord (gjk.c:667-669, :979-981) */
static void ccd_minors(mjtNum M[3], const mjtNum a[3], const mjtNum b[3], const mjtNum c[3]) {
  M[0] = b[1]*c[2] - b[2]*c[1] - a[1]*c[2] + a[2]*c[1] + a[1]*b[2] - a[2]*b[1];
  M[1] = b[0]*c[2] - b[2]*c[0] - a[0]*c[2] + a[2]*c[0] + a[0]*b[2] - a[2]*b[0];
  M[2] = b[0]*c[1] - b[1]*c[0] - a[0]*c[1] + a[1]*c[0] + a[0]*b[1] - a[1]*b[0];
}

/* the axes kept after dropping the one of largest projection; returns M_max */
static mjtNum ccd_axes(const mjtNum M[3], int* x, int* y) {
  mjtNum m1 = fabs(M[0]), m2 = fabs(M[1]), m3 = fabs(M[2]);
  if (m1 >= m2 && m1 >= m3) { *x = 1; *y = 2; return M[0]; }
  if (m2 >= m3) { *x = 0; *y = 2; return M[1]; }
  *x = 0; *y = 1;
  return M[2];
}

/* signed area cofactor of (p, u, w) in the kept axes (gjk.c:722-731) */
static mjtNum ccd_area(const mjtNum* p, const mjtNum* u, const mjtNum* w, int x, int y) {
  return p[x]*u[y] + p[y]*w[x] + u[x]*w[y] - p[x]*w[y] - p[y]*u[x] - w[x]*u[y];
}

/* S2D (gjk.c:653-783) */
static void ccd_S2D(mjtNum lam[3], const mjtNum a[3], const mjtNum b[3], const mjtNum c[3]) {
  mjtNum p[3];
  if (ccd_projPlane(p, a, b, c)) {
    ccd_S1D(lam, a, b);
    lam[2] = 0;
    return;
  }
  mjtNum M[3];
  int x, y;
  ccd_minors(M, a, b, c);
  mjtNum Mmax = ccd_axes(M, &x, &y);
  mjtNum C1 = ccd_area(p, b, c, x, y), C2 = ccd_area(p, c, a, x, y), C3 = ccd_area(p, a, b, x, y);
  int k1 = ccd_sameSign(Mmax, C1), k2 = ccd_sameSign(Mmax, C2), k3 = ccd_sameSign(Mmax, C3);
  if (k1 && k2 && k3) {
    lam[0] = C1 / Mmax;
    lam[1] = C2 / Mmax;
    lam[2] = C3 / Mmax;
    return;
  }
  mjtNum dmin = mjhipMAXVAL, l[2], q[3], dd;
  if (!k1) {
    ccd_S1D(l, b, c);
    ccd_lincomb(q, l, 2, b, c, NULL, NULL);
    dd = mju_dot3(q, q);
    lam[0] = 0; lam[1] = l[0]; lam[2] = l[1];
    dmin = dd;
  }
  if (!k2) {
    ccd_S1D(l, a, c);
    ccd_lincomb(q, l, 2, a, c, NULL, NULL);
    dd = mju_dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = 0; lam[2] = l[1];
      dmin = dd;
    }
  }
  if (!k3) {
    ccd_S1D(l, a, b);
    ccd_lincomb(q, l, 2, a, b, NULL, NULL);
    dd = mju_dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = l[1]; lam[2] = 0;
    }
  }
}

/* S3D (gjk.c:560-649) */
static void ccd_S3D(mjtNum lam[4], const mjtNum a[3], const mjtNum b[3], const mjtNum c[3],
                    const mjtNum e[3]) {
  mjtNum C1 = -ccd_det3(b, c, e), C2 = ccd_det3(a, c, e), C3 = -ccd_det3(a, b, e),
         C4 = ccd_det3(a, b, c);
  mjtNum det = C1 + C2 + C3 + C4;
  int k1 = ccd_sameSign(det, C1), k2 = ccd_sameSign(det, C2), k3 = ccd_sameSign(det, C3),
      k4 = ccd_sameSign(det, C4);
  if (k1 && k2 && k3 && k4) {
    lam[0] = C1 / det;
    lam[1] = C2 / det;
    lam[2] = C3 / det;
    lam[3] = C4 / det;
    return;
  }
  mjtNum dmin = mjhipMAXVAL, l[3], q[3], dd;
  if (!k1) {
    ccd_S2D(l, b, c, e);
    ccd_lincomb(q, l, 3, b, c, e, NULL);
    dd = mju_dot3(q, q);
    lam[0] = 0; lam[1] = l[0]; lam[2] = l[1]; lam[3] = l[2];
    dmin = dd;
  }
  if (!k2) {
    ccd_S2D(l, a, c, e);
    ccd_lincomb(q, l, 3, a, c, e, NULL);
    dd = mju_dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = 0; lam[2] = l[1]; lam[3] = l[2];
      dmin = dd;
    }
  }
  if (!k3) {
    ccd_S2D(l, a, b, e);
    ccd_lincomb(q, l, 3, a, b, e, NULL);
    dd = mju_dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = l[1]; lam[2] = 0; lam[3] = l[2];
      dmin = dd;
    }
  }
  if (!k4) {
    ccd_S2D(l, a, b, c);
    ccd_lincomb(q, l, 3, a, b, c, NULL);
    dd = mju_dot3(q, q);
    if (dd < dmin) {
      lam[0] = l[0]; lam[1] = l[1]; lam[2] = l[2]; lam[3] = 0;
    }
  }
}

/* the solver state of one mjc_ccd call (mjCCDStatus, gjk.h:70-89, the fields this path uses) */
#define OR_MAXCONPAIR 50       /* mjMAXCONPAIR: the status's witness capacity */
typedef struct {
  mjtNum dist, x1[3*OR_MAXCONPAIR], x2[3*OR_MAXCONPAIR];
  int nx, iters, nsimplex;
  int kmax, maxc;
  int unsupported;          /* a multicontact feature the restatement does not cover (none) */
  mjtNum tol, cutoff;
  orVtx simplex[4];
} orCCD;

/* gjkIntersect (gjk.c:393-448): 1 contact, 0 none, -1 inconclusive */
static mjtNum ccd_faceDist(mjtNum n[3], const orVtx* a, const orVtx* b, const orVtx* c) {
  mjtNum d1[3], d2[3];
  mju_sub3(d1, c->v, a->v);
  mju_sub3(d2, b->v, a->v);
  mju_cross(n, d1, d2);
  mjtNum nn = mju_dot3(n, n);
  if (nn > mjMINVAL*mjMINVAL && nn < mjhipMAXVAL*mjhipMAXVAL) {
    nn = 1/sqrt(nn);
    mju_scl3(n, n, nn);
    return mju_dot3(n, a->v);
  }
  return mjhipMAXVAL;
}

static int ccd_intersect(orCCD* st, orShape* A, orShape* B) {
  orVtx s[4] = {st->simplex[0], st->simplex[1], st->simplex[2], st->simplex[3]};
  int o[4] = {0, 1, 2, 3};
  int k = st->iters;
  for (; k < st->kmax; k++) {
    mjtNum dist[4], nrm[12];
    dist[0] = ccd_faceDist(nrm + 0, s + o[2], s + o[1], s + o[3]);
    dist[1] = ccd_faceDist(nrm + 3, s + o[0], s + o[2], s + o[3]);
    dist[2] = ccd_faceDist(nrm + 6, s + o[1], s + o[0], s + o[3]);
    dist[3] = ccd_faceDist(nrm + 9, s + o[0], s + o[1], s + o[2]);
    if (!dist[3] || !dist[2] || !dist[1] || !dist[0]) {
      st->iters = k;
      return -1;
    }
    int i = dist[0] < dist[1] ? 0 : 1, j = dist[2] < dist[3] ? 2 : 3;
    int w = dist[i] < dist[j] ? i : j;
    if (dist[w] > 0) {
      st->nsimplex = 4;
      for (int q = 0; q < 4; q++) st->simplex[q] = s[o[q]];
      st->iters = k;
      return 1;
    }
    mjtNum ndir[3] = {-nrm[3*w], -nrm[3*w+1], -nrm[3*w+2]};
    ccd_support(s + o[w], A, B, nrm + 3*w, ndir);
    if (mju_dot3(nrm + 3*w, s[o[w]].v) < 0) {
      st->nsimplex = 0;
      st->iters = k;
      return 0;
    }
    i = (w + 1) & 3;
    j = (w + 2) & 3;
    int t = o[i];
    o[i] = o[j];
    o[j] = t;
  }
  st->iters = k;
  return -1;
}

/* gjk (gjk.c:163-272) */
static void ccd_gjk(orCCD* st, orShape* A, orShape* B) {
  const int get_dist = st->cutoff > 0;
  int backup = !get_dist, n = 0, k = 0;
  orVtx* S = st->simplex;
  mjtNum x[3], lam[4] = {1, 0, 0, 0}, cut2 = st->cutoff*st->cutoff;
  /* discreteGeoms (gjk.c:150-158) */
  const int dA = A->gtype == mjhipGEOM_BOX || A->gtype == mjhipGEOM_MESH ||
                 A->gtype == mjhipGEOM_HFIELD;
  const int dB = B->gtype == mjhipGEOM_BOX || B->gtype == mjhipGEOM_MESH ||
                 B->gtype == mjhipGEOM_HFIELD;
  const int discrete = A->margin == 0 && B->margin == 0 && dA && dB;
  const mjtNum eps = discrete ? 0 : st->tol*st->tol;
  mju_sub3(x, st->x1, st->x2);
  for (; k < st->kmax; k++) {
    /* gjkSupport (:301-323) */
    mjtNum dir[3] = {-1, 0, 0}, ndir[3] = {1, 0, 0};
    mjtNum nn = mju_dot3(x, x);
    if (nn > mjMINVAL*mjMINVAL) {
      nn = 1/sqrt(nn);
      mju_scl3(ndir, x, nn);
      mju_scl3(dir, ndir, -1);
    }
    ccd_support(S + n, A, B, dir, ndir);
    const mjtNum* sk = S[n].v;
    mjtNum diff[3];
    mju_sub3(diff, x, sk);
    if (2*mju_dot3(x, diff) < eps) {
      if (!k) n = 1;
      break;
    }
    if (!get_dist) {
      if (mju_dot3(x, sk) > 0) {
        st->iters = k;
        st->nsimplex = 0;
        st->nx = 0;
        st->dist = mjhipMAXVAL;
        return;
      }
    } else if (st->cutoff < mjhipMAXVAL) {
      mjtNum vs = mju_dot3(x, sk), vv = mju_dot3(x, x);
      if (mju_dot3(x, sk) > 0 && (vs*vs / vv) >= cut2) {
        st->iters = k;
        st->nsimplex = 0;
        st->nx = 0;
        st->dist = mjhipMAXVAL;
        return;
      }
    }
    if (n == 3 && backup) {
      st->iters = k;
      int r = ccd_intersect(st, A, B);
      if (r != -1) {
        st->nx = 0;
        st->dist = r > 0 ? 0 : mjhipMAXVAL;
        return;
      }
      k = st->iters;
      backup = 0;
    }
    /* subdistance (:544-556) */
    lam[0] = lam[1] = lam[2] = lam[3] = 0;
    if (n + 1 == 4) ccd_S3D(lam, S[0].v, S[1].v, S[2].v, S[3].v);
    else if (n + 1 == 3) ccd_S2D(lam, S[0].v, S[1].v, S[2].v);
    else if (n + 1 == 2) ccd_S1D(lam, S[0].v, S[1].v);
    else lam[0] = 1;
    n = 0;
    for (int i = 0; i < 4; i++) {
      if (lam[i] == 0) continue;
      S[n] = S[i];
      lam[n++] = lam[i];
    }
    mjtNum nx[3];
    ccd_lincomb(nx, lam, n, S[0].v, S[1].v, S[2].v, S[3].v);
    if (fabs(nx[0] - x[0]) < mjMINVAL && fabs(nx[1] - x[1]) < mjMINVAL &&
        fabs(nx[2] - x[2]) < mjMINVAL) {
      break;
    }
    mju_copy3(x, nx);
    if (n == 4) break;
  }
  ccd_lincomb(st->x1, lam, n, S[0].p1, S[1].p1, S[2].p1, S[3].p1);
  ccd_lincomb(st->x2, lam, n, S[0].p2, S[1].p2, S[2].p2, S[3].p2);
  st->nx = 1;
  st->iters = k;
  st->nsimplex = n;
  st->dist = mju_norm3(x);
}

/*------------------------------- EPA (gjk.c:820-1459) ----------------------------------------*/
typedef struct {
  int vi[3], adj[3];
  mjtNum proj[3], dist;
  int slot;              /* position in the candidate list; -1 not listed; -2 deleted */
} orFace;

typedef struct {
  orVtx* vtx;
  int nvtx;
  orFace* face;
  int nface, maxface;
  int* list;             /* candidate faces (the reference's map) */
  int nlist;
  int* hface;            /* horizon: faces and their edges */
  int* hedge;
  int nh;
  const mjtNum* w;
} orPoly;

static int ccd_addVertex(orPoly* P, const orVtx* v) {
  orVtx* t = P->vtx + P->nvtx;
  mju_copy3(t->p1, v->p1);
  mju_copy3(t->p2, v->p2);
  t->i1 = v->i1;
  t->i2 = v->i2;
  mju_sub3(t->v, v->p1, v->p2);
  return P->nvtx++;
}

/* epaSupport (:328-353) */
static int ccd_newVertex(orPoly* P, orShape* A, orShape* B, const mjtNum d[3],
                         mjtNum dn) {
  mjtNum dir[3] = {1, 0, 0}, ndir[3] = {-1, 0, 0};
  if (dn > mjMINVAL) {
    dir[0] = d[0] / dn;
    dir[1] = d[1] / dn;
    dir[2] = d[2] / dn;
    mju_scl3(ndir, dir, -1);
  }
  ccd_support(P->vtx + P->nvtx, A, B, dir, ndir);
  return P->nvtx++;
}

/* attachFace (:1192-1213) */
static mjtNum ccd_attach(orPoly* P, int a, int b, int c, int j1, int j2, int j3) {
  orFace* f = P->face + P->nface++;
  f->vi[0] = a; f->vi[1] = b; f->vi[2] = c;
  f->adj[0] = j1; f->adj[1] = j2; f->adj[2] = j3;
  if (ccd_projPlane(f->proj, P->vtx[c].v, P->vtx[b].v, P->vtx[a].v)) return 0;
  f->dist = mju_norm3(f->proj);
  f->slot = -1;
  return f->dist;
}

static void ccd_listAll(orPoly* P, int n) {
  for (int i = 0; i < n; i++) {
    P->list[i] = i;
    P->face[i].slot = i;
  }
  P->nlist = n;
}

/* replaceSimplex3 (:820-837) */
static void ccd_toTriangle(orPoly* P, orCCD* st, int a, int b, int c) {
  st->nsimplex = 3;
  const int id[3] = {a, b, c};
  for (int i = 0; i < 3; i++) {
    mju_copy3(st->simplex[i].p1, P->vtx[id[i]].p1);
    mju_copy3(st->simplex[i].p2, P->vtx[id[i]].p2);
    mju_copy3(st->simplex[i].v, P->vtx[id[i]].v);
  }
  P->nface = 0;
  P->nvtx = 0;
}

/* sameSide / testTetra (:842-868) */
static int ccd_sameSide(const mjtNum p0[3], const mjtNum p1[3], const mjtNum p2[3],
                        const mjtNum p3[3]) {
  mjtNum e1[3], e2[3], e3[3], e4[3], n[3];
  mju_sub3(e1, p1, p0);
  mju_sub3(e2, p2, p0);
  mju_cross(n, e1, e2);
  mju_sub3(e3, p3, p0);
  mjtNum d1 = mju_dot3(n, e3);
  mju_scl3(e4, p0, -1);
  mjtNum d2 = mju_dot3(n, e4);
  return (d1 > 0 && d2 > 0) || (d1 < 0 && d2 < 0);
}

static int ccd_inTetra(const mjtNum* a, const mjtNum* b, const mjtNum* c, const mjtNum* d) {
  return ccd_sameSide(a, b, c, d) && ccd_sameSide(b, c, d, a) && ccd_sameSide(c, d, a, b) &&
         ccd_sameSide(d, a, b, c);
}

/* triAffineCoord / triPointIntersect (:976-1035) */
static void ccd_affine(mjtNum lam[3], const mjtNum a[3], const mjtNum b[3], const mjtNum c[3],
                       const mjtNum p[3]) {
  mjtNum M[3];
  int x, y;
  ccd_minors(M, a, b, c);
  mjtNum Mmax = ccd_axes(M, &x, &y);
  lam[0] = ccd_area(p, b, c, x, y) / Mmax;
  lam[1] = ccd_area(p, c, a, x, y) / Mmax;
  lam[2] = ccd_area(p, a, b, x, y) / Mmax;
}

static int ccd_onTriangle(const mjtNum a[3], const mjtNum b[3], const mjtNum c[3],
                          const mjtNum p[3]) {
  mjtNum lam[3], q[3], d[3];
  ccd_affine(lam, a, b, c, p);
  if (lam[0] < 0 || lam[1] < 0 || lam[2] < 0) return 0;
  q[0] = a[0]*lam[0] + b[0]*lam[1] + c[0]*lam[2];
  q[1] = a[1]*lam[0] + b[1]*lam[1] + c[1]*lam[2];
  q[2] = a[2]*lam[0] + b[2]*lam[1] + c[2]*lam[2];
  mju_sub3(d, q, p);
  return mju_norm3(d) < mjMINVAL;
}

/* polytope3 (:1040-1117) */
static int ccd_fromTriangle(orPoly* P, orCCD* st, orShape* A, orShape* B) {
  const mjtNum *a = st->simplex[0].v, *b = st->simplex[1].v, *c = st->simplex[2].v;
  mjtNum e1[3], e2[3], n[3], nn[3];
  mju_sub3(e1, b, a);
  mju_sub3(e2, c, a);
  mju_cross(n, e1, e2);
  mjtNum nrm = mju_norm3(n);
  if (nrm < mjMINVAL) return 4;                        /* mjEPA_P3_BAD_NORMAL */
  mju_scl3(nn, n, -1);
  int i1 = ccd_addVertex(P, st->simplex + 0);
  int i2 = ccd_addVertex(P, st->simplex + 1);
  int i3 = ccd_addVertex(P, st->simplex + 2);
  int i5 = ccd_newVertex(P, A, B, nn, nrm);
  int i4 = ccd_newVertex(P, A, B, n, nrm);
  const mjtNum *v4 = P->vtx[i4].v, *v5 = P->vtx[i5].v;
  if (ccd_onTriangle(a, b, c, v4)) return 5;            /* mjEPA_P3_INVALID_V4 */
  if (ccd_onTriangle(a, b, c, v5)) return 6;            /* mjEPA_P3_INVALID_V5 */
  if (st->dist > 10*mjMINVAL && !ccd_inTetra(a, b, c, v4) && !ccd_inTetra(a, b, c, v5)) {
    return 7;                                          /* mjEPA_P3_MISSING_ORIGIN */
  }
  if (ccd_attach(P, i4, i1, i2, 1, 3, 2) < mjMINVAL) return 8;
  if (ccd_attach(P, i4, i3, i1, 2, 4, 0) < mjMINVAL) return 8;
  if (ccd_attach(P, i4, i2, i3, 0, 5, 1) < mjMINVAL) return 8;
  if (ccd_attach(P, i5, i2, i1, 5, 0, 4) < mjMINVAL) return 8;
  if (ccd_attach(P, i5, i1, i3, 3, 1, 5) < mjMINVAL) return 8;
  if (ccd_attach(P, i5, i3, i2, 4, 2, 3) < mjMINVAL) return 8;   /* mjEPA_P3_ORIGIN_ON_FACE */
  ccd_listAll(P, 6);
  return 0;
}

/* rotmat (:873-887): 120 degrees about axis */
static void ccd_rot120(mjtNum R[9], const mjtNum axis[3]) {
  mjtNum n = mju_norm3(axis);
  mjtNum u1 = axis[0] / n, u2 = axis[1] / n, u3 = axis[2] / n;
  const mjtNum s = 0.86602540378, c = -0.5;
  R[0] = c + u1*u1*(1 - c);
  R[1] = u1*u2*(1 - c) - u3*s;
  R[2] = u1*u3*(1 - c) + u2*s;
  R[3] = u2*u1*(1 - c) + u3*s;
  R[4] = c + u2*u2*(1 - c);
  R[5] = u2*u3*(1 - c) - u1*s;
  R[6] = u1*u3*(1 - c) - u2*s;
  R[7] = u2*u3*(1 - c) + u1*s;
  R[8] = c + u3*u3*(1 - c);
}

/* polytope2 (:892-971) */
static int ccd_fromSegment(orPoly* P, orCCD* st, orShape* A, orShape* B) {
  const mjtNum *a = st->simplex[0].v, *b = st->simplex[1].v;
  mjtNum d[3];
  mju_sub3(d, b, a);
  mjtNum best = mjhipMAXVAL;
  int ix = 0;
  for (int i = 0; i < 3; i++) {
    if (fabs(d[i]) < best) {
      best = fabs(d[i]);
      ix = i;
    }
  }
  mjtNum e[3] = {0, 0, 0}, d1[3], d2[3], d3[3], R[9];
  e[ix] = 1;
  mju_cross(d1, e, d);
  ccd_rot120(R, d);
  mju_mulMatVec3(d2, R, d1);
  mju_mulMatVec3(d3, R, d2);
  int i1 = ccd_addVertex(P, st->simplex + 0);
  int i2 = ccd_addVertex(P, st->simplex + 1);
  int i3 = ccd_newVertex(P, A, B, d1, mju_norm3(d1));
  int i4 = ccd_newVertex(P, A, B, d2, mju_norm3(d2));
  int i5 = ccd_newVertex(P, A, B, d3, mju_norm3(d3));
  const int tri[6][6] = {{i1, i3, i4, 1, 3, 2}, {i1, i5, i3, 2, 4, 0}, {i1, i4, i5, 0, 5, 1},
                         {i2, i4, i3, 5, 0, 4}, {i2, i3, i5, 3, 1, 5}, {i2, i5, i4, 4, 2, 3}};
  for (int f = 0; f < 6; f++) {
    if (ccd_attach(P, tri[f][0], tri[f][1], tri[f][2], tri[f][3], tri[f][4], tri[f][5]) <
        mjMINVAL) {
      ccd_toTriangle(P, st, tri[f][0], tri[f][1], tri[f][2]);
      return ccd_fromTriangle(P, st, A, B);
    }
  }
  const mjtNum *v1 = P->vtx[i1].v, *v2 = P->vtx[i2].v, *v3 = P->vtx[i3].v,
               *v4 = P->vtx[i4].v, *v5 = P->vtx[i5].v;
  if (st->dist > 10*mjMINVAL && !ccd_inTetra(v1, v3, v4, v5) && !ccd_inTetra(v2, v3, v4, v5)) {
    return 2;                                          /* mjEPA_P2_MISSING_ORIGIN */
  }
  ccd_listAll(P, 6);
  return 0;
}

/* polytope4 (:1122-1156) */
static int ccd_fromTetra(orPoly* P, orCCD* st, orShape* A, orShape* B) {
  int i1 = ccd_addVertex(P, st->simplex + 0);
  int i2 = ccd_addVertex(P, st->simplex + 1);
  int i3 = ccd_addVertex(P, st->simplex + 2);
  int i4 = ccd_addVertex(P, st->simplex + 3);
  const int tri[4][6] = {{i1, i2, i3, 1, 3, 2}, {i1, i4, i2, 2, 3, 0}, {i1, i3, i4, 0, 3, 1},
                         {i4, i3, i2, 2, 0, 1}};
  for (int f = 0; f < 4; f++) {
    if (ccd_attach(P, tri[f][0], tri[f][1], tri[f][2], tri[f][3], tri[f][4], tri[f][5]) <
        mjMINVAL) {
      ccd_toTriangle(P, st, tri[f][0], tri[f][1], tri[f][2]);
      return ccd_fromTriangle(P, st, A, B);
    }
  }
  if (!ccd_inTetra(P->vtx[i1].v, P->vtx[i2].v, P->vtx[i3].v, P->vtx[i4].v)) return 9;
  ccd_listAll(P, 4);
  return 0;
}

/* deleteFace (:1174-1180) */
static void ccd_unlist(orPoly* P, int f) {
  orFace* F = P->face + f;
  if (F->slot >= 0) {
    P->list[F->slot] = P->list[--P->nlist];
    P->face[P->list[F->slot]].slot = F->slot;
  }
  F->slot = -2;
}

static int ccd_edgeOf(const orFace* F, int v) {
  if (F->vi[0] == v) return 0;
  if (F->vi[1] == v) return 1;
  return 2;
}

/* horizonRec (:1246-1267) */
static int ccd_visible(orPoly* P, int f, int e) {
  orFace* F = P->face + f;
  mjtNum d2 = F->dist*F->dist;
  if (mju_dot3(F->proj, P->w) >= d2) {
    ccd_unlist(P, f);
    for (int k = 1; k < 3; k++) {
      int i = (e + k) % 3;
      int g = F->adj[i];
      if (P->face[g].slot > -2) {
        int ge = ccd_edgeOf(P->face + g, F->vi[(i + 1) % 3]);
        if (!ccd_visible(P, g, ge)) {
          P->hface[P->nh] = g;
          P->hedge[P->nh++] = ge;
        }
      }
    }
    return 1;
  }
  return 0;
}

/* horizon (:1272-1295) */
static void ccd_horizon(orPoly* P, int f) {
  ccd_unlist(P, f);
  const orFace* F = P->face + f;
  for (int k = 0; k < 3; k++) {
    int g = F->adj[k];
    int ge = ccd_edgeOf(P->face + g, F->vi[(k + 1) % 3]);
    if ((k == 0 || P->face[g].slot > -2) && !ccd_visible(P, g, ge)) {
      P->hface[P->nh] = g;
      P->hedge[P->nh++] = ge;
    }
  }
}

/* epa (:1329-1459) + epaWitness (:1300-1323); returns the face or -1 */
static int ccd_epa(orCCD* st, orPoly* P, orShape* A, orShape* B) {
  mjtNum lower, upper = FLT_MAX;
  int f = -1, pf = -1, k;
  P->nh = 0;
  for (k = 0; k < st->kmax; k++) {
    pf = f;
    lower = FLT_MAX;
    for (int i = 0; i < P->nlist; i++) {
      if (P->face[P->list[i]].dist < lower) {
        f = P->list[i];
        lower = P->face[f].dist;
      }
    }
    if (lower > upper || f < 0) {
      f = pf;
      break;
    }
    if (lower <= 0) break;                              /* warning: origin on a face */
    orFace* F = P->face + f;
    int wi = ccd_newVertex(P, A, B, F->proj, lower);
    const mjtNum* w = P->vtx[wi].v;
    mjtNum up = mju_dot3(F->proj, w) / lower;
    if (up < upper) upper = up;
    if (upper - lower < st->tol) break;
    P->w = w;
    ccd_horizon(P, f);
    if (P->nh < 3) {
      f = -1;
      break;
    }
    const int nf = P->nface, ne = P->nh;
    if (ne > P->maxface - P->nface) break;              /* warning: out of face memory */
    for (int i = 0; i < ne; i++) {
      const int cur = nf + i, prev = i ? cur - 1 : nf + ne - 1, next = nf + (i + 1) % ne;
      orFace* H = P->face + P->hface[i];
      const int e = P->hedge[i];
      const int a = H->vi[e], b = H->vi[(e + 1) % 3];
      H->adj[e] = cur;
      mjtNum dd = ccd_attach(P, wi, b, a, prev, P->hface[i], next);
      if (dd == 0) {
        f = -1;
        break;
      }
      if (dd >= lower && dd <= upper) {
        int s = P->nlist++;
        P->list[s] = P->nface - 1;
        P->face[P->nface - 1].slot = s;
      }
    }
    P->nh = 0;
    if (!P->nlist || f < 0) break;
  }
  if (f >= 0) {
    const orFace* F = P->face + f;
    mjtNum lam[3];
    ccd_affine(lam, P->vtx[F->vi[0]].v, P->vtx[F->vi[1]].v, P->vtx[F->vi[2]].v, F->proj);
    const mjtNum *a1 = P->vtx[F->vi[0]].p1, *b1 = P->vtx[F->vi[1]].p1, *c1 = P->vtx[F->vi[2]].p1;
    const mjtNum *a2 = P->vtx[F->vi[0]].p2, *b2 = P->vtx[F->vi[1]].p2, *c2 = P->vtx[F->vi[2]].p2;
    for (int i = 0; i < 3; i++) {
      st->x1[i] = a1[i]*lam[0] + b1[i]*lam[1] + c1[i]*lam[2];
      st->x2[i] = a2[i]*lam[0] + b2[i]*lam[1] + c2[i]*lam[2];
    }
    st->nx = 1;
    st->dist = -F->dist;
  } else {
    st->nx = 0;
    st->dist = 0;
  }
  return f;
}

/* mjc_ccd (:2215-2343) with max_contacts = 1 and the distance cutoff `cutoff` (0 for contacts,
 * mjc_Convex; the distance bound for mj_geomDistanceCCD); the geoms' margins are in
 * A->margin / B->margin */
/* obj->center: the geom position (mjc_center :78-98), or a prism's mean vertex
   (mjc_prism_center :103-110) */
static void ccd_center(mjtNum c[3], const orShape* s) {
  if (s->gtype == mjhipGEOM_HFIELD) {
    mju_zero3(c);
    for (int i = 0; i < 6; i++) mju_addTo3(c, s->prism[i]);
    mju_scl3(c, c, 1.0/6.0);
  } else {
    mju_copy3(c, s->pos);
  }
}

/*------------------ multicontact (engine_collision_gjk.c:1460-2193) ------------------------
 * With max_contacts > 1 the EPA's final face is turned into a contact polygon: the feature
 * (vertex, edge or face) of each geom the face's three vertices span, the geoms' face normals
 * around it, a pair of anti-aligned faces (or an edge perpendicular to a face), and the
 * clipping of one face polygon by the other, for boxes and meshes (the mesh polygons of
 * mjCMesh::MakePolygons, meshes.py make_polygons). */
#define OR_FACE_TOL 0.99999872      /* mjFACE_TOL (gjk.h:29) */
#define OR_EDGE_TOL 0.00159999931   /* mjEDGE_TOL (gjk.h:32) */
#define OR_MAX_POLYVERT 150         /* mjMAX_POLYVERT (gjk.h:35) */

static mjtNum mc_dot3(const mjtNum a[3], const mjtNum b[3]) {
  return a[0]*b[0] + a[1]*b[1] + a[2]*b[2];
}

/* equal3 (:116-120) */
static int mc_equal3(const mjtNum a[3], const mjtNum b[3]) {
  return fabs(a[0] - b[0]) < mjMINVAL && fabs(a[1] - b[1]) < mjMINVAL &&
         fabs(a[2] - b[2]) < mjMINVAL;
}

/* area4 (:1463-1476) */
static mjtNum mc_area4(const mjtNum a[3], const mjtNum b[3], const mjtNum c[3],
                       const mjtNum d[3]) {
  mjtNum ad[3] = {d[0] - a[0], d[1] - a[1], d[2] - a[2]};
  mjtNum db[3] = {b[0] - d[0], b[1] - d[1], b[2] - d[2]};
  mjtNum bc[3] = {c[0] - b[0], c[1] - b[1], c[2] - b[2]};
  mjtNum ca[3] = {a[0] - c[0], a[1] - c[1], a[2] - c[2]};
  mjtNum e[3], f[3], g[3];
  mju_cross(e, ad, db);
  mju_cross(f, bc, ca);
  mju_add3(g, e, f);
  return 0.5 * sqrt(mc_dot3(g, g));
}

/* next (:1481-1486), on vertex indices */
static int mc_next(int nvert, int i) { return i == nvert - 1 ? 0 : i + 1; }

/* polygonQuad (:1491-1535): the maximum-area quadrilateral, as vertex indices */
static void mc_polygonQuad(int res[4], const mjtNum* poly, int nvert) {
  int a = 0, b = 1, c = 2, d = 3;
  res[0] = a; res[1] = b; res[2] = c; res[3] = d;
  mjtNum m = mc_area4(poly + 3*a, poly + 3*b, poly + 3*c, poly + 3*d), mn;
  for (; a < nvert; a++) {
    while (1) {
      mn = mc_area4(poly + 3*a, poly + 3*b, poly + 3*c, poly + 3*mc_next(nvert, d));
      if (mn <= m) break;
      m = mn;
      d = mc_next(nvert, d);
      res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      while (1) {
        mn = mc_area4(poly + 3*a, poly + 3*b, poly + 3*mc_next(nvert, c), poly + 3*d);
        if (mn <= m) break;
        m = mn;
        c = mc_next(nvert, c);
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
      while (1) {
        mn = mc_area4(poly + 3*a, poly + 3*mc_next(nvert, b), poly + 3*c, poly + 3*d);
        if (mn <= m) break;
        m = mn;
        b = mc_next(nvert, b);
        res[0] = a; res[1] = b; res[2] = c; res[3] = d;
      }
    }
    if (b == a) {
      b = mc_next(nvert, b);
      if (c == b) {
        c = mc_next(nvert, c);
        if (d == c) d = mc_next(nvert, d);
      }
    }
  }
}

/* planeNormal (:1540-1549) */
static mjtNum mc_planeNormal(mjtNum res[3], const mjtNum v1[3], const mjtNum v2[3],
                             const mjtNum n[3]) {
  mjtNum v3[3], d1[3], d2[3];
  mju_add3(v3, v1, n);
  mju_sub3(d1, v2, v1);
  mju_sub3(d2, v3, v1);
  mju_cross(res, d1, d2);
  return mc_dot3(res, v1);
}

/* halfspace (:1553-1557) */
static int mc_halfspace(const mjtNum a[3], const mjtNum n[3], const mjtNum p[3]) {
  mjtNum diff[3] = {p[0] - a[0], p[1] - a[1], p[2] - a[2]};
  return mc_dot3(diff, n) > 0;
}

/* planeIntersect (:1561-1574) */
static mjtNum mc_planeIntersect(mjtNum res[3], const mjtNum pn[3], mjtNum pd, const mjtNum a[3],
                                const mjtNum b[3]) {
  mjtNum ab[3];
  mju_sub3(ab, b, a);
  mjtNum temp = mc_dot3(pn, ab);
  if (temp == 0.0) return mjhipMAXVAL;
  mjtNum t = (pd - mc_dot3(pn, a)) / temp;
  if (t >= 0.0 && t <= 1.0) {
    res[0] = a[0] + t*ab[0];
    res[1] = a[1] + t*ab[1];
    res[2] = a[2] + t*ab[2];
  }
  return t;
}

/* polygonClip (:1579-1690): face2 clipped by the edge planes of face1 (normal n); the
   vertices become the contacts' x2, x1 = x2 - dir */
static void mc_polygonClip(orCCD* st, const mjtNum* face1, int nface1, const mjtNum* face2,
                           int nface2, const mjtNum n[3], const mjtNum dir[3]) {
  if (nface1 < 3) return;
  mjtNum pn[3*OR_MAX_POLYVERT], pd[OR_MAX_POLYVERT];
  for (int i = 0; i < nface1 - 1; i++) {
    pd[i] = mc_planeNormal(pn + 3*i, face1 + 3*i, face1 + 3*i + 3, n);
  }
  pd[nface1 - 1] = mc_planeNormal(pn + 3*(nface1 - 1), face1 + 3*(nface1 - 1), face1, n);
  mjtNum buf1[6*OR_MAX_POLYVERT], buf2[6*OR_MAX_POLYVERT];
  mjtNum *polygon = buf1, *clipped = buf2;
  int npolygon = nface2, nclipped = 0;
  for (int i = 0; i < nface2; i++) mju_copy3(polygon + 3*i, face2 + 3*i);
  for (int e = 0; e < 3*nface1; e += 3) {
    for (int i = 0; i < npolygon; i++) {
      mjtNum* P = polygon + 3*i;
      mjtNum* Q = (i < npolygon - 1) ? polygon + 3*(i + 1) : polygon;
      int in1 = mc_halfspace(face1 + e, pn + e, P);
      int in2 = mc_halfspace(face1 + e, pn + e, Q);
      if (!in1 && !in2) continue;
      if (in1 && in2) {
        mju_copy3(clipped + 3*nclipped++, Q);
        continue;
      }
      mjtNum t = mc_planeIntersect(clipped + 3*nclipped++, pn + e, pd[e/3], P, Q);
      if (t < 0.0 || t > 1.0) nclipped--;
      if (in2) mju_copy3(clipped + 3*nclipped++, Q);
    }
    mjtNum* tmp = polygon;
    polygon = clipped;
    clipped = tmp;
    npolygon = nclipped;
    nclipped = 0;
  }
  if (npolygon < 1) return;
  if (st->maxc < 5 && npolygon > 4) {
    int rect[4];
    mc_polygonQuad(rect, polygon, npolygon);
    st->nx = 4;
    for (int i = 0; i < 4; i++) {
      mju_copy3(st->x2 + 3*i, polygon + 3*rect[i]);
      mju_sub3(st->x1 + 3*i, st->x2 + 3*i, dir);
    }
    return;
  }
  if (npolygon > OR_MAXCONPAIR) {
    st->nx = OR_MAXCONPAIR;
    for (int i = 0; i < 3*OR_MAXCONPAIR; i += 3) {
      mju_copy3(st->x2 + i, polygon + i);
      mju_sub3(st->x1 + i, st->x2 + i, dir);
    }
    return;
  }
  int k = 0;
  for (int i = 0; i < 3*npolygon; i += 3) {
    int skip = 0;
    for (int j = 0; j < k; j += 3) {
      if (mc_equal3(st->x2 + j, polygon + i)) {
        skip = 1;
        break;
      }
    }
    if (skip) continue;
    mju_copy3(st->x2 + k, polygon + i);
    mju_sub3(st->x1 + k, st->x2 + k, dir);
    k += 3;
  }
  st->nx = k/3;
}

/* globalcoord (:1695-1707) */
static void mc_global(mjtNum res[3], const mjtNum* mat, const mjtNum* pos, mjtNum l1, mjtNum l2,
                      mjtNum l3) {
  res[0] = mat[0]*l1 + mat[1]*l2 + mat[2]*l3;
  res[1] = mat[3]*l1 + mat[4]*l2 + mat[5]*l3;
  res[2] = mat[6]*l1 + mat[7]*l2 + mat[8]*l3;
  if (pos) {
    res[0] += pos[0];
    res[1] += pos[1];
    res[2] += pos[2];
  }
}

/* intersect (:1711-1723): up to 2 common entries of two arrays */
static int mc_intersect(int res[2], const int* a, const int* b, int n, int m) {
  int count = 0;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < m; j++) {
      if (a[i] == b[j]) {
        res[count++] = a[i];
        if (count == 2) return 2;
      }
    }
  }
  return count;
}

/* meshNormals (:1727-1792): the normals of the mesh polygons through the feature's vertices */
static int mc_meshNormals(mjtNum* res, int* resind, int dim, const orShape* s, int v1, int v2,
                          int v3) {
  const mjhipModel* m = s->model;
  const int polyadr = m->mesh_polyadr[s->meshid], vertadr = m->mesh_vertadr[s->meshid];
  const mjtNum* mat = s->mat;
  if (dim == 3) {
    const int a1 = m->mesh_polymapadr[vertadr + v1], n1 = m->mesh_polymapnum[vertadr + v1];
    const int a2 = m->mesh_polymapadr[vertadr + v2], n2 = m->mesh_polymapnum[vertadr + v2];
    const int a3 = m->mesh_polymapadr[vertadr + v3], n3 = m->mesh_polymapnum[vertadr + v3];
    int edgeset[2], faceset[2];
    int n = mc_intersect(edgeset, m->mesh_polymap + a1, m->mesh_polymap + a2, n1, n2);
    if (n == 0) return 0;
    n = mc_intersect(faceset, edgeset, m->mesh_polymap + a3, n, n3);
    if (n == 0) return 0;
    const mjtNum* nrm = m->mesh_polynormal + 3*(polyadr + faceset[0]);
    mc_global(res, mat, NULL, nrm[0], nrm[1], nrm[2]);
    resind[0] = faceset[0];
    return 1;
  }
  if (dim == 2) {
    const int a1 = m->mesh_polymapadr[vertadr + v1], n1 = m->mesh_polymapnum[vertadr + v1];
    const int a2 = m->mesh_polymapadr[vertadr + v2], n2 = m->mesh_polymapnum[vertadr + v2];
    int edgeset[2];
    const int n = mc_intersect(edgeset, m->mesh_polymap + a1, m->mesh_polymap + a2, n1, n2);
    for (int i = 0; i < n; i++) {
      const mjtNum* nrm = m->mesh_polynormal + 3*(polyadr + edgeset[i]);
      mc_global(res + 3*i, mat, NULL, nrm[0], nrm[1], nrm[2]);
      resind[i] = edgeset[i];
    }
    return n;
  }
  if (dim == 1) {
    const int a1 = m->mesh_polymapadr[vertadr + v1];
    int n1 = m->mesh_polymapnum[vertadr + v1];
    if (n1 > OR_MAX_POLYVERT) n1 = OR_MAX_POLYVERT;
    for (int i = 0; i < n1; i++) {
      const int index = m->mesh_polymap[a1 + i];
      const mjtNum* nrm = m->mesh_polynormal + 3*(polyadr + index);
      mc_global(res + 3*i, mat, NULL, nrm[0], nrm[1], nrm[2]);
      resind[i] = index;
    }
    return n1;
  }
  return 0;
}

/* meshEdgeNormals (:1796-1842): the directions of the mesh edges from the feature's vertex.
   As in the reference, the edge's other end is read at the polygon-local position k of the
   previous vertex (verts + 3k), not at that vertex's id. */
static int mc_meshEdgeNormals(mjtNum* res, mjtNum* endverts, int dim, const orShape* s,
                              const mjtNum v1[3], const mjtNum v2[3], int v1i) {
  if (dim == 2) {
    mju_copy3(endverts, v2);
    mju_sub3(res, v2, v1);
    mju_normalize3(res);
    return 1;
  }
  if (dim == 1) {
    const mjhipModel* m = s->model;
    const int polyadr = m->mesh_polyadr[s->meshid], vertadr = m->mesh_vertadr[s->meshid];
    const int a1 = m->mesh_polymapadr[vertadr + v1i];
    int n1 = m->mesh_polymapnum[vertadr + v1i];
    if (n1 > OR_MAX_POLYVERT) n1 = OR_MAX_POLYVERT;
    for (int i = 0; i < n1; i++) {
      const int idx = m->mesh_polymap[a1 + i];
      const int adr = m->mesh_polyvertadr[polyadr + idx];
      const int nvert = m->mesh_polyvertnum[polyadr + idx];
      for (int j = 0; j < nvert; j++) {
        if (m->mesh_polyvert[adr + j] == v1i) {
          const float* verts = m->mesh_vert + 3*vertadr;
          const int k = j == 0 ? nvert - 1 : j - 1;
          const float* vert = verts + 3*k;
          mc_global(endverts + 3*i, s->mat, s->pos, vert[0], vert[1], vert[2]);
          mju_sub3(res + 3*i, endverts + 3*i, v1);
          mju_normalize3(res + 3*i);
        }
      }
    }
    return n1;
  }
  return 0;
}

/* meshFace (:1994-2015): polygon idx's vertices, in reverse order, in the global frame */
static int mc_meshFace(mjtNum* res, const orShape* s, int idx) {
  const mjhipModel* m = s->model;
  const int polyadr = m->mesh_polyadr[s->meshid], vertadr = m->mesh_vertadr[s->meshid];
  const int adr = m->mesh_polyvertadr[polyadr + idx];
  int nvert = m->mesh_polyvertnum[polyadr + idx], j = 0;
  if (nvert > OR_MAX_POLYVERT) nvert = OR_MAX_POLYVERT;
  for (int i = nvert - 1; i >= 0; i--) {
    const float* vert = m->mesh_vert + 3*vertadr + 3*m->mesh_polyvert[adr + i];
    mc_global(res + 3*j++, s->mat, s->pos, vert[0], vert[1], vert[2]);
  }
  return nvert;
}

/* boxNormals (:1846-1899) */
static int mc_boxNormals(mjtNum res[9], int resind[3], int dim, const orShape* s, int v1, int v2,
                         int v3) {
  const mjtNum* mat = s->mat;
  if (dim == 3) {
    int x = ((v1 & 1) && (v2 & 1) && (v3 & 1)) - (!(v1 & 1) && !(v2 & 1) && !(v3 & 1));
    int y = ((v1 & 2) && (v2 & 2) && (v3 & 2)) - (!(v1 & 2) && !(v2 & 2) && !(v3 & 2));
    int z = ((v1 & 4) && (v2 & 4) && (v3 & 4)) - (!(v1 & 4) && !(v2 & 4) && !(v3 & 4));
    mc_global(res, mat, NULL, x, y, z);
    int sgn = x + y + z;
    if (x) resind[0] = 0;
    if (y) resind[0] = 2;
    if (z) resind[0] = 4;
    if (sgn == -1) resind[0]++;
    return 1;
  }
  if (dim == 2) {
    int x = ((v1 & 1) && (v2 & 1)) - (!(v1 & 1) && !(v2 & 1));
    int y = ((v1 & 2) && (v2 & 2)) - (!(v1 & 2) && !(v2 & 2));
    int z = ((v1 & 4) && (v2 & 4)) - (!(v1 & 4) && !(v2 & 4));
    if (x) {
      mc_global(res, mat, NULL, x, 0, 0);
      resind[0] = (x > 0) ? 0 : 1;
    }
    if (y) {
      int i = (x ? 1 : 0);
      mc_global(res + 3*i, mat, NULL, 0, y, 0);
      resind[i] = (y > 0) ? 2 : 3;
    }
    if (z) {
      mc_global(res + 3, mat, NULL, 0, 0, z);
      resind[1] = (z > 0) ? 4 : 5;
    }
    return 2;
  }
  if (dim == 1) {
    mjtNum x = (v1 & 1) ? 1 : -1, y = (v1 & 2) ? 1 : -1, z = (v1 & 4) ? 1 : -1;
    mc_global(res + 0, mat, NULL, x, 0, 0);
    mc_global(res + 3, mat, NULL, 0, y, 0);
    mc_global(res + 6, mat, NULL, 0, 0, z);
    resind[0] = (x > 0) ? 0 : 1;
    resind[1] = (y > 0) ? 2 : 3;
    resind[2] = (z > 0) ? 4 : 5;
    return 3;
  }
  return 0;
}

/* boxEdgeNormals (:1903-1938) */
static int mc_boxEdgeNormals(mjtNum res[9], mjtNum endverts[9], int dim, const orShape* s,
                             const mjtNum v1[3], const mjtNum v2[3], int v1i) {
  const mjtNum *mat = s->mat, *pos = s->pos, *size = s->size;
  if (dim == 2) {
    mju_copy3(endverts, v2);
    mju_sub3(res, v2, v1);
    mju_normalize3(res);
    return 1;
  }
  if (dim == 1) {
    mjtNum x = (v1i & 1) ? size[0] : -size[0];
    mjtNum y = (v1i & 2) ? size[1] : -size[1];
    mjtNum z = (v1i & 4) ? size[2] : -size[2];
    mc_global(endverts, mat, pos, -x, y, z);
    mju_sub3(res, endverts, v1);
    mju_normalize3(res);
    mc_global(endverts + 3, mat, pos, x, -y, z);
    mju_sub3(res + 3, endverts + 3, v1);
    mju_normalize3(res + 3);
    mc_global(endverts + 6, mat, pos, x, y, -z);
    mju_sub3(res + 6, endverts + 6, v1);
    mju_normalize3(res + 6);
    return 3;
  }
  return 0;
}

/* boxFace (:1942-1990) */
static int mc_boxFace(mjtNum res[12], const orShape* s, int idx) {
  const mjtNum *mat = s->mat, *pos = s->pos, *z = s->size;
  static const signed char corner[6][4][3] = {
    {{ 1,  1,  1}, { 1,  1, -1}, { 1, -1, -1}, { 1, -1,  1}},     /* right */
    {{-1,  1, -1}, {-1,  1,  1}, {-1, -1,  1}, {-1, -1, -1}},     /* left */
    {{-1,  1, -1}, { 1,  1, -1}, { 1,  1,  1}, {-1,  1,  1}},     /* top */
    {{-1, -1,  1}, { 1, -1,  1}, { 1, -1, -1}, {-1, -1, -1}},     /* bottom */
    {{-1,  1,  1}, { 1,  1,  1}, { 1, -1,  1}, {-1, -1,  1}},     /* front */
    {{ 1,  1, -1}, {-1,  1, -1}, {-1, -1, -1}, { 1, -1, -1}}};    /* back */
  if (idx < 0 || idx > 5) return 0;
  for (int k = 0; k < 4; k++) {
    const signed char* c = corner[idx][k];
    mc_global(res + 3*k, mat, pos, c[0] > 0 ? z[0] : -z[0], c[1] > 0 ? z[1] : -z[1],
              c[2] > 0 ? z[2] : -z[2]);
  }
  return 4;
}

/* alignedFaces (:2019-2031) */
static int mc_alignedFaces(int res[2], const mjtNum* v, int nv, const mjtNum* w, int nw) {
  for (int i = 0; i < nv; i++) {
    for (int j = 0; j < nw; j++) {
      if (mc_dot3(v + 3*i, w + 3*j) < -OR_FACE_TOL) {
        res[0] = i;
        res[1] = j;
        return 1;
      }
    }
  }
  return 0;
}

/* alignedFaceEdge (:2036-2048) */
static int mc_alignedFaceEdge(int res[2], const mjtNum* edge, int nedge, const mjtNum* face,
                              int nface) {
  for (int i = 0; i < nface; i++) {
    for (int j = 0; j < nedge; j++) {
      if (fabs(mc_dot3(edge + 3*j, face + 3*i)) < OR_EDGE_TOL) {
        res[0] = j;
        res[1] = i;
        return 1;
      }
    }
  }
  return 0;
}

/* simplexDim (:2052-2067) */
static int mc_simplexDim(int* v1i, int* v2i, int* v3i, const mjtNum** v1, const mjtNum** v2,
                         const mjtNum** v3) {
  int a = *v1i, b = *v2i, c = *v3i;
  if (a != b) return (c == a || c == b) ? 2 : 3;
  if (a != c) {
    *v2i = *v3i;
    *v2 = *v3;
    return 2;
  }
  return 1;
}

/* multicontact (:2071-2193) */
static void ccd_multicontact(orCCD* st, const orPoly* P, int f, const orShape* A,
                             const orShape* B) {
  const orFace* F = P->face + f;
  const orVtx *p0 = P->vtx + F->vi[0], *p1 = P->vtx + F->vi[1], *p2 = P->vtx + F->vi[2];
  int v11i = p0->i1, v12i = p1->i1, v13i = p2->i1;
  int v21i = p0->i2, v22i = p1->i2, v23i = p2->i2;
  const mjtNum *v11 = p0->p1, *v12 = p1->p1, *v13 = p2->p1;
  const mjtNum *v21 = p0->p2, *v22 = p1->p2, *v23 = p2->p2;
  int nface1 = mc_simplexDim(&v11i, &v12i, &v13i, &v11, &v12, &v13);
  int nface2 = mc_simplexDim(&v21i, &v22i, &v23i, &v21, &v22, &v23);
  int nn1 = 0, nn2 = 0, idx1[OR_MAX_POLYVERT], idx2[OR_MAX_POLYVERT];
  mjtNum n1[3*OR_MAX_POLYVERT], n2[3*OR_MAX_POLYVERT], endverts[3*OR_MAX_POLYVERT];
  mjtNum face1[3*OR_MAX_POLYVERT], face2[3*OR_MAX_POLYVERT];
  if (A->gtype == mjhipGEOM_BOX) nn1 = mc_boxNormals(n1, idx1, nface1, A, v11i, v12i, v13i);
  else if (A->gtype == mjhipGEOM_MESH) {
    nn1 = mc_meshNormals(n1, idx1, nface1, A, v11i, v12i, v13i);
  }
  if (B->gtype == mjhipGEOM_BOX) nn2 = mc_boxNormals(n2, idx2, nface2, B, v21i, v22i, v23i);
  else if (B->gtype == mjhipGEOM_MESH) {
    nn2 = mc_meshNormals(n2, idx2, nface2, B, v21i, v22i, v23i);
  }
  int res[2], edgecon1 = 0, edgecon2 = 0;
  if (!mc_alignedFaces(res, n1, nn1, n2, nn2)) {
    if (nface1 < 3 && nface1 <= nface2) {
      nn1 = 0;
      if (A->gtype == mjhipGEOM_BOX) {
        nn1 = mc_boxEdgeNormals(n1, endverts, nface1, A, v11, v12, v11i);
      } else if (A->gtype == mjhipGEOM_MESH) {
        nn1 = mc_meshEdgeNormals(n1, endverts, nface1, A, v11, v12, v11i);
      }
      if (!mc_alignedFaceEdge(res, n1, nn1, n2, nn2)) return;
      edgecon1 = 1;
    } else if (nface2 < 3) {
      nn2 = 0;
      if (B->gtype == mjhipGEOM_BOX) {
        nn2 = mc_boxEdgeNormals(n2, endverts, nface2, B, v21, v22, v21i);
      } else if (B->gtype == mjhipGEOM_MESH) {
        nn2 = mc_meshEdgeNormals(n2, endverts, nface2, B, v21, v22, v21i);
      }
      if (!mc_alignedFaceEdge(res, n2, nn2, n1, nn1)) return;
      edgecon2 = 1;
    } else {
      return;
    }
  }
  int i = res[0], j = res[1];
  if (edgecon1) {
    mju_copy3(face1, p0->p1);
    mju_copy3(face1 + 3, endverts + 3*i);
    nface1 = 2;
  } else {
    const int ind = edgecon2 ? idx1[j] : idx1[i];
    nface1 = A->gtype == mjhipGEOM_BOX ? mc_boxFace(face1, A, ind) : mc_meshFace(face1, A, ind);
  }
  if (edgecon2) {
    mju_copy3(face2, p0->p2);
    mju_copy3(face2 + 3, endverts + 3*i);
    nface2 = 2;
  } else {
    nface2 = B->gtype == mjhipGEOM_BOX ? mc_boxFace(face2, B, idx2[j])
                                       : mc_meshFace(face2, B, idx2[j]);
  }
  mjtNum diff[3], dir[3];
  mju_sub3(diff, st->x2, st->x1);
  const mjtNum nd = sqrt(mc_dot3(diff, diff));
  if (edgecon1) {
    mju_scl3(dir, n2 + 3*j, nd);
    mc_polygonClip(st, face2, nface2, face1, nface1, n2 + 3*j, dir);
    return;
  }
  if (edgecon2) {
    mju_scl3(dir, n1 + 3*j, -nd);
    mc_polygonClip(st, face1, nface1, face2, nface2, n1 + 3*j, dir);
    return;
  }
  mju_scl3(dir, n2 + 3*j, nd);
  mc_polygonClip(st, face1, nface1, face2, nface2, n1 + 3*i, dir);
}

static mjtNum or_ccd(orCCD* st, orShape* A, orShape* B, int kmax, mjtNum tol, mjtNum cutoff,
                     int maxc) {
  ccd_center(st->x1, A);
  ccd_center(st->x2, B);
  st->iters = 0;
  st->tol = tol;
  st->kmax = kmax;
  st->maxc = maxc;
  st->unsupported = 0;
  st->cutoff = cutoff;
  const int shrinkA = A->gtype == mjhipGEOM_SPHERE || A->gtype == mjhipGEOM_CAPSULE;
  const int shrinkB = B->gtype == mjhipGEOM_SPHERE || B->gtype == mjhipGEOM_CAPSULE;
  if (shrinkA || shrinkB) {
    mjtNum full1 = 0, full2 = 0, m1 = A->margin, m2 = B->margin;
    if (shrinkA) {
      full1 = A->size[0] + 0.5*m1;
      A->kind = A->gtype == mjhipGEOM_SPHERE ? CCD_POINT : CCD_LINE;
      A->margin = 0;
    }
    if (shrinkB) {
      full2 = B->size[0] + 0.5*m2;
      B->kind = B->gtype == mjhipGEOM_SPHERE ? CCD_POINT : CCD_LINE;
      B->margin = 0;
    }
    st->cutoff += full1 + full2;
    ccd_gjk(st, A, B);
    st->cutoff = cutoff;
    A->margin = m1;
    B->margin = m2;
    A->kind = A->gtype;
    B->kind = B->gtype;
    if (st->dist > st->tol) {               /* shallow: inflate (:2195-2210) */
      mjtNum n[3];
      mju_sub3(n, st->x2, st->x1);
      mju_normalize3(n);
      if (full1) {
        st->x1[0] += full1*n[0];
        st->x1[1] += full1*n[1];
        st->x1[2] += full1*n[2];
      }
      if (full2) {
        st->x2[0] -= full2*n[0];
        st->x2[1] -= full2*n[1];
        st->x2[2] -= full2*n[2];
      }
      st->dist -= (full1 + full2);
      if (st->dist > st->cutoff) st->dist = mjhipMAXVAL;
      return st->dist;
    }
    if (!maxc) {                            /* contact not needed (:2267-2272) */
      st->nx = 0;
      st->dist = 0;
      return 0;
    }
    st->iters = 0;
    ccd_center(st->x1, A);
    ccd_center(st->x2, B);
  }
  ccd_gjk(st, A, B);
  if (!maxc) return st->dist;               /* penetration recovery not needed (:2280-2283) */
  if (st->dist <= tol && st->nsimplex > 1) {
    st->dist = 0;
    const int N = kmax;
    orPoly P;
    P.maxface = 6*N > 1000 ? 6*N : 1000;
    P.vtx = (orVtx*)malloc(sizeof(orVtx)*(5 + N));
    P.face = (orFace*)malloc(sizeof(orFace)*P.maxface);
    P.list = (int*)malloc(sizeof(int)*P.maxface);
    P.hface = (int*)malloc(sizeof(int)*(6 + N));
    P.hedge = (int*)malloc(sizeof(int)*(6 + N));
    P.nvtx = P.nface = P.nlist = P.nh = 0;
    int ret = st->nsimplex == 2 ? ccd_fromSegment(&P, st, A, B) :
              st->nsimplex == 3 ? ccd_fromTriangle(&P, st, A, B) : ccd_fromTetra(&P, st, A, B);
    if (!ret) {
      const int f = ccd_epa(st, &P, A, B);
      if (maxc > 1 && f >= 0) ccd_multicontact(st, &P, f, A, B);
    }
    free(P.vtx);
    free(P.face);
    free(P.list);
    free(P.hface);
    free(P.hedge);
  }
  return st->dist;
}

static void or_shape(orShape* s, const mjhipModel* m, const mjhipData* d, int g, mjtNum margin) {
  s->kind = s->gtype = m->geom_type[g];
  s->pos = d->geom_xpos + 3*g;
  s->mat = d->geom_xmat + 9*g;
  s->size = m->geom_size + 3*g;
  s->margin = margin;
  s->vert = NULL;
  s->graph = NULL;
  s->nvert = 0;
  s->vertindex = s->meshindex = -1;
  s->model = m;
  s->meshid = -1;
  if (s->gtype == mjhipGEOM_MESH) {
    const int id = m->geom_dataid[g];
    s->meshid = id;
    s->vert = m->mesh_vert + 3*m->mesh_vertadr[id];
    s->nvert = m->mesh_vertnum[id];
    s->graph = m->mesh_graphadr[id] >= 0 ? m->mesh_graph + m->mesh_graphadr[id] : NULL;
  }
}

/* mjc_CCDIteration (convex.c:792-819), native solver, one contact, on the shapes' current
 * frames */
static int col_ccdIteration(orRaw* c, const mjhipModel* m, orShape* A, orShape* B,
                            mjtNum margin) {
  orCCD st;
  mjtNum dist = or_ccd(&st, A, B, m->opt.ccd_iterations, m->opt.ccd_tolerance, 0, 1);
  if (!(dist < 0) || st.nx < 1) return 0;
  c->dist = margin + dist;
  mju_sub3(c->frame, st.x1, st.x2);
  mju_normalize3(c->frame);
  c->pos[0] = 0.5*(st.x1[0] + st.x2[0]);
  c->pos[1] = 0.5*(st.x1[1] + st.x2[1]);
  c->pos[2] = 0.5*(st.x1[2] + st.x2[2]);
  mju_zero3(c->frame + 3);
  return 1;
}

static mjtNum mju_dist3(const mjtNum a[3], const mjtNum b[3]);

/* mju_mulMatMat3 (engine_util_blas.c:193-203) */
static void mju_mulMatMat3(mjtNum r[9], const mjtNum a[9], const mjtNum b[9]) {
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) {
      r[3*i+j] = a[3*i]*b[j] + a[3*i+1]*b[3+j] + a[3*i+2]*b[6+j];
    }
  }
}

/* mju_rotateFrame (convex.c:862-880): the frame rotated by rot about origin */
static void or_rotateFrame(const mjtNum origin[3], const mjtNum rot[9], mjtNum xmat[9],
                           mjtNum xpos[3]) {
  mjtNum mat[9], vec[3], rel[3];
  mju_mulMatMat3(mat, rot, xmat);
  mju_copy(xmat, mat, 9);
  mju_sub3(rel, origin, xpos);
  mju_mulMatVec3(vec, rot, rel);
  mju_sub3(vec, vec, rel);
  mju_sub3(xpos, xpos, vec);
}

/* mjc_Convex (convex.c:915-1001) through mjc_CCDIteration (:792-819), native solver: one
 * contact; with mjENBL_MULTICCD, a box / mesh pair without margin (singlePass :895-909) asks
 * mjc_ccd for up to 4 contacts (the multicontact polygon) and stops there; other pairs without
 * a sphere or an ellipsoid add the extra contacts of the perturbed frames (:933-999): both
 * geoms rotated about the first
 * contact by -+1e-3 rad around its frame's y and z axes (geom 2 the other way), each new
 * contact farther than 1e-3 min(rbound) from every earlier one kept with the first one's
 * depth. The frames are perturbed on local copies (the reference rotates mjData's in place
 * and restores them). */
static int col_convex(orRaw* c, const mjhipModel* m, const mjhipData* d, int g1, int g2,
                      mjtNum margin) {
  orShape A, B;
  mjtNum xpos1[3], xmat1[9], xpos2[3], xmat2[9];
  mju_copy3(xpos1, d->geom_xpos + 3*g1);
  mju_copy(xmat1, d->geom_xmat + 9*g1, 9);
  mju_copy3(xpos2, d->geom_xpos + 3*g2);
  mju_copy(xmat2, d->geom_xmat + 9*g2, 9);
  or_shape(&A, m, d, g1, margin);
  or_shape(&B, m, d, g2, margin);
  mjtNum p1[3], r1[9], p2[3], r2[9];
  mju_copy3(p1, xpos1);
  mju_copy(r1, xmat1, 9);
  mju_copy3(p2, xpos2);
  mju_copy(r2, xmat2, 9);
  A.pos = p1; A.mat = r1;
  B.pos = p2; B.mat = r2;
  const int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  if (mjENABLED(mjhipENBL_MULTICCD) && margin <= 0 &&
      (t1 == mjhipGEOM_BOX || t1 == mjhipGEOM_MESH) &&
      (t2 == mjhipGEOM_BOX || t2 == mjhipGEOM_MESH)) {
    orCCD st;                         /* mjc_CCDIteration with max_contacts 4 (:792-819) */
    const mjtNum dist = or_ccd(&st, &A, &B, m->opt.ccd_iterations, m->opt.ccd_tolerance, 0, 4);
    if (!(dist < 0)) return 0;
    for (int i = 0; i < st.nx; i++) {
      c[i].dist = margin + dist;
      mju_sub3(c[i].frame, st.x1 + 3*i, st.x2 + 3*i);
      mju_normalize3(c[i].frame);
      c[i].pos[0] = 0.5*(st.x1[3*i] + st.x2[3*i]);
      c[i].pos[1] = 0.5*(st.x1[3*i + 1] + st.x2[3*i + 1]);
      c[i].pos[2] = 0.5*(st.x1[3*i + 2] + st.x2[3*i + 2]);
      mju_zero3(c[i].frame + 3);
    }
    return st.nx;
  }
  int ncon = col_ccdIteration(c, m, &A, &B, margin);
  if (ncon == 1 && mjENABLED(mjhipENBL_MULTICCD) && t1 != mjhipGEOM_ELLIPSOID &&
      t1 != mjhipGEOM_SPHERE && t2 != mjhipGEOM_ELLIPSOID && t2 != mjhipGEOM_SPHERE) {
    const mjtNum relative_tolerance = 1e-3, perturbation_angle = 1e-3;
    mjtNum frame[9];
    mju_copy(frame, c[0].frame, 9);
    mju_makeFrame(frame);
    const mjtNum tolerance = relative_tolerance * mjMIN(m->geom_rbound[g1], m->geom_rbound[g2]);
    const mjtNum* axes[2] = {frame + 3, frame + 6};
    const mjtNum angles[2] = {-perturbation_angle, perturbation_angle};
    for (int ai = 0; ai < 2; ai++) {
      for (int gi = 0; gi < 2; gi++) {
        mjtNum quat[4], rot[9], invrot[9];
        mju_axisAngle2Quat(quat, axes[ai], angles[gi]);
        mju_quat2Mat(rot, quat);
        or_rotateFrame(c[0].pos, rot, r1, p1);
        for (int i = 0; i < 3; i++) {
          for (int j = 0; j < 3; j++) invrot[3*j+i] = rot[3*i+j];
        }
        or_rotateFrame(c[0].pos, invrot, r2, p2);
        int fresh = col_ccdIteration(c + ncon, m, &A, &B, margin);
        if (fresh) {                          /* mjc_isDistinctContact (:851-858) */
          for (int i = 0; i < ncon; i++) {
            if (mju_dist3(c[i].pos, c[ncon].pos) <= tolerance) {
              fresh = 0;
              break;
            }
          }
        }
        if (fresh) {
          c[ncon].dist = c[0].dist;
          ncon++;
        }
        mju_copy3(p1, xpos1);
        mju_copy(r1, xmat1, 9);
        mju_copy3(p2, xpos2);
        mju_copy(r2, xmat2, 9);
      }
    }
  }
  return ncon;
}

/* mju_sign (engine_util_misc.c:1018-1026), mju_dist3 (engine_util_blas.c:157-160),
   mju_mulMatTMat3 (:208-218) */
static mjtNum mju_sign(mjtNum x) { return x < 0 ? -1 : (x > 0 ? 1 : 0); }

static mjtNum mju_dist3(const mjtNum a[3], const mjtNum b[3]) {
  mjtNum dif[3] = {a[0]-b[0], a[1]-b[1], a[2]-b[2]};
  return sqrt(dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2]);
}

static void mju_mulMatTMat3(mjtNum r[9], const mjtNum a[9], const mjtNum b[9]) {
  r[0] = a[0]*b[0] + a[3]*b[3] + a[6]*b[6];
  r[1] = a[0]*b[1] + a[3]*b[4] + a[6]*b[7];
  r[2] = a[0]*b[2] + a[3]*b[5] + a[6]*b[8];
  r[3] = a[1]*b[0] + a[4]*b[3] + a[7]*b[6];
  r[4] = a[1]*b[1] + a[4]*b[4] + a[7]*b[7];
  r[5] = a[1]*b[2] + a[4]*b[5] + a[7]*b[8];
  r[6] = a[2]*b[0] + a[5]*b[3] + a[8]*b[6];
  r[7] = a[2]*b[1] + a[5]*b[4] + a[8]*b[7];
  r[8] = a[2]*b[2] + a[5]*b[5] + a[8]*b[8];
}

/* mjccd_support (convex.c:501-704), the libccd-style support of a geom at unit direction dir
   in its current frame (s->pos / s->mat): the mesh case hill-climbs from s->meshindex with the
   start vertex's own value as the first bound and records the result in s->meshindex; the
   result is inflated by half the object's margin */
static void or_ccdSupportLib(mjtNum r[3], orShape* s, const mjtNum dir[3]) {
  mjtNum ld[3], res[3];
  mju_mulMatTVec3(ld, s->mat, dir);
  const mjtNum* size = s->size;
  switch (s->gtype) {
  case mjhipGEOM_SPHERE:
    mju_scl3(res, ld, size[0]);
    break;
  case mjhipGEOM_CAPSULE:
    mju_scl3(res, ld, size[0]);
    res[2] += mju_sign(ld[2]) * size[1];
    break;
  case mjhipGEOM_ELLIPSOID:
    for (int i = 0; i < 3; i++) res[i] = ld[i] * size[i];
    mju_normalize3(res);
    for (int i = 0; i < 3; i++) res[i] *= size[i];
    break;
  case mjhipGEOM_CYLINDER: {
    mjtNum tmp = sqrt(ld[0]*ld[0] + ld[1]*ld[1]);
    if (tmp > mjMINVAL) {
      res[0] = ld[0]/tmp*size[0];
      res[1] = ld[1]/tmp*size[0];
    } else {
      res[0] = res[1] = 0;
    }
    res[2] = mju_sign(ld[2]) * size[1];
    break;
  }
  case mjhipGEOM_BOX:
    for (int i = 0; i < 3; i++) res[i] = mju_sign(ld[i]) * size[i];
    break;
  default: {                            /* mesh */
    const float* V = s->vert;
    mjtNum tmp = -1E+10;
    int ibest = -1;
    if (!s->graph) {
      for (int i = 0; i < s->nvert; i++) {
        mjtNum vdot = ld[0]*(mjtNum)V[3*i] + ld[1]*(mjtNum)V[3*i+1] + ld[2]*(mjtNum)V[3*i+2];
        if (vdot > tmp) {
          tmp = vdot;
          ibest = i;
        }
      }
      s->meshindex = ibest;
    } else {
      const int numvert = s->graph[0];
      const int* edgeadr = s->graph + 2;
      const int* globalid = s->graph + 2 + numvert;
      const int* localid = s->graph + 2 + 2*numvert;
      ibest = s->meshindex < 0 ? 0 : s->meshindex;
      tmp = ld[0]*(mjtNum)V[3*globalid[ibest]] + ld[1]*(mjtNum)V[3*globalid[ibest]+1] +
            ld[2]*(mjtNum)V[3*globalid[ibest]+2];
      int change = 1, locid;
      while (change) {
        change = 0;
        int i = edgeadr[ibest];
        while ((locid = localid[i]) >= 0) {
          mjtNum vdot = ld[0]*(mjtNum)V[3*globalid[locid]] + ld[1]*(mjtNum)V[3*globalid[locid]+1] +
                        ld[2]*(mjtNum)V[3*globalid[locid]+2];
          if (vdot > tmp) {
            tmp = vdot;
            ibest = locid;
            change = 1;
          }
          i++;
        }
      }
      s->meshindex = ibest;
      ibest = globalid[ibest];
    }
    if (ibest < 0) {
      mju_zero3(res);
    } else {
      for (int i = 0; i < 3; i++) res[i] = (mjtNum)V[3*ibest + i];
    }
    break;
  }
  }
  for (int i = 0; i < 3; i++) res[i] += ld[i] * s->margin/2;
  mju_mulMatVec3(res, s->mat, res);
  mju_addTo3(res, s->pos);
  mju_copy3(r, res);
}

/* addplanemesh (convex.c:1010-1040) */
static int or_addPlaneMesh(orRaw* c, const float vertex[3], const mjtNum pos1[3],
                           const mjtNum normal1[3], const mjtNum pos2[3], const mjtNum mat2[9],
                           const mjtNum first[3], mjtNum rbound) {
  mjtNum pnt[3], v[3] = {vertex[0], vertex[1], vertex[2]}, dif[3];
  mju_mulMatVec3(pnt, mat2, v);
  mju_addTo3(pnt, pos2);
  if (mju_dist3(pnt, first) < 0.3*rbound) return 0;
  mju_sub3(dif, pnt, pos1);
  c->dist = mju_dot3(normal1, dif);
  mju_copy3(c->pos, pnt);
  mju_addToScl3(c->pos, normal1, -0.5*c->dist);
  mju_copy3(c->frame, normal1);
  mju_zero3(c->frame + 3);
  return 1;
}

/* mjc_PlaneConvex (convex.c:1045-1141): the libccd support of geom 2 at -normal gives the first
   contact; for a mesh, up to maxplanemesh = 3 in all with the vertices below the margin around
   the support vertex (the hull graph's neighbours, else every vertex) */
static int col_planeConvex(orRaw* c, const mjhipModel* m, const mjhipData* d, int g1, int g2,
                           mjtNum margin) {
  const mjtNum *pos1 = d->geom_xpos + 3*g1, *mat1 = d->geom_xmat + 9*g1;
  const mjtNum *pos2 = d->geom_xpos + 3*g2, *mat2 = d->geom_xmat + 9*g2;
  mjtNum normal[3] = {mat1[2], mat1[5], mat1[8]}, dir[3] = {-mat1[2], -mat1[5], -mat1[8]};
  mjtNum v[3], dif[3];
  orShape obj;
  or_shape(&obj, m, d, g2, 0);
  or_ccdSupportLib(v, &obj, dir);
  mju_sub3(dif, v, pos1);
  mjtNum dist = mju_dot3(normal, dif);
  if (dist > margin) return 0;
  c->dist = dist;
  mju_copy3(c->pos, v);
  mju_addToScl3(c->pos, normal, -0.5*dist);
  mju_copy3(c->frame, normal);
  mju_zero3(c->frame + 3);
  int count = 1;
  const int id = m->geom_dataid[g2];
  if (id == -1) return count;
  const float* vertdata = m->mesh_vert + 3*m->mesh_vertadr[id];
  mjtNum locdir[3];
  mju_mulMatTVec3(locdir, mat2, dir);
  mju_sub3(dif, pos2, pos1);
  const mjtNum threshold = mju_dot3(normal, dif) - margin;
  const mjtNum rbound = m->geom_rbound[g2];
  if (m->mesh_graphadr[id] < 0) {
    for (int i = 0; i < m->mesh_vertnum[id] && count < 3; i++) {
      mjtNum vdot = locdir[0]*(mjtNum)vertdata[3*i] + locdir[1]*(mjtNum)vertdata[3*i+1] +
                    locdir[2]*(mjtNum)vertdata[3*i+2];
      if (vdot > threshold && i != obj.meshindex) {
        count += or_addPlaneMesh(c + count, vertdata + 3*i, pos1, normal, pos2, mat2, c->pos,
                                 rbound);
      }
    }
  } else if (obj.meshindex >= 0) {
    const int* graph = m->mesh_graph + m->mesh_graphadr[id];
    const int numvert = graph[0];
    const int* edgeadr = graph + 2;
    const int* globalid = graph + 2 + numvert;
    const int* localid = graph + 2 + 2*numvert;
    int i = edgeadr[obj.meshindex], locid;
    while ((locid = localid[i]) >= 0 && count < 3) {
      const float* vx = vertdata + 3*globalid[locid];
      mjtNum vdot = locdir[0]*(mjtNum)vx[0] + locdir[1]*(mjtNum)vx[1] + locdir[2]*(mjtNum)vx[2];
      if (vdot > threshold) {
        count += or_addPlaneMesh(c + count, vx, pos1, normal, pos2, mat2, c->pos, rbound);
      }
      i++;
    }
  }
  return count;
}

/* mjc_ellipsoidInside (convex.c:1363-1414) and mjc_ellipsoidOutside (:1419-1464) */
static int or_ellipsoidInside(mjtNum nrm[3], const mjtNum pos[3], const mjtNum size[3]) {
  mjtNum S2inv[3] = {1/(size[0]*size[0]), 1/(size[1]*size[1]), 1/(size[2]*size[2])};
  mjtNum C = pos[0]*pos[0]*S2inv[0] + pos[1]*pos[1]*S2inv[1] + pos[2]*pos[2]*S2inv[2] - 1;
  if (C > 0) return 0;
  mju_normalize3(nrm);
  for (int iter = 0; iter < 30; iter++) {
    mjtNum A = nrm[0]*nrm[0]*S2inv[0] + nrm[1]*nrm[1]*S2inv[1] + nrm[2]*nrm[2]*S2inv[2];
    mjtNum B = pos[0]*nrm[0]*S2inv[0] + pos[1]*nrm[1]*S2inv[1] + pos[2]*nrm[2]*S2inv[2];
    mjtNum det = B*B - A*C;
    if (det < mjMINVAL || A < mjMINVAL) return iter > 0;
    mjtNum x = (-B + sqrt(det))/A;
    if (x < 0) return iter > 0;
    mjtNum pnt[3];
    mju_addScl3(pnt, pos, nrm, x);
    mjtNum newnrm[3] = {pnt[0]*S2inv[0], pnt[1]*S2inv[1], pnt[2]*S2inv[2]};
    mju_normalize3(newnrm);
    mjtNum change = mju_dist3(nrm, newnrm);
    mju_copy3(nrm, newnrm);
    if (change < 1e-6) break;
  }
  return 1;
}

static int or_ellipsoidOutside(mjtNum nrm[3], const mjtNum pos[3], const mjtNum size[3]) {
  mjtNum S2[3] = {size[0]*size[0], size[1]*size[1], size[2]*size[2]};
  mjtNum PS2[3] = {pos[0]*pos[0]*S2[0], pos[1]*pos[1]*S2[1], pos[2]*pos[2]*S2[2]};
  mjtNum la = 0;
  for (int iter = 0; iter < 30; iter++) {
    mjtNum R[3] = {1/(S2[0]+la), 1/(S2[1]+la), 1/(S2[2]+la)};
    mjtNum val = PS2[0]*R[0]*R[0] + PS2[1]*R[1]*R[1] + PS2[2]*R[2]*R[2] - 1;
    if (val < 1e-6) break;
    mjtNum deriv = -2*(PS2[0]*R[0]*R[0]*R[0] + PS2[1]*R[1]*R[1]*R[1] + PS2[2]*R[2]*R[2]*R[2]);
    if (deriv > -mjMINVAL) break;
    mjtNum delta = -val/deriv;
    if (delta < 1e-6) break;
    la += delta;
  }
  nrm[0] = pos[0]/(S2[0]+la);
  nrm[1] = pos[1]/(S2[1]+la);
  nrm[2] = pos[2]/(S2[2]+la);
  mju_normalize3(nrm);
  return 1;
}

/* mjc_fixNormal (convex.c:1469-1614): the contact normal from the smooth geom's surface */
static void or_fixNormal(const mjhipModel* m, const mjhipData* d, orRaw* con, int g1, int g2) {
  int gid[2] = {g1, g2}, type[2];
  for (int i = 0; i < 2; i++) {
    type[i] = m->geom_type[gid[i]];
    if (type[i] != mjhipGEOM_SPHERE && type[i] != mjhipGEOM_CAPSULE &&
        type[i] != mjhipGEOM_ELLIPSOID && type[i] != mjhipGEOM_CYLINDER) {
      type[i] = -1;
    }
  }
  if (type[0] == -1 && type[1] == -1) return;
  mjtNum normal[2][3] = {{con->frame[0], con->frame[1], con->frame[2]},
                         {-con->frame[0], -con->frame[1], -con->frame[2]}};
  int processed[2] = {0, 0};
  for (int i = 0; i < 2; i++) {
    if (type[i] == -1) continue;
    const mjtNum* mat = d->geom_xmat + 9*gid[i];
    const mjtNum* size = m->geom_size + 3*gid[i];
    mjtNum dif[3], pos[3], nrm[3], dst1, dst2;
    mju_sub3(dif, con->pos, d->geom_xpos + 3*gid[i]);
    mju_mulMatTVec3(pos, mat, dif);
    mju_mulMatTVec3(nrm, mat, normal[i]);
    switch (type[i]) {
    case mjhipGEOM_SPHERE:
      mju_copy3(nrm, pos);
      processed[i] = 1;
      break;
    case mjhipGEOM_CAPSULE:
      if (pos[2] < -size[1]) {
        nrm[2] = pos[2] + size[1];
      } else if (pos[2] > size[1]) {
        nrm[2] = pos[2] - size[1];
      } else {
        nrm[2] = 0;
      }
      nrm[0] = pos[0];
      nrm[1] = pos[1];
      processed[i] = 1;
      break;
    case mjhipGEOM_ELLIPSOID:
      if (size[0] < mjMINVAL || size[1] < mjMINVAL || size[2] < mjMINVAL) break;
      dst1 = pos[0]*pos[0]/(size[0]*size[0]) + pos[1]*pos[1]/(size[1]*size[1]) +
             pos[2]*pos[2]/(size[2]*size[2]);
      processed[i] = dst1 <= 1 ? or_ellipsoidInside(nrm, pos, size)
                               : or_ellipsoidOutside(nrm, pos, size);
      break;
    default:                                /* cylinder */
      if (fabs(pos[2]) > 0.95*size[1]) break;
      dst1 = fabs(size[1] - fabs(pos[2]));
      dst2 = fabs(size[0] - sqrt(pos[0]*pos[0] + pos[1]*pos[1]));
      if (dst1 < 0.25*dst2) break;
      nrm[0] = pos[0];
      nrm[1] = pos[1];
      nrm[2] = 0;
      processed[i] = 1;
      break;
    }
    if (processed[i]) {
      mju_normalize3(nrm);
      mju_mulMatVec3(normal[i], mat, nrm);
    }
  }
  if (processed[0] && processed[1]) {
    mju_sub3(con->frame, normal[0], normal[1]);
    mju_normalize3(con->frame);
  } else if (processed[0]) {
    mju_copy3(con->frame, normal[0]);
  } else if (processed[1]) {
    mju_scl3(con->frame, normal[1], -1);
  }
  if (processed[0] || processed[1]) mju_zero3(con->frame + 3);
}

/* addVert (convex.c:1154-1168) */
static void or_prismAddVert(int* nvert, orShape* s, mjtNum x, mjtNum y, mjtNum z) {
  mju_copy3(s->prism[0], s->prism[1]);
  mju_copy3(s->prism[1], s->prism[2]);
  mju_copy3(s->prism[3], s->prism[4]);
  mju_copy3(s->prism[4], s->prism[5]);
  s->prism[2][0] = s->prism[5][0] = x;
  s->prism[2][1] = s->prism[5][1] = y;
  s->prism[5][2] = z;
  (*nvert)++;
}

/* most contacts of mjc_ConvexHField for a height field: one per triangular prism of the grid,
   at most mjMAXCONPAIR (50) */
static int or_hfieldMaxContacts(const mjhipModel* m, int hid) {
  int n = 2*(m->hfield_nrow[hid] - 1)*(m->hfield_ncol[hid] - 1);
  return n < 50 ? n : 50;
}

/* mjc_ConvexHField (convex.c:1173-1356): geom 2 expressed in the height field's frame, its
   support box against the field's box, then the native solver (mjc_penetration :34-68, one
   contact) against every triangular prism of the covered sub-grid, each contact's normal fixed
   by mjc_fixNormal. The solver's warm starts of geom 2 carry over from the support-box calls
   through every prism, as in the reference's single mjCCDObj. */
static int col_convexHField(orRaw* con, const mjhipModel* m, const mjhipData* d, int g1, int g2,
                            mjtNum margin) {
  const mjtNum *pos1 = d->geom_xpos + 3*g1, *mat1 = d->geom_xmat + 9*g1;
  const mjtNum *pos2 = d->geom_xpos + 3*g2, *mat2 = d->geom_xmat + 9*g2;
  const int hid = m->geom_dataid[g1];
  const int nrow = m->hfield_nrow[hid], ncol = m->hfield_ncol[hid];
  const float* data = m->hfield_data + m->hfield_adr[hid];
  const mjtNum* size1 = m->hfield_size + 4*hid;
  mjtNum vec[3], pos[3], mat[9];
  mju_sub3(vec, pos2, pos1);
  mju_mulMatTVec(pos, mat1, vec, 3, 3);
  const mjtNum r2 = m->geom_rbound[g2];
  for (int i = 0; i < 2; i++) {
    if ((size1[i] < pos[i] - r2 - margin) || (-size1[i] > pos[i] + r2 + margin)) return 0;
  }
  if (size1[2] < pos[2] - r2 - margin) return 0;
  if (-size1[3] > pos[2] + r2 + margin) return 0;
  mju_mulMatTMat3(mat, mat1, mat2);
  /* geom 2 in the field's frame (the reference overwrites its geom_xmat/xpos meanwhile) */
  orShape B;
  or_shape(&B, m, d, g2, 0);
  B.pos = pos;
  B.mat = mat;
  mjtNum sv[3], xmin, xmax, ymin, ymax, zmin, zmax;
  const mjtNum ax[6][3] = {{1, 0, 0}, {-1, 0, 0}, {0, 1, 0}, {0, -1, 0}, {0, 0, 1}, {0, 0, -1}};
  or_ccdSupportLib(sv, &B, ax[0]); xmax = sv[0];
  or_ccdSupportLib(sv, &B, ax[1]); xmin = sv[0];
  or_ccdSupportLib(sv, &B, ax[2]); ymax = sv[1];
  or_ccdSupportLib(sv, &B, ax[3]); ymin = sv[1];
  or_ccdSupportLib(sv, &B, ax[4]); zmax = sv[2];
  or_ccdSupportLib(sv, &B, ax[5]); zmin = sv[2];
  if ((xmin - margin > size1[0]) || (xmax + margin < -size1[0]) ||
      (ymin - margin > size1[1]) || (ymax + margin < -size1[1]) ||
      (zmin - margin > size1[2]) || (zmax + margin < -size1[3])) {
    return 0;
  }
  int cmin = (int)floor((xmin + size1[0]) / (2*size1[0]) * (ncol - 1));
  int cmax = (int)ceil((xmax + size1[0]) / (2*size1[0]) * (ncol - 1));
  int rmin = (int)floor((ymin + size1[1]) / (2*size1[1]) * (nrow - 1));
  int rmax = (int)ceil((ymax + size1[1]) / (2*size1[1]) * (nrow - 1));
  cmin = mjMAX(0, cmin);
  cmax = mjMIN(ncol - 1, cmax);
  rmin = mjMAX(0, rmin);
  rmax = mjMIN(nrow - 1, rmax);
  B.margin = margin;
  orShape A;
  memset(&A, 0, sizeof(A));
  A.kind = A.gtype = mjhipGEOM_HFIELD;
  A.vertindex = A.meshindex = -1;
  const mjtNum dx = (2.0*size1[0]) / (ncol - 1), dy = (2.0*size1[1]) / (nrow - 1);
  const int dr[2] = {1, 0};
  A.prism[0][2] = A.prism[1][2] = A.prism[2][2] = -size1[3];
  int cnt = 0;
  for (int r = rmin; r < rmax; r++) {
    int nvert = 0;
    for (int c = cmin; c <= cmax; c++) {
      for (int i = 0; i < 2; i++) {
        or_prismAddVert(&nvert, &A, dx*c - size1[0], dy*(r + dr[i]) - size1[1],
                        data[(r + dr[i])*ncol + c]*size1[2] + margin);
        if (nvert <= 2) continue;
        if (A.prism[3][2] < zmin && A.prism[4][2] < zmin && A.prism[5][2] < zmin) continue;
        orCCD st;
        const mjtNum dist = or_ccd(&st, &A, &B, m->opt.ccd_iterations, m->opt.ccd_tolerance, 0, 1);
        if (!(dist < 0)) continue;              /* mjc_penetration: no penetration */
        mjtNum dir[3], vp[3];
        mju_sub3(dir, st.x1, st.x2);
        mju_normalize3(dir);
        vp[0] = 0.5*(st.x1[0] + st.x2[0]);
        vp[1] = 0.5*(st.x1[1] + st.x2[1]);
        vp[2] = 0.5*(st.x1[2] + st.x2[2]);
        if (dir[0] == 0 && dir[1] == 0 && dir[2] == 0) continue;   /* ccdVec3Eq(dir, origin) */
        con[cnt].dist = dist;                    /* -depth */
        mju_mulMatVec3(con[cnt].frame, mat1, dir);
        mju_mulMatVec3(con[cnt].pos, mat1, vp);
        mju_addTo3(con[cnt].pos, pos1);
        mju_zero3(con[cnt].frame + 3);
        if (++cnt >= 50) {
          r = rmax + 1;
          c = cmax + 1;
          break;
        }
      }
    }
  }
  for (int i = 0; i < cnt; i++) or_fixNormal(m, d, con + i, g1, g2);
  return cnt;
}

/* Test hook restating the reference's Penetration helper (test/engine/
   engine_collision_gjk_test.cc:86-150): mjc_ccd on geoms g1, g2 with the given margin,
   tolerance and iterations, one contact, no distance cutoff. Returns the number of contacts
   (0 or 1); out = {dist, dir[3], pos[3]}. */
int or_ccdPenetration(const mjhipModel* m, const mjhipData* d, int g1, int g2, mjtNum margin,
                      mjtNum tol, int kmax, mjtNum* out) {
  orShape A, B;
  or_shape(&A, m, d, g1, margin);
  or_shape(&B, m, d, g2, margin);
  orCCD st;
  mjtNum dist = or_ccd(&st, &A, &B, kmax, tol, 0, 1);
  if (!(dist < 0) || st.nx < 1) return 0;
  out[0] = dist;
  mju_sub3(out + 1, st.x1, st.x2);
  mju_normalize3(out + 1);
  for (int k = 0; k < 3; k++) out[4 + k] = 0.5*(st.x1[k] + st.x2[k]);
  return 1;
}

/* mjc_ccd (engine_collision_gjk.c:2215-2343) as the reference's GJK tests call it
   (engine_collision_gjk_test.cc:62-84 GeomDist, :86-150 Penetration): geoms g1, g2 at the
   data's current frames, object margin `margin` on both, config {kmax, tol, maxc, cutoff}.
   out: dist, nx, unsupported (always 0), x1[3*50], x2[3*50]. Returns dist. */
mjtNum or_ccdGeneral(const mjhipModel* m, const mjhipData* d, int g1, int g2, mjtNum margin,
                     mjtNum tol, int kmax, int maxc, mjtNum cutoff, mjtNum* out) {
  orShape A, B;
  or_shape(&A, m, d, g1, margin);
  or_shape(&B, m, d, g2, margin);
  orCCD st;
  st.nx = 0;
  mjtNum dist = or_ccd(&st, &A, &B, kmax, tol, cutoff, maxc);
  out[0] = dist;
  out[1] = st.nx;
  out[2] = st.unsupported;
  for (int k = 0; k < 3*OR_MAXCONPAIR; k++) {
    out[3 + k] = st.x1[k];
    out[3 + 3*OR_MAXCONPAIR + k] = st.x2[k];
  }
  return dist;
}

/* pairs served by mjc_Convex in mjCOLLISIONFUNC (capsule-ellipsoid/cylinder, sphere-ellipsoid,
 * ellipsoid and cylinder pairs among themselves and with boxes) */
static int or_isConvexPair(int t1, int t2) {
  if (t1 == mjhipGEOM_PLANE || t1 == mjhipGEOM_HFIELD) return 0;
  if (t2 == mjhipGEOM_ELLIPSOID || t2 == mjhipGEOM_MESH) return 1;
  if (t2 == mjhipGEOM_CYLINDER) return t1 == mjhipGEOM_CAPSULE || t1 == mjhipGEOM_CYLINDER ||
                                        t1 == mjhipGEOM_ELLIPSOID;
  if (t2 == mjhipGEOM_BOX) return t1 == mjhipGEOM_ELLIPSOID || t1 == mjhipGEOM_CYLINDER;
  return 0;
}

/* mjCOLLISIONFUNC (:41-52) for type-ordered t1 <= t2: 0 = no function, otherwise the most
 * contacts the function returns when it is one of the primitives restated here (a height
 * field's, 50, is bounded per field by or_pairMaxContacts), or -1 for a function outside the
 * subset (SDFs, libccd's MPR) */
static int or_collisionFunc(const mjhipModel* m, int t1, int t2) {
  static const int table[9][9] = {
    /*           PLANE HFIELD SPHERE CAPSULE ELLIPS CYL BOX MESH SDF */
    /*PLANE  */ {0,    0,     1,     2,      1,     4,  4,  3,   -1},
    /*HFIELD */ {0,    0,     50,    50,     50,    50, 50, 50,  -1},
    /*SPHERE */ {0,    0,     1,     1,      1,     1,  1,  1,   -1},
    /*CAPSULE*/ {0,    0,     0,     2,      1,     1,  2,  1,   -1},
    /*ELLIPS */ {0,    0,     0,     0,      1,     1,  1,  1,   -1},
    /*CYL    */ {0,    0,     0,     0,      0,     1,  1,  1,   -1},
    /*BOX    */ {0,    0,     0,     0,      0,     0,  24, 1,   -1},
    /*MESH   */ {0,    0,     0,     0,      0,     0,  0,  1,   -1},
    /*SDF    */ {0,    0,     0,     0,      0,     0,  0,  0,   -1}};
  if (t1 < 0 || t2 < 0 || t1 > 8 || t2 > 8) return -1;
  const int k = table[t1][t2];
  if (k > 0 && (t1 == mjhipGEOM_HFIELD || (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_MESH))) {
    /* mjc_ConvexHField / the plane-mesh path through mjc_penetration / the native solver */
    if (mjDISABLED(mjhipDSBL_NATIVECCD) && t1 == mjhipGEOM_HFIELD) return -1;
  }
  if (k > 0 && or_isConvexPair(t1, t2)) {
    /* mjc_Convex with the libccd MPR fallback: not restated. MULTICCD (pairs without a
       sphere or ellipsoid): up to 5 contacts (the first and four perturbed ones,
       convex.c:933-999; a box / mesh pair without margin: up to 4 from one pass) */
    if (mjDISABLED(mjhipDSBL_NATIVECCD)) return -1;
    if (mjENABLED(mjhipENBL_MULTICCD) && t1 != mjhipGEOM_SPHERE && t1 != mjhipGEOM_ELLIPSOID &&
        t2 != mjhipGEOM_ELLIPSOID) {
      return 5;
    }
  }
  return k;
}

/* the most contacts of type-ordered geoms g1, g2 (0: no function, -1: outside the subset) */
static int or_pairMaxContacts(const mjhipModel* m, int g1, int g2) {
  const int k = or_collisionFunc(m, m->geom_type[g1], m->geom_type[g2]);
  if (k > 0 && m->geom_type[g1] == mjhipGEOM_HFIELD) {
    return or_hfieldMaxContacts(m, m->geom_dataid[g1]);
  }
  return k;
}

/* add_pair :937-990: geom-level (OR over the body's geoms) bitmask check, ordered ids */
static void or_addPair(const mjhipModel* m, int b1, int b2, int* npair, int* pair) {
  int ct[2] = {0, 0}, ca[2] = {0, 0}, b[2] = {b1, b2};
  for (int k = 0; k < 2; k++) {
    for (int g = m->body_geomadr[b[k]]; g < m->body_geomadr[b[k]] + m->body_geomnum[b[k]];
         g++) {
      ct[k] |= m->geom_contype[g];
      ca[k] |= m->geom_conaffinity[g];
    }
  }
  if (!(ct[0] & ca[1]) && !(ct[1] & ca[0])) return;
  pair[(*npair)++] = b1 < b2 ? (b1 << 16) + b2 : (b2 << 16) + b1;
}

/* mju_eig3 (engine_util_solve.c:683-781): Jacobi iterations on a quaternion */
static void or_eig3(mjtNum eigval[3], mjtNum eigvec[9], const mjtNum mat[9]) {
  const mjtNum eigEPS = 1e-12;
  mjtNum quat[4] = {1, 0, 0, 0}, D[9], tmp[9];
  for (int iter = 0; iter < 500; iter++) {
    mju_quat2Mat(eigvec, quat);
    for (int i = 0; i < 3; i++) {         /* tmp = eigvec' * mat (mju_mulMatTMat3) */
      for (int j = 0; j < 3; j++) {
        tmp[3*i+j] = eigvec[i]*mat[j] + eigvec[3+i]*mat[3+j] + eigvec[6+i]*mat[6+j];
      }
    }
    for (int i = 0; i < 3; i++) {         /* D = tmp * eigvec (mju_mulMatMat3) */
      for (int j = 0; j < 3; j++) {
        D[3*i+j] = tmp[3*i]*eigvec[j] + tmp[3*i+1]*eigvec[3+j] + tmp[3*i+2]*eigvec[6+j];
      }
    }
    eigval[0] = D[0];
    eigval[1] = D[4];
    eigval[2] = D[8];
    int rk, ck, rotk;
    if (fabs(D[1]) > fabs(D[2]) && fabs(D[1]) > fabs(D[5])) {
      rk = 0; ck = 1; rotk = 2;
    } else if (fabs(D[2]) > fabs(D[5])) {
      rk = 0; ck = 2; rotk = 1;
    } else {
      rk = 1; ck = 2; rotk = 0;
    }
    if (fabs(D[3*rk+ck]) < eigEPS) break;
    mjtNum tau = (D[4*ck]-D[4*rk])/(2*D[3*rk+ck]), t;
    if (tau >= 0) {
      t = 1.0/(tau + sqrt(1 + tau*tau));
    } else {
      t = -1.0/(-tau + sqrt(1 + tau*tau));
    }
    mjtNum c = 1.0/sqrt(1 + t*t);
    if (c > 1.0-eigEPS) break;
    tmp[1] = tmp[2] = tmp[3] = 0;
    tmp[rotk+1] = (tau >= 0 ? -sqrt(0.5-0.5*c) : sqrt(0.5-0.5*c));
    if (rotk == 1) tmp[rotk+1] = -tmp[rotk+1];
    tmp[0] = sqrt(1.0 - tmp[rotk+1]*tmp[rotk+1]);
    mju_normalize4(tmp);
    mju_mulQuat(quat, quat, tmp);
    mju_normalize4(quat);
  }
  /* the broadphase uses only the frame's rows; the reference sorts the eigenpairs in
   * decreasing order (bubble sort 0, 1, 0, swapping columns and eigenvalues) */
  for (int j = 0; j < 3; j++) {
    int j1 = j % 2;
    if (eigval[j1] + eigEPS < eigval[j1+1]) {
      mjtNum e = eigval[j1];
      eigval[j1] = eigval[j1+1];
      eigval[j1+1] = e;
      for (int k = 0; k < 3; k++) {
        mjtNum v = eigvec[3*k+j1];
        eigvec[3*k+j1] = eigvec[3*k+j1+1];
        eigvec[3*k+j1+1] = v;
      }
    }
  }
}

/* makeAAMM :862-895 for a body: geom centers in `frame`, inflated by rbound + margin */
static void or_makeAAMM(const mjhipModel* m, const mjhipData* d, mjtNum aamm[6], int b,
                        const mjtNum frame[9]) {
  for (int i = 0; i < m->body_geomnum[b]; i++) {
    int g = m->body_geomadr[b] + i;
    mjtNum margin = mjENABLED(mjhipENBL_OVERRIDE) ? 0.5*m->opt.o_margin : m->geom_margin[g];
    mjtNum a[6];
    for (int j = 0; j < 3; j++) {
      const mjtNum* x = d->geom_xpos + 3*g;
      mjtNum cen = x[0]*frame[3*j] + x[1]*frame[3*j+1] + x[2]*frame[3*j+2];
      a[j] = cen - m->geom_rbound[g] - margin;
      a[j+3] = cen + m->geom_rbound[g] + margin;
    }
    if (i == 0) {
      for (int j = 0; j < 6; j++) aamm[j] = a[j];
    } else {
      for (int j = 0; j < 3; j++) {
        aamm[j] = mjMIN(aamm[j], a[j]);
        aamm[j+3] = mjMAX(aamm[j+3], a[j+3]);
      }
    }
  }
}

/* mj_SAP :1006-1100 along axis 0: float keys, stable sort (mjSORT is stable), active list */
typedef struct { float value; int id_ismax; } orSAP;

static int or_SAP(const mjtNum* aamm, int n, int* pair) {
  orSAP* sb = (orSAP*)malloc(sizeof(orSAP) * 2 * (n > 0 ? n : 1));
  orSAP* ab = (orSAP*)malloc(sizeof(orSAP) * 2 * (n > 0 ? n : 1));
  for (int i = 0; i < n; i++) {
    sb[2*i].id_ismax = i;
    sb[2*i].value = (float)aamm[6*i];
    sb[2*i+1].id_ismax = i + 0x10000;
    sb[2*i+1].value = (float)aamm[6*i+3];
  }
  for (int j = 1; j < 2*n; j++) {         /* stable insertion sort by value */
    orSAP t = sb[j];
    int k = j - 1;
    for (; k >= 0 && sb[k].value > t.value; k--) sb[k+1] = sb[k];
    sb[k+1] = t;
  }
  int cnt = 0, npair = 0;
  for (int i = 0; i < 2*n; i++) {
    if (!(sb[i].id_ismax & 0x10000)) {
      for (int j = 0; j < cnt; j++) {
        int id1 = ab[j].id_ismax, id2 = sb[i].id_ismax;
        if (aamm[6*id1+1] > aamm[6*id2+4] || aamm[6*id1+2] > aamm[6*id2+5] ||
            aamm[6*id2+1] > aamm[6*id1+4] || aamm[6*id2+2] > aamm[6*id1+5]) {
          continue;
        }
        pair[npair++] = (id1 << 16) + id2;
      }
      ab[cnt++] = sb[i];
    } else {
      int toremove = sb[i].id_ismax & 0xFFFF;
      for (int j = 0; j < cnt; j++) {
        if (ab[j].id_ismax == toremove) {
          for (int k = j; k < cnt - 1; k++) ab[k] = ab[k+1];
          cnt--;
          break;
        }
      }
    }
  }
  free(sb);
  free(ab);
  return npair;
}

/* mj_broadphase :1148-1286: always-colliding pairs of the world body (or a world-welded body
 * with a plane), then SAP pairs in the geom covariance frame filtered by weld; the result is
 * sorted by signature (duplicates are skipped by the caller) */
static int or_broadphase(const mjhipModel* m, const mjhipData* d, int* pair) {
  int npair = 0, nbody = m->nbody;
  int dsbl_filterparent = mjDISABLED(mjhipDSBL_FILTERPARENT);
  for (int b1 = 0; b1 < nbody; b1++) {
    if (!or_canCollide(m, b1)) continue;
    if ((b1 == 0 && m->body_geomnum[b1] > 0) || (m->body_weldid[b1] == 0 && or_hasPlane(m, b1))) {
      for (int b2 = 0; b2 < nbody; b2++) {
        if (!or_canCollide(m, b2)) continue;
        int weld2 = m->body_weldid[b2];
        int pweld2 = m->body_weldid[m->body_parentid[weld2]];
        if (or_filterBodyPair(0, 0, weld2, pweld2, dsbl_filterparent)) continue;
        or_addPair(m, b1, b2, &npair, pair);
      }
    }
  }
  int cnt = 0;
  mjtNum cen[3] = {0, 0, 0};
  for (int i = 0; i < m->ngeom; i++) {
    if (m->geom_bodyid[i]) {
      for (int k = 0; k < 3; k++) cen[k] += d->geom_xpos[3*i+k];
      cnt++;
    }
  }
  if (cnt == 0) goto sort;
  for (int k = 0; k < 3; k++) cen[k] *= 1.0/cnt;
  {
    mjtNum cov[9] = {0}, eigval[3], frame[9];
    for (int i = 0; i < m->ngeom; i++) {
      if (!m->geom_bodyid[i]) continue;
      const mjtNum* v = d->geom_xpos + 3*i;
      mjtNum dif[3] = {v[0]-cen[0], v[1]-cen[1], v[2]-cen[2]};
      mjtNum D00 = dif[0]*dif[0], D01 = dif[0]*dif[1], D02 = dif[0]*dif[2];
      mjtNum D11 = dif[1]*dif[1], D12 = dif[1]*dif[2], D22 = dif[2]*dif[2];
      cov[0] += D00; cov[1] += D01; cov[2] += D02;
      cov[3] += D01; cov[4] += D11; cov[5] += D12;
      cov[6] += D02; cov[7] += D12; cov[8] += D22;
    }
    for (int k = 0; k < 9; k++) cov[k] *= 1.0/cnt;
    or_eig3(eigval, frame, cov);
    int* bid = (int*)malloc(sizeof(int) * nbody);
    int ncollide = 0;
    for (int i = 1; i < nbody; i++) {
      if (or_canCollide(m, i)) bid[ncollide++] = i;
    }
    if (ncollide > 1) {
      mjtNum* aamm = (mjtNum*)malloc(sizeof(mjtNum) * 6 * ncollide);
      int* sap = (int*)malloc(sizeof(int) * ncollide * (ncollide - 1) / 2);
      for (int i = 0; i < ncollide; i++) or_makeAAMM(m, d, aamm + 6*i, bid[i], frame);
      int nsap = or_SAP(aamm, ncollide, sap);
      for (int i = 0; i < nsap; i++) {
        int b1 = bid[sap[i] >> 16], b2 = bid[sap[i] & 0xFFFF];
        int weld1 = m->body_weldid[b1], weld2 = m->body_weldid[b2];
        int pweld1 = m->body_weldid[m->body_parentid[weld1]];
        int pweld2 = m->body_weldid[m->body_parentid[weld2]];
        if (or_filterBodyPair(weld1, pweld1, weld2, pweld2, dsbl_filterparent)) continue;
        or_addPair(m, b1, b2, &npair, pair);
      }
      free(aamm);
      free(sap);
    }
    free(bid);
  }
sort:
  for (int j = 1; j < npair; j++) {       /* bfsort: unsigned signature order */
    int t = pair[j], k = j - 1;
    for (; k >= 0 && (unsigned)pair[k] > (unsigned)t; k--) pair[k+1] = pair[k];
    pair[k+1] = t;
  }
  return npair;
}

/* contacts enabled at all (mj_collision :282-287; nconmax is unbounded here) */
static int or_contactsEnabled(const mjhipModel* m) {
  return !mjDISABLED(mjhipDSBL_CONSTRAINT) && !mjDISABLED(mjhipDSBL_CONTACT) && m->nbody >= 2;
}

/* mj_collideGeomPair's merged test (:499-523): geoms g1, g2 (either order) form one of the
 * predefined pairs [startadr, pairadr) merged for this body pair */
static int or_mergedPair(const mjhipModel* m, int g1, int g2, int startadr, int pairadr) {
  for (int k = startadr; k < pairadr; k++) {
    if ((m->pair_geom1[k] == g1 && m->pair_geom2[k] == g2) ||
        (m->pair_geom1[k] == g2 && m->pair_geom2[k] == g1)) {
      return 1;
    }
  }
  return 0;
}

/* condim of a geom pair as mj_contactParam (:1289-1384) resolves it */
static int or_pairCondim(const mjhipModel* m, int g1, int g2) {
  int p1 = m->geom_priority[g1], p2 = m->geom_priority[g2];
  if (p1 != p2) return p1 > p2 ? m->geom_condim[g1] : m->geom_condim[g2];
  return mjMAX(m->geom_condim[g1], m->geom_condim[g2]);
}

/* Array sizing of the oracle's contact and constraint buffers (test infrastructure, not a
 * reference rule: the reference sizes its arena by nconmax/njmax). Worst case over every
 * body pair the broadphase could return: the most contacts of each geom pair's restated
 * function, with the pyramidal/elliptic rows per contact (mj_instantiateContact). */
static void or_contactBounds(const mjhipModel* m, int* ncon, int* nrow) {
  *ncon = *nrow = 0;
  if (!or_contactsEnabled(m)) return;
  int dsbl_filterparent = mjDISABLED(mjhipDSBL_FILTERPARENT);
  int ell = m->opt.cone == mjhipCONE_ELLIPTIC;
  for (int b1 = 0; b1 < m->nbody; b1++) {
    for (int b2 = b1 + 1; b2 < m->nbody; b2++) {
      if (!or_canCollide(m, b1) || !or_canCollide(m, b2) || !or_canCollide2(m, b1, b2)) continue;
      int weld1 = m->body_weldid[b1], weld2 = m->body_weldid[b2];
      int pweld1 = m->body_weldid[m->body_parentid[weld1]];
      int pweld2 = m->body_weldid[m->body_parentid[weld2]];
      if (or_filterBodyPair(weld1, pweld1, weld2, pweld2, dsbl_filterparent)) continue;
      int excluded = 0;
      for (int i = 0; i < m->nexclude; i++) excluded |= m->exclude_signature[i] == (b1 << 16) + b2;
      if (excluded) continue;
      for (int g1 = m->body_geomadr[b1]; g1 < m->body_geomadr[b1] + m->body_geomnum[b1]; g1++) {
        for (int g2 = m->body_geomadr[b2]; g2 < m->body_geomadr[b2] + m->body_geomnum[b2]; g2++) {
          if (or_mergedPair(m, g1, g2, 0, m->npair)) continue;   /* counted below */
          const int flip = m->geom_type[g1] > m->geom_type[g2];
          int k = or_pairMaxContacts(m, flip ? g2 : g1, flip ? g1 : g2);
          if (k > 0 && !or_filterBitmask(m->geom_contype[g1], m->geom_conaffinity[g1],
                                         m->geom_contype[g2], m->geom_conaffinity[g2])) {
            int condim = or_pairCondim(m, g1, g2);
            *ncon += k;
            *nrow += k * (condim == 1 ? 1 : (ell ? condim : 2*(condim - 1)));
          }
        }
      }
    }
  }
  for (int p = 0; p < m->npair; p++) {      /* predefined pairs: no bitmask, their condim */
    const int a = m->pair_geom1[p], b = m->pair_geom2[p];
    const int flip = m->geom_type[a] > m->geom_type[b];
    const int k = or_pairMaxContacts(m, flip ? b : a, flip ? a : b);
    if (k > 0) {
      const int condim = m->pair_dim[p];
      *ncon += k;
      *nrow += k * (condim == 1 ? 1 : (ell ? condim : 2*(condim - 1)));
    }
  }
}

int or_contactCapacity(const mjhipModel* m) {
  int ncon, nrow;
  or_contactBounds(m, &ncon, &nrow);
  return ncon;
}

int or_efcCapacity(const mjhipModel* m) {
  int n = 0;
  for (int i = 0; i < m->njnt; i++) {
    if (m->jnt_limited[i]) n += (m->jnt_type[i] == mjhipJNT_BALL) ? 1 : 2;
  }
  for (int i = 0; i < m->ntendon; i++) {
    if (m->tendon_limited[i]) n += 2;
  }
  for (int i = 0; i < m->nv; i++) {
    if (m->dof_frictionloss[i] > 0) n++;
  }
  for (int i = 0; i < m->ntendon; i++) {
    if (m->tendon_frictionloss[i] > 0) n++;
  }
  for (int i = 0; i < m->neq; i++) {
    int t = m->eq_type[i];
    n += t == mjhipEQ_CONNECT ? 3 : (t == mjhipEQ_WELD ? 6 : 1);
  }
  int ncon, nrow;
  or_contactBounds(m, &ncon, &nrow);
  return n + nrow;
}

/* the narrowphase of type-ordered geoms g1, g2 (mjCOLLISIONFUNC's primitive and convex
 * functions): raw contacts closer than margin into raw[] (<= 50), their count */
static int or_narrow(const mjhipModel* m, const mjhipData* d, int g1, int g2, mjtNum margin,
                     orRaw* raw) {
  const int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const mjtNum *pos1 = d->geom_xpos + 3*g1, *mat1 = d->geom_xmat + 9*g1;
  const mjtNum *pos2 = d->geom_xpos + 3*g2, *mat2 = d->geom_xmat + 9*g2;
  const mjtNum *size1 = m->geom_size + 3*g1, *size2 = m->geom_size + 3*g2;
  int num = 0;
  if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_CYLINDER) {
    num = col_planeCylinder(raw, margin, pos1, mat1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_BOX) {
    num = col_planeBox(raw, margin, pos1, mat1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_SPHERE) {
    num = raw_planeSphere(raw, margin, pos1, mat1, pos2, size2[0]);
  } else if (t1 == mjhipGEOM_PLANE && t2 == mjhipGEOM_CAPSULE) {
    num = col_planeCapsule(raw, margin, pos1, mat1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_SPHERE) {
    num = raw_sphereSphere(raw, margin, pos1, mat1, size1[0], pos2, mat2, size2[0]);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_CAPSULE) {
    num = col_sphereCapsule(raw, margin, pos1, mat1, size1[0], pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_CYLINDER) {
    num = col_sphereCylinder(raw, margin, pos1, mat1, size1[0], pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_CAPSULE && t2 == mjhipGEOM_BOX) {
    num = col_capsuleBox(raw, margin, pos1, mat1, size1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_SPHERE && t2 == mjhipGEOM_BOX) {
    num = raw_sphereBox(raw, margin, pos1, size1[0], pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_CAPSULE && t2 == mjhipGEOM_CAPSULE) {
    num = col_capsuleCapsule(raw, margin, pos1, mat1, size1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX) {
    num = col_boxBox(raw, margin, pos1, mat1, size1, pos2, mat2, size2);
    if (num) num = or_boxBoxFilter(raw, num, margin, pos1, mat1, size1, pos2, mat2, size2);
  } else if (t1 == mjhipGEOM_PLANE && (t2 == mjhipGEOM_ELLIPSOID || t2 == mjhipGEOM_MESH)) {
    num = col_planeConvex(raw, m, d, g1, g2, margin);
  } else if (t1 == mjhipGEOM_HFIELD) {
    num = col_convexHField(raw, m, d, g1, g2, margin);
  } else if (or_isConvexPair(t1, t2)) {
    num = col_convex(raw, m, d, g1, g2, margin);
  }
  return num;
}

/* mj_collideGeoms (engine_collision_driver.c:1440-1632: dynamic filters, narrowphase,
 * mj_setContact) for geoms of two bodies (ipair = -1), or for predefined pair ipair (g1, g2
 * its geoms): no bitmask filter, the pair's margin (mj_assignMargin), condim, gap, solref,
 * solimp, friction, and its solreffriction when either value is nonzero (:1597-1609) */
static void or_collideGeoms(const mjhipModel* m, const mjhipData* d, orEfc* e, int g1, int g2,
                            int ipair) {
  if (m->geom_type[g1] > m->geom_type[g2]) { int t = g1; g1 = g2; g2 = t; }
  int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const int kmax = or_collisionFunc(m, t1, t2);
  if (kmax == 0) return;
  if (ipair < 0 && or_filterBitmask(m->geom_contype[g1], m->geom_conaffinity[g1],
                                    m->geom_contype[g2], m->geom_conaffinity[g2])) {
    return;
  }
  mjtNum margin = mjENABLED(mjhipENBL_OVERRIDE) ? m->opt.o_margin :
                  ipair >= 0 ? m->pair_margin[ipair] :
                  mjMAX(m->geom_margin[g1], m->geom_margin[g2]);
  if (or_filterSphere(m, d, g1, g2, margin)) return;
  if (kmax < 0) {              /* a collision function outside the subset would run: flag */
    ((mjhipData*)d)->status |= MJHIP_INST_UNSUPPORTED;
    return;
  }
  orRaw raw[50];
  const int num = or_narrow(m, d, g1, g2, margin, raw);
  if (!num) return;
  int condim;
  mjtNum gap, solref[2], solimp[5], friction[5], solreffriction[2] = {0, 0};
  if (ipair < 0) {
    or_contactParam(m, g1, g2, &condim, &gap, solref, solimp, friction);
  } else {
    condim = m->pair_dim[ipair];
    gap = m->pair_gap[ipair];
    mju_copy(solref, m->pair_solref + 2*ipair, 2);
    mju_copy(solimp, m->pair_solimp + 5*ipair, 5);
    mju_copy(friction, m->pair_friction + 5*ipair, 5);
    if (m->pair_solreffriction[2*ipair] || m->pair_solreffriction[2*ipair + 1]) {
      mju_copy(solreffriction, m->pair_solreffriction + 2*ipair, 2);
    }
  }
  for (int k = 0; k < num; k++) {
    int i = e->ncon;
    if (i >= e->con_capacity) return;   /* cannot happen: capacity is exact */
    e->con_dist[i] = raw[k].dist;
    mju_copy3(e->con_pos + 3*i, raw[k].pos);
    mju_copy(e->con_frame + 9*i, raw[k].frame, 9);
    e->con_geom[2*i] = g1;
    e->con_geom[2*i+1] = g2;
    /* mj_setContact :1387-1415 with mj_assignRef/Imp/Friction (constraint.c:122-165) */
    e->con_dim[i] = condim;
    e->con_includemargin[i] = margin - gap;
    const int ovr = mjENABLED(mjhipENBL_OVERRIDE) != 0;
    mju_copy(e->con_solref + 2*i, ovr ? m->opt.o_solref : solref, 2);
    mju_copy(e->con_solreffriction + 2*i, ovr ? m->opt.o_solref : solreffriction, 2);
    mju_copy(e->con_solimp + 5*i, ovr ? m->opt.o_solimp : solimp, 5);
    for (int j = 0; j < 5; j++) {
      e->con_friction[5*i+j] = mjMAX(1e-5, ovr ? m->opt.o_friction[j] : friction[j]);
    }
    e->con_exclude[i] = (e->con_dist[i] >= e->con_includemargin[i]);
    mju_makeFrame(e->con_frame + 9*i);
    e->con_efc_address[i] = -1;
    e->con_mu[i] = 0;
    e->ncon = i + 1;
  }
}

/* engine_support.c:1407-1450 mj_geomDistance (with mj_geomDistanceCCD :1379-1402): the
 * smallest signed distance between two geoms up to distmax, and the segment between the
 * nearest points in fromto (zeros when none is found). mjc_Convex and box-box pairs go
 * through the native solver with the distance bound as its cutoff; the other functions
 * return their contacts closer than distmax. Functions outside the subset flag the state. */
static mjtNum or_geomDistance(const mjhipModel* m, mjhipData* d, int geom1, int geom2,
                              mjtNum distmax, mjtNum fromto[6]) {
  mjtNum dist = distmax;
  mju_zero(fromto, 6);
  const int flip = m->geom_type[geom1] > m->geom_type[geom2];
  const int g1 = flip ? geom2 : geom1, g2 = flip ? geom1 : geom2;
  const int t1 = m->geom_type[g1], t2 = m->geom_type[g2];
  const int ccd = or_isConvexPair(t1, t2) || (t1 == mjhipGEOM_BOX && t2 == mjhipGEOM_BOX);
  const int kmax = or_collisionFunc(m, t1, t2);
  if (kmax == 0) return dist;                 /* no collision function */
  if (kmax < 0 && !(ccd && !mjDISABLED(mjhipDSBL_NATIVECCD))) {
    d->status |= MJHIP_INST_UNSUPPORTED;      /* mesh, height field, SDF or libccd's MPR */
    return dist;
  }
  if (ccd && !mjDISABLED(mjhipDSBL_NATIVECCD)) {
    orShape A, B;
    or_shape(&A, m, d, g1, 0);
    or_shape(&B, m, d, g2, 0);
    orCCD st;
    const mjtNum r = or_ccd(&st, &A, &B, m->opt.ccd_iterations, m->opt.ccd_tolerance, distmax, 1);
    if (st.nx > 0) {
      mju_copy3(fromto, st.x1);
      mju_copy3(fromto + 3, st.x2);
    }
    return r;
  }
  orRaw raw[50];
  const int num = or_narrow(m, d, g1, g2, distmax, raw);
  int best = -1;
  for (int i = 0; i < num; i++) {
    if (raw[i].dist < dist) {
      dist = raw[i].dist;
      best = i;
    }
  }
  if (best >= 0) {
    const mjtNum sign = flip ? -1 : 1;
    mju_addScl3(fromto, raw[best].pos, raw[best].frame, -0.5*sign*dist);
    mju_addScl3(fromto + 3, raw[best].pos, raw[best].frame, 0.5*sign*dist);
  }
  return dist;
}

/* contactcompare (engine_collision_driver.c:223-257) on the geom ids of two contacts */
static int or_contactLess(const mjhipModel* m, const orEfc* e, int a, int b) {
  int a1 = e->con_geom[2*a], a2 = e->con_geom[2*a+1];
  int b1 = e->con_geom[2*b], b2 = e->con_geom[2*b+1];
  if (m->geom_type[a1] > m->geom_type[a2]) { int t = a1; a1 = a2; a2 = t; }
  if (m->geom_type[b1] > m->geom_type[b2]) { int t = b1; b1 = b2; b2 = t; }
  return a1 < b1 || (a1 == b1 && a2 < b2);
}

static void or_swapContacts(orEfc* e, int a, int b) {
#define SWP(arr, k) for (int j = 0; j < (k); j++) { mjtNum t = e->arr[(k)*a+j]; \
    e->arr[(k)*a+j] = e->arr[(k)*b+j]; e->arr[(k)*b+j] = t; }
#define SWPI(arr, k) for (int j = 0; j < (k); j++) { int t = e->arr[(k)*a+j]; \
    e->arr[(k)*a+j] = e->arr[(k)*b+j]; e->arr[(k)*b+j] = t; }
  SWP(con_dist, 1) SWP(con_pos, 3) SWP(con_frame, 9) SWP(con_includemargin, 1)
  SWP(con_friction, 5) SWP(con_solref, 2) SWP(con_solreffriction, 2) SWP(con_solimp, 5)
  SWP(con_mu, 1) SWPI(con_dim, 1) SWPI(con_geom, 2) SWPI(con_exclude, 1)
  SWPI(con_efc_address, 1)
#undef SWP
#undef SWPI
}

/* mj_collision (engine_collision_driver.c:265-497): the broadphase's body pairs in signature
 * order (repeats skipped); ahead of each, the predefined pairs whose signature is not above
 * its own (:316-327, before the filters); then the body bitmask and exclude filters, then a
 * single-geom pair, the midphase (mj_collideTree, whose contacts are stably sorted by
 * contactcompare) or all-to-all, skipping the geom pairs merged as predefined pairs; the
 * predefined pairs left after the sweep last (:432-437). The midphase's bounding-volume tests
 * are inflated by the margins, so visiting the pair's geoms all-to-all yields the same
 * contacts before the sort. */
static void or_collision(const mjhipModel* m, const mjhipData* d, orEfc* e) {
  e->ncon = 0;
  if (!or_contactsEnabled(m)) return;
  int nb = m->nbody;
  int* pair = (int*)malloc(sizeof(int) * (nb*nb + nb*(nb - 1)/2 + 1));
  int np = or_broadphase(m, d, pair);
  unsigned last_signature = (unsigned)-1;
  int pairadr = 0;
  for (int i = 0; i < np; i++) {
    int b1 = (pair[i] >> 16) & 0xFFFF, b2 = pair[i] & 0xFFFF;
    unsigned signature = ((unsigned)b1 << 16) + b2;
    if (signature == last_signature) continue;
    last_signature = signature;
    int merged = 0, startadr = pairadr;
    while (pairadr < m->npair && (unsigned)m->pair_signature[pairadr] <= signature) {
      if ((unsigned)m->pair_signature[pairadr] == signature) merged = 1;
      or_collideGeoms(m, d, e, m->pair_geom1[pairadr], m->pair_geom2[pairadr], pairadr);
      pairadr++;
    }
    if (!or_canCollide2(m, b1, b2)) continue;
    int exadr = 0;
    while (exadr < m->nexclude && (unsigned)m->exclude_signature[exadr] < signature) exadr++;
    if (exadr < m->nexclude && (unsigned)m->exclude_signature[exadr] == signature) continue;
    int n1 = m->body_geomnum[b1], n2 = m->body_geomnum[b2];
    int before = e->ncon;
    for (int a = 0; a < n1; a++) {
      for (int c = 0; c < n2; c++) {
        const int g1 = m->body_geomadr[b1] + a, g2 = m->body_geomadr[b2] + c;
        if (merged && or_mergedPair(m, g1, g2, startadr, pairadr)) continue;
        or_collideGeoms(m, d, e, g1, g2, -1);
      }
    }
    int midphase = !mjDISABLED(mjhipDSBL_MIDPHASE) && !(n1 == 1 && n2 == 1);
    if (midphase) {   /* stable insertion sort (mjSORT is stable) */
      for (int a = before + 1; a < e->ncon; a++) {
        for (int b = a; b > before && or_contactLess(m, e, b, b - 1); b--) {
          or_swapContacts(e, b, b - 1);
        }
      }
    }
  }
  while (pairadr < m->npair) {
    or_collideGeoms(m, d, e, m->pair_geom1[pairadr], m->pair_geom2[pairadr], pairadr);
    pairadr++;
  }
  free(pair);
}

/* mju_mulMatMat (engine_util_blas.c:818-831) */
static void mju_mulMatMat(mjtNum* res, const mjtNum* mat1, const mjtNum* mat2, int r1, int c1,
                          int c2) {
  mju_zero(res, r1*c2);
  for (int i = 0; i < r1; i++) {
    for (int k = 0; k < c1; k++) {
      mjtNum tmp = mat1[i*c1+k];
      if (tmp) mju_addToScl(res + i*c2, mat2 + k*c2, tmp, c2);
    }
  }
}

/* :265-356 mj_addConstraint: dense rows are dropped when all-zero (non-contact types); sparse
 * rows copy the chain and are dropped only when it is empty */
static void mj_addConstraint(const mjhipModel* m, orEfc* e, const mjtNum* jac, const mjtNum* pos,
                             const mjtNum* margin, mjtNum frictionloss, int size, int type,
                             int id, int NV, const int* chain) {
  int nv = m->nv, nefc = e->nefc;
  int *nnz = e->efc_J_rownnz, *adr = e->efc_J_rowadr, *ind = e->efc_J_colind;
  int empty = !(type == orCNSTR_CONTACT_FRICTIONLESS || type == orCNSTR_CONTACT_PYRAMIDAL ||
                type == orCNSTR_CONTACT_ELLIPTIC);
  if (!mj_isSparse(m)) {
    for (int i = 0; empty && i < size*nv; i++) {
      if (jac[i]) empty = 0;
    }
    if (!empty) mju_copy(e->efc_J + nefc*nv, jac, size*nv);
  } else {
    NV = mjMAX(0, NV);
    if (NV) {
      empty = 0;
    } else if (empty) {
      return;
    }
    for (int i = 0; i < size; i++) {
      adr[nefc+i] = (nefc+i ? adr[nefc+i-1]+nnz[nefc+i-1] : 0);
      nnz[nefc+i] = NV;
      if (NV) {
        memcpy(ind + adr[nefc+i], chain, NV*sizeof(int));
        mju_copy(e->efc_J + adr[nefc+i], jac + i*NV, NV);
      }
    }
  }
  if (empty) return;
  for (int i = 0; i < size; i++) {
    e->efc_pos[nefc+i] = (pos ? pos[i] : 0);
    e->efc_margin[nefc+i] = (margin ? margin[i] : 0);
    e->efc_frictionloss[nefc+i] = frictionloss;
    e->efc_type[nefc+i] = type;
    e->efc_id[nefc+i] = id;
  }
  e->nefc += size;
  if (type == orCNSTR_EQUALITY) {
    e->ne += size;
  } else if (type == orCNSTR_FRICTION_DOF || type == orCNSTR_FRICTION_TENDON) {
    e->nf += size;
  } else if (type == orCNSTR_LIMIT_JOINT || type == orCNSTR_LIMIT_TENDON) {
    e->nl += size;
  }
}

/* engine_util_spatial.c:81-92 */
static void mju_mulQuatAxis(mjtNum res[4], const mjtNum quat[4], const mjtNum axis[3]) {
  mjtNum tmp[4] = {-quat[1]*axis[0] - quat[2]*axis[1] - quat[3]*axis[2],
                   quat[0]*axis[0] + quat[2]*axis[2] - quat[3]*axis[1],
                   quat[0]*axis[1] + quat[3]*axis[0] - quat[1]*axis[2],
                   quat[0]*axis[2] + quat[1]*axis[1] - quat[2]*axis[0]};
  res[0] = tmp[0]; res[1] = tmp[1]; res[2] = tmp[2]; res[3] = tmp[3];
}

/* mj_instantiateEquality :493-764: connect, weld, joint and tendon (flex is outside the
 * supported subset), dense (NV = nv) or over the merged chain of a sparse model. eq_active is
 * the model's eq_active0 (mj_resetData). */
static void or_instantiateEquality(const mjhipModel* m, mjhipData* d, orEfc* e) {
  int nv = m->nv, issparse = mj_isSparse(m);
  if (mjDISABLED(mjhipDSBL_EQUALITY) || m->neq == 0) return;
  size_t n6 = 6*(size_t)nv + 1;
  mjtNum* jac[2] = {(mjtNum*)calloc(n6, sizeof(mjtNum)), (mjtNum*)calloc(n6, sizeof(mjtNum))};
  mjtNum* jacdif = (mjtNum*)calloc(n6, sizeof(mjtNum));
  mjtNum* sparse_buf = (mjtNum*)calloc(nv + 1, sizeof(mjtNum));
  int* chain = (int*)calloc(nv + 1, sizeof(int));
  int* chain2 = (int*)calloc(nv + 1, sizeof(int));
  int* buf_ind = (int*)calloc(nv + 1, sizeof(int));
  for (int i = 0; i < m->neq; i++) {
    if (!m->eq_active0[i]) continue;
    const mjtNum* data = m->eq_data + mjhipNEQDATA*i;
    int id[2] = {m->eq_obj1id[i], m->eq_obj2id[i]}, body_id[2], size = 0, NV = 0, NV2 = 0;
    mjtNum cpos[6], pos[2][3], ref[2], quat[4], quat1[4], quat2[4], quat3[4], axis[3];
    switch (m->eq_type[i]) {
    case mjhipEQ_CONNECT:
      if (m->eq_objtype[i] == OBJ_BODY) {
        for (int j = 0; j < 2; j++) {
          mju_mulMatVec3(pos[j], d->xmat + 9*id[j], data + 3*j);
          mju_addTo3(pos[j], d->xpos + 3*id[j]);
          body_id[j] = id[j];
        }
      } else {
        for (int j = 0; j < 2; j++) {
          mju_copy3(pos[j], d->site_xpos + 3*id[j]);
          body_id[j] = m->site_bodyid[id[j]];
        }
      }
      mju_sub3(cpos, pos[0], pos[1]);
      /* Jacobian difference (opposite of contact: 0 - 1) */
      NV = mj_jacDifPair(m, d, chain, body_id[1], body_id[0], pos[1], pos[0], jac[1], jac[0],
                         jacdif, NULL, NULL, NULL);
      mju_copy(jac[0], jacdif, 3*NV);
      size = 3;
      break;
    case mjhipEQ_WELD: {
      if (m->eq_objtype[i] == OBJ_BODY) {
        for (int j = 0; j < 2; j++) {
          const mjtNum* anchor = data + 3*(1-j);
          mju_mulMatVec3(pos[j], d->xmat + 9*id[j], anchor);
          mju_addTo3(pos[j], d->xpos + 3*id[j]);
          body_id[j] = id[j];
        }
      } else {
        for (int j = 0; j < 2; j++) {
          mju_copy3(pos[j], d->site_xpos + 3*id[j]);
          body_id[j] = m->site_bodyid[id[j]];
        }
      }
      mju_sub3(cpos, pos[0], pos[1]);
      mjtNum torquescale = data[10];
      NV = mj_jacDifPair(m, d, chain, body_id[1], body_id[0], pos[1], pos[0], jac[1], jac[0],
                         jacdif, jac[1] + 3*nv, jac[0] + 3*nv, jacdif + 3*nv);
      /* translation:rotation compressed to NV columns each */
      mju_copy(jac[0], jacdif, 3*NV);
      mju_copy(jac[0] + 3*NV, jacdif + 3*nv, 3*NV);
      if (m->eq_objtype[i] == OBJ_BODY) {
        mju_mulQuat(quat, d->xquat + 4*id[0], data + 6);
        mju_copy4(quat1, d->xquat + 4*id[1]);
      } else {
        mjtNum qs1[4];
        mju_mulQuat(quat, d->xquat + 4*body_id[0], m->site_quat + 4*id[0]);
        mju_mulQuat(qs1, d->xquat + 4*body_id[1], m->site_quat + 4*id[1]);
        mju_copy4(quat1, qs1);
      }
      quat1[1] = -quat1[1]; quat1[2] = -quat1[2]; quat1[3] = -quat1[3];
      mju_mulQuat(quat2, quat1, quat);
      mju_scl3(cpos + 3, quat2 + 1, torquescale);
      for (int j = 0; j < NV; j++) {
        axis[0] = jac[0][3*NV + j];
        axis[1] = jac[0][4*NV + j];
        axis[2] = jac[0][5*NV + j];
        mju_mulQuatAxis(quat2, quat1, axis);
        mju_mulQuat(quat3, quat2, quat);
        jac[0][3*NV + j] = 0.5*quat3[1];
        jac[0][4*NV + j] = 0.5*quat3[2];
        jac[0][5*NV + j] = 0.5*quat3[3];
      }
      mju_scl(jac[0] + 3*NV, jac[0] + 3*NV, torquescale, 3*NV);
      size = 6;
      break;
    }
    case mjhipEQ_JOINT:
    case mjhipEQ_TENDON: {
      for (int j = 0; j < 1 + (id[1] >= 0); j++) {
        if (m->eq_type[i] == mjhipEQ_JOINT) {
          pos[j][0] = d->qpos[m->jnt_qposadr[id[j]]];
          ref[j] = m->qpos0[m->jnt_qposadr[id[j]]];
          if (issparse) {
            *(j == 0 ? &NV : &NV2) = 1;
            (j == 0 ? chain : chain2)[0] = m->jnt_dofadr[id[j]];
            jac[j][0] = 1;
          } else {
            mju_zero(jac[j], nv);
            jac[j][m->jnt_dofadr[id[j]]] = 1;
          }
        } else {
          pos[j][0] = d->ten_length[id[j]];
          ref[j] = m->tendon_length0[id[j]];
          if (issparse) {
            int tn = d->ten_J_rownnz[id[j]], ta = d->ten_J_rowadr[id[j]];
            *(j == 0 ? &NV : &NV2) = tn;
            memcpy(j == 0 ? chain : chain2, d->ten_J_colind + ta, tn*sizeof(int));
            mju_copy(jac[j], d->ten_J + ta, tn);
          } else {
            mju_copy(jac[j], d->ten_J + id[j]*nv, nv);
          }
        }
      }
      if (id[1] >= 0) {
        mjtNum dif = pos[1][0] - ref[1];
        cpos[0] = pos[0][0] - ref[0] - data[0] -
                  (data[1]*dif + data[2]*dif*dif + data[3]*dif*dif*dif +
                   data[4]*dif*dif*dif*dif);
        mjtNum deriv = data[1] + 2*data[2]*dif + 3*data[3]*dif*dif + 4*data[4]*dif*dif*dif;
        if (issparse) {
          NV = mju_combineSparse(jac[0], jac[1], 1, -deriv, NV, NV2, chain, chain2, sparse_buf,
                                 buf_ind);
        } else {
          mju_addToScl(jac[0], jac[1], -deriv, nv);
        }
      } else {
        cpos[0] = pos[0][0] - ref[0] - data[0];
      }
      size = 1;
      break;
    }
    }
    if (size) {
      mj_addConstraint(m, e, jac[0], cpos, 0, 0, size, orCNSTR_EQUALITY, i,
                       issparse ? NV : 0, issparse ? chain : NULL);
    }
  }
  free(jac[0]); free(jac[1]); free(jacdif); free(sparse_buf);
  free(chain); free(chain2); free(buf_ind);
}

/* mj_instantiateFriction :768-822: dof friction, then tendon friction on the tendon's ten_J
   row (dense: a row whose Jacobian is all zero is skipped; sparse: one whose chain is) */
static void or_instantiateFriction(const mjhipModel* m, mjhipData* d, orEfc* e, mjtNum* jac) {
  int nv = m->nv, issparse = mj_isSparse(m);
  if (mjDISABLED(mjhipDSBL_FRICTIONLOSS)) return;
  for (int i = 0; i < nv; i++) {
    if (m->dof_frictionloss[i] > 0) {
      if (issparse) {
        jac[0] = 1;
      } else {
        mju_zero(jac, nv);
        jac[i] = 1;
      }
      mj_addConstraint(m, e, jac, 0, 0, m->dof_frictionloss[i], 1, orCNSTR_FRICTION_DOF, i,
                       issparse ? 1 : 0, issparse ? &i : NULL);
    }
  }
  for (int i = 0; i < m->ntendon; i++) {
    if (m->tendon_frictionloss[i] > 0) {
      mj_addConstraint(m, e, d->ten_J + (issparse ? d->ten_J_rowadr[i] : i*nv), 0, 0,
                       m->tendon_frictionloss[i], 1, orCNSTR_FRICTION_TENDON, i,
                       issparse ? d->ten_J_rownnz[i] : 0,
                       issparse ? d->ten_J_colind + d->ten_J_rowadr[i] : NULL);
    }
  }
}

/* :824-959 */
static void or_instantiateLimit(const mjhipModel* m, mjhipData* d, orEfc* e, mjtNum* jac) {
  int side, nv = m->nv, issparse = mj_isSparse(m);
  mjtNum margin, value, dist, angleAxis[3];
  if (mjDISABLED(mjhipDSBL_LIMIT)) return;
  for (int i = 0; i < m->njnt; i++) {
    if (m->jnt_limited[i]) {
      margin = m->jnt_margin[i];
      if (m->jnt_type[i] == mjhipJNT_SLIDE || m->jnt_type[i] == mjhipJNT_HINGE) {
        value = d->qpos[m->jnt_qposadr[i]];
        for (side = -1; side <= 1; side += 2) {
          dist = side * (m->jnt_range[2*i+(side+1)/2] - value);
          if (dist < margin) {
            if (issparse) {
              jac[0] = -(mjtNum)side;
            } else {
              mju_zero(jac, nv);
              jac[m->jnt_dofadr[i]] = -(mjtNum)side;
            }
            mj_addConstraint(m, e, jac, &dist, &margin, 0, 1, orCNSTR_LIMIT_JOINT, i,
                             issparse ? 1 : 0, issparse ? m->jnt_dofadr + i : NULL);
          }
        }
      } else if (m->jnt_type[i] == mjhipJNT_BALL) {
        int adr = m->jnt_qposadr[i];
        mjtNum quat[4] = {d->qpos[adr], d->qpos[adr+1], d->qpos[adr+2], d->qpos[adr+3]};
        mju_normalize4(quat);
        mju_quat2Vel(angleAxis, quat, 1);
        value = mju_normalize3(angleAxis);
        dist = mjMAX(m->jnt_range[2*i], m->jnt_range[2*i+1]) - value;
        if (dist < margin) {
          if (issparse) {
            int chain[3] = {m->jnt_dofadr[i], m->jnt_dofadr[i] + 1, m->jnt_dofadr[i] + 2};
            mju_scl3(jac, angleAxis, -1);
            mj_addConstraint(m, e, jac, &dist, &margin, 0, 1, orCNSTR_LIMIT_JOINT, i, 3, chain);
          } else {
            mju_zero(jac, nv);
            mju_scl3(jac + m->jnt_dofadr[i], angleAxis, -1);
            mj_addConstraint(m, e, jac, &dist, &margin, 0, 1, orCNSTR_LIMIT_JOINT, i, 0, NULL);
          }
        }
      }
    }
  }
  for (int i = 0; i < m->ntendon; i++) {
    if (m->tendon_limited[i]) {
      value = d->ten_length[i];
      margin = m->tendon_margin[i];
      for (side = -1; side <= 1; side += 2) {
        dist = side * (m->tendon_range[2*i+(side+1)/2] - value);
        if (dist < margin) {
          if (issparse) {
            mju_scl(jac, d->ten_J + d->ten_J_rowadr[i], -side, d->ten_J_rownnz[i]);
          } else {
            mju_scl(jac, d->ten_J+i*nv, -side, nv);
          }
          mj_addConstraint(m, e, jac, &dist, &margin, 0, 1, orCNSTR_LIMIT_TENDON, i,
                           issparse ? d->ten_J_rownnz[i] : 0,
                           issparse ? d->ten_J_colind + d->ten_J_rowadr[i] : NULL);
        }
      }
    }
  }
}

/* mj_instantiateContact :964-1131, pyramidal, elliptic or frictionless, dense (NV = nv) or
 * over the merged chain of a sparse model (a contact whose chain is empty is excluded,
 * exclude = 3) */
static void or_instantiateContact(const mjhipModel* m, mjhipData* d, orEfc* e) {
  int nv = m->nv, issparse = mj_isSparse(m);
  if (mjDISABLED(mjhipDSBL_CONTACT) || e->ncon == 0 || nv == 0) return;
  mjtNum* jac = (mjtNum*)malloc(6*nv*sizeof(mjtNum));
  mjtNum* jacdif = (mjtNum*)malloc(6*nv*sizeof(mjtNum));
  mjtNum* jac1p = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
  mjtNum* jac2p = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
  mjtNum* jac1r = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
  mjtNum* jac2r = (mjtNum*)malloc(3*nv*sizeof(mjtNum));
  int* chain = (int*)malloc(nv*sizeof(int));
  mjtNum *jacdifp = jacdif, *jacdifr = jacdif + 3*nv;
  for (int i = 0; i < e->ncon; i++) {
    if (e->con_exclude[i]) continue;
    int dim = e->con_dim[i];
    e->con_efc_address[i] = e->nefc;
    int b1 = m->geom_bodyid[e->con_geom[2*i]], b2 = m->geom_bodyid[e->con_geom[2*i+1]];
    const mjtNum* cpos_ = e->con_pos + 3*i;
    int NV = mj_jacDifPair(m, d, chain, b1, b2, cpos_, cpos_, jac1p, jac2p, jacdifp,
                           dim > 3 ? jac1r : NULL, dim > 3 ? jac2r : NULL,
                           dim > 3 ? jacdifr : NULL);
    if (NV == 0) {                         /* :1071-1076 */
      e->con_efc_address[i] = -1;
      e->con_exclude[i] = 3;
      continue;
    }
    /* rotate to the contact frame */
    const mjtNum* frame = e->con_frame + 9*i;
    mju_mulMatMat(jac, frame, jacdifp, dim > 1 ? 3 : 1, 3, NV);
    if (dim > 3) mju_mulMatMat(jac + 3*NV, frame, jacdifr, dim-3, 3, NV);
    if (dim == 1) {
      mj_addConstraint(m, e, jac, e->con_dist + i, e->con_includemargin + i, 0, 1,
                       orCNSTR_CONTACT_FRICTIONLESS, i, issparse ? NV : 0,
                       issparse ? chain : NULL);
    } else if (m->opt.cone == mjhipCONE_ELLIPTIC) {
      /* elliptic cone :1113-1126: the dim rotated rows, pos = (dist, 0, ...) */
      mjtNum cpos[6] = {0}, cmargin[6] = {0};
      cpos[0] = e->con_dist[i];
      cmargin[0] = e->con_includemargin[i];
      mj_addConstraint(m, e, jac, cpos, cmargin, 0, dim, orCNSTR_CONTACT_ELLIPTIC, i,
                       issparse ? NV : 0, issparse ? chain : NULL);
    } else {
      mjtNum cpos[2] = {e->con_dist[i], e->con_dist[i]};
      mjtNum cmargin[2] = {e->con_includemargin[i], e->con_includemargin[i]};
      for (int k = 1; k < dim; k++) {
        mjtNum f = e->con_friction[5*i + k-1];
        for (int j = 0; j < NV; j++) jacdifp[j] = jac[j] + jac[k*NV+j]*f;
        for (int j = 0; j < NV; j++) jacdifp[NV+j] = jac[j] + jac[k*NV+j]*(-f);
        mj_addConstraint(m, e, jacdifp, cpos, cmargin, 0, 2, orCNSTR_CONTACT_PYRAMIDAL, i,
                         issparse ? NV : 0, issparse ? chain : NULL);
      }
    }
  }
  free(jac); free(jacdif); free(jac1p); free(jac2p); free(jac1r); free(jac2r); free(chain);
}

/* :1138-1311 (limit, friction and contact rows) */
static void or_diagApprox(const mjhipModel* m, orEfc* e) {
  int weldcnt = 0;
  for (int i = 0; i < e->nefc; i++) {
    int id = e->efc_id[i], b1, b2;
    switch (e->efc_type[i]) {
    case orCNSTR_EQUALITY:
      switch (m->eq_type[id]) {
      case mjhipEQ_CONNECT:
      case mjhipEQ_WELD:
        b1 = m->eq_obj1id[id];
        b2 = m->eq_obj2id[id];
        if (m->eq_objtype[id] == OBJ_SITE) {
          b1 = m->site_bodyid[b1];
          b2 = m->site_bodyid[b2];
        }
        if (m->eq_type[id] == mjhipEQ_CONNECT) {
          e->efc_diagApprox[i] = m->body_invweight0[2*b1] + m->body_invweight0[2*b2];
        } else {
          e->efc_diagApprox[i] = m->body_invweight0[2*b1 + (weldcnt > 2)] +
                                 m->body_invweight0[2*b2 + (weldcnt > 2)];
          weldcnt = (weldcnt + 1) % 6;
        }
        break;
      default:
        e->efc_diagApprox[i] = m->eq_type[id] == mjhipEQ_JOINT ?
            m->dof_invweight0[m->jnt_dofadr[m->eq_obj1id[id]]] :
            m->tendon_invweight0[m->eq_obj1id[id]];
        if (m->eq_obj2id[id] >= 0) {
          e->efc_diagApprox[i] += m->eq_type[id] == mjhipEQ_JOINT ?
              m->dof_invweight0[m->jnt_dofadr[m->eq_obj2id[id]]] :
              m->tendon_invweight0[m->eq_obj2id[id]];
        }
        break;
      }
      break;
    case orCNSTR_FRICTION_DOF:
      e->efc_diagApprox[i] = m->dof_invweight0[id];
      break;
    case orCNSTR_LIMIT_JOINT:
      e->efc_diagApprox[i] = m->dof_invweight0[m->jnt_dofadr[id]];
      break;
    case orCNSTR_FRICTION_TENDON:
    case orCNSTR_LIMIT_TENDON:
      e->efc_diagApprox[i] = m->tendon_invweight0[id];
      break;
    case orCNSTR_CONTACT_FRICTIONLESS:
    case orCNSTR_CONTACT_PYRAMIDAL:
    case orCNSTR_CONTACT_ELLIPTIC: {
      int dim = e->con_dim[id];
      mjtNum tran = 0, rot = 0;
      for (int side = 0; side < 2; side++) {
        int b = m->geom_bodyid[e->con_geom[2*id+side]];
        tran += m->body_invweight0[2*b] * 1.0;
        rot += m->body_invweight0[2*b+1] * 1.0;
      }
      if (e->efc_type[i] == orCNSTR_CONTACT_FRICTIONLESS) {
        e->efc_diagApprox[i] = tran;
      } else if (e->efc_type[i] == orCNSTR_CONTACT_ELLIPTIC) {
        for (int j = 0; j < dim; j++) e->efc_diagApprox[i+j] = j < 3 ? tran : rot;
        i += dim - 1;
      } else {
        for (int j = 0; j < dim-1; j++) {
          mjtNum fri = e->con_friction[5*id+j];
          e->efc_diagApprox[i+2*j] = e->efc_diagApprox[i+2*j+1] =
              tran + fri*fri*(j < 2 ? tran : rot);
        }
        i += 2*dim - 3;
      }
      break;
    }
    }
  }
}

/* :1316-1371 (limit and friction rows; solreffriction only applies to contacts) */
static void getsolparam(const mjhipModel* m, const orEfc* e, int i, mjtNum* solref,
                        mjtNum* solreffriction, mjtNum* solimp) {
  int id = e->efc_id[i];
  mju_zero(solreffriction, 2);
  switch (e->efc_type[i]) {
  case orCNSTR_EQUALITY:
    mju_copy(solref, m->eq_solref+2*id, 2);
    mju_copy(solimp, m->eq_solimp+5*id, 5);
    break;
  case orCNSTR_CONTACT_FRICTIONLESS:
  case orCNSTR_CONTACT_PYRAMIDAL:
  case orCNSTR_CONTACT_ELLIPTIC:
    mju_copy(solref, e->con_solref+2*id, 2);
    mju_copy(solreffriction, e->con_solreffriction+2*id, 2);
    mju_copy(solimp, e->con_solimp+5*id, 5);
    break;
  case orCNSTR_LIMIT_JOINT:
    mju_copy(solref, m->jnt_solref+2*id, 2);
    mju_copy(solimp, m->jnt_solimp+5*id, 5);
    break;
  case orCNSTR_FRICTION_DOF:
    mju_copy(solref, m->dof_solref+2*id, 2);
    mju_copy(solimp, m->dof_solimp+5*id, 5);
    break;
  case orCNSTR_LIMIT_TENDON:
    mju_copy(solref, m->tendon_solref_lim+2*id, 2);
    mju_copy(solimp, m->tendon_solimp_lim+5*id, 5);
    break;
  case orCNSTR_FRICTION_TENDON:
    mju_copy(solref, m->tendon_solref_fri+2*id, 2);
    mju_copy(solimp, m->tendon_solimp_fri+5*id, 5);
    break;
  }
  if ((solref[0] > 0) ^ (solref[1] > 0)) {   /* mixed format: default (0.02, 1) */
    solref[0] = 0.02;
    solref[1] = 1;
  }
  if (!mjDISABLED(mjhipDSBL_REFSAFE) && solref[0] > 0) {
    solref[0] = mjMAX(solref[0], 2*m->opt.timestep);
  }
  if ((solreffriction[0] > 0) ^ (solreffriction[1] > 0)) mju_zero(solreffriction, 2);
  if (!mjDISABLED(mjhipDSBL_REFSAFE) && solreffriction[0] > 0) {
    solreffriction[0] = mjMAX(solreffriction[0], 2*m->opt.timestep);
  }
  solimp[0] = mjMIN(mjhipMAXIMP, mjMAX(mjhipMINIMP, solimp[0]));
  solimp[1] = mjMIN(mjhipMAXIMP, mjMAX(mjhipMINIMP, solimp[1]));
  solimp[2] = mjMAX(0, solimp[2]);
  solimp[3] = mjMIN(mjhipMAXIMP, mjMAX(mjhipMINIMP, solimp[3]));
  solimp[4] = mjMAX(1, solimp[4]);
}

/* :1413-1421 */
static mjtNum power(mjtNum a, mjtNum b) {
  if (b == 1) return a;
  else if (b == 2) return a*a;
  return pow(a, b);
}

/* :1425-1480 */
static void getimpedance(const mjtNum* solimp, mjtNum pos, mjtNum margin, mjtNum* imp,
                         mjtNum* impP) {
  if (solimp[0] == solimp[1] || solimp[2] <= mjMINVAL) {
    *imp = 0.5*(solimp[0] + solimp[1]);
    *impP = 0;
    return;
  }
  mjtNum x = (pos-margin) / solimp[2];
  mjtNum sgn = 1;
  if (x < 0) {
    x = -x;
    sgn = -1;
  }
  if (x >= 1 || x <= 0) {
    *imp = (x >= 1 ? solimp[1] : solimp[0]);
    *impP = 0;
    return;
  }
  mjtNum y, yP;
  if (solimp[4] == 1) {
    y = x;
    yP = 1;
  } else if (x <= solimp[3]) {
    mjtNum a = 1/power(solimp[3], solimp[4]-1);
    y = a*power(x, solimp[4]);
    yP = solimp[4] * a*power(x, solimp[4]-1);
  } else {
    mjtNum b = 1/power(1-solimp[3], solimp[4]-1);
    y = 1-b*power(1-x, solimp[4]);
    yP = solimp[4] * b*power(1-x, solimp[4]-1);
  }
  *imp = solimp[0] + y*(solimp[1]-solimp[0]);
  *impP = yP * sgn * (solimp[1]-solimp[0]) / solimp[2];
}

/* :1494-1608; a pyramidal contact's 2*(condim-1) rows share one impedance */
static void or_makeImpedance(const mjhipModel* m, orEfc* e) {
  int nefc = e->nefc;
  mjtNum *R = e->efc_R, *KBIP = e->efc_KBIP;
  mjtNum imp, impP, solref[2], solreffriction[2], solimp[5];
  for (int i = 0; i < nefc; i++) {
    getsolparam(m, e, i, solref, solreffriction, solimp);
    /* getposdim :1392-1422 */
    int dim = e->efc_type[i] == orCNSTR_CONTACT_PYRAMIDAL ? 2*(e->con_dim[e->efc_id[i]]-1) :
              (e->efc_type[i] == orCNSTR_CONTACT_ELLIPTIC ? e->con_dim[e->efc_id[i]] : 1);
    mjtNum pos = e->efc_pos[i];
    if (e->efc_type[i] == orCNSTR_EQUALITY) {
      int t = m->eq_type[e->efc_id[i]];
      if (t == mjhipEQ_WELD || t == mjhipEQ_CONNECT) {
        dim = t == mjhipEQ_WELD ? 6 : 3;
        pos = mju_norm(e->efc_pos + i, dim);
      }
    }
    getimpedance(solimp, pos, e->efc_margin[i], &imp, &impP);
    for (int j = 0; j < dim; j++) {
      int r = i + j, tp = e->efc_type[r];
      R[r] = mjMAX(mjMINVAL, (1-imp)*e->efc_diagApprox[r]/imp);
      int elliptic_friction = tp == orCNSTR_CONTACT_ELLIPTIC && j > 0;
      const mjtNum* ref = elliptic_friction && (solreffriction[0] || solreffriction[1]) ?
                          solreffriction : solref;
      if (tp == orCNSTR_FRICTION_DOF || tp == orCNSTR_FRICTION_TENDON || elliptic_friction) {
        KBIP[4*r] = 0;
      } else if (ref[0] > 0) {
        KBIP[4*r] = 1 / mjMAX(mjMINVAL, solimp[1]*solimp[1] * ref[0]*ref[0] * ref[1]*ref[1]);
      } else {
        KBIP[4*r] = -ref[0] / mjMAX(mjMINVAL, solimp[1]*solimp[1]);
      }
      if (ref[1] > 0) {
        KBIP[4*r+1] = 2 / mjMAX(mjMINVAL, solimp[1]*ref[0]);
      } else {
        KBIP[4*r+1] = -ref[1] / mjMAX(mjMINVAL, solimp[1]);
      }
      KBIP[4*r+2] = imp;
      KBIP[4*r+3] = impP;
    }
    i += dim - 1;
  }
  /* frictional contacts: R in the friction directions, contact mu (:1562-1598) */
  for (int i = e->ne + e->nf; i < nefc; i++) {
    if (e->efc_type[i] == orCNSTR_CONTACT_ELLIPTIC) {
      int id = e->efc_id[i], dim = e->con_dim[id];
      const mjtNum* friction = e->con_friction + 5*id;
      R[i+1] = R[i]/mjMAX(mjMINVAL, m->opt.impratio);
      e->con_mu[id] = friction[0] * sqrt(R[i+1]/R[i]);
      for (int j = 1; j < dim-1; j++) {
        R[i+j+1] = R[i+1]*friction[0]*friction[0]/(friction[j]*friction[j]);
      }
      i += dim - 1;
    } else if (e->efc_type[i] == orCNSTR_CONTACT_PYRAMIDAL) {
      int id = e->efc_id[i], dim = e->con_dim[id];
      const mjtNum* friction = e->con_friction + 5*id;
      R[i+1] = R[i]/mjMAX(mjMINVAL, m->opt.impratio);
      e->con_mu[id] = friction[0] * sqrt(R[i+1]/R[i]);
      mjtNum Rpy = 2*e->con_mu[id]*e->con_mu[id]*R[i];
      for (int j = 0; j < 2*(dim-1); j++) R[i+j] = Rpy;
      i += 2*(dim-1) - 1;
    }
  }
  for (int i = 0; i < nefc; i++) e->efc_D[i] = 1 / R[i];
  for (int i = 0; i < nefc; i++) {
    e->efc_diagApprox[i] = R[i] * KBIP[4*i+2] / (1-KBIP[4*i+2]);
  }
}

/* :2005-2116 (dense; equality and contacts are outside the supported subset) */
static void or_makeConstraint(const mjhipModel* m, mjhipData* d, orEfc* e) {
  e->ne = e->nf = e->nl = e->nefc = 0;
  if (mjDISABLED(mjhipDSBL_CONSTRAINT)) return;
  mjtNum* jac = (mjtNum*)malloc((m->nv > 0 ? m->nv : 1)*sizeof(mjtNum));
  or_instantiateEquality(m, d, e);
  or_instantiateFriction(m, d, e, jac);
  or_instantiateLimit(m, d, e, jac);
  free(jac);
  or_instantiateContact(m, d, e);
  e->nJ = 0;
  if (!e->nefc) return;
  /* transpose the sparse Jacobian (:2083-2104; the row supernodes only select the AVX
     kernels, whose per-row sums group as mju_dotSparse's) */
  if (mj_isSparse(m)) {
    e->nJ = e->efc_J_rowadr[e->nefc-1] + e->efc_J_rownnz[e->nefc-1];
    mju_transposeSparse(e->efc_JT, e->efc_J, e->nefc, m->nv, e->efc_JT_rownnz, e->efc_JT_rowadr,
                        e->efc_JT_colind, e->efc_J_rownnz, e->efc_J_rowadr, e->efc_J_colind);
  }
  or_diagApprox(m, e);
  or_makeImpedance(m, e);
}

/* mj_mulJacVec :361-377: res = J*vec (sparse: mju_mulMatVecSparse over the rows) */
static void or_mulJacVec(const mjhipModel* m, const orEfc* e, mjtNum* res, const mjtNum* vec) {
  if (!e->nefc) return;
  if (mj_isSparse(m)) {
    mju_mulMatVecSparse(res, e->efc_J, vec, e->nefc, e->efc_J_rownnz, e->efc_J_rowadr,
                        e->efc_J_colind);
  } else {
    mju_mulMatVec(res, e->efc_J, vec, e->nefc, m->nv);
  }
}

/* mj_mulJacTVec :426-442: res = J'*vec (sparse: mju_mulMatVecSparse over the rows of JT,
 * each dof's terms grouped by their position in its JT row) */
static void or_mulJacTVec(const mjhipModel* m, const orEfc* e, mjtNum* res, const mjtNum* vec) {
  if (!e->nefc) return;
  if (mj_isSparse(m)) {
    mju_mulMatVecSparse(res, e->efc_JT, vec, m->nv, e->efc_JT_rownnz, e->efc_JT_rowadr,
                        e->efc_JT_colind);
  } else {
    mju_mulMatTVec(res, e->efc_J, vec, e->nefc, m->nv);
  }
}

/* :2362-2375 */
static void or_referenceConstraint(const mjhipModel* m, mjhipData* d, orEfc* e) {
  int nefc = e->nefc;
  mjtNum* KBIP = e->efc_KBIP;
  or_mulJacVec(m, e, e->efc_vel, d->qvel);
  for (int i = 0; i < nefc; i++) {
    e->efc_aref[i] = -KBIP[4*i+1]*e->efc_vel[i]
                     -KBIP[4*i]*KBIP[4*i+2]*(e->efc_pos[i]-e->efc_margin[i]);
  }
}

/* :2387-2549 (island < 0, cost = NULL); elliptic-cone rows come only from contacts, which
 * are outside the supported subset */
static void or_constraintUpdate(const mjhipModel* m, mjhipData* d, orEfc* e, const mjtNum* jar) {
  int ne = e->ne, nf = e->nf, nefc = e->nefc;
  const mjtNum *D = e->efc_D, *R = e->efc_R, *floss = e->efc_frictionloss;
  mjtNum* force = e->efc_force;
  if (!nefc) {
    mju_zero(d->qfrc_constraint, m->nv);
    return;
  }
  for (int i = 0; i < nefc; i++) force[i] = -D[i] * jar[i];
  for (int i = 0; i < nefc; i++) {
    if (i < ne) {
      e->efc_state[i] = orCNSTRSTATE_QUADRATIC;
      continue;
    }
    if (i < ne + nf) {
      if (jar[i] <= -R[i] * floss[i]) {
        force[i] = floss[i];
        e->efc_state[i] = orCNSTRSTATE_LINEARNEG;
      } else if (jar[i] >= R[i] * floss[i]) {
        force[i] = -floss[i];
        e->efc_state[i] = orCNSTRSTATE_LINEARPOS;
      } else {
        e->efc_state[i] = orCNSTRSTATE_QUADRATIC;
      }
      continue;
    }
    if (e->efc_type[i] != orCNSTR_CONTACT_ELLIPTIC) {
      if (jar[i] >= 0) {
        force[i] = 0;
        e->efc_state[i] = orCNSTRSTATE_SATISFIED;
      } else {
        e->efc_state[i] = orCNSTRSTATE_QUADRATIC;
      }
    } else {
      /* elliptic cone :2459-2540 (no cost, no cone Hessian) */
      int id = e->efc_id[i], dim = e->con_dim[id];
      mjtNum mu = e->con_mu[id];
      const mjtNum* friction = e->con_friction + 5*id;
      mjtNum U[6];
      U[0] = jar[i]*mu;
      for (int j = 1; j < dim; j++) U[j] = jar[i+j]*friction[j-1];
      mjtNum N = U[0], T = mju_norm(U+1, dim-1);
      if (N >= mu*T || (T <= 0 && N >= 0)) {
        mju_zero(force+i, dim);
        e->efc_state[i] = orCNSTRSTATE_SATISFIED;
      } else if (mu*N + T <= 0 || (T <= 0 && N < 0)) {
        e->efc_state[i] = orCNSTRSTATE_QUADRATIC;
      } else {
        mjtNum Dm = D[i] / (mu*mu*(1 + mu*mu));
        mjtNum NmT = N - mu*T;
        force[i] = -Dm*NmT*mu;
        for (int j = 1; j < dim; j++) force[i+j] = -force[i]/T*U[j]*friction[j-1];
        e->efc_state[i] = orCNSTRSTATE_CONE;
      }
      for (int j = 1; j < dim; j++) e->efc_state[i+j] = e->efc_state[i];
      i += dim - 1;
    }
  }
  /* mj_mulJacTVec_island(island < 0) = mj_mulJacTVec (engine_core_constraint.c:426-442) */
  or_mulJacTVec(m, e, d->qfrc_constraint, e->efc_force);
}

/*============================ engine_forward.c / engine_inverse.c =========================*/

/* engine_forward.c:193-231 */
static void or_fwdVelocity(const mjhipModel* m, mjhipData* d, orEfc* e) {
  /* tendon velocity: dense or sparse (:206-212) */
  if (mj_isSparse(m)) {
    mju_mulMatVecSparse(d->ten_velocity, d->ten_J, d->qvel, m->ntendon, d->ten_J_rownnz,
                        d->ten_J_rowadr, d->ten_J_colind);
  } else {
    mju_mulMatVec(d->ten_velocity, d->ten_J, d->qvel, m->ntendon, m->nv);
  }
  if (!mjDISABLED(mjhipDSBL_ACTUATION)) {
    for (int r = 0; r < m->nu; r++) {
      d->actuator_velocity[r] = mju_dotSparse(d->actuator_moment + m->moment_rowadr[r], d->qvel,
                                              m->moment_rownnz[r],
                                              m->moment_colind + m->moment_rowadr[r]);
    }
  }
  or_comVel(m, d);
  or_passive(m, d);
  or_referenceConstraint(m, d, e);
  or_rne(m, d, 0, d->qfrc_bias);
}

/* engine_inverse.c:37-68 (mj_collision: no contacts in the supported subset) */
void or_invPosition(const mjhipModel* m, mjhipData* d, orEfc* e) {
  or_kinematics(m, d);
  or_comPos(m, d);
  or_camlight(m, d);
  or_tendon(m, d);
  or_crb(m, d);
  or_factorM(m, d);
  or_collision(m, d, e);
  or_makeConstraint(m, d, e);
  or_transmission(m, d, e);
}

/* engine_inverse.c:73-76 */
void or_invVelocity(const mjhipModel* m, mjhipData* d, orEfc* e) {
  or_fwdVelocity(m, d, e);
}

/* engine_inverse.c:169-192 */
void or_invConstraint(const mjhipModel* m, mjhipData* d, orEfc* e) {
  int nefc = e->nefc;
  if (!nefc) {
    mju_zero(d->qfrc_constraint, m->nv);
    return;
  }
  mjtNum* jar = (mjtNum*)malloc(nefc*sizeof(mjtNum));
  or_mulJacVec(m, e, jar, d->qacc);
  mju_subFrom(jar, e->efc_aref, nefc);
  or_constraintUpdate(m, d, e, jar);
  free(jar);
}

/* engine_inverse.c:197-261 (sensors/energy: none in the supported subset;
 * mjENBL_INVDISCRETE is not supported by the oracle) */
/* engine_support.c:966-1017 mj_mulM (res = M*vec from the sparse qM) */
static void or_mulM(const mjhipModel* m, const mjhipData* d, mjtNum* res, const mjtNum* vec) {
  int nv = m->nv;
  const mjtNum* M = d->qM;
  mju_zero(res, nv);
  for (int i = 0; i < nv; i++) {
    int adr = m->dof_Madr[i];
    res[i] = M[adr]*vec[i];
    if (m->dof_simplenum[i]) continue;
    int j = m->dof_parentid[i];
    while (j >= 0) {
      adr++;
      res[i] += M[adr]*vec[j];
      res[j] += M[adr]*vec[i];
      j = m->dof_parentid[j];
    }
  }
}

/* dense value of the sparse actuator_moment row `i` at column `col` */
static mjtNum moment_at(const mjhipModel* m, const mjhipData* d, int i, int col) {
  int adr = m->moment_rowadr[i];
  for (int k = 0; k < m->moment_rownnz[i]; k++) {
    if (m->moment_colind[adr+k] == col) return d->actuator_moment[adr+k];
  }
  return 0;
}

/* qDeriv(r, c) of mjd_smooth_vel(flg_bias = 0) (engine_derivative.c:1522-1536): actuator
 * velocity terms (mjd_actuator_vel :812-870, addJTBJ :693-724), then dof damping and tendon
 * damping (mjd_passive_vel :1432-1519), in the reference's order of accumulation. Only the
 * entries on qM's sparsity are needed (the implicitfast reduction through mapD2M). */
static mjtNum or_qDeriv(const mjhipModel* m, const mjhipData* d, int r, int c) {
  mjtNum q = 0;
  if (!mjDISABLED(mjhipDSBL_ACTUATION)) {
    for (int i = 0; i < m->nu; i++) {
      mjtNum bias_vel = 0, gain_vel = 0;
      if (m->actuator_biastype[i] == mjhipBIAS_AFFINE) bias_vel = m->actuator_biasprm[10*i+2];
      if (m->actuator_gaintype[i] == mjhipGAIN_AFFINE) gain_vel = m->actuator_gainprm[10*i+2];
      if (gain_vel != 0) bias_vel += gain_vel * d->ctrl[i];
      if (bias_vel != 0) {
        mjtNum mr = moment_at(m, d, i, r);
        if (mr) q += moment_at(m, d, i, c) * (mr * bias_vel);
      }
    }
  }
  if (!mjDISABLED(mjhipDSBL_PASSIVE)) {
    if (r == c) q -= m->dof_damping[r];
    for (int t = 0; t < m->ntendon; t++) {
      if (m->tendon_damping[t] > 0) {
        mjtNum B = -m->tendon_damping[t];
        /* addJTBJ :693-724, or addJTBJSparse :729-755 for a sparse model, whose only extra
           terms are exact zeros (structural entries of value 0) */
        mjtNum Jr = ten_J_at(m, d, t, r);
        if (Jr) q += ten_J_at(m, d, t, c) * (Jr * B);
      }
    }
  }
  return q;
}

/*---------------- mjd_rne_vel: d qfrc_bias / d qvel (the implicit integrator) ---------------*/

/* 6x6 Jacobians of the spatial helpers (engine_derivative.c:65-186). Each lists the nonzero
 * entries (row, col, value) of the partial derivative of the helper's output in the given
 * argument; everything else is zero. */
static void or_set36(mjtNum D[36], const int* rc, const mjtNum* val, int n) {
  mju_zero(D, 36);
  for (int k = 0; k < n; k++) D[rc[2*k]*6 + rc[2*k+1]] = val[k];
}

/* crossMotion(vel, v) w.r.t. vel (:65-99) */
static void or_crossMotion_vel(mjtNum D[36], const mjtNum v[6]) {
  static const int rc[] = {0,2, 0,1, 1,2, 1,0, 2,1, 2,0, 3,2, 3,1, 3,5, 3,4,
                           4,2, 4,0, 4,5, 4,3, 5,1, 5,0, 5,4, 5,3};
  const mjtNum val[] = {-v[1], v[2], v[0], -v[2], -v[0], v[1], -v[4], v[5], -v[1], v[2],
                        v[3], -v[5], v[0], -v[2], -v[3], v[4], -v[0], v[1]};
  or_set36(D, rc, val, 18);
}

/* crossForce(vel, f) w.r.t. vel (:103-136) */
static void or_crossForce_vel(mjtNum D[36], const mjtNum f[6]) {
  static const int rc[] = {0,2, 0,1, 0,5, 0,4, 1,2, 1,0, 1,5, 1,3, 2,1, 2,0, 2,4, 2,3,
                           3,2, 3,1, 4,2, 4,0, 5,1, 5,0};
  const mjtNum val[] = {-f[1], f[2], -f[4], f[5], f[0], -f[2], f[3], -f[5], -f[0], f[1],
                        -f[3], f[4], -f[4], f[5], f[3], -f[5], -f[3], f[4]};
  or_set36(D, rc, val, 18);
}

/* crossForce(vel, f) w.r.t. f (:140-173) */
static void or_crossForce_frc(mjtNum D[36], const mjtNum vel[6]) {
  static const int rc[] = {0,1, 0,2, 0,4, 0,5, 1,0, 1,2, 1,3, 1,5, 2,0, 2,1, 2,3, 2,4,
                           3,4, 3,5, 4,3, 4,5, 5,3, 5,4};
  const mjtNum val[] = {-vel[2], vel[1], -vel[5], vel[4], vel[2], -vel[0], vel[5], -vel[3],
                        -vel[1], vel[0], -vel[4], vel[3], -vel[2], vel[1], vel[2], -vel[0],
                        -vel[1], vel[0]};
  or_set36(D, rc, val, 18);
}

/* mulInertVec(i, v) w.r.t. v (:178-213) */
static void or_mulInertVec_vel(mjtNum D[36], const mjtNum i[10]) {
  static const int rc[] = {0,0, 0,1, 0,2, 0,4, 0,5, 1,0, 1,1, 1,2, 1,3, 1,5, 2,0, 2,1,
                           2,2, 2,3, 2,4, 3,1, 3,2, 3,3, 4,2, 4,0, 4,4, 5,0, 5,1, 5,5};
  const mjtNum val[] = {i[0], i[3], i[4], -i[8], i[7], i[3], i[1], i[5], i[8], -i[6],
                        i[4], i[5], i[2], -i[7], i[6], i[8], -i[7], i[9], i[6], -i[8],
                        i[9], i[7], -i[6], i[9]};
  or_set36(D, rc, val, 24);
}

static void or_transpose6(mjtNum res[36], const mjtNum mat[36]) {
  for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) res[c*6+r] = mat[r*6+c];
}

/* number of dof ancestors of dof j (engine_derivative.c:542) */
static int or_Jadr(const mjhipModel* m, int j) {
  return (j < m->nv - 1 ? m->dof_Madr[j+1] : m->nM) - (m->dof_Madr[j] + 1);
}

/* :484-500 copyFromParent: body n's B row starts with its ancestors' dofs, as does its
 * parent's row */
static void or_copyFromParent(const mjhipModel* m, mjtNum* mat, int n) {
  if (n == 0 || m->body_weldid[m->body_parentid[n]] == 0) return;
  int ndof = 0;
  for (int p = m->body_weldid[m->body_parentid[n]]; p > 0;
       p = m->body_weldid[m->body_parentid[p]]) {
    ndof += m->body_dofnum[p];
  }
  mju_copy(mat + 6*m->B_rowadr[n], mat + 6*m->B_rowadr[m->body_parentid[n]], 6*ndof);
}

/* :505-531 addToParent: add body n's row into its parent's at matching columns */
static void or_addToParent(const mjhipModel* m, mjtNum* mat, int n) {
  if (n == 0 || m->body_weldid[m->body_parentid[n]] == 0) return;
  int np = m->body_parentid[n];
  const int* cn = m->B_colind + m->B_rowadr[n];
  const int* cp = m->B_colind + m->B_rowadr[np];
  for (int i = 0, ip = 0; i < m->B_rownnz[n] && ip < m->B_rownnz[np]; ) {
    if (cn[i] == cp[ip]) {
      mju_addTo(mat + 6*(m->B_rowadr[np] + ip), mat + 6*(m->B_rowadr[n] + i), 6);
      i++;
      ip++;
    } else {
      ip++;                             /* child columns are a subset of the parent's */
    }
  }
}

/* :535-600 mjd_comVel_vel: Dcvel (B sparsity) and Dcdofdot (D sparsity), each nonzero a
 * 6-vector */
static void or_comVel_vel(const mjhipModel* m, const mjhipData* d, mjtNum* Dcvel,
                          mjtNum* Dcdofdot) {
  mjtNum mat[36], matT[36];
  for (int i = 1; i < m->nbody; i++) {
    or_copyFromParent(m, Dcvel, i);
    mjtNum* row = Dcvel + 6*m->B_rowadr[i];
    int last = m->body_dofadr[i] + m->body_dofnum[i];
    for (int j = m->body_dofadr[i]; j < last; j++) {
      int Jadr = or_Jadr(m, j);
      int t = m->jnt_type[m->dof_jntid[j]];
      int nrot = 1;                     /* rotational dofs handled below */
      if (t == mjhipJNT_FREE) {         /* translations: Dcdofdot stays zero */
        for (int k = 0; k < 3; k++) mju_addTo(row + 6*(Jadr + k), d->cdof + 6*(j + k), 6);
        j += 3;
        Jadr += 3;
        nrot = 3;
      } else if (t == mjhipJNT_BALL) {
        nrot = 3;
      }
      for (int k = 0; k < nrot; k++) {
        or_crossMotion_vel(mat, d->cdof + 6*(j + k));
        or_transpose6(matT, mat);
        mju_mulMatMat(Dcdofdot + 6*m->D_rowadr[j + k], row, matT, Jadr + k, 6, 6);
      }
      for (int k = 0; k < nrot; k++) mju_addTo(row + 6*(Jadr + k), d->cdof + 6*(j + k), 6);
      j += nrot - 1;
    }
  }
}

/* :604-690 mjd_rne_vel: qDeriv -= d qfrc_bias / d qvel on the D sparsity */
static void or_rne_vel(const mjhipModel* m, const mjhipData* d, mjtNum* qDeriv) {
  const int nB = m->nB, nD = m->nD;
  mjtNum* Dcdofdot = (mjtNum*)calloc(6*(size_t)nD + 1, sizeof(mjtNum));
  mjtNum* Dcvel = (mjtNum*)calloc(6*(size_t)nB + 1, sizeof(mjtNum));
  mjtNum* Dcacc = (mjtNum*)calloc(6*(size_t)nB + 1, sizeof(mjtNum));
  mjtNum* Dcfrc = (mjtNum*)calloc(6*(size_t)nB + 1, sizeof(mjtNum));
  mjtNum* tmp6 = (mjtNum*)calloc(6*(size_t)m->nv + 1, sizeof(mjtNum));
  mjtNum mat[36], mat1[36], mat2[36], dmul[36], tmp[6];
  or_comVel_vel(m, d, Dcvel, Dcdofdot);
  for (int i = 1; i < m->nbody; i++) {
    or_copyFromParent(m, Dcacc, i);
    const int nnz = m->B_rownnz[i];
    mjtNum* acc = Dcacc + 6*m->B_rowadr[i];
    int last = m->body_dofadr[i] + m->body_dofnum[i];
    for (int j = m->body_dofadr[i]; j < last; j++) {
      mju_addTo(acc + 6*or_Jadr(m, j), d->cdof_dot + 6*j, 6);
      mju_addToScl(acc, Dcdofdot + 6*m->D_rowadr[j], d->qvel[j], 6*nnz);
    }
    /* Dcfrc = (d mulInertVec / d cacc) Dcacc + (d crossForce / d cvel
     *         + d crossForce / d f * d mulInertVec / d cvel) Dcvel */
    or_mulInertVec_vel(dmul, d->cinert + 10*i);
    or_transpose6(mat1, dmul);
    mju_mulMatMat(Dcfrc + 6*m->B_rowadr[i], acc, mat1, nnz, 6, 6);
    mju_mulInertVec(tmp, d->cinert + 10*i, d->cvel + 6*i);
    or_crossForce_vel(mat, tmp);
    or_crossForce_frc(mat1, d->cvel + 6*i);
    mju_mulMatMat(mat2, mat1, dmul, 6, 6, 6);
    mju_addTo(mat, mat2, 36);
    or_transpose6(mat1, mat);
    mju_mulMatMat(tmp6, Dcvel + 6*m->B_rowadr[i], mat1, nnz, 6, 6);
    mju_addTo(Dcfrc + 6*m->B_rowadr[i], tmp6, 6*nnz);
  }
  for (int i = m->nbody - 1; i > 0; i--) or_addToParent(m, Dcfrc, i);
  for (int j = 0; j < m->nv; j++) {
    int i = m->dof_bodyid[j];
    mju_mulMatVec(tmp6, Dcfrc + 6*m->B_rowadr[i], d->cdof + 6*j, m->B_rownnz[i], 6);
    mju_subFrom(qDeriv + m->D_rowadr[j], tmp6, m->B_rownnz[i]);
  }
  free(Dcdofdot); free(Dcvel); free(Dcacc); free(Dcfrc); free(tmp6);
}

/*---------------- fluid force derivatives (mjd_passive_vel's fluid part) ---------------------*/

static mjtNum or_maxMoment(const mjtNum s[3], int k);
static void or_semiAxes(const mjhipModel* m, int g, mjtNum ax[3]);
static void or_objectVelocity(const mjhipModel* m, const mjhipData* d, int type, int id,
                              mjtNum res[6], int flg_local);
static void mju_transformSpatial(mjtNum res[6], const mjtNum vec[6], int flg_force,
                                 const mjtNum newpos[3], const mjtNum oldpos[3],
                                 const mjtNum* rotnew2old);

/* addJTBJ :693-724: qDeriv (D sparsity) += J' B J for the n x n matrix B and the n rows of J */
static void or_addJTBJ(const mjhipModel* m, mjtNum* qDeriv, const mjtNum* J, const mjtNum* B,
                       int n) {
  const int nv = m->nv;
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < n; j++) {
      if (!B[i*n+j]) continue;
      for (int k = 0; k < nv; k++) {
        if (!J[i*nv+k]) continue;
        const mjtNum s = J[i*nv+k] * B[i*n+j];
        for (int a = m->D_rowadr[k]; a < m->D_rowadr[k] + m->D_rownnz[k]; a++) {
          qDeriv[a] += J[j*nv + m->D_colind[a]] * s;
        }
      }
    }
  }
}

/* :898-909 addToQuadrant (B is indexed column-major in 3x3 blocks) */
static void or_addToQuadrant(mjtNum* B, const mjtNum D[9], int col_quad, int row_quad) {
  const int r = 3*row_quad, c = 3*col_quad;
  for (int k = 0; k < 3; k++) {
    for (int l = 0; l < 3; l++) B[6*(c+k) + r+l] += D[3*k+l];
  }
}

/* :38-61 mjd_cross */
static void or_dcross(const mjtNum a[3], const mjtNum b[3], mjtNum* Da, mjtNum* Db) {
  mju_zero(Da, 9);
  Da[1] =  b[2]; Da[2] = -b[1]; Da[3] = -b[2]; Da[5] =  b[0]; Da[6] =  b[1]; Da[7] = -b[0];
  mju_zero(Db, 9);
  Db[1] = -a[2]; Db[2] =  a[1]; Db[3] =  a[2]; Db[5] = -a[0]; Db[6] = -a[1]; Db[7] =  a[0];
}

static void or_addToScl3(mjtNum* r, const mjtNum* a, mjtNum s) {
  r[0] += a[0]*s; r[1] += a[1]*s; r[2] += a[2]*s;
}

/* :916-957 mjd_addedMassForces */
static void or_dAddedMass(mjtNum* B, const mjtNum lv[6], mjtNum rho, const mjtNum vm[3],
                          const mjtNum vi[3]) {
  const mjtNum lin[3] = {lv[3], lv[4], lv[5]}, ang[3] = {lv[0], lv[1], lv[2]};
  const mjtNum plin[3] = {rho*vm[0]*lin[0], rho*vm[1]*lin[1], rho*vm[2]*lin[2]};
  const mjtNum pang[3] = {rho*vi[0]*ang[0], rho*vi[1]*ang[1], rho*vi[2]*ang[2]};
  mjtNum Da[9], Db[9];
  or_dcross(pang, ang, Da, Db);
  or_addToQuadrant(B, Db, 0, 0);
  for (int i = 0; i < 9; i++) Da[i] *= rho * vi[i % 3];
  or_addToQuadrant(B, Da, 0, 0);
  or_dcross(plin, lin, Da, Db);
  or_addToQuadrant(B, Db, 0, 1);
  for (int i = 0; i < 9; i++) Da[i] *= rho * vm[i % 3];
  or_addToQuadrant(B, Da, 0, 1);
  or_dcross(plin, ang, Da, Db);
  or_addToQuadrant(B, Db, 1, 0);
  for (int i = 0; i < 9; i++) Da[i] *= rho * vm[i % 3];
  or_addToQuadrant(B, Da, 1, 1);
}

/* :962-1011 mjd_viscous_torque */
static void or_dViscousTorque(mjtNum* D, const mjtNum lv[6], mjtNum rho, mjtNum mu,
                              const mjtNum s[3], mjtNum slender, mjtNum angdrag) {
  const mjtNum dmax = mjMAX(mjMAX(s[0], s[1]), s[2]);
  const mjtNum dmin = mjMIN(mjMIN(s[0], s[1]), s[2]);
  const mjtNum dmid = s[0] + s[1] + s[2] - dmax - dmin;
  const mjtNum eqD = 2.0/3.0 * (s[0] + s[1] + s[2]);
  const mjtNum lin_visc = mjhipPI * eqD*eqD*eqD;
  const mjtNum Imax = 8.0/15.0 * mjhipPI * dmid * (dmax*dmax)*(dmax*dmax);
  const mjtNum II[3] = {or_maxMoment(s, 0), or_maxMoment(s, 1), or_maxMoment(s, 2)};
  const mjtNum x = lv[0], y = lv[1], z = lv[2];
  const mjtNum mc[3] = {angdrag*II[0] + slender*(Imax - II[0]),
                        angdrag*II[1] + slender*(Imax - II[1]),
                        angdrag*II[2] + slender*(Imax - II[2])};
  const mjtNum mv[3] = {x * mc[0], y * mc[1], z * mc[2]};
  const mjtNum density = rho / mjMAX(mjMINVAL, mju_norm3(mv));
  const mjtNum msq[3] = {-density * x * mc[0] * mc[0], -density * y * mc[1] * mc[1],
                         -density * z * mc[2] * mc[2]};
  const mjtNum lin_coef = mu * lin_visc;
  mju_zero(D, 9);
  D[0] = D[4] = D[8] = x*msq[0] + y*msq[1] + z*msq[2] - lin_coef;
  or_addToScl3(D, msq, x);
  or_addToScl3(D+3, msq, y);
  or_addToScl3(D+6, msq, z);
}

/* :1016-1079 mjd_viscous_drag */
static void or_dViscousDrag(mjtNum* D, const mjtNum lv[6], mjtNum rho, mjtNum mu,
                            const mjtNum s[3], mjtNum blunt, mjtNum slender) {
  const mjtNum dmax = mjMAX(mjMAX(s[0], s[1]), s[2]);
  const mjtNum dmin = mjMIN(mjMIN(s[0], s[1]), s[2]);
  const mjtNum dmid = s[0] + s[1] + s[2] - dmax - dmin;
  const mjtNum eqD = 2.0/3.0 * (s[0] + s[1] + s[2]);
  const mjtNum Amax = mjhipPI * dmax * dmid;
  const mjtNum a = (s[1]*s[2])*(s[1]*s[2]), b = (s[2]*s[0])*(s[2]*s[0]);
  const mjtNum c = (s[0]*s[1])*(s[0]*s[1]);
  const mjtNum aa = a*a, bb = b*b, cc = c*c;
  const mjtNum x = lv[3], y = lv[4], z = lv[5];
  const mjtNum xx = x*x, yy = y*y, zz = z*z, xy = x*y, yz = y*z, xz = x*z;
  const mjtNum pden = aa*xx + bb*yy + cc*zz;
  const mjtNum pnum = a*xx + b*yy + c*zz;
  const mjtNum dA = mjhipPI / mjMAX(mjMINVAL, sqrt(pnum*pnum*pnum * pden));
  const mjtNum Aproj = mjhipPI * sqrt(pden/mjMAX(mjMINVAL, pnum));
  const mjtNum norm = sqrt(xx + yy + zz);
  const mjtNum inv_norm = 1.0 / mjMAX(mjMINVAL, norm);
  const mjtNum lin_coef = mu * 3.0 * mjhipPI * eqD;
  const mjtNum quad_coef = rho * (Aproj*blunt + slender*(Amax - Aproj));
  const mjtNum Ac = rho * norm * (blunt - slender);
  const mjtNum dAv[3] = {Ac * dA * a * x * (b * yy * (a - b) + c * zz * (a - c)),
                         Ac * dA * b * y * (a * xx * (b - a) + c * zz * (b - c)),
                         Ac * dA * c * z * (a * xx * (c - a) + b * yy * (c - b))};
  D[0] = xx; D[1] = xy; D[2] = xz;
  D[3] = xy; D[4] = yy; D[5] = yz;
  D[6] = xz; D[7] = yz; D[8] = zz;
  const mjtNum inner = xx + yy + zz;
  D[0] += inner; D[4] += inner; D[8] += inner;
  mju_scl(D, D, -quad_coef*inv_norm, 9);
  or_addToScl3(D+0, dAv, -x);
  or_addToScl3(D+3, dAv, -y);
  or_addToScl3(D+6, dAv, -z);
  D[0] -= lin_coef; D[4] -= lin_coef; D[8] -= lin_coef;
}

/* :1084-1133 mjd_kutta_lift */
static void or_dKuttaLift(mjtNum* D, const mjtNum lv[6], mjtNum rho, const mjtNum s[3],
                          mjtNum kutta) {
  const mjtNum a = (s[1]*s[2])*(s[1]*s[2]), b = (s[2]*s[0])*(s[2]*s[0]);
  const mjtNum c = (s[0]*s[1])*(s[0]*s[1]);
  const mjtNum aa = a*a, bb = b*b, cc = c*c;
  const mjtNum x = lv[3], y = lv[4], z = lv[5];
  const mjtNum xx = x*x, yy = y*y, zz = z*z, xy = x*y, yz = y*z, xz = x*z;
  const mjtNum pden = aa*xx + bb*yy + cc*zz;
  const mjtNum pnum = a*xx + b*yy + c*zz;
  const mjtNum norm2 = xx + yy + zz;
  const mjtNum df_denom = mjhipPI * kutta * rho / mjMAX(mjMINVAL, sqrt(pden * pnum * norm2));
  const mjtNum dfx = yy * (a - b) + zz * (a - c);
  const mjtNum dfy = xx * (b - a) + zz * (b - c);
  const mjtNum dfz = xx * (c - a) + yy * (c - b);
  const mjtNum proj_term = pnum / mjMAX(mjMINVAL, pden);
  const mjtNum cos_term = pnum / mjMAX(mjMINVAL, norm2);
  D[0] = a-a; D[1] = b-a; D[2] = c-a;
  D[3] = a-b; D[4] = b-b; D[5] = c-b;
  D[6] = a-c; D[7] = b-c; D[8] = c-c;
  mju_scl(D, D, 2 * pnum, 9);
  const mjtNum inner[3] = {aa * proj_term - a + cos_term, bb * proj_term - b + cos_term,
                           cc * proj_term - c + cos_term};
  or_addToScl3(D + 0, inner, dfx);
  or_addToScl3(D + 3, inner, dfy);
  or_addToScl3(D + 6, inner, dfz);
  D[0] *= xx; D[1] *= xy; D[2] *= xz;
  D[3] *= xy; D[4] *= yy; D[5] *= yz;
  D[6] *= xz; D[7] *= yz; D[8] *= zz;
  D[0] -= dfx * pnum;
  D[4] -= dfy * pnum;
  D[8] -= dfz * pnum;
  mju_scl(D, D, df_denom, 9);
}

/* :1138-1161 mjd_magnus_force */
static void or_dMagnus(mjtNum* B, const mjtNum lv[6], mjtNum rho, const mjtNum s[3],
                       mjtNum magnus) {
  const mjtNum volume = 4.0/3.0 * mjhipPI * s[0] * s[1] * s[2];
  const mjtNum coef = magnus * rho * volume;
  mjtNum Dlin[9], Dang[9];
  const mjtNum lin[3] = {coef * lv[3], coef * lv[4], coef * lv[5]};
  const mjtNum ang[3] = {coef * lv[0], coef * lv[1], coef * lv[2]};
  or_dcross(ang, lin, Dang, Dlin);
  or_addToQuadrant(B, Dang, 1, 0);
  or_addToQuadrant(B, Dlin, 1, 1);
}

/* the local 6 x nv Jacobian of a frame (rotation rows, then translation): mj_jac at `point`,
 * each half rotated by mju_mulMatTMat(xmat, ., 3, 3, nv) (engine_util_blas.c:884-897) */
static void or_localJac(const mjhipModel* m, const mjhipData* d, mjtNum* J, mjtNum* tmp,
                        const mjtNum* point, const mjtNum* xmat, int body) {
  const int nv = m->nv;
  mj_jac(m, d, J + 3*nv, J, point, body);
  for (int h = 0; h < 2; h++) {
    mju_zero(tmp, 3*nv);
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++) {
        if (xmat[3*i+j]) mju_addToScl(tmp + j*nv, J + 3*h*nv + i*nv, xmat[3*i+j], nv);
      }
    }
    mju_copy(J + 3*h*nv, tmp, 3*nv);
  }
}

/* :1168-1270 mjd_ellipsoidFluid (dense) */
static void or_dEllipsoidFluid(const mjhipModel* m, const mjhipData* d, mjtNum* qDeriv,
                               int b, mjtNum* J, mjtNum* tmp) {
  for (int j = 0; j < m->body_geomnum[b]; j++) {
    const int g = m->body_geomadr[b] + j;
    const mjtNum* c = m->geom_fluid + 12*g;
    mjtNum ax[3], lvel[6], wind[6], lwind[6], B[36], D[9];
    or_semiAxes(m, g, ax);
    if (c[0] == 0.0) continue;
    or_objectVelocity(m, d, OBJ_GEOM, g, lvel, 1);
    mju_zero(wind, 6);
    mju_copy3(wind+3, m->opt.wind);
    mju_transformSpatial(lwind, wind, 0, d->geom_xpos + 3*g,
                         d->subtree_com + 3*m->body_rootid[b], d->geom_xmat + 9*g);
    lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
    or_localJac(m, d, J, tmp, d->geom_xpos + 3*g, d->geom_xmat + 9*g, m->geom_bodyid[g]);
    mju_zero(B, 36);
    or_dMagnus(B, lvel, m->opt.density, ax, c[5]);
    or_dKuttaLift(D, lvel, m->opt.density, ax, c[4]);
    or_addToQuadrant(B, D, 1, 1);
    or_dViscousDrag(D, lvel, m->opt.density, m->opt.viscosity, ax, c[1], c[2]);
    or_addToQuadrant(B, D, 1, 1);
    or_dViscousTorque(D, lvel, m->opt.density, m->opt.viscosity, ax, c[2], c[3]);
    or_addToQuadrant(B, D, 0, 0);
    or_dAddedMass(B, lvel, m->opt.density, c + 6, c + 9);
    if (m->opt.integrator == mjhipINT_IMPLICITFAST) {     /* mju_symmetrize (blas.c:794-801) */
      for (int r = 0; r < 6; r++) {
        for (int k = 0; k < r; k++) B[r*6+k] = B[k*6+r] = 0.5 * (B[r*6+k] + B[k*6+r]);
      }
    }
    or_addJTBJ(m, qDeriv, J, B, 6);
  }
}

/* :1275-1425 mjd_inertiaBoxFluid (dense) */
static void or_dInertiaBoxFluid(const mjhipModel* m, const mjhipData* d, mjtNum* qDeriv,
                                int i, mjtNum* J, mjtNum* tmp) {
  const int nv = m->nv;
  const mjtNum* inertia = m->body_inertia + 3*i;
  const mjtNum rho = m->opt.density, mu = m->opt.viscosity;
  mjtNum lvel[6], wind[6], lwind[6], box[3], B;
  box[0] = sqrt(mjMAX(mjMINVAL, (inertia[1] + inertia[2] - inertia[0])) / m->body_mass[i] * 6.0);
  box[1] = sqrt(mjMAX(mjMINVAL, (inertia[0] + inertia[2] - inertia[1])) / m->body_mass[i] * 6.0);
  box[2] = sqrt(mjMAX(mjMINVAL, (inertia[0] + inertia[1] - inertia[2])) / m->body_mass[i] * 6.0);
  or_objectVelocity(m, d, OBJ_BODY, i, lvel, 1);
  mju_zero(wind, 6);
  mju_copy3(wind+3, m->opt.wind);
  mju_transformSpatial(lwind, wind, 0, d->xipos+3*i, d->subtree_com+3*m->body_rootid[i],
                       d->ximat+9*i);
  lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
  or_localJac(m, d, J, tmp, d->xipos + 3*i, d->ximat + 9*i, i);
  if (mu > 0) {
    const mjtNum diam = (box[0] + box[1] + box[2])/3.0;
    B = -mjhipPI*diam*diam*diam*mu;
    for (int j = 0; j < 3; j++) or_addJTBJ(m, qDeriv, J + j*nv, &B, 1);
    B = -3.0*mjhipPI*diam*mu;
    for (int j = 0; j < 3; j++) or_addJTBJ(m, qDeriv, J + 3*nv + j*nv, &B, 1);
  }
  if (rho > 0) {
    B = -rho*box[0]*(box[1]*box[1]*box[1]*box[1]+box[2]*box[2]*box[2]*box[2])*
        2*fabs(lvel[0])/64.0;
    or_addJTBJ(m, qDeriv, J, &B, 1);
    B = -rho*box[1]*(box[0]*box[0]*box[0]*box[0]+box[2]*box[2]*box[2]*box[2])*
        2*fabs(lvel[1])/64.0;
    or_addJTBJ(m, qDeriv, J + nv, &B, 1);
    B = -rho*box[2]*(box[0]*box[0]*box[0]*box[0]+box[1]*box[1]*box[1]*box[1])*
        2*fabs(lvel[2])/64.0;
    or_addJTBJ(m, qDeriv, J + 2*nv, &B, 1);
    B = -0.5*rho*box[1]*box[2]*2*fabs(lvel[3]);
    or_addJTBJ(m, qDeriv, J + 3*nv, &B, 1);
    B = -0.5*rho*box[0]*box[2]*2*fabs(lvel[4]);
    or_addJTBJ(m, qDeriv, J + 4*nv, &B, 1);
    B = -0.5*rho*box[0]*box[1]*2*fabs(lvel[5]);
    or_addJTBJ(m, qDeriv, J + 5*nv, &B, 1);
  }
}

/* mjd_passive_vel :1494-1513: the fluid models' derivatives, per body as mj_fluid chooses */
static void or_dFluid(const mjhipModel* m, const mjhipData* d, mjtNum* qDeriv) {
  if (mjDISABLED(mjhipDSBL_PASSIVE) || !(m->opt.viscosity > 0 || m->opt.density > 0)) return;
  mjtNum* J = (mjtNum*)malloc((6*(size_t)m->nv + 1)*sizeof(mjtNum));
  mjtNum* tmp = (mjtNum*)malloc((3*(size_t)m->nv + 1)*sizeof(mjtNum));
  for (int i = 1; i < m->nbody; i++) {
    if (m->body_mass[i] < mjMINVAL) continue;
    int ell = 0;
    for (int j = 0; j < m->body_geomnum[i] && ell == 0; j++) {
      ell += m->geom_fluid[12*(m->body_geomadr[i] + j)] > 0;
    }
    if (ell) or_dEllipsoidFluid(m, d, qDeriv, i, J, tmp);
    else or_dInertiaBoxFluid(m, d, qDeriv, i, J, tmp);
  }
  free(J);
  free(tmp);
}

/* mjd_smooth_vel (engine_derivative.c:1522-1536) on the D sparsity: uses the position/velocity
 * quantities already in d */
void or_smoothVel(const mjhipModel* m, const mjhipData* d, mjtNum* qDeriv, int flg_bias) {
  for (int r = 0; r < m->nv; r++) {
    for (int k = 0; k < m->D_rownnz[r]; k++) {
      qDeriv[m->D_rowadr[r] + k] = or_qDeriv(m, d, r, m->D_colind[m->D_rowadr[r] + k]);
    }
  }
  or_dFluid(m, d, qDeriv);
  if (flg_bias) or_rne_vel(m, d, qDeriv);
}

/* address of (r, c) in the D sparsity (mapD2M's inverse lookup; c is an ancestor of r) */
static int or_Dadr(const mjhipModel* m, int r, int c) {
  for (int a = m->D_rowadr[r]; a < m->D_rowadr[r] + m->D_rownnz[r]; a++) {
    if (m->D_colind[a] == c) return a;
  }
  return -1;                                  /* SHOULD NOT OCCUR */
}

/* engine_inverse.c:81-164 mj_discreteAcc:
 *   Euler: qacc <- M^-1 (M + h*diag(B)) qacc when implicit damping applies
 *   implicitfast: qacc <- M^-1 (M - h*qDeriv) qacc, qDeriv reduced to qM's sparsity
 *   implicit: qacc <- M^-1 (M - h*qDeriv) qacc with the full qDeriv (incl. mjd_rne_vel) on
 *   the D sparsity (the reference's qLU before factorization)
 * RK4 is an error in the reference: MJHIP_INST_UNSUPPORTED, qacc unchanged. */
static void or_discreteAcc(const mjhipModel* m, mjhipData* d) {
  int nv = m->nv;
  if (m->opt.integrator == mjhipINT_IMPLICITFAST) {
    /* mjd_smooth_vel(flg_bias = 0) on the D sparsity, reduced to qM's (mapD2M) */
    mjtNum* qMsave = (mjtNum*)malloc(m->nM*sizeof(mjtNum));
    mjtNum* qfrc = (mjtNum*)malloc(nv*sizeof(mjtNum));
    mjtNum* qDeriv = (mjtNum*)malloc((m->nD + 1)*sizeof(mjtNum));
    or_smoothVel(m, d, qDeriv, 0);
    mju_copy(qMsave, d->qM, m->nM);
    for (int r = 0; r < nv; r++) {          /* qM += qDerivReduced * -h */
      int adr = m->dof_Madr[r];
      for (int c = r; c >= 0; c = m->dof_parentid[c]) {
        d->qM[adr] = d->qM[adr] + qDeriv[or_Dadr(m, r, c)] * -m->opt.timestep;
        adr++;
      }
    }
    free(qDeriv);
    or_mulM(m, d, qfrc, d->qacc);
    mju_copy(d->qM, qMsave, m->nM);
    or_solveM(m, d, d->qacc, qfrc, 1);
    free(qMsave);
    free(qfrc);
    return;
  }
  if (m->opt.integrator == mjhipINT_IMPLICIT) {
    /* mjd_smooth_vel(flg_bias = 1) on the D sparsity, qLU = qM (via mapM2D) - h*qDeriv,
     * qfrc = qLU*qacc (mju_mulMatVecSparse, engine_util_sparse.c:156-166) */
    mjtNum* qDeriv = (mjtNum*)malloc((m->nD + 1)*sizeof(mjtNum));
    mjtNum* qfrc = (mjtNum*)malloc((nv + 1)*sizeof(mjtNum));
    or_smoothVel(m, d, qDeriv, 1);
    for (int i = 0; i < m->nD; i++) {
      qDeriv[i] = d->qM[m->mapM2D[i]] + qDeriv[i] * -m->opt.timestep;   /* now qLU */
    }
    for (int r = 0; r < nv; r++) {
      qfrc[r] = mju_dotSparse(qDeriv + m->D_rowadr[r], d->qacc, m->D_rownnz[r],
                              m->D_colind + m->D_rowadr[r]);
    }
    or_solveM(m, d, d->qacc, qfrc, 1);
    free(qDeriv);
    free(qfrc);
    return;
  }
  if (m->opt.integrator != mjhipINT_EULER) {
    d->status |= MJHIP_INST_UNSUPPORTED;
    return;
  }
  int dof_damping = 0;
  if (!mjDISABLED(mjhipDSBL_EULERDAMP)) {
    for (int i = 0; i < nv; i++) {
      if (m->dof_damping[i] > 0) {
        dof_damping = 1;
        break;
      }
    }
  }
  if (!dof_damping) return;
  mjtNum* qfrc = (mjtNum*)malloc(nv*sizeof(mjtNum));
  or_mulM(m, d, qfrc, d->qacc);
  for (int i = 0; i < nv; i++) qfrc[i] += m->opt.timestep * m->dof_damping[i] * d->qacc[i];
  or_solveM(m, d, d->qacc, qfrc, 1);
  free(qfrc);
}

/* engine_sensor.c:920-1008 mj_energyPos: gravity, joint and tendon spring energy (no flex).
 * As the reference, the free joint's translational term normalizes (x, y, z, qw) as a
 * quaternion before differencing, and the ball term differences the raw qpos quaternion. */
static void or_energyPos(const mjhipModel* m, mjhipData* d) {
  mjtNum dif[3], quat[4];
  d->energy[0] = 0;
  if (!mjDISABLED(mjhipDSBL_GRAVITY)) {
    for (int i = 1; i < m->nbody; i++) {
      d->energy[0] -= m->body_mass[i] * mju_dot3(m->opt.gravity, d->xipos + 3*i);
    }
  }
  if (mjDISABLED(mjhipDSBL_PASSIVE)) return;
  for (int i = 0; i < m->njnt; i++) {
    mjtNum k = m->jnt_stiffness[i];
    int padr = m->jnt_qposadr[i];
    int t = m->jnt_type[i];
    if (t == mjhipJNT_FREE || t == mjhipJNT_BALL) {
      if (t == mjhipJNT_FREE) {
        mju_copy(quat, d->qpos + padr, 4);
        mju_normalize4(quat);
        mju_sub3(dif, quat, m->qpos_spring + padr);
        d->energy[0] += 0.5*k*mju_dot3(dif, dif);
        padr += 3;
      }
      mju_subQuat(dif, d->qpos + padr, m->qpos_spring + padr);
      d->energy[0] += 0.5*k*mju_dot3(dif, dif);
    } else {
      mjtNum x = d->qpos[padr] - m->qpos_spring[padr];
      d->energy[0] += 0.5*k*x*x;
    }
  }
  for (int i = 0; i < m->ntendon; i++) {
    mjtNum len = d->ten_length[i], disp = 0;
    mjtNum lo = m->tendon_lengthspring[2*i], hi = m->tendon_lengthspring[2*i+1];
    if (len > hi) disp = hi - len;
    else if (len < lo) disp = lo - len;
    d->energy[0] += 0.5*m->tendon_stiffness[i]*disp*disp;
  }
}

/* engine_sensor.c:1011-1020 mj_energyVel: 0.5 qvel' M qvel */
static void or_energyVel(const mjhipModel* m, mjhipData* d) {
  mjtNum* vec = (mjtNum*)malloc((m->nv + 1)*sizeof(mjtNum));
  or_mulM(m, d, vec, d->qvel);
  d->energy[1] = 0.5*mju_dot(vec, d->qvel, m->nv);
  free(vec);
}

/*============================ engine_sensor.c =============================================*/

/* mjtSensor / mjtObj / mjtDataType values (mjmodel.h) */
enum { SENS_TOUCH = 0, SENS_ACCELEROMETER, SENS_VELOCIMETER, SENS_GYRO, SENS_FORCE, SENS_TORQUE,
       SENS_MAGNETOMETER, SENS_RANGEFINDER, SENS_CAMPROJECTION, SENS_JOINTPOS, SENS_JOINTVEL,
       SENS_TENDONPOS, SENS_TENDONVEL, SENS_ACTUATORPOS, SENS_ACTUATORVEL, SENS_ACTUATORFRC,
       SENS_JOINTACTFRC, SENS_BALLQUAT, SENS_BALLANGVEL, SENS_JOINTLIMITPOS,
       SENS_JOINTLIMITVEL, SENS_JOINTLIMITFRC, SENS_TENDONLIMITPOS, SENS_TENDONLIMITVEL,
       SENS_TENDONLIMITFRC, SENS_FRAMEPOS, SENS_FRAMEQUAT, SENS_FRAMEXAXIS, SENS_FRAMEYAXIS,
       SENS_FRAMEZAXIS, SENS_FRAMELINVEL, SENS_FRAMEANGVEL, SENS_FRAMELINACC,
       SENS_FRAMEANGACC, SENS_SUBTREECOM, SENS_SUBTREELINVEL, SENS_SUBTREEANGMOM,
       SENS_GEOMDIST, SENS_GEOMNORMAL, SENS_GEOMFROMTO, SENS_E_POTENTIAL, SENS_E_KINETIC,
       SENS_CLOCK };
enum { DATATYPE_REAL = 0, DATATYPE_POSITIVE = 1 };

/* engine_util_blas.c:179-188 */
static void mju_mulMatTVec3(mjtNum res[3], const mjtNum mat[9], const mjtNum vec[3]) {
  mjtNum tmp[3] = {mat[0]*vec[0] + mat[3]*vec[1] + mat[6]*vec[2],
                   mat[1]*vec[0] + mat[4]*vec[1] + mat[7]*vec[2],
                   mat[2]*vec[0] + mat[5]*vec[1] + mat[8]*vec[2]};
  res[0] = tmp[0]; res[1] = tmp[1]; res[2] = tmp[2];
}

/* engine_util_spatial.c:495-523 */
static void mju_transformSpatial(mjtNum res[6], const mjtNum vec[6], int flg_force,
                                 const mjtNum newpos[3], const mjtNum oldpos[3],
                                 const mjtNum* rotnew2old) {
  mjtNum cros[3], dif[3], tran[6];
  mju_copy(tran, vec, 6);
  mju_sub3(dif, newpos, oldpos);
  if (flg_force) {
    mju_cross(cros, dif, vec+3);
    mju_sub3(tran, vec, cros);
  } else {
    mju_cross(cros, dif, vec);
    mju_sub3(tran+3, vec+3, cros);
  }
  if (rotnew2old) {
    mju_mulMatTVec3(res, rotnew2old, tran);
    mju_mulMatTVec3(res+3, rotnew2old, tran+3);
  } else {
    mju_copy(res, tran, 6);
  }
}

/* object frame (pos, rot) and body of a sensorized object: the switch shared by
 * mj_objectVelocity/mj_objectAcceleration (engine_support.c:1265-1312, :1317-1361) and
 * get_xpos_xmat (engine_sensor.c:69-94) */
static int obj_frame(const mjhipModel* m, const mjhipData* d, int type, int id,
                     const mjtNum** pos, const mjtNum** mat) {
  switch (type) {
  case OBJ_BODY:   *pos = d->xipos + 3*id;     *mat = d->ximat + 9*id;     return id;
  case OBJ_XBODY:  *pos = d->xpos + 3*id;      *mat = d->xmat + 9*id;      return id;
  case OBJ_GEOM:   *pos = d->geom_xpos + 3*id; *mat = d->geom_xmat + 9*id; return m->geom_bodyid[id];
  case OBJ_SITE:   *pos = d->site_xpos + 3*id; *mat = d->site_xmat + 9*id; return m->site_bodyid[id];
  default:         *pos = d->cam_xpos + 3*id;  *mat = d->cam_xmat + 9*id;  return m->cam_bodyid[id];
  }
}

/* engine_support.c:1265-1312 */
static void or_objectVelocity(const mjhipModel* m, const mjhipData* d, int type, int id,
                              mjtNum res[6], int flg_local) {
  const mjtNum *pos, *mat;
  int b = obj_frame(m, d, type, id, &pos, &mat);
  mju_transformSpatial(res, d->cvel + 6*b, 0, pos, d->subtree_com + 3*m->body_rootid[b],
                       flg_local ? mat : NULL);
}

/* engine_support.c:1317-1371 */
static void or_objectAcceleration(const mjhipModel* m, const mjhipData* d, int type, int id,
                                  mjtNum res[6], int flg_local) {
  const mjtNum *pos, *mat;
  mjtNum correction[3], vel[6];
  int b = obj_frame(m, d, type, id, &pos, &mat);
  const mjtNum* com = d->subtree_com + 3*m->body_rootid[b];
  mju_transformSpatial(vel, d->cvel + 6*b, 0, pos, com, flg_local ? mat : NULL);
  mju_transformSpatial(res, d->cacc + 6*b, 0, pos, com, flg_local ? mat : NULL);
  mju_cross(correction, vel, vel+3);
  mju_addTo3(res+3, correction);
}

/* engine_sensor.c:96-118 get_xquat */
static void or_xquat(const mjhipModel* m, const mjhipData* d, int type, int id, mjtNum q[4]) {
  switch (type) {
  case OBJ_XBODY: mju_copy4(q, d->xquat + 4*id); break;
  case OBJ_BODY:  mju_mulQuat(q, d->xquat + 4*id, m->body_iquat + 4*id); break;
  case OBJ_GEOM:  mju_mulQuat(q, d->xquat + 4*m->geom_bodyid[id], m->geom_quat + 4*id); break;
  case OBJ_SITE:  mju_mulQuat(q, d->xquat + 4*m->site_bodyid[id], m->site_quat + 4*id); break;
  default:        mju_mulQuat(q, d->xquat + 4*m->cam_bodyid[id], m->cam_quat + 4*id); break;
  }
}

/* engine_passive.c:527-585 mj_inertiaBoxFluidModel */
static void or_inertiaBoxFluid(const mjhipModel* m, mjhipData* d, int i) {
  mjtNum lvel[6], wind[6], lwind[6], lfrc[6], bfrc[6], box[3], diam;
  const mjtNum* inertia = m->body_inertia + 3*i;
  box[0] = sqrt(mjMAX(mjMINVAL, (inertia[1] + inertia[2] - inertia[0])) / m->body_mass[i] * 6.0);
  box[1] = sqrt(mjMAX(mjMINVAL, (inertia[0] + inertia[2] - inertia[1])) / m->body_mass[i] * 6.0);
  box[2] = sqrt(mjMAX(mjMINVAL, (inertia[0] + inertia[1] - inertia[2])) / m->body_mass[i] * 6.0);
  or_objectVelocity(m, d, OBJ_BODY, i, lvel, 1);
  mju_zero(wind, 6);
  mju_copy3(wind+3, m->opt.wind);
  mju_transformSpatial(lwind, wind, 0, d->xipos+3*i, d->subtree_com+3*m->body_rootid[i],
                       d->ximat+9*i);
  lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
  mju_zero(lfrc, 6);
  if (m->opt.viscosity > 0) {
    diam = (box[0] + box[1] + box[2])/3.0;
    mju_scl3(lfrc, lvel, -mjhipPI*diam*diam*diam*m->opt.viscosity);
    mju_scl3(lfrc+3, lvel+3, -3.0*mjhipPI*diam*m->opt.viscosity);
  }
  if (m->opt.density > 0) {
    lfrc[3] -= 0.5*m->opt.density*box[1]*box[2]*fabs(lvel[3])*lvel[3];
    lfrc[4] -= 0.5*m->opt.density*box[0]*box[2]*fabs(lvel[4])*lvel[4];
    lfrc[5] -= 0.5*m->opt.density*box[0]*box[1]*fabs(lvel[5])*lvel[5];
    lfrc[0] -= m->opt.density*box[0]*(box[1]*box[1]*box[1]*box[1]+box[2]*box[2]*box[2]*box[2])*
               fabs(lvel[0])*lvel[0]/64.0;
    lfrc[1] -= m->opt.density*box[1]*(box[0]*box[0]*box[0]*box[0]+box[2]*box[2]*box[2]*box[2])*
               fabs(lvel[1])*lvel[1]/64.0;
    lfrc[2] -= m->opt.density*box[2]*(box[0]*box[0]*box[0]*box[0]+box[1]*box[1]*box[1]*box[1])*
               fabs(lvel[2])*lvel[2]/64.0;
  }
  mju_mulMatVec3(bfrc, d->ximat+9*i, lfrc);
  mju_mulMatVec3(bfrc+3, d->ximat+9*i, lfrc+3);
  mj_applyFT(m, d, bfrc+3, bfrc, d->xipos+3*i, i, d->qfrc_fluid);
}

/* engine_passive.c:650-687 mj_addedMassForces without accelerations */
static void or_addedMass(const mjtNum v[6], mjtNum rho, const mjtNum vm[3], const mjtNum vi[3],
                         mjtNum f[6]) {
  const mjtNum lin[3] = {v[3], v[4], v[5]}, ang[3] = {v[0], v[1], v[2]};
  const mjtNum plin[3] = {rho*vm[0]*lin[0], rho*vm[1]*lin[1], rho*vm[2]*lin[2]};
  const mjtNum pang[3] = {rho*vi[0]*ang[0], rho*vi[1]*ang[1], rho*vi[2]*ang[2]};
  mjtNum fa[3], t1[3], t2[3];
  mju_cross(fa, plin, ang);
  mju_cross(t1, plin, lin);
  mju_cross(t2, pang, ang);
  mju_addTo3(f, t1);
  mju_addTo3(f, t2);
  mju_addTo3(f+3, fa);
}

static mjtNum or_pow4(mjtNum x) { return (x*x)*(x*x); }

/* engine_passive.c:697-701 */
static mjtNum or_maxMoment(const mjtNum s[3], int k) {
  const mjtNum d0 = s[k], d1 = s[(k+1) % 3], d2 = s[(k+2) % 3];
  return 8.0/15.0 * mjhipPI * d0 * or_pow4(mjMAX(d1, d2));
}

/* engine_passive.c:705-790 mj_viscousForces */
static void or_viscousForces(const mjtNum v[6], mjtNum rho, mjtNum mu, const mjtNum s[3],
                             mjtNum magnus, mjtNum kutta, mjtNum blunt, mjtNum slender,
                             mjtNum angdrag, mjtNum f[6]) {
  const mjtNum lin[3] = {v[3], v[4], v[5]}, ang[3] = {v[0], v[1], v[2]};
  const mjtNum volume = 4.0/3.0 * mjhipPI * s[0] * s[1] * s[2];
  const mjtNum dmax = mjMAX(mjMAX(s[0], s[1]), s[2]);
  const mjtNum dmin = mjMIN(mjMIN(s[0], s[1]), s[2]);
  const mjtNum dmid = s[0] + s[1] + s[2] - dmax - dmin;
  const mjtNum Amax = mjhipPI * dmax * dmid;
  mjtNum mf[3];
  mju_cross(mf, ang, lin);
  mf[0] *= magnus * rho * volume;
  mf[1] *= magnus * rho * volume;
  mf[2] *= magnus * rho * volume;
  const mjtNum den = or_pow4(s[1]*s[2]) * (lin[0]*lin[0]) + or_pow4(s[2]*s[0]) * (lin[1]*lin[1]) +
                     or_pow4(s[0]*s[1]) * (lin[2]*lin[2]);
  const mjtNum num = (s[1]*s[2]*lin[0])*(s[1]*s[2]*lin[0]) + (s[2]*s[0]*lin[1])*(s[2]*s[0]*lin[1]) +
                     (s[0]*s[1]*lin[2])*(s[0]*s[1]*lin[2]);
  const mjtNum Aproj = mjhipPI * sqrt(den/mjMAX(mjMINVAL, num));
  const mjtNum nrm[3] = {(s[1]*s[2])*(s[1]*s[2]) * lin[0], (s[2]*s[0])*(s[2]*s[0]) * lin[1],
                         (s[0]*s[1])*(s[0]*s[1]) * lin[2]};
  const mjtNum cosa = num / mjMAX(mjMINVAL, mju_norm3(lin) * den);
  mjtNum kc[3], kf[3];
  mju_cross(kc, nrm, lin);
  kc[0] *= kutta * rho * cosa * Aproj;
  kc[1] *= kutta * rho * cosa * Aproj;
  kc[2] *= kutta * rho * cosa * Aproj;
  mju_cross(kf, kc, lin);
  const mjtNum D = 2.0/3.0 * (s[0] + s[1] + s[2]);
  const mjtNum cf = 3.0 * mjhipPI * D, ct = mjhipPI * D*D*D;
  const mjtNum Imax = 8.0/15.0 * mjhipPI * dmid * or_pow4(dmax);
  const mjtNum II[3] = {or_maxMoment(s, 0), or_maxMoment(s, 1), or_maxMoment(s, 2)};
  const mjtNum mom[3] = {ang[0] * (angdrag*II[0] + slender*(Imax - II[0])),
                         ang[1] * (angdrag*II[1] + slender*(Imax - II[1])),
                         ang[2] * (angdrag*II[2] + slender*(Imax - II[2]))};
  const mjtNum dlin = mu*cf + rho*mju_norm3(lin)*(Aproj*blunt + slender*(Amax - Aproj));
  const mjtNum dang = mu * ct + rho * mju_norm3(mom);
  f[0] -= dang * ang[0];
  f[1] -= dang * ang[1];
  f[2] -= dang * ang[2];
  f[3] += mf[0] + kf[0] - dlin*lin[0];
  f[4] += mf[1] + kf[1] - dlin*lin[1];
  f[5] += mf[2] + kf[2] - dlin*lin[2];
}

/* engine_util_misc.c:425-451 mju_geomSemiAxes */
static void or_semiAxes(const mjhipModel* m, int g, mjtNum ax[3]) {
  const mjtNum* s = m->geom_size + 3*g;
  switch (m->geom_type[g]) {
  case mjhipGEOM_SPHERE:   ax[0] = s[0]; ax[1] = s[0]; ax[2] = s[0]; break;
  case mjhipGEOM_CAPSULE:  ax[0] = s[0]; ax[1] = s[0]; ax[2] = s[1] + s[0]; break;
  case mjhipGEOM_CYLINDER: ax[0] = s[0]; ax[1] = s[0]; ax[2] = s[1]; break;
  default:                 ax[0] = s[0]; ax[1] = s[1]; ax[2] = s[2];
  }
}

/* engine_passive.c:588-646 mj_ellipsoidFluidModel */
static void or_ellipsoidFluid(const mjhipModel* m, mjhipData* d, int b) {
  for (int j = 0; j < m->body_geomnum[b]; j++) {
    const int g = m->body_geomadr[b] + j;
    const mjtNum* c = m->geom_fluid + 12*g;    /* readFluidGeomInteraction (:793-821) */
    mjtNum ax[3], lvel[6], wind[6], lwind[6], lfrc[6], bfrc[6];
    or_semiAxes(m, g, ax);
    if (c[0] == 0.0) continue;
    or_objectVelocity(m, d, OBJ_GEOM, g, lvel, 1);
    mju_zero(wind, 6);
    mju_copy3(wind+3, m->opt.wind);
    mju_transformSpatial(lwind, wind, 0, d->geom_xpos + 3*g,
                         d->subtree_com + 3*m->body_rootid[b], d->geom_xmat + 9*g);
    lvel[3] -= lwind[3]; lvel[4] -= lwind[4]; lvel[5] -= lwind[5];
    mju_zero(lfrc, 6);
    or_addedMass(lvel, m->opt.density, c + 6, c + 9, lfrc);
    or_viscousForces(lvel, m->opt.density, m->opt.viscosity, ax, c[5], c[4], c[1], c[2], c[3],
                     lfrc);
    mju_scl(lfrc, lfrc, c[0], 6);
    mju_mulMatVec3(bfrc, d->geom_xmat + 9*g, lfrc);
    mju_mulMatVec3(bfrc+3, d->geom_xmat + 9*g, lfrc+3);
    mj_applyFT(m, d, bfrc+3, bfrc, d->geom_xpos + 3*g, b, d->qfrc_fluid);
  }
}

/* engine_passive.c:402-428 mj_fluid: the ellipsoid model for a body with a geom that uses
 * it (geom_fluid[0] > 0), the inertia-box model otherwise */
static int or_fluid(const mjhipModel* m, mjhipData* d) {
  int has_fluid = m->opt.viscosity > 0 || m->opt.density > 0;
  if (has_fluid) {
    for (int i = 1; i < m->nbody; i++) {
      if (m->body_mass[i] < mjMINVAL) continue;
      int ell = 0;
      for (int j = 0; j < m->body_geomnum[i] && ell == 0; j++) {
        ell += m->geom_fluid[12*(m->body_geomadr[i] + j)] > 0;
      }
      if (ell) or_ellipsoidFluid(m, d, i);
      else or_inertiaBoxFluid(m, d, i);
    }
  }
  return has_fluid;
}

/* engine_core_smooth.c:1900-1958 */
static void or_subtreeVel(const mjhipModel* m, mjhipData* d) {
  int nbody = m->nbody;
  mjtNum dx[3], dv[3], dp[3], dL[3];
  mjtNum* body_vel = (mjtNum*)malloc(6*(size_t)nbody*sizeof(mjtNum));
  for (int i = 0; i < nbody; i++) {
    or_objectVelocity(m, d, OBJ_BODY, i, body_vel + 6*i, 0);
    mju_scl3(d->subtree_linvel + 3*i, body_vel + 6*i + 3, m->body_mass[i]);
    mju_mulMatTVec3(dv, d->ximat + 9*i, body_vel + 6*i);
    dv[0] *= m->body_inertia[3*i];
    dv[1] *= m->body_inertia[3*i+1];
    dv[2] *= m->body_inertia[3*i+2];
    mju_mulMatVec3(d->subtree_angmom + 3*i, d->ximat + 9*i, dv);
  }
  for (int i = nbody-1; i >= 0; i--) {
    if (i) mju_addTo3(d->subtree_linvel + 3*m->body_parentid[i], d->subtree_linvel + 3*i);
    mju_scl3(d->subtree_linvel + 3*i, d->subtree_linvel + 3*i,
             1/mjMAX(mjMINVAL, m->body_subtreemass[i]));
  }
  for (int i = nbody-1; i > 0; i--) {
    int parent = m->body_parentid[i];
    mju_sub3(dx, d->xipos + 3*i, d->subtree_com + 3*i);
    mju_sub3(dv, body_vel + 6*i + 3, d->subtree_linvel + 3*i);
    mju_scl3(dp, dv, m->body_mass[i]);
    mju_cross(dL, dx, dp);
    mju_addTo3(d->subtree_angmom + 3*i, dL);
    mju_addTo3(d->subtree_angmom + 3*parent, d->subtree_angmom + 3*i);
    mju_sub3(dx, d->subtree_com + 3*i, d->subtree_com + 3*parent);
    mju_sub3(dv, d->subtree_linvel + 3*i, d->subtree_linvel + 3*parent);
    mju_scl3(dv, dv, m->body_subtreemass[i]);
    mju_cross(dL, dx, dv);
    mju_addTo3(d->subtree_angmom + 3*parent, dL);
  }
  free(body_vel);
}

/* engine_util_misc.c:830-850 */
static void mju_decodePyramid(mjtNum* force, const mjtNum* pyramid, const mjtNum* mu, int dim) {
  if (dim == 1) {
    force[0] = pyramid[0];
    return;
  }
  force[0] = 0;
  for (int i = 0; i < 2*(dim-1); i++) force[0] += pyramid[i];
  for (int i = 0; i < dim-1; i++) force[i+1] = (pyramid[2*i] - pyramid[2*i+1]) * mu[i];
}

/* engine_support.c:1459-1480 mj_contactForce (pyramidal cones: the supported subset) */
static void or_contactForce(const mjhipModel* m, const orEfc* e, int id, mjtNum result[6]) {
  mju_zero(result, 6);
  if (id >= 0 && id < e->ncon && e->con_efc_address[id] >= 0) {
    if (m->opt.cone != mjhipCONE_ELLIPTIC) {
      mju_decodePyramid(result, e->efc_force + e->con_efc_address[id], e->con_friction + 5*id,
                        e->con_dim[id]);
    } else {
      mju_copy(result, e->efc_force + e->con_efc_address[id], e->con_dim[id]);
    }
  }
}

/* engine_core_smooth.c:2027-2181 (no equality constraints in the supported subset) */
static void or_rnePostConstraint(const mjhipModel* m, mjhipData* d, const orEfc* e) {
  int nbody = m->nbody;
  mjtNum cfrc_com[6], cfrc[6], lfrc[6];
  mju_zero(d->cacc, 6);
  if (!mjDISABLED(mjhipDSBL_GRAVITY)) mju_scl3(d->cacc + 3, m->opt.gravity, -1);
  mju_zero(d->cfrc_ext, 6*nbody);
  for (int i = 1; i < nbody; i++) {
    if (!mju_isZero(d->xfrc_applied + 6*i, 6)) {
      mju_copy3(cfrc, d->xfrc_applied + 6*i + 3);
      mju_copy3(cfrc + 3, d->xfrc_applied + 6*i);
      mju_transformSpatial(cfrc_com, cfrc, 1, d->subtree_com + 3*m->body_rootid[i],
                           d->xipos + 3*i, NULL);
      mju_addTo(d->cfrc_ext + 6*i, cfrc_com, 6);
    }
  }
  for (int i = 0; i < e->ncon; i++) {
    if (e->con_efc_address[i] < 0) continue;
    const int* geom = e->con_geom + 2*i;
    if (geom[0] < 0 || geom[1] < 0) continue;
    or_contactForce(m, e, i, lfrc);
    const mjtNum* frame = e->con_frame + 9*i;
    mju_mulMatTVec3(cfrc, frame, lfrc + 3);
    mju_mulMatTVec3(cfrc + 3, frame, lfrc);
    int k;
    if ((k = m->geom_bodyid[geom[0]])) {
      mju_transformSpatial(cfrc_com, cfrc, 1, d->subtree_com + 3*m->body_rootid[k],
                           e->con_pos + 3*i, NULL);
      mju_subFrom(d->cfrc_ext + 6*k, cfrc_com, 6);
    }
    if ((k = m->geom_bodyid[geom[1]])) {
      mju_transformSpatial(cfrc_com, cfrc, 1, d->subtree_com + 3*m->body_rootid[k],
                           e->con_pos + 3*i, NULL);
      mju_addTo(d->cfrc_ext + 6*k, cfrc_com, 6);
    }
  }
  /* connect and weld forces (:2102-2158); joint/tendon rows apply no body force */
  for (int i = 0; i < e->ne;) {
    int id = e->efc_id[i], t = m->eq_type[id];
    const mjtNum* eq_data = m->eq_data + mjhipNEQDATA*id;
    if (t == mjhipEQ_CONNECT || t == mjhipEQ_WELD) {
      mjtNum pos[3], *offset;
      mju_copy3(cfrc + 3, e->efc_force + i);
      if (t == mjhipEQ_WELD) mju_copy3(cfrc, e->efc_force + i + 3);
      else mju_zero3(cfrc);
      int body_semantic = m->eq_objtype[id] == OBJ_BODY;
      int obj1 = m->eq_obj1id[id], k = body_semantic ? obj1 : m->site_bodyid[obj1];
      if (k) {
        offset = body_semantic ? (mjtNum*)eq_data + 3*(t == mjhipEQ_WELD) : m->site_pos + 3*obj1;
        mj_local2Global(d, pos, 0, offset, 0, k, 0);
        mju_transformSpatial(cfrc_com, cfrc, 1, d->subtree_com + 3*m->body_rootid[k], pos, NULL);
        mju_addTo(d->cfrc_ext + 6*k, cfrc_com, 6);
      }
      int obj2 = m->eq_obj2id[id];
      k = body_semantic ? obj2 : m->site_bodyid[obj2];
      if (k) {
        offset = body_semantic ? (mjtNum*)eq_data + 3*(t == mjhipEQ_CONNECT) : m->site_pos + 3*obj2;
        mj_local2Global(d, pos, 0, offset, 0, k, 0);
        mju_transformSpatial(cfrc_com, cfrc, 1, d->subtree_com + 3*m->body_rootid[k], pos, NULL);
        mju_subFrom(d->cfrc_ext + 6*k, cfrc_com, 6);
      }
      i += t == mjhipEQ_WELD ? 6 : 3;
    } else {
      i++;
    }
  }
  mjtNum cacc[6], cfrc_body[6], cfrc_corr[6];
  mju_zero(d->cfrc_int, 6);
  for (int j = 1; j < nbody; j++) {
    int bda = m->body_dofadr[j];
    mju_mulDofVec(cacc, d->cdof_dot + 6*bda, d->qvel + bda, m->body_dofnum[j]);
    mju_add(d->cacc + 6*j, d->cacc + 6*m->body_parentid[j], cacc, 6);
    mju_mulDofVec(cacc, d->cdof + 6*bda, d->qacc + bda, m->body_dofnum[j]);
    mju_addTo(d->cacc + 6*j, cacc, 6);
    mju_mulInertVec(cfrc_body, d->cinert + 10*j, d->cacc + 6*j);
    mju_mulInertVec(cfrc_corr, d->cinert + 10*j, d->cvel + 6*j);
    mju_crossForce(cfrc, d->cvel + 6*j, cfrc_corr);
    mju_addTo(cfrc_body, cfrc, 6);
    mju_sub(d->cfrc_int + 6*j, cfrc_body, d->cfrc_ext + 6*j, 6);
  }
  for (int j = nbody-1; j > 0; j--) {
    mju_addTo(d->cfrc_int + 6*m->body_parentid[j], d->cfrc_int + 6*j, 6);
  }
}

/* engine_sensor.c:38-66 */
static void or_applyCutoff(const mjhipModel* m, mjhipData* d, int stage) {
  for (int i = 0; i < m->nsensor; i++) {
    if (m->sensor_needstage[i] == stage && m->sensor_cutoff[i] > 0) {
      if (m->sensor_type[i] == SENS_GEOMFROMTO) continue;   /* :44-47 */
      int adr = m->sensor_adr[i], dim = m->sensor_dim[i];
      mjtNum cutoff = m->sensor_cutoff[i];
      for (int j = 0; j < dim; j++) {
        if (m->sensor_datatype[i] == DATATYPE_REAL) {
          d->sensordata[adr+j] = mju_clip(d->sensordata[adr+j], -cutoff, cutoff);
        } else if (m->sensor_datatype[i] == DATATYPE_POSITIVE) {
          d->sensordata[adr+j] = mjMIN(cutoff, d->sensordata[adr+j]);
        }
      }
    }
  }
}

/* first limit row of (type, id) among rows ne+nf..nefc (engine_sensor.c:286-304) */
static int or_limitRow(const orEfc* e, int type, int id) {
  for (int j = e->ne + e->nf; j < e->nefc; j++) {
    if (e->efc_type[j] == type && e->efc_id[j] == id) return j;
  }
  return -1;
}

/* engine_sensor.c:126-215 cam_project: the pixel coordinates of a point in a camera's image,
 * through the reference's explicit 4x4 product image * focal * rotation * translation (every
 * term in its loop order, zeros included) */
static void or_camProject(mjtNum out[2], const mjtNum* target, const mjtNum* cpos,
                          const mjtNum* cmat, const int* res, mjtNum fovy, const float* intr,
                          const float* size) {
  mjtNum T[4][4] = {{0}}, Rm[4][4] = {{0}}, F[3][4] = {{0}}, I[3][3] = {{0}}, P[3][4] = {{0}};
  mjtNum fx, fy;
  for (int i = 0; i < 4; i++) T[i][i] = Rm[i][i] = 1;
  for (int i = 0; i < 3; i++) T[i][3] = -cpos[i];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) Rm[i][j] = cmat[3*j+i];
  }
  if (size[0] && size[1]) {
    fx = intr[0] / size[0] * res[0];
    fy = intr[1] / size[1] * res[1];
  } else {
    fx = fy = .5 / tan(fovy * mjhipPI / 360.) * res[1];
  }
  F[0][0] = -fx;
  F[1][1] = fy;
  F[2][2] = 1.0;
  I[0][0] = I[1][1] = I[2][2] = 1;
  I[0][2] = (mjtNum)res[0] / 2.0;
  I[1][2] = (mjtNum)res[1] / 2.0;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      for (int k = 0; k < 4; k++)
        for (int l = 0; l < 4; l++)
          for (int n = 0; n < 4; n++) P[i][n] += I[i][j] * F[j][k] * Rm[k][l] * T[l][n];
  const mjtNum ph[4] = {target[0], target[1], target[2], 1};
  mjtNum px[3] = {0, 0, 0};
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 4; j++) px[i] += P[i][j] * ph[j];
  }
  mjtNum den = px[2];
  if (fabs(den) < mjMINVAL) den = den < 0 ? mjMIN(den, -mjMINVAL) : mjMAX(den, mjMINVAL);
  out[0] = px[0] / den;
  out[1] = px[1] / den;
}

/* mj_ray for the rangefinder (defined with the touch sensor's ray functions below) */
static mjtNum or_ray(const mjhipModel* m, const mjhipData* d, const mjtNum* pnt,
                     const mjtNum* vec, int bodyexclude, int* geomid);

static void or_energyPos(const mjhipModel* m, mjhipData* d);
static void or_energyVel(const mjhipModel* m, mjhipData* d);

/* engine_sensor.c:209-513 mj_sensorPos (no user/plugin sensors) */
static void or_sensorPos(const mjhipModel* m, mjhipData* d, const orEfc* e) {
  if (mjDISABLED(mjhipDSBL_SENSOR)) return;
  for (int i = 0; i < m->nsensor; i++) {
    if (m->sensor_needstage[i] != mjhipSTAGE_POS) continue;
    int type = m->sensor_type[i], objtype = m->sensor_objtype[i], objid = m->sensor_objid[i];
    int refid = m->sensor_refid[i], reftype = m->sensor_reftype[i], adr = m->sensor_adr[i];
    mjtNum* out = d->sensordata + adr;
    mjtNum rvec[3];
    const mjtNum *xpos, *xmat, *xpos_ref, *xmat_ref;
    int r;
    switch (type) {
    case SENS_MAGNETOMETER:
      mju_mulMatTVec(out, d->site_xmat + 9*objid, m->opt.magnetic, 3, 3);
      break;
    case SENS_CAMPROJECTION:
      or_camProject(out, d->site_xpos + 3*objid, d->cam_xpos + 3*refid, d->cam_xmat + 9*refid,
                    m->cam_resolution + 2*refid, m->cam_fovy[refid],
                    m->cam_intrinsic + 4*refid, m->cam_sensorsize + 2*refid);
      break;
    case SENS_RANGEFINDER:                   /* the site's z axis, its own body excluded */
      rvec[0] = d->site_xmat[9*objid+2];
      rvec[1] = d->site_xmat[9*objid+5];
      rvec[2] = d->site_xmat[9*objid+8];
      out[0] = or_ray(m, d, d->site_xpos + 3*objid, rvec, m->site_bodyid[objid], NULL);
      break;
    case SENS_JOINTPOS:
      out[0] = d->qpos[m->jnt_qposadr[objid]];
      break;
    case SENS_TENDONPOS:
      out[0] = d->ten_length[objid];
      break;
    case SENS_ACTUATORPOS:
      out[0] = d->actuator_length[objid];
      break;
    case SENS_BALLQUAT:
      mju_copy4(out, d->qpos + m->jnt_qposadr[objid]);
      mju_normalize4(out);
      break;
    case SENS_JOINTLIMITPOS:
    case SENS_TENDONLIMITPOS:
      out[0] = 0;
      r = or_limitRow(e, type == SENS_JOINTLIMITPOS ? orCNSTR_LIMIT_JOINT : orCNSTR_LIMIT_TENDON,
                      objid);
      if (r >= 0) out[0] = e->efc_pos[r] - e->efc_margin[r];
      break;
    case SENS_FRAMEPOS:
    case SENS_FRAMEXAXIS:
    case SENS_FRAMEYAXIS:
    case SENS_FRAMEZAXIS:
      obj_frame(m, d, objtype, objid, &xpos, &xmat);
      if (refid == -1) {
        if (type == SENS_FRAMEPOS) {
          mju_copy3(out, xpos);
        } else {
          int offset = type - SENS_FRAMEXAXIS;
          out[0] = xmat[offset];
          out[1] = xmat[offset+3];
          out[2] = xmat[offset+6];
        }
      } else {
        obj_frame(m, d, reftype, refid, &xpos_ref, &xmat_ref);
        if (type == SENS_FRAMEPOS) {
          mju_sub3(rvec, xpos, xpos_ref);
          mju_mulMatTVec3(out, xmat_ref, rvec);
        } else {
          int offset = type - SENS_FRAMEXAXIS;
          mjtNum axis[3] = {xmat[offset], xmat[offset+3], xmat[offset+6]};
          mju_mulMatTVec3(out, xmat_ref, axis);
        }
      }
      break;
    case SENS_FRAMEQUAT: {
      mjtNum objquat[4], refquat[4];
      or_xquat(m, d, objtype, objid, objquat);
      if (refid == -1) {
        mju_copy4(out, objquat);
      } else {
        or_xquat(m, d, reftype, refid, refquat);
        refquat[1] = -refquat[1]; refquat[2] = -refquat[2]; refquat[3] = -refquat[3];
        mju_mulQuat(out, refquat, objquat);
      }
      break;
    }
    case SENS_SUBTREECOM:
      mju_copy3(out, d->subtree_com + 3*objid);
      break;
    case SENS_GEOMDIST:
    case SENS_GEOMNORMAL:
    case SENS_GEOMFROMTO: {
      /* :378-460: the smallest distance over the geom pairs of the two bodies/geoms, cutoff
       * as the bound (the reference shares one evaluation among consecutive sensors of the
       * same pair and cutoff; recomputing gives the same values) */
      const mjtNum margin = m->sensor_cutoff[i];
      mjtNum dist = margin, fromto[6] = {0, 0, 0, 0, 0, 0};
      const int n1 = objtype == OBJ_BODY ? m->body_geomnum[objid] : 1;
      const int id1 = objtype == OBJ_BODY ? m->body_geomadr[objid] : objid;
      const int n2 = reftype == OBJ_BODY ? m->body_geomnum[refid] : 1;
      const int id2 = reftype == OBJ_BODY ? m->body_geomadr[refid] : refid;
      for (int a = id1; a < id1 + n1; a++) {
        for (int b = id2; b < id2 + n2; b++) {
          mjtNum ft[6];
          const mjtNum dn = or_geomDistance(m, d, a, b, margin, ft);
          if (dn < dist) {
            dist = dn;
            mju_copy(fromto, ft, 6);
          }
        }
      }
      if (type == SENS_GEOMDIST) {
        out[0] = dist;
      } else if (type == SENS_GEOMNORMAL) {
        mjtNum nrm[3] = {fromto[3]-fromto[0], fromto[4]-fromto[1], fromto[5]-fromto[2]};
        if (nrm[0] || nrm[1] || nrm[2]) mju_normalize3(nrm);
        mju_copy3(out, nrm);
      } else {
        mju_copy(out, fromto, 6);
      }
      break;
    }
    case SENS_E_POTENTIAL:
      or_energyPos(m, d);
      out[0] = d->energy[0];
      break;
    case SENS_E_KINETIC:
      or_energyVel(m, d);
      out[0] = d->energy[1];
      break;
    case SENS_CLOCK:
      out[0] = d->time;
      break;
    }
  }
  or_applyCutoff(m, d, mjhipSTAGE_POS);
}

/* engine_sensor.c:521-672 mj_sensorVel */
static void or_sensorVel(const mjhipModel* m, mjhipData* d, const orEfc* e) {
  if (mjDISABLED(mjhipDSBL_SENSOR)) return;
  int subtreeVel = 0;
  mjtNum xvel[6];
  for (int i = 0; i < m->nsensor; i++) {
    if (m->sensor_needstage[i] != mjhipSTAGE_VEL) continue;
    int type = m->sensor_type[i], objtype = m->sensor_objtype[i], objid = m->sensor_objid[i];
    int refid = m->sensor_refid[i], reftype = m->sensor_reftype[i], adr = m->sensor_adr[i];
    mjtNum* out = d->sensordata + adr;
    int r;
    if (!subtreeVel && (type == SENS_SUBTREELINVEL || type == SENS_SUBTREEANGMOM)) {
      or_subtreeVel(m, d);
      subtreeVel = 1;
    }
    switch (type) {
    case SENS_VELOCIMETER:
      or_objectVelocity(m, d, OBJ_SITE, objid, xvel, 1);
      mju_copy3(out, xvel + 3);
      break;
    case SENS_GYRO:
      or_objectVelocity(m, d, OBJ_SITE, objid, xvel, 1);
      mju_copy3(out, xvel);
      break;
    case SENS_JOINTVEL:
      out[0] = d->qvel[m->jnt_dofadr[objid]];
      break;
    case SENS_TENDONVEL:
      out[0] = d->ten_velocity[objid];
      break;
    case SENS_ACTUATORVEL:
      out[0] = d->actuator_velocity[objid];
      break;
    case SENS_BALLANGVEL:
      mju_copy3(out, d->qvel + m->jnt_dofadr[objid]);
      break;
    case SENS_JOINTLIMITVEL:
    case SENS_TENDONLIMITVEL:
      out[0] = 0;
      r = or_limitRow(e, type == SENS_JOINTLIMITVEL ? orCNSTR_LIMIT_JOINT : orCNSTR_LIMIT_TENDON,
                      objid);
      if (r >= 0) out[0] = e->efc_vel[r];
      break;
    case SENS_FRAMELINVEL:
    case SENS_FRAMEANGVEL:
      or_objectVelocity(m, d, objtype, objid, xvel, 0);
      if (refid > -1) {
        const mjtNum *xpos, *xmat, *xpos_ref, *xmat_ref;
        mjtNum xvel_ref[6], rel_vel[6], cross[3], rvec[3];
        obj_frame(m, d, objtype, objid, &xpos, &xmat);
        obj_frame(m, d, reftype, refid, &xpos_ref, &xmat_ref);
        or_objectVelocity(m, d, reftype, refid, xvel_ref, 0);
        mju_sub(rel_vel, xvel, xvel_ref, 6);
        mju_sub3(rvec, xpos, xpos_ref);
        mju_cross(cross, rvec, xvel_ref);
        mju_addTo3(rel_vel + 3, cross);
        mju_mulMatTVec3(xvel, xmat_ref, rel_vel);
        mju_mulMatTVec3(xvel + 3, xmat_ref, rel_vel + 3);
      }
      mju_copy3(out, type == SENS_FRAMELINVEL ? xvel + 3 : xvel);
      break;
    case SENS_SUBTREELINVEL:
      mju_copy3(out, d->subtree_linvel + 3*objid);
      break;
    case SENS_SUBTREEANGMOM:
      mju_copy3(out, d->subtree_angmom + 3*objid);
      break;
    }
  }
  or_applyCutoff(m, d, mjhipSTAGE_VEL);
}

/*================================= engine_ray.c (touch zones) =============================*/

/* ray_map :37-52: ray in the geom's local frame */
static void or_rayMap(const mjtNum* pos, const mjtNum* mat, const mjtNum* pnt, const mjtNum* vec,
                      mjtNum* lpnt, mjtNum* lvec) {
  const mjtNum dif[3] = {pnt[0]-pos[0], pnt[1]-pos[1], pnt[2]-pos[2]};
  lpnt[0] = mat[0]*dif[0] + mat[3]*dif[1] + mat[6]*dif[2];
  lpnt[1] = mat[1]*dif[0] + mat[4]*dif[1] + mat[7]*dif[2];
  lpnt[2] = mat[2]*dif[0] + mat[5]*dif[1] + mat[8]*dif[2];
  lvec[0] = mat[0]*vec[0] + mat[3]*vec[1] + mat[6]*vec[2];
  lvec[1] = mat[1]*vec[0] + mat[4]*vec[1] + mat[7]*vec[2];
  lvec[2] = mat[2]*vec[0] + mat[5]*vec[1] + mat[8]*vec[2];
}

/* ray_quad :105-127: a x^2 + 2 b x + c = 0, smallest non-negative root or -1 */
static mjtNum or_rayQuad(mjtNum a, mjtNum b, mjtNum c, mjtNum* x) {
  mjtNum det = b*b - a*c;
  if (det < mjMINVAL) {
    x[0] = -1;
    x[1] = -1;
    return -1;
  }
  det = sqrt(det);
  x[0] = (-b-det)/a;
  x[1] = (-b+det)/a;
  if (x[0] >= 0) return x[0];
  if (x[1] >= 0) return x[1];
  return -1;
}

/* ray_plane :191-218 */
static mjtNum or_rayPlane(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                          const mjtNum* pnt, const mjtNum* vec) {
  mjtNum lpnt[3], lvec[3];
  or_rayMap(pos, mat, pnt, vec, lpnt, lvec);
  if (lvec[2] > -mjMINVAL) return -1;
  const mjtNum x = -lpnt[2]/lvec[2];
  if (x < 0) return -1;
  mjtNum p0 = lpnt[0] + x*lvec[0], p1 = lpnt[1] + x*lvec[1];
  if ((size[0] <= 0 || fabs(p0) <= size[0]) && (size[1] <= 0 || fabs(p1) <= size[1])) return x;
  return -1;
}

/* ray_sphere :222-235 (mat unused) */
static mjtNum or_raySphere(const mjtNum* pos, mjtNum dist_sqr, const mjtNum* pnt,
                           const mjtNum* vec) {
  mjtNum dif[3] = {pnt[0]-pos[0], pnt[1]-pos[1], pnt[2]-pos[2]};
  mjtNum a = vec[0]*vec[0] + vec[1]*vec[1] + vec[2]*vec[2];
  mjtNum b = vec[0]*dif[0] + vec[1]*dif[1] + vec[2]*dif[2];
  mjtNum c = dif[0]*dif[0] + dif[1]*dif[1] + dif[2]*dif[2] - dist_sqr;
  mjtNum xx[2];
  return or_rayQuad(a, b, c, xx);
}

/* ray_capsule :238-301: round side between the flat sides, then the two hemispheres */
static mjtNum or_rayCapsule(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                            const mjtNum* pnt, const mjtNum* vec) {
  mjtNum ssz = size[0] + size[1];
  if (or_raySphere(pos, ssz*ssz, pnt, vec) < 0) return -1;
  mjtNum lpnt[3], lvec[3];
  or_rayMap(pos, mat, pnt, vec, lpnt, lvec);
  mjtNum x = -1, sol, xx[2];
  mjtNum a = lvec[0]*lvec[0] + lvec[1]*lvec[1];
  mjtNum b = lvec[0]*lpnt[0] + lvec[1]*lpnt[1];
  mjtNum c = lpnt[0]*lpnt[0] + lpnt[1]*lpnt[1] - size[0]*size[0];
  sol = or_rayQuad(a, b, c, xx);
  if (sol >= 0 && fabs(lpnt[2]+sol*lvec[2]) <= size[1]) {
    if (x < 0 || sol < x) x = sol;
  }
  mjtNum ldif[3] = {lpnt[0], lpnt[1], lpnt[2]-size[1]};
  a = lvec[0]*lvec[0] + lvec[1]*lvec[1] + lvec[2]*lvec[2];
  b = lvec[0]*ldif[0] + lvec[1]*ldif[1] + lvec[2]*ldif[2];
  c = ldif[0]*ldif[0] + ldif[1]*ldif[1] + ldif[2]*ldif[2] - size[0]*size[0];
  or_rayQuad(a, b, c, xx);
  for (int i = 0; i < 2; i++) {
    if (xx[i] >= 0 && lpnt[2]+xx[i]*lvec[2] >= size[1]) {
      if (x < 0 || xx[i] < x) x = xx[i];
    }
  }
  ldif[2] = lpnt[2]+size[1];
  b = lvec[0]*ldif[0] + lvec[1]*ldif[1] + lvec[2]*ldif[2];
  c = ldif[0]*ldif[0] + ldif[1]*ldif[1] + ldif[2]*ldif[2] - size[0]*size[0];
  or_rayQuad(a, b, c, xx);
  for (int i = 0; i < 2; i++) {
    if (xx[i] >= 0 && lpnt[2]+xx[i]*lvec[2] <= -size[1]) {
      if (x < 0 || xx[i] < x) x = xx[i];
    }
  }
  return x;
}

/* ray_ellipsoid :305-323 */
static mjtNum or_rayEllipsoid(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                              const mjtNum* pnt, const mjtNum* vec) {
  mjtNum lpnt[3], lvec[3];
  or_rayMap(pos, mat, pnt, vec, lpnt, lvec);
  mjtNum s[3] = {1/(size[0]*size[0]), 1/(size[1]*size[1]), 1/(size[2]*size[2])};
  mjtNum a = s[0]*lvec[0]*lvec[0] + s[1]*lvec[1]*lvec[1] + s[2]*lvec[2]*lvec[2];
  mjtNum b = s[0]*lvec[0]*lpnt[0] + s[1]*lvec[1]*lpnt[1] + s[2]*lvec[2]*lpnt[2];
  mjtNum c = s[0]*lpnt[0]*lpnt[0] + s[1]*lpnt[1]*lpnt[1] + s[2]*lpnt[2]*lpnt[2] - 1;
  mjtNum xx[2];
  return or_rayQuad(a, b, c, xx);
}

/* ray_cylinder :327-383: the flat sides, then the round side between them */
static mjtNum or_rayCylinder(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                             const mjtNum* pnt, const mjtNum* vec) {
  mjtNum ssz = size[0]*size[0] + size[1]*size[1];
  if (or_raySphere(pos, ssz, pnt, vec) < 0) return -1;
  mjtNum lpnt[3], lvec[3];
  or_rayMap(pos, mat, pnt, vec, lpnt, lvec);
  mjtNum x = -1, sol;
  if (fabs(lvec[2]) > mjMINVAL) {
    for (int side = -1; side <= 1; side += 2) {
      sol = (side*size[1]-lpnt[2])/lvec[2];
      if (sol >= 0) {
        mjtNum p0 = lpnt[0] + sol*lvec[0], p1 = lpnt[1] + sol*lvec[1];
        if (p0*p0 + p1*p1 <= size[0]*size[0]) {
          if (x < 0 || sol < x) x = sol;
        }
      }
    }
  }
  mjtNum a = lvec[0]*lvec[0] + lvec[1]*lvec[1];
  mjtNum b = lvec[0]*lpnt[0] + lvec[1]*lpnt[1];
  mjtNum c = lpnt[0]*lpnt[0] + lpnt[1]*lpnt[1] - size[0]*size[0];
  mjtNum xx[2];
  sol = or_rayQuad(a, b, c, xx);
  if (sol >= 0 && fabs(lpnt[2]+sol*lvec[2]) <= size[1]) {
    if (x < 0 || sol < x) x = sol;
  }
  return x;
}

/* ray_box :387-445; all (may be NULL): each face's hit, -1 for none */
static mjtNum or_rayBoxAll(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                           const mjtNum* pnt, const mjtNum* vec, mjtNum* all) {
  if (all) {
    for (int i = 0; i < 6; i++) all[i] = -1;
  }
  mjtNum ssz = size[0]*size[0] + size[1]*size[1] + size[2]*size[2];
  if (or_raySphere(pos, ssz, pnt, vec) < 0) return -1;
  const int iface[3][2] = {{1, 2}, {0, 2}, {0, 1}};
  mjtNum lpnt[3], lvec[3];
  or_rayMap(pos, mat, pnt, vec, lpnt, lvec);
  mjtNum x = -1, sol;
  for (int i = 0; i < 3; i++) {
    if (fabs(lvec[i]) > mjMINVAL) {
      for (int side = -1; side <= 1; side += 2) {
        sol = (side*size[i]-lpnt[i])/lvec[i];
        if (sol >= 0) {
          mjtNum p0 = lpnt[iface[i][0]] + sol*lvec[iface[i][0]];
          mjtNum p1 = lpnt[iface[i][1]] + sol*lvec[iface[i][1]];
          if (fabs(p0) <= size[iface[i][0]] && fabs(p1) <= size[iface[i][1]]) {
            if (x < 0 || sol < x) x = sol;
            if (all) all[2*i + (side + 1)/2] = sol;
          }
        }
      }
    }
  }
  return x;
}

static mjtNum or_rayBox(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                        const mjtNum* pnt, const mjtNum* vec) {
  return or_rayBoxAll(pos, mat, size, pnt, vec, NULL);
}

/* ray_triangle :132-186 */
static mjtNum or_rayTriangle(mjtNum v[][3], const mjtNum* lpnt, const mjtNum* lvec,
                             const mjtNum* b0, const mjtNum* b1) {
  mjtNum dif[3][3], planar[3][2];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) dif[i][j] = v[i][j] - lpnt[j];
  }
  for (int i = 0; i < 3; i++) {
    planar[i][0] = mju_dot3(b0, dif[i]);
    planar[i][1] = mju_dot3(b1, dif[i]);
  }
  if ((planar[0][0] > 0 && planar[1][0] > 0 && planar[2][0] > 0) ||
      (planar[0][0] < 0 && planar[1][0] < 0 && planar[2][0] < 0) ||
      (planar[0][1] > 0 && planar[1][1] > 0 && planar[2][1] > 0) ||
      (planar[0][1] < 0 && planar[1][1] < 0 && planar[2][1] < 0)) {
    return -1;
  }
  mjtNum A[4] = {planar[0][0]-planar[2][0], planar[1][0]-planar[2][0],
                 planar[0][1]-planar[2][1], planar[1][1]-planar[2][1]};
  mjtNum b[2] = {-planar[2][0], -planar[2][1]};
  mjtNum det = A[0]*A[3] - A[1]*A[2];
  if (fabs(det) < mjMINVAL) return -1;
  mjtNum t0 = (A[3]*b[0] - A[1]*b[1]) / det;
  mjtNum t1 = (-A[2]*b[0] + A[0]*b[1]) / det;
  if (t0 < 0 || t1 < 0 || t0 + t1 > 1) return -1;
  mju_sub3(dif[0], v[0], v[2]);
  mju_sub3(dif[1], v[1], v[2]);
  mju_sub3(dif[2], lpnt, v[2]);
  mjtNum nrm[3];
  mju_cross(nrm, dif[0], dif[1]);
  mjtNum denom = mju_dot3(lvec, nrm);
  if (fabs(denom) < mjMINVAL) return -1;
  return -mju_dot3(dif[2], nrm) / denom;
}

/* the basis b0, b1 of the plane normal to the local ray (mj_rayHfield :497-509, mju_rayTree
   :651-663) */
static void or_rayBasis(const mjtNum lvec[3], mjtNum b0[3], mjtNum b1[3]) {
  b0[0] = b0[1] = b0[2] = 1;
  if (fabs(lvec[0]) >= fabs(lvec[1]) && fabs(lvec[0]) >= fabs(lvec[2])) {
    b0[0] = 0;
  } else if (fabs(lvec[1]) >= fabs(lvec[2])) {
    b0[1] = 0;
  } else {
    b0[2] = 0;
  }
  mju_addScl3(b1, b0, lvec, -mju_dot3(lvec, b0)/mju_dot3(lvec, lvec));
  mju_normalize3(b1);
  mju_cross(b0, b1, lvec);
  mju_normalize3(b0);
}

/* mj_rayHfield :453-595 (the reference's side-face indexing by nrow kept) */
static mjtNum or_rayHfield(const mjhipModel* m, const mjhipData* d, int id, const mjtNum* pnt,
                           const mjtNum* vec) {
  const int hid = m->geom_dataid[id];
  const int nrow = m->hfield_nrow[hid], ncol = m->hfield_ncol[hid];
  const mjtNum* size = m->hfield_size + 4*hid;
  const float* data = m->hfield_data + m->hfield_adr[hid];
  const mjtNum* xpos = d->geom_xpos + 3*id;
  const mjtNum* xmat = d->geom_xmat + 9*id;
  mjtNum base_size[3] = {size[0], size[1], size[3]*0.5};
  mjtNum base_pos[3] = {xpos[0] - xmat[2]*size[3]*0.5, xpos[1] - xmat[5]*size[3]*0.5,
                        xpos[2] - xmat[8]*size[3]*0.5};
  mjtNum top_size[3] = {size[0], size[1], size[2]*0.5};
  mjtNum top_pos[3] = {xpos[0] + xmat[2]*size[2]*0.5, xpos[1] + xmat[5]*size[2]*0.5,
                       xpos[2] + xmat[8]*size[2]*0.5};
  mjtNum x = or_rayBoxAll(base_pos, xmat, base_size, pnt, vec, NULL);
  mjtNum all[6];
  mjtNum top_intersect = or_rayBoxAll(top_pos, xmat, top_size, pnt, vec, all);
  if (top_intersect < 0) return x;
  mjtNum lpnt[3], lvec[3], b0[3], b1[3];
  or_rayMap(xpos, xmat, pnt, vec, lpnt, lvec);
  or_rayBasis(lvec, b0, b1);
  mjtNum seg[2] = {0, top_intersect};
  for (int i = 0; i < 6; i++) {
    if (all[i] > seg[1]) {
      seg[0] = top_intersect;
      seg[1] = all[i];
    }
  }
  mjtNum dx = (2.0*size[0]) / (ncol-1), dy = (2.0*size[1]) / (nrow-1), SX[2], SY[2];
  for (int i = 0; i < 2; i++) {
    SX[i] = (lpnt[0] + seg[i]*lvec[0] + size[0]) / dx;
    SY[i] = (lpnt[1] + seg[i]*lvec[1] + size[1]) / dy;
  }
  int cmin = mjMAX(0, (int)floor(mjMIN(SX[0], SX[1]))-1);
  int cmax = mjMIN(ncol-1, (int)ceil(mjMAX(SX[0], SX[1]))+1);
  int rmin = mjMAX(0, (int)floor(mjMIN(SY[0], SY[1]))-1);
  int rmax = mjMIN(nrow-1, (int)ceil(mjMAX(SY[0], SY[1]))+1);
  for (int r = rmin; r < rmax; r++) {
    for (int c = cmin; c < cmax; c++) {
      mjtNum va[3][3] = {
        {dx*c-size[0], dy*r-size[1], data[r*ncol+c]*size[2]},
        {dx*(c+1)-size[0], dy*(r+1)-size[1], data[(r+1)*ncol+(c+1)]*size[2]},
        {dx*(c+1)-size[0], dy*r-size[1], data[r*ncol+(c+1)]*size[2]}};
      mjtNum sol = or_rayTriangle(va, lpnt, lvec, b0, b1);
      if (sol >= 0 && (x < 0 || sol < x)) x = sol;
      mjtNum vb[3][3] = {
        {dx*c-size[0], dy*r-size[1], data[r*ncol+c]*size[2]},
        {dx*(c+1)-size[0], dy*(r+1)-size[1], data[(r+1)*ncol+(c+1)]*size[2]},
        {dx*c-size[0], dy*(r+1)-size[1], data[(r+1)*ncol+c]*size[2]}};
      sol = or_rayTriangle(vb, lpnt, lvec, b0, b1);
      if (sol >= 0 && (x < 0 || sol < x)) x = sol;
    }
  }
  for (int i = 0; i < 4; i++) {
    if (all[i] >= 0 && (all[i] < x || x < 0)) {
      mjtNum z = (lpnt[2] + all[i]*lvec[2]) / size[2];
      mjtNum y, y0, z0, z1;
      if (i < 2) {
        y = (lpnt[1] + all[i]*lvec[1] + size[1]) / dy;
        y0 = mjMAX(0, mjMIN(nrow-2, floor(y)));
        z0 = (mjtNum)data[(int)round(y0)*nrow + (i == 1 ? ncol-1 : 0)];
        z1 = (mjtNum)data[(int)round(y0+1)*nrow + (i == 1 ? ncol-1 : 0)];
      } else {
        y = (lpnt[0] + all[i]*lvec[0] + size[0]) / dx;
        y0 = mjMAX(0, mjMIN(ncol-2, floor(y)));
        z0 = (mjtNum)data[(int)round(y0) + (i == 3 ? (nrow-1)*ncol : 0)];
        z1 = (mjtNum)data[(int)round(y0+1) + (i == 3 ? (nrow-1)*ncol : 0)];
      }
      if (z < z0*(y0+1-y) + z1*(y-y0)) x = all[i];
    }
  }
  return x;
}

/* mj_rayMesh :800-813: the bounding box, then every face (mju_rayTree :628-730 visits the
   faces whose bounding volumes the ray crosses; the nearest hit over all faces is the same) */
static mjtNum or_rayMesh(const mjhipModel* m, const mjhipData* d, int id, const mjtNum* pnt,
                         const mjtNum* vec) {
  const mjtNum* xpos = d->geom_xpos + 3*id;
  const mjtNum* xmat = d->geom_xmat + 9*id;
  if (or_rayBoxAll(xpos, xmat, m->geom_size + 3*id, pnt, vec, NULL) < 0) return -1;
  const int mid = m->geom_dataid[id];
  mjtNum lpnt[3], lvec[3], b0[3], b1[3];
  or_rayMap(xpos, xmat, pnt, vec, lpnt, lvec);
  or_rayBasis(lvec, b0, b1);
  mjtNum x = -1;
  for (int f = m->mesh_faceadr[mid]; f < m->mesh_faceadr[mid] + m->mesh_facenum[mid]; f++) {
    mjtNum v[3][3];
    for (int i = 0; i < 3; i++) {
      const float* vf = m->mesh_vert + 3*(m->mesh_face[3*f + i] + m->mesh_vertadr[mid]);
      for (int j = 0; j < 3; j++) v[i][j] = (mjtNum)vf[j];
    }
    mjtNum sol = or_rayTriangle(v, lpnt, lvec, b0, b1);
    if (sol >= 0 && (x < 0 || sol < x)) x = sol;
  }
  return x;
}

/* mju_rayGeom :818-846 for the primitive types a site can have */
static mjtNum or_rayGeom(const mjtNum* pos, const mjtNum* mat, const mjtNum* size,
                         const mjtNum* pnt, const mjtNum* vec, int type) {
  switch (type) {
  case mjhipGEOM_PLANE:     return or_rayPlane(pos, mat, size, pnt, vec);
  case mjhipGEOM_SPHERE:    return or_raySphere(pos, size[0]*size[0], pnt, vec);
  case mjhipGEOM_CAPSULE:   return or_rayCapsule(pos, mat, size, pnt, vec);
  case mjhipGEOM_ELLIPSOID: return or_rayEllipsoid(pos, mat, size, pnt, vec);
  case mjhipGEOM_CYLINDER:  return or_rayCylinder(pos, mat, size, pnt, vec);
  case mjhipGEOM_BOX:       return or_rayBox(pos, mat, size, pnt, vec);
  default:                  return -1;
  }
}

/* the rangefinder (engine_sensor.c mjSENS_RANGEFINDER): mj_ray from the site along its z
 * axis, geomgroup NULL, flg_static 1, the site's body excluded */
/* :69-100 ray_eliminate with geomgroup NULL and flg_static 1: the excluded body's geoms and
 * invisible geoms (alpha 0 of the geom, or of its material) */
static int or_rayEliminate(const mjhipModel* m, int g, int bodyexclude) {
  if (m->geom_bodyid[g] == bodyexclude) return 1;
  const int mat = m->geom_matid[g];
  if (mat < 0 && m->geom_rgba[4*g+3] == 0) return 1;
  if (mat >= 0 && m->mat_rgba[4*mat+3] == 0) return 1;
  return 0;
}

/* :1145-1185 mj_ray (geomgroup NULL, flg_static 1): the nearest hit, -1 for none; the geom hit
 * in *geomid (exported below for the tests as or_rayTest) */
static mjtNum or_ray(const mjhipModel* m, const mjhipData* d, const mjtNum* pnt, const mjtNum* vec,
              int bodyexclude, int* geomid);
mjtNum or_rayTest(const mjhipModel* m, const mjhipData* d, const mjtNum* pnt,
                  const mjtNum* vec, int bodyexclude, int* geomid) {
  return or_ray(m, d, pnt, vec, bodyexclude, geomid);
}
static mjtNum or_ray(const mjhipModel* m, const mjhipData* d, const mjtNum* pnt, const mjtNum* vec,
              int bodyexclude, int* geomid) {
  mjtNum dist = -1;
  if (geomid) *geomid = -1;
  for (int g = 0; g < m->ngeom; g++) {
    if (or_rayEliminate(m, g, bodyexclude)) continue;
    const int t = m->geom_type[g];
    const mjtNum nd = t == mjhipGEOM_MESH ? or_rayMesh(m, d, g, pnt, vec) :
                      t == mjhipGEOM_HFIELD ? or_rayHfield(m, d, g, pnt, vec) :
                      or_rayGeom(d->geom_xpos+3*g, d->geom_xmat+9*g, m->geom_size+3*g, pnt, vec,
                                 t);
    if (nd >= 0 && (nd < dist || dist < 0)) {
      dist = nd;
      if (geomid) *geomid = g;
    }
  }
  return dist;
}


/* the touch sensor (engine_sensor.c:750-793): normal forces of the contacts of the site's
 * body whose normal ray, from the contact point, hits the site's zone */
static mjtNum or_touch(const mjhipModel* m, const mjhipData* d, const orEfc* e, int objid) {
  int bodyid = m->site_bodyid[objid];
  mjtNum total = 0, conforce[6], conray[3];
  for (int j = 0; j < e->ncon; j++) {
    int conbody[2];
    for (int k = 0; k < 2; k++) {
      int g = e->con_geom[2*j+k];
      conbody[k] = g >= 0 ? m->geom_bodyid[g] : -1;
    }
    if (e->con_efc_address[j] >= 0 && (bodyid == conbody[0] || bodyid == conbody[1])) {
      or_contactForce(m, e, j, conforce);
      if (conforce[0] <= 0) continue;
      mju_scl3(conray, e->con_frame + 9*j, conforce[0]);
      mju_normalize3(conray);
      if (bodyid == conbody[1]) mju_scl3(conray, conray, -1);
      if (or_rayGeom(d->site_xpos + 3*objid, d->site_xmat + 9*objid, m->site_size + 3*objid,
                     e->con_pos + 3*j, conray, m->site_type[objid]) >= 0) {
        total += conforce[0];
      }
    }
  }
  return total;
}

/* engine_sensor.c:677-915 mj_sensorAcc */
static void or_sensorAcc(const mjhipModel* m, mjhipData* d, const orEfc* e) {
  if (mjDISABLED(mjhipDSBL_SENSOR)) return;
  int rnePost = 0;
  mjtNum tmp[6];
  for (int i = 0; i < m->nsensor; i++) {
    if (m->sensor_needstage[i] != mjhipSTAGE_ACC) continue;
    int type = m->sensor_type[i], objtype = m->sensor_objtype[i], objid = m->sensor_objid[i];
    mjtNum* out = d->sensordata + m->sensor_adr[i];
    int r, bodyid, rootid;
    if (!rnePost && (type == SENS_ACCELEROMETER || type == SENS_FORCE || type == SENS_TORQUE ||
                     type == SENS_FRAMELINACC || type == SENS_FRAMEANGACC)) {
      or_rnePostConstraint(m, d, e);
      rnePost = 1;
    }
    switch (type) {
    case SENS_TOUCH:
      out[0] = or_touch(m, d, e, objid);
      break;
    case SENS_ACCELEROMETER:
      or_objectAcceleration(m, d, OBJ_SITE, objid, tmp, 1);
      mju_copy3(out, tmp + 3);
      break;
    case SENS_FORCE:
    case SENS_TORQUE:
      bodyid = m->site_bodyid[objid];
      rootid = m->body_rootid[bodyid];
      mju_transformSpatial(tmp, d->cfrc_int + 6*bodyid, 1, d->site_xpos + 3*objid,
                           d->subtree_com + 3*rootid, d->site_xmat + 9*objid);
      mju_copy3(out, type == SENS_FORCE ? tmp + 3 : tmp);
      break;
    case SENS_ACTUATORFRC:
      out[0] = d->actuator_force[objid];
      break;
    case SENS_JOINTACTFRC:
      out[0] = d->qfrc_actuator[m->jnt_dofadr[objid]];
      break;
    case SENS_JOINTLIMITFRC:
    case SENS_TENDONLIMITFRC:
      out[0] = 0;
      r = or_limitRow(e, type == SENS_JOINTLIMITFRC ? orCNSTR_LIMIT_JOINT : orCNSTR_LIMIT_TENDON,
                      objid);
      if (r >= 0) out[0] = e->efc_force[r];
      break;
    case SENS_FRAMELINACC:
    case SENS_FRAMEANGACC:
      or_objectAcceleration(m, d, objtype, objid, tmp, 0);
      mju_copy3(out, type == SENS_FRAMELINACC ? tmp + 3 : tmp);
      break;
    }
  }
  or_applyCutoff(m, d, mjhipSTAGE_ACC);
}

void or_inverseSkip(const mjhipModel* m, mjhipData* d, orEfc* e, int skipstage,
                    int skipsensor) {
  int nv = m->nv;
  mjtNum* qacc = NULL;
  d->status = or_checkInputs(m, d, skipstage < mjhipSTAGE_POS, skipstage < mjhipSTAGE_VEL, 1);
  if (skipstage < mjhipSTAGE_POS) {
    or_invPosition(m, d, e);
    if (!skipsensor) or_sensorPos(m, d, e);
    if (mjENABLED(mjhipENBL_ENERGY)) or_energyPos(m, d);
  }
  if (skipstage < mjhipSTAGE_VEL) {
    or_fwdVelocity(m, d, e);
    if (!skipsensor) or_sensorVel(m, d, e);
    if (mjENABLED(mjhipENBL_ENERGY)) or_energyVel(m, d);
  }
  if (mjENABLED(mjhipENBL_INVDISCRETE)) {
    qacc = (mjtNum*)malloc(nv*sizeof(mjtNum));
    mju_copy(qacc, d->qacc, nv);
    or_discreteAcc(m, d);
  }
  or_invConstraint(m, d, e);
  or_rne(m, d, 1, d->qfrc_inverse);
  if (!skipsensor) or_sensorAcc(m, d, e);
  for (int i = 0; i < nv; i++) {
    d->qfrc_inverse[i] += m->dof_armature[i] * d->qacc[i]
                          - d->qfrc_passive[i] - d->qfrc_constraint[i];
  }
  if (qacc) {
    mju_copy(d->qacc, qacc, nv);
    free(qacc);
  }
  d->nefc = e->nefc;
}

/* engine_inverse.c:266-269 */
void or_inverse(const mjhipModel* m, mjhipData* d, orEfc* e) {
  or_inverseSkip(m, d, e, mjhipSTAGE_NONE, 0);
}

/*============================ forward harness (engine_forward.c) ===========================*/

/* mj_fwdActuation :276-515 for gain fixed/affine, bias none/affine, no dynamics, joint
 * transmission; qfrc_actuator = moment' * force */
static void or_fwdActuation(const mjhipModel* m, mjhipData* d) {
  int nv = m->nv, nu = m->nu;
  mju_zero(d->qfrc_actuator, nv);
  mju_zero(d->actuator_force, nu);
  if (mjDISABLED(mjhipDSBL_ACTUATION) || !nu) return;
  mjtNum* force = d->actuator_force;
  for (int i = 0; i < nu; i++) {
    mjtNum ctrl = d->ctrl ? d->ctrl[i] : 0;
    if (m->actuator_ctrllimited[i] && !mjDISABLED(mjhipDSBL_CLAMPCTRL)) {
      mjtNum* r = m->actuator_ctrlrange + 2*i;
      ctrl = ctrl < r[0] ? r[0] : (ctrl > r[1] ? r[1] : ctrl);
    }
    mjtNum* prm = m->actuator_gainprm + 10*i;
    mjtNum gain = prm[0];
    if (m->actuator_gaintype[i] == mjhipGAIN_AFFINE) {
      gain = prm[0] + prm[1]*d->actuator_length[i] + prm[2]*d->actuator_velocity[i];
    }
    force[i] = gain * ctrl;
    if (m->actuator_biastype[i] == mjhipBIAS_AFFINE) {
      prm = m->actuator_biasprm + 10*i;
      force[i] += prm[0] + prm[1]*d->actuator_length[i] + prm[2]*d->actuator_velocity[i];
    }
    if (m->actuator_forcelimited[i]) {
      mjtNum* r = m->actuator_forcerange + 2*i;
      force[i] = force[i] < r[0] ? r[0] : (force[i] > r[1] ? r[1] : force[i]);
    }
  }
  for (int i = 0; i < nu; i++) {       /* mju_mulMatTVecSparse */
    if (!force[i]) continue;
    int adr = m->moment_rowadr[i];
    for (int j = 0; j < m->moment_rownnz[i]; j++) {
      d->qfrc_actuator[m->moment_colind[adr+j]] += d->actuator_moment[adr+j]*force[i];
    }
  }
}

/* mj_forward for constraint-free states: position, velocity, actuation, acceleration,
 * with qacc = qacc_smooth (engine_forward.c:520-531, :654-: nefc = 0) */
int or_forward(const mjhipModel* m, mjhipData* d, orEfc* e) {
  int nv = m->nv;
  d->status = or_checkInputs(m, d, 1, 1, 0);
  or_invPosition(m, d, e);
  or_fwdVelocity(m, d, e);
  or_fwdActuation(m, d);
  /* mj_fwdAcceleration engine_forward.c:520-531 */
  mju_sub(d->qfrc_smooth, d->qfrc_passive, d->qfrc_bias, nv);
  mju_addTo(d->qfrc_smooth, d->qfrc_applied, nv);
  mju_addTo(d->qfrc_smooth, d->qfrc_actuator, nv);
  or_xfrcAccumulate(m, d, d->qfrc_smooth);
  or_solveM(m, d, d->qacc_smooth, d->qfrc_smooth, 1);
  /* mj_fwdConstraint with nefc = 0: qacc = qacc_smooth, no constraint force */
  mju_copy(d->qacc, d->qacc_smooth, nv);
  mju_zero(d->qfrc_constraint, nv);
  d->status |= or_checkInputs(m, d, 0, 0, 1);      /* mj_checkAcc after mj_forward */
  d->nefc = e->nefc;
  return e->nefc;
}

/* mj_RungeKutta(m, d, 4), engine_forward.c:842-941 (na = 0) */
void or_rungeKutta4(const mjhipModel* m, mjhipData* d, orEfc* e) {
  static const mjtNum A[9] = {0.5, 0, 0, 0, 0.5, 0, 0, 0, 1};
  static const mjtNum Bt[4] = {1.0/6.0, 1.0/3.0, 1.0/3.0, 1.0/6.0};
  int nv = m->nv, nq = m->nq, N = 4;
  mjtNum h = m->opt.timestep;
  mjtNum *X[4], *F[4];
  mjtNum* dX = (mjtNum*)malloc(2*nv*sizeof(mjtNum));
  for (int i = 0; i < N; i++) {
    X[i] = (mjtNum*)malloc((nq+nv)*sizeof(mjtNum));
    F[i] = (mjtNum*)malloc(nv*sizeof(mjtNum));
  }
  mju_copy(X[0], d->qpos, nq);
  mju_copy(X[0]+nq, d->qvel, nv);
  mju_copy(F[0], d->qacc, nv);
  for (int i = 1; i < N; i++) {
    mju_zero(dX, 2*nv);
    for (int j = 0; j < i; j++) {
      mju_addToScl(dX, X[j]+nq, A[(i-1)*(N-1)+j], nv);
      mju_addToScl(dX+nv, F[j], A[(i-1)*(N-1)+j], nv);
    }
    mju_copy(X[i], X[0], nq+nv);
    mj_integratePos(m, X[i], dX, h);
    mju_addToScl(X[i]+nq, dX+nv, h, nv);
    mju_copy(d->qpos, X[i], nq);
    mju_copy(d->qvel, X[i]+nq, nv);
    or_forward(m, d, e);
    mju_copy(F[i], d->qacc, nv);
  }
  mju_zero(dX, 2*nv);
  for (int j = 0; j < N; j++) {
    mju_addToScl(dX, X[j]+nq, Bt[j], nv);
    mju_addToScl(dX+nv, F[j], Bt[j], nv);
  }
  mju_copy(d->qpos, X[0], nq);
  mju_copy(d->qvel, X[0]+nq, nv);
  /* mj_advance(m, d, 0, dX+nv, dX): qvel += h*qacc, then integratePos with dX */
  mju_addToScl(d->qvel, dX+nv, h, nv);
  mj_integratePos(m, d->qpos, dX, h);
  for (int i = 0; i < N; i++) {
    free(X[i]);
    free(F[i]);
  }
  free(dX);
}

/*============================ engine_derivative_fd.c ======================================*/

/* :48-53 */
static void diff(mjtNum* dx, const mjtNum* x1, const mjtNum* x2, mjtNum h, int n) {
  mjtNum inv_h = 1/h;
  for (int i = 0; i < n; i++) dx[i] = inv_h * (x2[i] - x1[i]);
}

/* engine_derivative_fd.c:160-168: one evaluation, force = qfrc_inverse (- qfrc_actuator of
 * mj_fwdActuation when flg_actuation) */
static void fd_eval(const mjhipModel* m, mjhipData* d, orEfc* e, int stage, int skipsensor,
                    int flg_actuation, mjtNum* force) {
  or_inverseSkip(m, d, e, stage, skipsensor);
  mju_copy(force, d->qfrc_inverse, m->nv);
  if (flg_actuation) {
    or_fwdActuation(m, d);
    for (int i = 0; i < m->nv; i++) force[i] -= d->qfrc_actuator[i];
  }
}

/* engine_derivative_fd.c:611-719 mjd_inverseFD */
void or_inverseFDEx(const mjhipModel* m, mjhipData* d, orEfc* e, mjtNum eps, int flg_actuation,
                    mjtNum* DfDq, mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv,
                    mjtNum* DsDa, mjtNum* DmDq) {
  int nq = m->nq, nv = m->nv, nM = m->nM, ns = m->nsensordata;
  int skipsensor = !DsDq && !DsDv && !DsDa;
  mjtNum* pos = (mjtNum*)malloc(nq*sizeof(mjtNum));
  mjtNum* force = (mjtNum*)malloc(nv*sizeof(mjtNum));
  mjtNum* force_plus = (mjtNum*)malloc(nv*sizeof(mjtNum));
  mjtNum* sensor = (mjtNum*)malloc((ns + 1)*sizeof(mjtNum));
  mjtNum* mass = (mjtNum*)malloc(nM*sizeof(mjtNum));
  mjtNum* dpos = (mjtNum*)calloc(nv, sizeof(mjtNum));
  mju_copy(pos, d->qpos, nq);
  fd_eval(m, d, e, mjhipSTAGE_NONE, skipsensor, flg_actuation, force);
  if (!skipsensor) mju_copy(sensor, d->sensordata, ns);
  mju_copy(mass, d->qM, nM);
  if (DfDa || DsDa) {
    for (int i = 0; i < nv; i++) {
      mjtNum tmp = d->qacc[i];
      d->qacc[i] += eps;
      fd_eval(m, d, e, mjhipSTAGE_VEL, skipsensor, flg_actuation, force_plus);
      d->qacc[i] = tmp;
      if (DfDa) diff(DfDa + i*nv, force, force_plus, eps, nv);
      if (DsDa) diff(DsDa + i*ns, sensor, d->sensordata, eps, ns);
    }
  }
  if (DfDv || DsDv) {
    for (int i = 0; i < nv; i++) {
      mjtNum tmp = d->qvel[i];
      d->qvel[i] += eps;
      fd_eval(m, d, e, mjhipSTAGE_POS, skipsensor, flg_actuation, force_plus);
      d->qvel[i] = tmp;
      if (DfDv) diff(DfDv + i*nv, force, force_plus, eps, nv);
      if (DsDv) diff(DsDv + i*ns, sensor, d->sensordata, eps, ns);
    }
  }
  if (DfDq || DsDq || DmDq) {
    for (int i = 0; i < nv; i++) {
      mju_zero(dpos, nv);
      dpos[i] = 1;
      mj_integratePos(m, d->qpos, dpos, eps);
      fd_eval(m, d, e, mjhipSTAGE_NONE, skipsensor, flg_actuation, force_plus);
      mju_copy(d->qpos, pos, nq);
      if (DfDq) diff(DfDq + i*nv, force, force_plus, eps, nv);
      if (DsDq) diff(DsDq + i*ns, sensor, d->sensordata, eps, ns);
      if (DmDq) diff(DmDq + i*nM, mass, d->qM, eps, nM);
    }
  }
  /* like the reference, d keeps the outputs of the last perturbed evaluation */
  free(pos); free(force); free(force_plus); free(sensor); free(mass); free(dpos);
}

void or_inverseFD(const mjhipModel* m, mjhipData* d, orEfc* e, mjtNum eps, mjtNum* DfDq,
                  mjtNum* DfDv, mjtNum* DfDa, mjtNum* DsDq, mjtNum* DsDv, mjtNum* DsDa,
                  mjtNum* DmDq) {
  or_inverseFDEx(m, d, e, eps, 0, DfDq, DfDv, DfDa, DsDq, DsDv, DsDa, DmDq);
}

/* engine_inverse.c:275-316 mj_compareFwdInv: with rows from a forward pass in e, the
 * inverse of the forward qacc against the forward constraint force and applied forces */
void or_compareFwdInv(const mjhipModel* m, mjhipData* d, orEfc* e) {
  int nv = m->nv, nefc = e->nefc;
  d->solver_fwdinv[0] = d->solver_fwdinv[1] = 0;
  if (!nefc) return;
  mjtNum* qforce = (mjtNum*)malloc(nv*sizeof(mjtNum));
  mjtNum* dif = (mjtNum*)malloc(nv*sizeof(mjtNum));
  mjtNum* save_qfrc_constraint = (mjtNum*)malloc(nv*sizeof(mjtNum));
  mjtNum* save_efc_force = (mjtNum*)malloc(nefc*sizeof(mjtNum));
  for (int i = 0; i < nv; i++) qforce[i] = d->qfrc_applied[i] + d->qfrc_actuator[i];
  or_xfrcAccumulate(m, d, qforce);
  mju_copy(save_qfrc_constraint, d->qfrc_constraint, nv);
  mju_copy(save_efc_force, e->efc_force, nefc);
  or_inverseSkip(m, d, e, mjhipSTAGE_VEL, 1);
  for (int i = 0; i < nv; i++) dif[i] = save_qfrc_constraint[i] - d->qfrc_constraint[i];
  d->solver_fwdinv[0] = mju_norm(dif, nv);
  for (int i = 0; i < nv; i++) dif[i] = qforce[i] - d->qfrc_inverse[i];
  d->solver_fwdinv[1] = mju_norm(dif, nv);
  mju_copy(d->qfrc_constraint, save_qfrc_constraint, nv);
  mju_copy(e->efc_force, save_efc_force, nefc);
  free(qforce); free(dif); free(save_qfrc_constraint); free(save_efc_force);
}

/*============================ CPU baseline =================================================*/

typedef struct {
  const mjhipModel* m;
  const mjtNum *qpos, *qvel, *qacc;
  mjtNum* qfrc;
  int B, chunk;
  int* next;               /* shared chunk counter */
  pthread_mutex_t* lock;
} orJob;

static mjtNum* alloc_data(const mjhipModel* m, mjhipData* d, orEfc* e) {
  size_t total = 0;
  int cap = or_efcCapacity(m);
#define MJ_M(n) m->n
#define XD(name, d0, d1, stage) total += (size_t)(m->d0) * (d1);
  MJHIP_DATA_FIELDS
#undef XD
  total += 2*(size_t)m->nv + 6*(size_t)m->nbody + 2*(size_t)m->nu;
#define XD(name, d0, d1, stage) total += (size_t)(m->d0) * (d1);
  MJHIP_DATA_SENSOR_AUX
#undef XD
  total += (size_t)cap * (m->nv + 14);
  mjtNum* buf = (mjtNum*)calloc(total + 1, sizeof(mjtNum));
  mjtNum* p = buf;
  memset(d, 0, sizeof(*d));
#define XD(name, d0, d1, stage) d->name = p; p += (size_t)(m->d0) * (d1);
  MJHIP_DATA_FIELDS
#undef XD
#undef MJ_M
  d->qfrc_applied = p; p += m->nv;
  d->qfrc_actuator = p; p += m->nv;
  d->xfrc_applied = p; p += 6*m->nbody;
  d->ctrl = p; p += m->nu;
  d->actuator_force = p; p += m->nu;
#define XD(name, d0, d1, stage) d->name = p; p += (size_t)(m->d0) * (d1);
  MJHIP_DATA_SENSOR_AUX
#undef XD
  memset(e, 0, sizeof(*e));
  e->capacity = cap;
  e->efc_J = p; p += (size_t)cap*m->nv;
  e->efc_pos = p; p += cap;
  e->efc_margin = p; p += cap;
  e->efc_frictionloss = p; p += cap;
  e->efc_diagApprox = p; p += cap;
  e->efc_KBIP = p; p += 4*(size_t)cap;
  e->efc_D = p; p += cap;
  e->efc_R = p; p += cap;
  e->efc_vel = p; p += cap;
  e->efc_aref = p; p += cap;
  e->efc_force = p; p += cap;
  e->efc_type = (int*)calloc(3*(size_t)cap + 1, sizeof(int));
  e->efc_id = e->efc_type + cap;
  e->efc_state = e->efc_id + cap;
  if (mj_isSparse(m)) {                    /* compressed rows and tendon Jacobians */
    size_t cn = (size_t)cap*m->nv, tn = (size_t)m->ntendon;
    int* ip = (int*)calloc(2*tn + tn*m->nv + 2*(size_t)cap + 2*cn + 2*(size_t)m->nv + 1,
                           sizeof(int));
    e->efc_JT = (mjtNum*)calloc(cn + 1, sizeof(mjtNum));
    d->ten_J_rownnz = ip; ip += tn;
    d->ten_J_rowadr = ip; ip += tn;
    d->ten_J_colind = ip; ip += tn*m->nv;
    e->efc_J_rownnz = ip; ip += cap;
    e->efc_J_rowadr = ip; ip += cap;
    e->efc_J_colind = ip; ip += cn;
    e->efc_JT_rownnz = ip; ip += m->nv;
    e->efc_JT_rowadr = ip; ip += m->nv;
    e->efc_JT_colind = ip;
  }
  return buf;
}

static void* worker(void* arg) {
  orJob* J = (orJob*)arg;
  const mjhipModel* m = J->m;
  mjhipData d;
  orEfc e;
  mjtNum* buf = alloc_data(m, &d, &e);
  for (;;) {
    pthread_mutex_lock(J->lock);
    int start = *J->next;
    *J->next += J->chunk;
    pthread_mutex_unlock(J->lock);
    if (start >= J->B) break;
    int end = start + J->chunk < J->B ? start + J->chunk : J->B;
    for (int k = start; k < end; k++) {
      mju_copy(d.qpos, J->qpos + (size_t)k*m->nq, m->nq);
      mju_copy(d.qvel, J->qvel + (size_t)k*m->nv, m->nv);
      mju_copy(d.qacc, J->qacc + (size_t)k*m->nv, m->nv);
      or_inverse(m, &d, &e);
      mju_copy(J->qfrc + (size_t)k*m->nv, d.qfrc_inverse, m->nv);
    }
  }
  free(e.efc_type);
  free(d.ten_J_rownnz);
  free(e.efc_JT);
  free(buf);
  return NULL;
}

double or_inverseBatch(const mjhipModel* m, int B, const mjtNum* qpos, const mjtNum* qvel,
                       const mjtNum* qacc, mjtNum* qfrc_inverse, int nthread) {
  if (nthread < 1) nthread = 1;
  int chunk = B / (10*nthread);
  if (chunk < 1) chunk = 1;
  int next = 0;
  pthread_mutex_t lock = PTHREAD_MUTEX_INITIALIZER;
  orJob job = {m, qpos, qvel, qacc, qfrc_inverse, B, chunk, &next, &lock};
  pthread_t* th = (pthread_t*)malloc(nthread*sizeof(pthread_t));
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int i = 0; i < nthread; i++) pthread_create(&th[i], NULL, worker, &job);
  for (int i = 0; i < nthread; i++) pthread_join(th[i], NULL);
  clock_gettime(CLOCK_MONOTONIC, &t1);
  free(th);
  return (t1.tv_sec - t0.tv_sec) + 1e-9*(t1.tv_nsec - t0.tv_nsec);
}
