/*
 * deftri_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library.  The product (triangulation-in-deformable-scenes_amd/) never links or calls it.
 *
 * A plain-C restatement of the reference hot path: the g2o Levenberg–Marquardt solve that
 * `arapOptimization` runs (reference Modules/Optimization/g2oBundleAdjustment.cc:608-1008,
 * LM call at :962), with the reference's edge types:
 *   - EdgeSE3ProjectXYZPerKeyFrameOnlyPoints  g2oTypes.h:267-298, linearizeOplus g2oTypes.cc:270-283
 *   - EdgeDepthCorrection                     g2oTypes.h:390-421 (numeric Jacobian)
 *   - EdgeARAP                                g2oTypes.h:300-349 (numeric Jacobian; analytic one
 *                                             commented out at g2oTypes.cc:308-331)
 *   - KannalaBrandt8::project / projectJac    Modules/Calibration/KannalaBrandt8.cc:32-49, 85-114 (fp32)
 * and the third-party semantics g2o contributes (not vendored in the reference; version
 * unpinned — SURVEY §8c / Appendix A), restated from upstream g2o's published code:
 *   - BaseMultiEdge / BaseBinaryEdge numeric linearizeOplus: central differences, delta 1e-9
 *   - RobustKernelHuber::robustify, robustInformation = rho'·Omega
 *   - OptimizationAlgorithmLevenberg::solve: lambda init tau*max diag (tau 1e-5), rho test with
 *     scale = dx·(lambda dx + b) + 1e-3, lambda *= max(1/3, min(2/3, 1-(2rho-1)^3)) / lambda *= ni,
 *     ni *= 2, at most 10 trials
 *   - SE3Quat (map, exp, product, normalizeRotation) and Eigen's quaternion<->matrix formulas
 *   - LinearSolverEigen = Eigen SimplicialLDLT: up-looking sparse LDL^T (T. Davis' LDL algorithm,
 *     which Eigen's SimplicialCholesky implements), zero pivot = failed solve.
 * Ordering: Eigen uses (block) AMD; this restatement uses a geometric nested dissection on the
 * point coordinates (same factor, different fill/rounding) — documented in DESIGN.md.
 *
 * Build: oracle/Makefile (gcc -O2 -fno-fast-math -ffp-contract=off).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/deftri.h"

/* ------------------------------------------------------------------------------------ */
/* quaternion / SE3Quat (g2o types_six_dof_expmap + Eigen Quaternion formulas)           */
/* ------------------------------------------------------------------------------------ */
typedef struct { double x, y, z, w; } quat;
typedef struct { quat r; double t[3]; } se3q;

static void q_normalize_rotation(quat *q) {        /* SE3Quat::normalizeRotation */
    if (q->w < 0) { q->x = -q->x; q->y = -q->y; q->z = -q->z; q->w = -q->w; }
    double n = sqrt(q->x * q->x + q->y * q->y + q->z * q->z + q->w * q->w);
    q->x /= n; q->y /= n; q->z /= n; q->w /= n;
}

static void q_to_mat(const quat *q, double R[9]) { /* Eigen QuaternionBase::toRotationMatrix */
    double tx = 2 * q->x, ty = 2 * q->y, tz = 2 * q->z;
    double twx = tx * q->w, twy = ty * q->w, twz = tz * q->w;
    double txx = tx * q->x, txy = ty * q->x, txz = tz * q->x;
    double tyy = ty * q->y, tyz = tz * q->y, tzz = tz * q->z;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}

static quat q_from_mat(const double m[9]) {        /* Eigen quaternionbase_assign_impl<3x3> */
    quat q;
    double t = m[0] + m[4] + m[8];
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[7] - m[5]) * t;
        q.y = (m[2] - m[6]) * t;
        q.z = (m[3] - m[1]) * t;
    } else {
        int i = 0;
        if (m[4] > m[0]) i = 1;
        if (m[8] > m[3 * i + i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        double c[3];
        t = sqrt(m[3 * i + i] - m[3 * j + j] - m[3 * k + k] + 1.0);
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[3 * k + j] - m[3 * j + k]) * t;
        c[j] = (m[3 * j + i] + m[3 * i + j]) * t;
        c[k] = (m[3 * k + i] + m[3 * i + k]) * t;
        q.x = c[0]; q.y = c[1]; q.z = c[2];
    }
    return q;
}

static void q_rotate(const quat *q, const double v[3], double out[3]) { /* Eigen _transformVector */
    double uv[3] = {q->y * v[2] - q->z * v[1], q->z * v[0] - q->x * v[2], q->x * v[1] - q->y * v[0]};
    uv[0] += uv[0]; uv[1] += uv[1]; uv[2] += uv[2];
    double c[3] = {q->y * uv[2] - q->z * uv[1], q->z * uv[0] - q->x * uv[2], q->x * uv[1] - q->y * uv[0]};
    out[0] = v[0] + q->w * uv[0] + c[0];
    out[1] = v[1] + q->w * uv[1] + c[1];
    out[2] = v[2] + q->w * uv[2] + c[2];
}

static quat q_mul(const quat *a, const quat *b) {
    quat r;
    r.w = a->w * b->w - a->x * b->x - a->y * b->y - a->z * b->z;
    r.x = a->w * b->x + a->x * b->w + a->y * b->z - a->z * b->y;
    r.y = a->w * b->y + a->y * b->w + a->z * b->x - a->x * b->z;
    r.z = a->w * b->z + a->z * b->w + a->x * b->y - a->y * b->x;
    return r;
}

static void se3_map(const se3q *T, const double p[3], double out[3]) {   /* SE3Quat::map */
    q_rotate(&T->r, p, out);
    out[0] += T->t[0]; out[1] += T->t[1]; out[2] += T->t[2];
}

static se3q se3_from7(const double *a) {
    se3q T;
    T.r.x = a[0]; T.r.y = a[1]; T.r.z = a[2]; T.r.w = a[3];
    T.t[0] = a[4]; T.t[1] = a[5]; T.t[2] = a[6];
    q_normalize_rotation(&T.r);                     /* SE3Quat(q, t) constructor */
    return T;
}
static void se3_to7(const se3q *T, double *a) {
    a[0] = T->r.x; a[1] = T->r.y; a[2] = T->r.z; a[3] = T->r.w;
    a[4] = T->t[0]; a[5] = T->t[1]; a[6] = T->t[2];
}

static se3q se3_exp(const double u[6]) {           /* SE3Quat::exp (omega, upsilon) */
    const double *w = u, *ups = u + 3;
    double theta = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    double O[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double O2[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += O[3 * i + k] * O[3 * k + j];
            O2[3 * i + j] = s;
        }
    double R[9], V[9], a, b, c, d;
    if (theta < 0.00001) { a = 1; b = 0.5; c = 0.5; d = 1.0 / 6.0; }
    else {
        a = sin(theta) / theta;
        b = (1 - cos(theta)) / (theta * theta);
        c = (1 - cos(theta)) / (theta * theta);
        d = (theta - sin(theta)) / pow(theta, 3);
    }
    for (int i = 0; i < 9; i++) {
        double I = (i % 4 == 0) ? 1.0 : 0.0;
        R[i] = I + a * O[i] + b * O2[i];
        V[i] = I + c * O[i] + d * O2[i];
    }
    se3q T;
    T.r = q_from_mat(R);
    for (int i = 0; i < 3; i++) T.t[i] = V[3 * i] * ups[0] + V[3 * i + 1] * ups[1] + V[3 * i + 2] * ups[2];
    q_normalize_rotation(&T.r);
    return T;
}

static se3q se3_mul(const se3q *A, const se3q *B) { /* SE3Quat::operator* */
    se3q r = *A;
    double tb[3];
    q_rotate(&A->r, B->t, tb);
    r.t[0] += tb[0]; r.t[1] += tb[1]; r.t[2] += tb[2];
    r.r = q_mul(&A->r, &B->r);
    q_normalize_rotation(&r.r);
    return r;
}

static void se3_oplus(se3q *T, const double u[6]) { /* VertexSE3Expmap::oplusImpl */
    se3q E = se3_exp(u);
    *T = se3_mul(&E, T);
}

/* ------------------------------------------------------------------------------------ */
/* Kannala–Brandt 8 (fp32 like the reference: project takes p.cast<float>())            */
/* ------------------------------------------------------------------------------------ */
static void kb8_project(const float *k, const float p[3], float uv[2]) {
    const float x2_plus_y2 = p[0] * p[0] + p[1] * p[1];
    const float theta = atan2f(sqrtf(x2_plus_y2), p[2]);
    const float psi = atan2f(p[1], p[0]);
    const float theta2 = theta * theta;
    const float theta3 = theta * theta2;
    const float theta5 = theta3 * theta2;
    const float theta7 = theta5 * theta2;
    const float theta9 = theta7 * theta2;
    const float r = theta + k[4] * theta3 + k[5] * theta5 + k[6] * theta7 + k[7] * theta9;
    uv[0] = k[0] * r * cosf(psi) + k[2];
    uv[1] = k[1] * r * sinf(psi) + k[3];
}

static void kb8_project_jac(const float *k, const float p[3], float J[6]) {
    float x2 = p[0] * p[0], y2 = p[1] * p[1], z2 = p[2] * p[2];
    float r2 = x2 + y2;
    float r = sqrtf(r2);
    float r3 = r2 * r;
    float theta = atan2f(r, p[2]);
    float theta2 = theta * theta, theta3 = theta2 * theta;
    float theta4 = theta2 * theta2, theta5 = theta4 * theta;
    float theta6 = theta2 * theta4, theta7 = theta6 * theta;
    float theta8 = theta4 * theta4, theta9 = theta8 * theta;
    float f = theta + theta3 * k[4] + theta5 * k[5] + theta7 * k[6] + theta9 * k[7];
    float fd = 1 + 3 * k[4] * theta2 + 5 * k[5] * theta4 + 7 * k[6] * theta6 + 9 * k[7] * theta8;
    J[0] = k[0] * (fd * p[2] * x2 / (r2 * (r2 + z2)) + f * y2 / r3);
    J[1] = k[0] * (fd * p[2] * p[1] * p[0] / (r2 * (r2 + z2)) - f * p[1] * p[0] / r3);
    J[2] = -k[0] * fd * p[0] / (r2 + z2);
    J[3] = k[1] * (fd * p[2] * p[1] * p[0] / (r2 * (r2 + z2)) - f * p[1] * p[0] / r3);
    J[4] = k[1] * (fd * p[2] * y2 / (r2 * (r2 + z2)) + f * x2 / r3);
    J[5] = -k[1] * fd * p[1] / (r2 + z2);
}

/* ------------------------------------------------------------------------------------ */
/* problem + state                                                                         */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    const deftri_problem_desc *d;
    se3q *cams;          /* [C] */
    double *camR;        /* [C*9] rotation matrices of the camera poses */
    /* vertex / dof layout: T_g (6) per pair, scales (1), points (3) */
    int64_t nv, ndof;
    int64_t *voff;       /* [nv] */
    int *vdim;           /* [nv] */
} problem;

typedef struct {
    double *points;   /* [P*3] */
    double *scales;   /* [S] */
    se3q *tg;         /* [Q] */
} state;

static int64_t vid_tg(const problem *pb, int q) { (void)pb; return q; }
static int64_t vid_scale(const problem *pb, int s) { return pb->d->n_pairs + s; }
static int64_t vid_point(const problem *pb, int p) { return pb->d->n_pairs + pb->d->n_scales + p; }

static void state_alloc(const problem *pb, state *s) {
    const deftri_problem_desc *d = pb->d;
    s->points = (double *)malloc(sizeof(double) * 3 * (size_t)d->n_points);
    s->scales = (double *)malloc(sizeof(double) * (size_t)(d->n_scales ? d->n_scales : 1));
    s->tg = (se3q *)malloc(sizeof(se3q) * (size_t)(d->n_pairs ? d->n_pairs : 1));
}
static void state_free(state *s) { free(s->points); free(s->scales); free(s->tg); }
static void state_copy(const problem *pb, state *dst, const state *src) {
    const deftri_problem_desc *d = pb->d;
    memcpy(dst->points, src->points, sizeof(double) * 3 * (size_t)d->n_points);
    memcpy(dst->scales, src->scales, sizeof(double) * (size_t)d->n_scales);
    memcpy(dst->tg, src->tg, sizeof(se3q) * (size_t)d->n_pairs);
}

/* --- edge errors ----------------------------------------------------------------------- */
static void rep_error(const problem *pb, const state *s, int e, double err[2]) {
    const deftri_problem_desc *d = pb->d;
    const double *p = s->points + 3 * (size_t)d->rep_point[e];
    int c = d->rep_cam[e];
    double pc[3];
    se3_map(&pb->cams[c], p, pc);
    float pf[3] = {(float)pc[0], (float)pc[1], (float)pc[2]}, uv[2];
    kb8_project(d->cam_kb8 + 8 * c, pf, uv);
    err[0] = d->rep_obs[2 * e] - (double)uv[0];
    err[1] = d->rep_obs[2 * e + 1] - (double)uv[1];
}

static double depth_error_v(const problem *pb, int e, const double *p, double scale) {
    const deftri_problem_desc *d = pb->d;
    double pc[3];
    se3_map(&pb->cams[d->dep_cam[e]], p, pc);
    double error = pow((d->dep_meas[e] / scale - pc[2]), 2);
    if (scale <= 0.0) error = error * 500;
    return error;
}

static double arap_error_v(const problem *pb, int e, const double *v1i, const double *v2i,
                           const double *v1j, const double *v2j, const se3q *T) {
    const deftri_problem_desc *d = pb->d;
    double Rg[9];
    q_to_mat(&T->r, Rg);
    const double *t = T->t;
    double dg[3];
    for (int k = 0; k < 3; k++) {
        double a = Rg[3 * k] * v2i[0] + Rg[3 * k + 1] * v2i[1] + Rg[3 * k + 2] * v2i[2];
        double b = Rg[3 * k] * v2j[0] + Rg[3 * k + 1] * v2j[1] + Rg[3 * k + 2] * v2j[2];
        dg[k] = ((a - t[k]) - v1i[k]) + ((b - t[k]) - v1j[k]);
    }
    double energyGlobal = dg[0] * dg[0] + dg[1] * dg[1] + dg[2] * dg[2];
    const double *Ri = d->rot + 9 * (size_t)d->arap_rot[2 * e];
    const double *Rj = d->rot + 9 * (size_t)d->arap_rot[2 * e + 1];
    int q = d->arap_pair[e];
    double area = d->pair_area[q];
    double d1i[3], d2i[3], d1j[3], d2j[3], f[3], g[3];
    for (int k = 0; k < 3; k++) {
        d1i[k] = v1i[k] - v1j[k]; d2i[k] = v2i[k] - v2j[k];
        d1j[k] = v1j[k] - v1i[k]; d2j[k] = v2j[k] - v2i[k];
    }
    for (int k = 0; k < 3; k++) {
        f[k] = (d2i[k] - (Ri[3 * k] * d1i[0] + Ri[3 * k + 1] * d1i[1] + Ri[3 * k + 2] * d1i[2])) / area;
        g[k] = (d2j[k] - (Rj[3 * k] * d1j[0] + Rj[3 * k + 1] * d1j[1] + Rj[3 * k + 2] * d1j[2])) / area;
    }
    double fn = f[0] * f[0] + f[1] * f[1] + f[2] * f[2];
    double gn = g[0] * g[0] + g[1] * g[1] + g[2] * g[2];
    double energyArap = (d->arap_w[e] * (fn + gn) + energyGlobal);
    return energyArap - 0.0;
}

static double arap_error(const problem *pb, const state *s, int e) {
    const int32_t *v = pb->d->arap_pts + 4 * (size_t)e;
    return arap_error_v(pb, e, s->points + 3 * (size_t)v[0], s->points + 3 * (size_t)v[1],
                        s->points + 3 * (size_t)v[2], s->points + 3 * (size_t)v[3],
                        &s->tg[pb->d->arap_pair[e]]);
}

/* RobustKernelHuber::robustify */
static void huber(double delta, double e2, double rho[3]) {
    double dsqr = delta * delta;
    if (e2 <= dsqr) { rho[0] = e2; rho[1] = 1.; rho[2] = 0.; }
    else {
        double sqrte = sqrt(e2);
        rho[0] = 2 * sqrte * delta - dsqr;
        rho[1] = delta / sqrte;
        rho[2] = -0.5 * rho[1] / e2;
    }
}

/* Edge order of the sums (tools/oracle_spread.py: the oracle's own spread over legal summation
   orders): 0 the descriptor's order (g2o's insertion order), 1 every edge type walked backwards —
   the chi2 sums and H / b accumulate in the opposite order. */
static int g_edge_rev = 0;
void oracle_set_edge_order(int reversed) { g_edge_rev = reversed ? 1 : 0; }
#define EDGE_IDX(i, n) (g_edge_rev ? (n) - 1 - (i) : (i))

/* SparseOptimizer::activeRobustChi2 (computeActiveErrors + chi2 + robustify) */
static double active_robust_chi2(const problem *pb, const state *s) {
    const deftri_problem_desc *d = pb->d;
    double chi = 0.0, rho[3];
    for (int i = 0; i < d->n_rep; i++) {
        const int e = EDGE_IDX(i, d->n_rep);
        double err[2];
        rep_error(pb, s, e, err);
        double om = d->rep_info[e];
        double c2 = err[0] * (om * err[0]) + err[1] * (om * err[1]);
        if (d->huber_delta > 0) { huber(d->huber_delta, c2, rho); chi += rho[0]; }
        else chi += c2;
    }
    for (int i = 0; i < d->n_depth; i++) {
        const int e = EDGE_IDX(i, d->n_depth);
        double err = depth_error_v(pb, e, s->points + 3 * (size_t)d->dep_point[e], s->scales[d->dep_scale[e]]);
        chi += err * (d->dep_info[e] * err);
    }
    for (int i = 0; i < d->n_arap; i++) {
        const int e = EDGE_IDX(i, d->n_arap);
        double err = arap_error(pb, s, e);
        chi += err * (d->pair_info[d->arap_pair[e]] * err);
    }
    return chi;
}

/* ------------------------------------------------------------------------------------ */
/* block-sparse H (vertex blocks) + b                                                      */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int64_t nv;
    int64_t *rowptr;    /* [nv+1] */
    int64_t *col;       /* vertex neighbours (sorted, incl. self) */
    int64_t *valoff;    /* offset of the dim_a x dim_b block (row-major) */
    double *val;
    int64_t nval;
    double *b;          /* [ndof] */
} bsr;

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* vertex adjacency of all edges */
static void bsr_build(const problem *pb, bsr *H) {
    const deftri_problem_desc *d = pb->d;
    int64_t nv = pb->nv;
    /* collect pairs (a,b) both directions, plus self */
    int64_t cap = nv + 2 * (int64_t)d->n_depth + 2 * 20 * (int64_t)d->n_arap + 16;
    int64_t *pa = (int64_t *)malloc(sizeof(int64_t) * 2 * cap), n = 0;
#define ADDP(a_, b_) do { pa[2 * n] = (a_); pa[2 * n + 1] = (b_); n++; } while (0)
    for (int64_t v = 0; v < nv; v++) ADDP(v, v);
    for (int e = 0; e < d->n_depth; e++) {
        int64_t a = vid_point(pb, d->dep_point[e]), b = vid_scale(pb, d->dep_scale[e]);
        ADDP(a, b); ADDP(b, a);
    }
    for (int e = 0; e < d->n_arap; e++) {
        int64_t v[5];
        for (int k = 0; k < 4; k++) v[k] = vid_point(pb, d->arap_pts[4 * (size_t)e + k]);
        v[4] = vid_tg(pb, d->arap_pair[e]);
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 5; j++)
                if (i != j) ADDP(v[i], v[j]);
    }
#undef ADDP
    /* sort pairs lexicographically via key */
    int64_t *key = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t i = 0; i < n; i++) key[i] = pa[2 * i] * nv + pa[2 * i + 1];
    qsort(key, (size_t)n, sizeof(int64_t), cmp_i64);
    int64_t m = 0;
    for (int64_t i = 0; i < n; i++)
        if (i == 0 || key[i] != key[i - 1]) key[m++] = key[i];
    H->nv = nv;
    H->rowptr = (int64_t *)calloc((size_t)nv + 1, sizeof(int64_t));
    H->col = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
    H->valoff = (int64_t *)malloc(sizeof(int64_t) * (size_t)m);
    int64_t off = 0;
    for (int64_t i = 0; i < m; i++) {
        int64_t a = key[i] / nv, b = key[i] % nv;
        H->rowptr[a + 1]++;
        H->col[i] = b;
        H->valoff[i] = off;
        off += (int64_t)pb->vdim[a] * pb->vdim[b];
    }
    for (int64_t v = 0; v < nv; v++) H->rowptr[v + 1] += H->rowptr[v];
    H->nval = off;
    H->val = (double *)calloc((size_t)off, sizeof(double));
    H->b = (double *)calloc((size_t)pb->ndof, sizeof(double));
    free(key);
    free(pa);
}

static void bsr_free(bsr *H) { free(H->rowptr); free(H->col); free(H->valoff); free(H->val); free(H->b); }

static double *bsr_block(bsr *H, int64_t a, int64_t b) {
    int64_t lo = H->rowptr[a], hi = H->rowptr[a + 1] - 1;
    while (lo <= hi) {
        int64_t mid = (lo + hi) / 2;
        if (H->col[mid] == b) return H->val + H->valoff[mid];
        if (H->col[mid] < b) lo = mid + 1; else hi = mid - 1;
    }
    return NULL;
}

/* add J_a^T W J_b into block (a,b) and, for a != b, its transpose into (b,a) */
static void add_block(bsr *H, const problem *pb, int64_t a, int64_t b, const double *Ja, int da,
                      const double *Jb, int db, int m, const double *W /* m x m */) {
    double *blk = bsr_block(H, a, b);
    double tmp[6 * 6];
    for (int i = 0; i < da; i++)
        for (int j = 0; j < db; j++) {
            double s = 0;
            for (int r = 0; r < m; r++)
                for (int c = 0; c < m; c++) s += Ja[r * da + i] * W[r * m + c] * Jb[c * db + j];
            tmp[i * db + j] = s;
        }
    for (int i = 0; i < da * db; i++) blk[i] += tmp[i];
    if (a != b) {
        double *bt = bsr_block(H, b, a);
        for (int i = 0; i < da; i++)
            for (int j = 0; j < db; j++) bt[j * da + i] += tmp[i * db + j];
    }
    (void)pb;
}

static void add_b(bsr *H, const problem *pb, int64_t a, const double *Ja, int da, int m, const double *wr) {
    double *bb = H->b + pb->voff[a];
    for (int i = 0; i < da; i++) {
        double s = 0;
        for (int r = 0; r < m; r++) s += Ja[r * da + i] * wr[r];
        bb[i] += s;
    }
}

/* analytic ARAP Jacobian (1x18: p1i p2i p1j p2j T(omega, upsilon)); derivation in DESIGN.md */
static void arap_jac_analytic(const problem *pb, const state *s, int e, double J[18]) {
    const deftri_problem_desc *d = pb->d;
    const int32_t *v = d->arap_pts + 4 * (size_t)e;
    const double *p1i = s->points + 3 * (size_t)v[0], *p2i = s->points + 3 * (size_t)v[1];
    const double *p1j = s->points + 3 * (size_t)v[2], *p2j = s->points + 3 * (size_t)v[3];
    const se3q *T = &s->tg[d->arap_pair[e]];
    double Rg[9];
    q_to_mat(&T->r, Rg);
    const double *Ri = d->rot + 9 * (size_t)d->arap_rot[2 * e];
    const double *Rj = d->rot + 9 * (size_t)d->arap_rot[2 * e + 1];
    double area = d->pair_area[d->arap_pair[e]], w = d->arap_w[e];
    double d1[3], d2[3], a[3], c[3], g[3], u[3], s2[3];
    for (int k = 0; k < 3; k++) { d1[k] = p1i[k] - p1j[k]; d2[k] = p2i[k] - p2j[k]; s2[k] = p2i[k] + p2j[k]; }
    for (int k = 0; k < 3; k++) {
        a[k] = d2[k] - (Ri[3 * k] * d1[0] + Ri[3 * k + 1] * d1[1] + Ri[3 * k + 2] * d1[2]);
        c[k] = d2[k] - (Rj[3 * k] * d1[0] + Rj[3 * k + 1] * d1[1] + Rj[3 * k + 2] * d1[2]);
        double rs = Rg[3 * k] * s2[0] + Rg[3 * k + 1] * s2[1] + Rg[3 * k + 2] * s2[2];
        u[k] = rs - 2 * T->t[k];
        g[k] = u[k] - (p1i[k] + p1j[k]);
    }
    double co = 2.0 * w / (area * area);
    double qv[3], rv[3], rg[3];
    for (int k = 0; k < 3; k++) {
        qv[k] = co * (a[k] + c[k]);
        rv[k] = co * ((Ri[k] * a[0] + Ri[3 + k] * a[1] + Ri[6 + k] * a[2]) +
                      (Rj[k] * c[0] + Rj[3 + k] * c[1] + Rj[6 + k] * c[2]));
        rg[k] = 2.0 * (Rg[k] * g[0] + Rg[3 + k] * g[1] + Rg[6 + k] * g[2]);
    }
    for (int k = 0; k < 3; k++) {
        J[0 + k] = -rv[k] - 2.0 * g[k];
        J[3 + k] = qv[k] + rg[k];
        J[6 + k] = rv[k] - 2.0 * g[k];
        J[9 + k] = -qv[k] + rg[k];
    }
    J[12] = 2.0 * (u[1] * g[2] - u[2] * g[1]);
    J[13] = 2.0 * (u[2] * g[0] - u[0] * g[2]);
    J[14] = 2.0 * (u[0] * g[1] - u[1] * g[0]);
    J[15] = -4.0 * g[0]; J[16] = -4.0 * g[1]; J[17] = -4.0 * g[2];
}

/* BaseMultiEdge::linearizeOplus numeric (delta 1e-9, push/oplus/computeError/pop) */
static void arap_jac_numeric(const problem *pb, const state *s, int e, double J[18]) {
    const deftri_problem_desc *d = pb->d;
    const int32_t *v = d->arap_pts + 4 * (size_t)e;
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    double pts[4][3];
    for (int k = 0; k < 4; k++) memcpy(pts[k], s->points + 3 * (size_t)v[k], sizeof(pts[k]));
    se3q T = s->tg[d->arap_pair[e]];
    for (int vi = 0; vi < 4; vi++) {
        for (int dd = 0; dd < 3; dd++) {
            double bak = pts[vi][dd];
            pts[vi][dd] = bak + delta;
            double ep = arap_error_v(pb, e, pts[0], pts[1], pts[2], pts[3], &T);
            pts[vi][dd] = bak;
            pts[vi][dd] = bak + (-delta);
            double em = arap_error_v(pb, e, pts[0], pts[1], pts[2], pts[3], &T);
            pts[vi][dd] = bak;
            J[3 * vi + dd] = scalar * (ep - em);
        }
    }
    for (int dd = 0; dd < 6; dd++) {
        double u[6] = {0, 0, 0, 0, 0, 0};
        se3q Tp = T, Tm = T;
        u[dd] = delta;
        se3_oplus(&Tp, u);
        double ep = arap_error_v(pb, e, pts[0], pts[1], pts[2], pts[3], &Tp);
        u[dd] = -delta;
        se3_oplus(&Tm, u);
        double em = arap_error_v(pb, e, pts[0], pts[1], pts[2], pts[3], &Tm);
        J[12 + dd] = scalar * (ep - em);
    }
}

/* BaseBinaryEdge::linearizeOplus numeric for EdgeDepthCorrection: [dp(3) ds(1)] */
static void depth_jac_numeric(const problem *pb, const state *s, int e, double J[4]) {
    const deftri_problem_desc *d = pb->d;
    const double delta = 1e-9, scalar = 1.0 / (2 * delta);
    double p[3];
    memcpy(p, s->points + 3 * (size_t)d->dep_point[e], sizeof(p));
    double sc = s->scales[d->dep_scale[e]];
    for (int dd = 0; dd < 3; dd++) {
        double bak = p[dd];
        p[dd] = bak + delta;
        double ep = depth_error_v(pb, e, p, sc);
        p[dd] = bak + (-delta);
        double em = depth_error_v(pb, e, p, sc);
        p[dd] = bak;
        J[dd] = scalar * (ep - em);
    }
    double ep = depth_error_v(pb, e, p, sc + delta);
    double em = depth_error_v(pb, e, p, sc + (-delta));
    J[3] = scalar * (ep - em);
}

static void depth_jac_analytic(const problem *pb, const state *s, int e, double J[4]) {
    const deftri_problem_desc *d = pb->d;
    const double *p = s->points + 3 * (size_t)d->dep_point[e];
    double sc = s->scales[d->dep_scale[e]], pc[3];
    int c = d->dep_cam[e];
    se3_map(&pb->cams[c], p, pc);
    double r = d->dep_meas[e] / sc - pc[2];
    double f = (sc <= 0.0) ? 500.0 : 1.0;
    const double *R = pb->camR + 9 * c;
    for (int k = 0; k < 3; k++) J[k] = f * 2.0 * r * (-R[6 + k]);
    J[3] = f * 2.0 * r * (-d->dep_meas[e] / (sc * sc));
}

/* BlockSolver::buildSystem: linearizeOplus + constructQuadraticForm of every edge */
static void build_system(const problem *pb, const state *s, bsr *H, int analytic) {
    const deftri_problem_desc *d = pb->d;
    memset(H->val, 0, sizeof(double) * (size_t)H->nval);
    memset(H->b, 0, sizeof(double) * (size_t)pb->ndof);
    for (int i = 0; i < d->n_rep; i++) {
        const int e = EDGE_IDX(i, d->n_rep);
        double err[2];
        rep_error(pb, s, e, err);
        const double *p = s->points + 3 * (size_t)d->rep_point[e];
        int c = d->rep_cam[e];
        double pc[3];
        se3_map(&pb->cams[c], p, pc);
        float pf[3] = {(float)pc[0], (float)pc[1], (float)pc[2]}, jf[6];
        kb8_project_jac(d->cam_kb8 + 8 * c, pf, jf);
        const double *R = pb->camR + 9 * c;
        double J[6];
        for (int r = 0; r < 2; r++)
            for (int k = 0; k < 3; k++)
                J[3 * r + k] = -(double)jf[3 * r] * R[k] - (double)jf[3 * r + 1] * R[3 + k] - (double)jf[3 * r + 2] * R[6 + k];
        double om = d->rep_info[e];
        double c2 = err[0] * (om * err[0]) + err[1] * (om * err[1]);
        double w = 1.0;
        if (d->huber_delta > 0) { double rho[3]; huber(d->huber_delta, c2, rho); w = rho[1]; }
        double W[4] = {w * om, 0, 0, w * om};
        double wr[2] = {-(w * om * err[0]), -(w * om * err[1])};
        int64_t a = vid_point(pb, d->rep_point[e]);
        add_block(H, pb, a, a, J, 3, J, 3, 2, W);
        add_b(H, pb, a, J, 3, 2, wr);
    }
    for (int i = 0; i < d->n_depth; i++) {
        const int e = EDGE_IDX(i, d->n_depth);
        double J[4];
        if (analytic) depth_jac_analytic(pb, s, e, J); else depth_jac_numeric(pb, s, e, J);
        double err = depth_error_v(pb, e, s->points + 3 * (size_t)d->dep_point[e], s->scales[d->dep_scale[e]]);
        double om = d->dep_info[e];
        double W[1] = {om}, wr[1] = {-(om * err)};
        int64_t a = vid_point(pb, d->dep_point[e]), b = vid_scale(pb, d->dep_scale[e]);
        add_block(H, pb, a, a, J, 3, J, 3, 1, W);
        add_block(H, pb, b, b, J + 3, 1, J + 3, 1, 1, W);
        add_block(H, pb, a, b, J, 3, J + 3, 1, 1, W);
        add_b(H, pb, a, J, 3, 1, wr);
        add_b(H, pb, b, J + 3, 1, 1, wr);
    }
    for (int i = 0; i < d->n_arap; i++) {
        const int e = EDGE_IDX(i, d->n_arap);
        double J[18];
        if (analytic) arap_jac_analytic(pb, s, e, J); else arap_jac_numeric(pb, s, e, J);
        double err = arap_error(pb, s, e);
        double om = d->pair_info[d->arap_pair[e]];
        double W[1] = {om}, wr[1] = {-(om * err)};
        int64_t v[5];
        const double *Jv[5];
        int dim[5] = {3, 3, 3, 3, 6};
        for (int k = 0; k < 4; k++) { v[k] = vid_point(pb, d->arap_pts[4 * (size_t)e + k]); Jv[k] = J + 3 * k; }
        v[4] = vid_tg(pb, d->arap_pair[e]); Jv[4] = J + 12;
        for (int i = 0; i < 5; i++) {
            add_block(H, pb, v[i], v[i], Jv[i], dim[i], Jv[i], dim[i], 1, W);
            add_b(H, pb, v[i], Jv[i], dim[i], 1, wr);
            for (int j = i + 1; j < 5; j++) add_block(H, pb, v[i], v[j], Jv[i], dim[i], Jv[j], dim[j], 1, W);
        }
    }
}

/* ------------------------------------------------------------------------------------ */
/* fill-reducing ordering: geometric nested dissection on point vertices, globals last    */
/* ------------------------------------------------------------------------------------ */
typedef struct { const double *xy; int64_t *nodes; } nd_ctx;
static const double *g_sort_xy; static int g_sort_axis;
static int cmp_axis(const void *a, const void *b) {
    double x = g_sort_xy[2 * *(const int64_t *)a + g_sort_axis];
    double y = g_sort_xy[2 * *(const int64_t *)b + g_sort_axis];
    if (x < y) return -1;
    if (x > y) return 1;
    int64_t i = *(const int64_t *)a, j = *(const int64_t *)b;
    return (i > j) - (i < j);
}

static void nd_rec(const bsr *H, const problem *pb, const double *xy, int64_t *nodes, int64_t n,
                   int64_t *out, int64_t *nout, int *side, int depth) {
    if (n <= 64 || depth > 60) {
        for (int64_t i = 0; i < n; i++) out[(*nout)++] = nodes[i];
        return;
    }
    double mn[2] = {1e300, 1e300}, mx[2] = {-1e300, -1e300};
    for (int64_t i = 0; i < n; i++)
        for (int k = 0; k < 2; k++) {
            double v = xy[2 * nodes[i] + k];
            if (v < mn[k]) mn[k] = v;
            if (v > mx[k]) mx[k] = v;
        }
    g_sort_xy = xy; g_sort_axis = (mx[0] - mn[0] >= mx[1] - mn[1]) ? 0 : 1;
    qsort(nodes, (size_t)n, sizeof(int64_t), cmp_axis);
    int64_t half = n / 2;
    /* side: 1 = left, 2 = right; separator = left nodes adjacent to a right node */
    for (int64_t i = 0; i < n; i++) side[nodes[i]] = (i < half) ? 1 : 2;
    int64_t nl = 0, nr = 0, ns = 0;
    int64_t *tmp = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t i = 0; i < half; i++) {
        int64_t v = pb->d->n_pairs + pb->d->n_scales + nodes[i];
        int sep = 0;
        for (int64_t k = H->rowptr[v]; k < H->rowptr[v + 1]; k++) {
            int64_t u = H->col[k] - pb->d->n_pairs - pb->d->n_scales;
            if (u >= 0 && side[u] == 2) { sep = 1; break; }
        }
        if (sep) side[nodes[i]] = 3;
    }
    for (int64_t i = 0; i < n; i++) if (side[nodes[i]] == 1) tmp[nl++] = nodes[i];
    for (int64_t i = 0; i < n; i++) if (side[nodes[i]] == 2) tmp[nl + nr++] = nodes[i];
    for (int64_t i = 0; i < n; i++) if (side[nodes[i]] == 3) tmp[nl + nr + ns++] = nodes[i];
    memcpy(nodes, tmp, sizeof(int64_t) * (size_t)n);
    free(tmp);
    for (int64_t i = 0; i < n; i++) side[nodes[i]] = 0;
    nd_rec(H, pb, xy, nodes, nl, out, nout, side, depth + 1);
    nd_rec(H, pb, xy, nodes + nl, nr, out, nout, side, depth + 1);
    for (int64_t i = 0; i < ns; i++) out[(*nout)++] = nodes[nl + nr + i];
}

/* An externally supplied elimination order (bench.py's CPU baseline: the device plan's nested
   dissection, so the oracle's SimplicialLDLT runs the same fill and flop count as the device). */
static int64_t *g_vorder = NULL, g_vorder_n = 0;
void oracle_set_vertex_order(const int64_t *order, int64_t nv) {
    free(g_vorder); g_vorder = NULL; g_vorder_n = 0;
    if (!order || nv <= 0) return;
    g_vorder = (int64_t *)malloc(sizeof(int64_t) * (size_t)nv);
    memcpy(g_vorder, order, sizeof(int64_t) * (size_t)nv);
    g_vorder_n = nv;
}

/* returns vertex permutation perm[k] = vertex eliminated k-th */
static int64_t *nd_order(const bsr *H, const problem *pb) {
    const deftri_problem_desc *d = pb->d;
    int64_t P = d->n_points, nv = pb->nv;
    if (g_vorder && g_vorder_n == nv) {
        int64_t *o = (int64_t *)malloc(sizeof(int64_t) * (size_t)nv);
        memcpy(o, g_vorder, sizeof(int64_t) * (size_t)nv);
        return o;
    }
    double *xy = (double *)malloc(sizeof(double) * 2 * (size_t)(P > 0 ? P : 1));
    for (int64_t p = 0; p < P; p++) {
        if (d->order_xy) { xy[2 * p] = d->order_xy[2 * p]; xy[2 * p + 1] = d->order_xy[2 * p + 1]; }
        else { xy[2 * p] = d->points[3 * p]; xy[2 * p + 1] = d->points[3 * p + 1]; }
    }
    int64_t *nodes = (int64_t *)malloc(sizeof(int64_t) * (size_t)(P > 0 ? P : 1));
    int64_t *out = (int64_t *)malloc(sizeof(int64_t) * (size_t)nv);
    int *side = (int *)calloc((size_t)(P > 0 ? P : 1), sizeof(int));
    for (int64_t p = 0; p < P; p++) nodes[p] = p;
    int64_t nout = 0;
    int64_t *pts = (int64_t *)malloc(sizeof(int64_t) * (size_t)(P > 0 ? P : 1));
    nd_rec(H, pb, xy, nodes, P, pts, &nout, side, 0);
    int64_t k = 0;
    for (int64_t i = 0; i < nout; i++) out[k++] = d->n_pairs + d->n_scales + pts[i];
    for (int64_t v = 0; v < d->n_pairs + d->n_scales; v++) out[k++] = v;   /* globals last */
    free(xy); free(nodes); free(side); free(pts);
    return out;
}

/* ------------------------------------------------------------------------------------ */
/* sparse LDL^T (up-looking, SimplicialLDLT semantics)                                    */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    int64_t n;
    int64_t *perm;      /* scalar dof eliminated k-th  */
    int64_t *pinv;
    /* upper triangle of permuted A in CSC: column k holds rows i <= k */
    int64_t *Ap, *Ai;
    double *Ax;
    int64_t *diagpos;   /* position of A(k,k) */
    int64_t *srcpos;    /* for each Ax entry: index into H->val (scalar) */
    /* factor */
    int64_t *Lp, *Parent, *Lnz, *Li, *Flag, *Pattern;
    double *Lx, *D, *Y;
    int64_t lnz;
} ldl;

static int64_t g_cmp_base;
static int cmp_pair_row(const void *a, const void *b) {
    int64_t x = ((const int64_t *)a)[0], y = ((const int64_t *)b)[0];
    return (x > y) - (x < y);
}

static void ldl_analyse(ldl *L, const problem *pb, const bsr *H, const int64_t *vperm) {
    int64_t n = pb->ndof, nv = pb->nv;
    L->n = n;
    L->perm = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    L->pinv = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    int64_t k = 0;
    for (int64_t i = 0; i < nv; i++) {
        int64_t v = vperm[i];
        for (int dd = 0; dd < pb->vdim[v]; dd++) L->perm[k++] = pb->voff[v] + dd;
    }
    for (int64_t i = 0; i < n; i++) L->pinv[L->perm[i]] = i;
    /* count entries of the upper triangle of P A P^T per column */
    int64_t *cnt = (int64_t *)calloc((size_t)n + 1, sizeof(int64_t));
    for (int64_t a = 0; a < nv; a++)
        for (int64_t q = H->rowptr[a]; q < H->rowptr[a + 1]; q++) {
            int64_t b = H->col[q];
            for (int i = 0; i < pb->vdim[a]; i++)
                for (int j = 0; j < pb->vdim[b]; j++) {
                    int64_t r = L->pinv[pb->voff[a] + i], c = L->pinv[pb->voff[b] + j];
                    if (r <= c) cnt[c + 1]++;
                }
        }
    L->Ap = (int64_t *)malloc(sizeof(int64_t) * ((size_t)n + 1));
    L->Ap[0] = 0;
    for (int64_t c = 0; c < n; c++) L->Ap[c + 1] = L->Ap[c] + cnt[c + 1];
    int64_t nnz = L->Ap[n];
    L->Ai = (int64_t *)malloc(sizeof(int64_t) * (size_t)nnz);
    L->Ax = (double *)malloc(sizeof(double) * (size_t)nnz);
    L->srcpos = (int64_t *)malloc(sizeof(int64_t) * (size_t)nnz);
    int64_t *fill = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t c = 0; c < n; c++) fill[c] = L->Ap[c];
    for (int64_t a = 0; a < nv; a++)
        for (int64_t q = H->rowptr[a]; q < H->rowptr[a + 1]; q++) {
            int64_t b = H->col[q];
            for (int i = 0; i < pb->vdim[a]; i++)
                for (int j = 0; j < pb->vdim[b]; j++) {
                    int64_t r = L->pinv[pb->voff[a] + i], c = L->pinv[pb->voff[b] + j];
                    if (r <= c) {
                        int64_t pos = fill[c]++;
                        L->Ai[pos] = r;
                        L->srcpos[pos] = H->valoff[q] + (int64_t)i * pb->vdim[b] + j;
                    }
                }
        }
    /* sort rows within each column (pairs row,src) */
    int64_t *buf = NULL; size_t bufcap = 0;
    for (int64_t c = 0; c < n; c++) {
        int64_t m = L->Ap[c + 1] - L->Ap[c];
        if ((size_t)m > bufcap) { bufcap = (size_t)m * 2; buf = (int64_t *)realloc(buf, sizeof(int64_t) * 2 * bufcap); }
        for (int64_t t = 0; t < m; t++) { buf[2 * t] = L->Ai[L->Ap[c] + t]; buf[2 * t + 1] = L->srcpos[L->Ap[c] + t]; }
        qsort(buf, (size_t)m, 2 * sizeof(int64_t), cmp_pair_row);
        for (int64_t t = 0; t < m; t++) { L->Ai[L->Ap[c] + t] = buf[2 * t]; L->srcpos[L->Ap[c] + t] = buf[2 * t + 1]; }
    }
    free(buf);
    L->diagpos = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    for (int64_t c = 0; c < n; c++) L->diagpos[c] = L->Ap[c + 1] - 1;   /* last row = c */
    free(fill); free(cnt);
    (void)g_cmp_base;
    /* symbolic (elimination tree + column counts) */
    L->Lp = (int64_t *)malloc(sizeof(int64_t) * ((size_t)n + 1));
    L->Parent = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    L->Lnz = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    L->Flag = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    L->Pattern = (int64_t *)malloc(sizeof(int64_t) * (size_t)n);
    L->D = (double *)malloc(sizeof(double) * (size_t)n);
    L->Y = (double *)malloc(sizeof(double) * (size_t)n);
    for (int64_t kk = 0; kk < n; kk++) {
        L->Parent[kk] = -1; L->Flag[kk] = kk; L->Lnz[kk] = 0;
        for (int64_t p = L->Ap[kk]; p < L->Ap[kk + 1]; p++) {
            int64_t i = L->Ai[p];
            if (i < kk) {
                for (; L->Flag[i] != kk; i = L->Parent[i]) {
                    if (L->Parent[i] == -1) L->Parent[i] = kk;
                    L->Lnz[i]++;
                    L->Flag[i] = kk;
                }
            }
        }
    }
    L->Lp[0] = 0;
    for (int64_t kk = 0; kk < n; kk++) L->Lp[kk + 1] = L->Lp[kk] + L->Lnz[kk];
    L->lnz = L->Lp[n];
    L->Li = (int64_t *)malloc(sizeof(int64_t) * (size_t)(L->lnz ? L->lnz : 1));
    L->Lx = (double *)malloc(sizeof(double) * (size_t)(L->lnz ? L->lnz : 1));
}

static void ldl_free(ldl *L) {
    free(L->perm); free(L->pinv); free(L->Ap); free(L->Ai); free(L->Ax); free(L->diagpos); free(L->srcpos);
    free(L->Lp); free(L->Parent); free(L->Lnz); free(L->Li); free(L->Flag); free(L->Pattern);
    free(L->Lx); free(L->D); free(L->Y);
}

/* numeric factorization of P (H + lambda I) P^T; returns 1 on success (no zero pivot) */
static int ldl_factor(ldl *L, const bsr *H, double lambda) {
    int64_t n = L->n;
    for (int64_t p = 0; p < L->Ap[n]; p++) L->Ax[p] = H->val[L->srcpos[p]];
    for (int64_t c = 0; c < n; c++) L->Ax[L->diagpos[c]] += lambda;
    for (int64_t k = 0; k < n; k++) {
        L->Y[k] = 0.0;
        int64_t top = n;
        L->Flag[k] = k;
        L->Lnz[k] = 0;
        for (int64_t p = L->Ap[k]; p < L->Ap[k + 1]; p++) {
            int64_t i = L->Ai[p];
            if (i <= k) {
                L->Y[i] += L->Ax[p];
                int64_t len = 0;
                for (; L->Flag[i] != k; i = L->Parent[i]) {
                    L->Pattern[len++] = i;
                    L->Flag[i] = k;
                }
                while (len > 0) L->Pattern[--top] = L->Pattern[--len];
            }
        }
        L->D[k] = L->Y[k];
        L->Y[k] = 0.0;
        for (; top < n; top++) {
            int64_t i = L->Pattern[top];
            double yi = L->Y[i];
            L->Y[i] = 0.0;
            int64_t p2 = L->Lp[i] + L->Lnz[i], p;
            for (p = L->Lp[i]; p < p2; p++) L->Y[L->Li[p]] -= L->Lx[p] * yi;
            double l_ki = yi / L->D[i];
            L->D[k] -= l_ki * yi;
            L->Li[p] = k;
            L->Lx[p] = l_ki;
            L->Lnz[i]++;
        }
        if (L->D[k] == 0.0) return 0;
    }
    return 1;
}

/* x = (P^T L D L^T P)^{-1} b */
static void ldl_solve(const ldl *L, const double *b, double *x) {
    int64_t n = L->n;
    double *y = (double *)malloc(sizeof(double) * (size_t)n);
    for (int64_t k = 0; k < n; k++) y[k] = b[L->perm[k]];
    for (int64_t j = 0; j < n; j++)
        for (int64_t p = L->Lp[j]; p < L->Lp[j + 1]; p++) y[L->Li[p]] -= L->Lx[p] * y[j];
    for (int64_t j = 0; j < n; j++) y[j] /= L->D[j];
    for (int64_t j = n - 1; j >= 0; j--)
        for (int64_t p = L->Lp[j]; p < L->Lp[j + 1]; p++) y[j] -= L->Lx[p] * y[L->Li[p]];
    for (int64_t k = 0; k < n; k++) x[L->perm[k]] = y[k];
    free(y);
}

/* ------------------------------------------------------------------------------------ */
/* problem setup + LM                                                                      */
/* ------------------------------------------------------------------------------------ */
static void problem_init(problem *pb, const deftri_problem_desc *d) {
    pb->d = d;
    pb->cams = (se3q *)malloc(sizeof(se3q) * (size_t)(d->n_cams ? d->n_cams : 1));
    pb->camR = (double *)malloc(sizeof(double) * 9 * (size_t)(d->n_cams ? d->n_cams : 1));
    for (int c = 0; c < d->n_cams; c++) {
        pb->cams[c] = se3_from7(d->cam_pose + 7 * c);
        q_to_mat(&pb->cams[c].r, pb->camR + 9 * c);
    }
    pb->nv = (int64_t)d->n_pairs + d->n_scales + d->n_points;
    pb->voff = (int64_t *)malloc(sizeof(int64_t) * (size_t)pb->nv);
    pb->vdim = (int *)malloc(sizeof(int) * (size_t)pb->nv);
    int64_t off = 0;
    for (int64_t v = 0; v < pb->nv; v++) {
        int dim = v < d->n_pairs ? 6 : (v < d->n_pairs + d->n_scales ? 1 : 3);
        pb->vdim[v] = dim; pb->voff[v] = off; off += dim;
    }
    pb->ndof = off;
}
static void problem_free(problem *pb) { free(pb->cams); free(pb->camR); free(pb->voff); free(pb->vdim); }

static void state_from_desc(const problem *pb, state *s) {
    const deftri_problem_desc *d = pb->d;
    memcpy(s->points, d->points, sizeof(double) * 3 * (size_t)d->n_points);
    memcpy(s->scales, d->scales, sizeof(double) * (size_t)d->n_scales);
    for (int q = 0; q < d->n_pairs; q++) s->tg[q] = se3_from7(d->tg + 7 * q);
}

/* OptimizableGraph::update via each vertex's oplusImpl */
static void state_update(const problem *pb, state *s, const double *dx) {
    const deftri_problem_desc *d = pb->d;
    for (int q = 0; q < d->n_pairs; q++) se3_oplus(&s->tg[q], dx + pb->voff[vid_tg(pb, q)]);
    for (int k = 0; k < d->n_scales; k++) s->scales[k] += dx[pb->voff[vid_scale(pb, k)]];
    for (int p = 0; p < d->n_points; p++) {
        const double *u = dx + pb->voff[vid_point(pb, p)];
        s->points[3 * p] += u[0]; s->points[3 * p + 1] += u[1]; s->points[3 * p + 2] += u[2];
    }
}

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

/* -------------------------------- exported API ------------------------------------------- */

int oracle_num_unknowns(const deftri_problem_desc *d, int64_t *n) {
    *n = 6 * (int64_t)d->n_pairs + d->n_scales + 3 * (int64_t)d->n_points;
    return 0;
}

/* chi2 at an explicit state (points/scales/tg may be NULL = the descriptor's initial state) */
int oracle_chi2(const deftri_problem_desc *d, const double *points, const double *scales,
                const double *tg, double *chi2) {
    problem pb; state s;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_from_desc(&pb, &s);
    if (points) memcpy(s.points, points, sizeof(double) * 3 * (size_t)d->n_points);
    if (scales) memcpy(s.scales, scales, sizeof(double) * (size_t)d->n_scales);
    if (tg) for (int q = 0; q < d->n_pairs; q++) s.tg[q] = se3_from7(tg + 7 * q);
    *chi2 = active_robust_chi2(&pb, &s);
    state_free(&s); problem_free(&pb);
    return 0;
}

/* per-edge errors at the initial state: rep [R*2], depth [D], arap [E] (any may be NULL) */
int oracle_edge_errors(const deftri_problem_desc *d, double *rep, double *dep, double *arap) {
    problem pb; state s;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_from_desc(&pb, &s);
    if (rep) for (int e = 0; e < d->n_rep; e++) rep_error(&pb, &s, e, rep + 2 * e);
    if (dep) for (int e = 0; e < d->n_depth; e++)
        dep[e] = depth_error_v(&pb, e, s.points + 3 * (size_t)d->dep_point[e], s.scales[d->dep_scale[e]]);
    if (arap) for (int e = 0; e < d->n_arap; e++) arap[e] = arap_error(&pb, &s, e);
    state_free(&s); problem_free(&pb);
    return 0;
}

/* ARAP Jacobians [E*18] at the initial state (analytic or numeric) */
int oracle_arap_jacobians(const deftri_problem_desc *d, int analytic, double *J) {
    problem pb; state s;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_from_desc(&pb, &s);
    for (int e = 0; e < d->n_arap; e++) {
        if (analytic) arap_jac_analytic(&pb, &s, e, J + 18 * (size_t)e);
        else arap_jac_numeric(&pb, &s, e, J + 18 * (size_t)e);
    }
    state_free(&s); problem_free(&pb);
    return 0;
}

/* Linearize at the initial state: b [n], and dense H [n*n] if Hdense != NULL (small n only),
   and y = H x if x,y != NULL. */
int oracle_linearize(const deftri_problem_desc *d, int analytic, double *b, double *Hdense,
                     const double *x, double *y) {
    problem pb; state s; bsr H;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_from_desc(&pb, &s);
    bsr_build(&pb, &H);
    build_system(&pb, &s, &H, analytic);
    int64_t n = pb.ndof;
    if (b) memcpy(b, H.b, sizeof(double) * (size_t)n);
    if (Hdense) {
        memset(Hdense, 0, sizeof(double) * (size_t)n * (size_t)n);
        for (int64_t a = 0; a < pb.nv; a++)
            for (int64_t q = H.rowptr[a]; q < H.rowptr[a + 1]; q++) {
                int64_t bb = H.col[q];
                for (int i = 0; i < pb.vdim[a]; i++)
                    for (int j = 0; j < pb.vdim[bb]; j++)
                        Hdense[(pb.voff[a] + i) * n + pb.voff[bb] + j] = H.val[H.valoff[q] + i * pb.vdim[bb] + j];
            }
    }
    if (x && y) {
        memset(y, 0, sizeof(double) * (size_t)n);
        for (int64_t a = 0; a < pb.nv; a++)
            for (int64_t q = H.rowptr[a]; q < H.rowptr[a + 1]; q++) {
                int64_t bb = H.col[q];
                for (int i = 0; i < pb.vdim[a]; i++)
                    for (int j = 0; j < pb.vdim[bb]; j++)
                        y[pb.voff[a] + i] += H.val[H.valoff[q] + i * pb.vdim[bb] + j] * x[pb.voff[bb] + j];
            }
    }
    bsr_free(&H); state_free(&s); problem_free(&pb);
    return 0;
}

/* The assembled H at the initial linearization as COO triplets (every stored block entry; nnz = 0 on
   entry asks for the count only).  Test infrastructure (tests/pcg_evidence.py). */
int oracle_hessian_coo(const deftri_problem_desc *d, int analytic, int64_t *nnz, int64_t *ri, int64_t *ci,
                       double *v) {
    problem pb; state s; bsr H;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_from_desc(&pb, &s);
    bsr_build(&pb, &H);
    build_system(&pb, &s, &H, analytic);
    int64_t k = 0;
    for (int64_t a = 0; a < pb.nv; a++)
        for (int64_t q = H.rowptr[a]; q < H.rowptr[a + 1]; q++) {
            int64_t bb = H.col[q];
            for (int i = 0; i < pb.vdim[a]; i++)
                for (int j = 0; j < pb.vdim[bb]; j++) {
                    if (*nnz > 0 && k < *nnz) {
                        ri[k] = pb.voff[a] + i; ci[k] = pb.voff[bb] + j;
                        v[k] = H.val[H.valoff[q] + i * pb.vdim[bb] + j];
                    }
                    k++;
                }
        }
    *nnz = k;
    bsr_free(&H); state_free(&s); problem_free(&pb);
    return 0;
}

/* Solve (H + lambda I) x = rhs at the initial linearization with the sparse LDL^T. */
int oracle_damped_solve(const deftri_problem_desc *d, int analytic, double lambda, const double *rhs,
                        double *x) {
    problem pb; state s; bsr H; ldl L;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_from_desc(&pb, &s);
    bsr_build(&pb, &H);
    build_system(&pb, &s, &H, analytic);
    int64_t *vperm = nd_order(&H, &pb);
    ldl_analyse(&L, &pb, &H, vperm);
    int ok = ldl_factor(&L, &H, lambda);
    if (ok) ldl_solve(&L, rhs, x);
    free(vperm); ldl_free(&L); bsr_free(&H); state_free(&s); problem_free(&pb);
    return ok ? 0 : DEFTRI_E_NUMERIC;
}

/* g2o SparseOptimizer::optimize(n) with OptimizationAlgorithmLevenberg + BlockSolverX +
   LinearSolverEigen.  Outputs the final state (points [P*3], scales [S], tg [Q*7]). */
int oracle_solve_lm(const deftri_problem_desc *d, const deftri_lm_params *prm, double *points_out,
                    double *scales_out, double *tg_out, deftri_report *rep) {
    double t_start = now_ms();
    problem pb; state s, sbak; bsr H; ldl L;
    problem_init(&pb, d);
    state_alloc(&pb, &s);
    state_alloc(&pb, &sbak);
    state_from_desc(&pb, &s);
    bsr_build(&pb, &H);
    int64_t *vperm = nd_order(&H, &pb);
    ldl_analyse(&L, &pb, &H, vperm);
    free(vperm);
    int64_t n = pb.ndof;
    double *dx = (double *)malloc(sizeof(double) * (size_t)n);
    memset(rep, 0, sizeof(*rep));
    rep->n_unknowns = n;
    rep->nnz_factor = L.lnz;
    int max_trials = prm->max_trials > 0 ? prm->max_trials : 10;
    double tau = prm->tau > 0 ? prm->tau : 1e-5;
    int analytic = prm->analytic_jacobians;
    double lambda = 0, ni = 2;
    double t_lin = 0, t_fac = 0, t_sol = 0, t_upd = 0;
    int status = DEFTRI_STATUS_OK, it;
    rep->chi2_initial = active_robust_chi2(&pb, &s);
    double currentChi = rep->chi2_initial;
    for (it = 0; it < prm->n_iterations; it++) {
        double t0 = now_ms();
        currentChi = active_robust_chi2(&pb, &s);           /* computeActiveErrors */
        build_system(&pb, &s, &H, analytic);
        t_lin += now_ms() - t0;
        if (it == 0) {
            if (prm->user_lambda > 0) lambda = prm->user_lambda;
            else {
                double maxDiag = 0;
                for (int64_t v = 0; v < pb.nv; v++) {
                    const double *blk = bsr_block(&H, v, v);
                    for (int k = 0; k < pb.vdim[v]; k++) {
                        double a = fabs(blk[k * pb.vdim[v] + k]);
                        if (a > maxDiag) maxDiag = a;
                    }
                }
                lambda = tau * maxDiag;
            }
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            state_copy(&pb, &sbak, &s);                        /* push */
            double t1 = now_ms();
            int ok2 = ldl_factor(&L, &H, lambda);
            double t2 = now_ms();
            if (ok2) ldl_solve(&L, H.b, dx); else memset(dx, 0, sizeof(double) * (size_t)n);
            double t3 = now_ms();
            t_fac += t2 - t1; t_sol += t3 - t2;
            state_update(&pb, &s, dx);
            double tempChi = active_robust_chi2(&pb, &s);
            t_upd += now_ms() - t3;
            if (!ok2) tempChi = 1.79769313486231570815e+308;
            rho = (currentChi - tempChi);
            double scale = 0;
            for (int64_t j = 0; j < n; j++) scale += dx[j] * (lambda * dx[j] + H.b[j]);
            scale += 1e-3;
            rho /= scale;
            rep->trials_total++;
            if (rho > 0 && isfinite(tempChi)) {
                double alpha = 1. - pow((2 * rho - 1), 3);
                alpha = alpha < (2. / 3.) ? alpha : (2. / 3.);
                double scaleFactor = (1. / 3.) > alpha ? (1. / 3.) : alpha;
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                state_copy(&pb, &s, &sbak);                    /* pop */
                rep->trials_rejected++;
            }
            qmax++;
        } while (rho < 0 && qmax < max_trials);
        if (it < DEFTRI_MAX_REPORT_ITERS) { rep->chi2_iter[it] = currentChi; rep->trials_iter[it] = qmax; }
        if (prm->verbose)
            fprintf(stderr, "[oracle] it %d chi2 %.9e lambda %.6e trials %d\n", it, currentChi, lambda, qmax);
        if (qmax == max_trials || rho == 0 || !isfinite(lambda)) { status = DEFTRI_STATUS_TERMINATE; it++; break; }
    }
    rep->status = status;
    rep->iterations = it;
    rep->chi2_final = active_robust_chi2(&pb, &s);
    rep->lambda_final = lambda;
    rep->ms_linearize = t_lin; rep->ms_factor = t_fac; rep->ms_solve = t_sol; rep->ms_update = t_upd;
    rep->ms_total = now_ms() - t_start;
    if (points_out) memcpy(points_out, s.points, sizeof(double) * 3 * (size_t)d->n_points);
    if (scales_out) memcpy(scales_out, s.scales, sizeof(double) * (size_t)d->n_scales);
    if (tg_out) for (int q = 0; q < d->n_pairs; q++) se3_to7(&s.tg[q], tg_out + 7 * q);
    free(dx); ldl_free(&L); bsr_free(&H); state_free(&s); state_free(&sbak); problem_free(&pb);
    return 0;
}

/* KB8 helpers exported for formula cross-checks */
void oracle_kb8_project(const float *k, const float *p, float *uv) { kb8_project(k, p, uv); }
void oracle_kb8_project_jac(const float *k, const float *p, float *J) { kb8_project_jac(k, p, J); }
void oracle_se3_exp(const double *u, double *out7) { se3q T = se3_exp(u); se3_to7(&T, out7); }
