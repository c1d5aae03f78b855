/*
 * ba_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker for the bundle-adjustment path).
 *
 * Only tests/ and __graft_entry__.smoke() may load this library (built into oracle/liboracle.so
 * together with deftri_oracle.c, whose SE3Quat / quaternion / KB8 / Huber helpers it reuses by
 * inclusion: one translation unit).  The product never links or calls it.
 *
 * A plain-C restatement of what the reference's BA entry points run in g2o
 * (Modules/Optimization/g2oBundleAdjustment.cc:38-138 bundleAdjustment, :140-243
 * poseOnlyOptimization, :245-444 localBundleAdjustment):
 *   - EdgeSE3ProjectXYZ::computeError / isDepthPositive   g2oTypes.h:165-189
 *   - EdgeSE3ProjectXYZ::linearizeOplus                   g2oTypes.cc:121-142
 *   - EdgeSE3ProjectXYZOnlyPose (points fixed)            g2oTypes.h:191-229, g2oTypes.cc:173-189
 * and the g2o machinery (external, version unpinned — SURVEY §8c), restated from upstream g2o:
 *   - SparseOptimizer::initializeOptimization(level): active edges = edges of that level with at
 *     least one non-fixed vertex; active vertices = vertices of active edges
 *   - BaseBinaryEdge::constructQuadraticForm with robust kernels (weightedOmega = rho' Omega,
 *     omega_r = -Omega e rho'), in edge order
 *   - BlockSolver<6,3>::setLambda / solve: Dinv = (Hll + lambda I).inverse() (Eigen 3x3 cofactor
 *     inverse), db = Dinv bl, coefficients_i += Bi db, Hschur(i1, i2) -= (Bi1 Dinv) Bi2^T for
 *     i2 >= i1, landmark by landmark; bschur = bp - coefficients; xl = Dinv (bl - Hpl^T xp)
 *   - LinearSolverEigen / LinearSolverDense on Hschur: a dense LDL^T here (natural order)
 *   - OptimizationAlgorithmLevenberg::solve (same rules as deftri_oracle.c)
 * Edge errors are cached exactly like g2o: only computeActiveErrors (active edges) or an explicit
 * computeError updates them.
 *
 * Build: oracle/Makefile (gcc -O2 -fno-fast-math -ffp-contract=off).
 */
#include "deftri_oracle.c"

typedef struct {
    const deftri_ba_desc *d;
    int K, P, E;
    se3q *poses;
    double *points;
    double *err;              /* [2E] cached errors (caller edge order) */
    const uint8_t *level, *robust;
    int alevel;
    /* activity */
    uint8_t *act;             /* [E] */
    int *sidx;                /* [K] Schur block of free active poses, -1 otherwise */
    uint8_t *pfree;           /* [P] */
    int nfree, nfree_pts;
} ba_problem;

static uint8_t ba_pose_fixed(const ba_problem *b, int k) { return b->d->pose_fixed ? b->d->pose_fixed[k] : 0; }
static uint8_t ba_point_fixed(const ba_problem *b, int l) { return b->d->point_fixed ? b->d->point_fixed[l] : 0; }

/* EdgeSE3ProjectXYZ::computeError (g2oTypes.h:165-182) */
static void ba_edge_error(const ba_problem *b, int e, double out[2]) {
    const deftri_ba_desc *d = b->d;
    int k = d->edge_pose[e], l = d->edge_point[e];
    double pc[3];
    se3_map(&b->poses[k], b->points + 3 * (size_t)l, pc);
    float pf[3] = {(float)pc[0], (float)pc[1], (float)pc[2]}, uv[2];
    kb8_project(d->pose_kb8 + 8 * k, pf, uv);
    out[0] = d->edge_obs[2 * e] - (double)uv[0];
    out[1] = d->edge_obs[2 * e + 1] - (double)uv[1];
}

static double ba_edge_chi2_raw(const ba_problem *b, int e) {   /* _error.dot(information() * _error) */
    double om = b->d->edge_info[e], e0 = b->err[2 * e], e1 = b->err[2 * e + 1];
    return e0 * (om * e0) + e1 * (om * e1);
}

static void ba_activate(ba_problem *b) {
    const deftri_ba_desc *d = b->d;
    uint8_t *pose_act = (uint8_t *)calloc((size_t)b->K + 1, 1);
    uint8_t *pt_act = (uint8_t *)calloc((size_t)b->P + 1, 1);
    for (int e = 0; e < b->E; e++) {
        int k = d->edge_pose[e], l = d->edge_point[e];
        int lev = b->level ? b->level[e] : 0;
        int all_fixed = ba_point_fixed(b, l) && ba_pose_fixed(b, k);
        b->act[e] = (lev == b->alevel && !all_fixed) ? 1 : 0;
        if (b->act[e]) { pose_act[k] = 1; pt_act[l] = 1; }
    }
    b->nfree = 0;
    for (int k = 0; k < b->K; k++) b->sidx[k] = (pose_act[k] && !ba_pose_fixed(b, k)) ? b->nfree++ : -1;
    b->nfree_pts = 0;
    for (int l = 0; l < b->P; l++) {
        b->pfree[l] = (pt_act[l] && !ba_point_fixed(b, l)) ? 1 : 0;
        b->nfree_pts += b->pfree[l];
    }
    free(pose_act); free(pt_act);
}

static void ba_init(ba_problem *b, const deftri_ba_desc *d, const uint8_t *level, const uint8_t *robust,
                    int alevel, const double *poses, const double *points, const double *err) {
    memset(b, 0, sizeof(*b));
    b->d = d; b->K = d->n_poses; b->P = d->n_points; b->E = d->n_edges;
    b->poses = (se3q *)malloc(sizeof(se3q) * ((size_t)b->K + 1));
    b->points = (double *)malloc(sizeof(double) * (3 * (size_t)b->P + 1));
    b->err = (double *)calloc(2 * (size_t)b->E + 1, sizeof(double));
    for (int k = 0; k < b->K; k++) b->poses[k] = se3_from7(poses + 7 * k);
    memcpy(b->points, points, sizeof(double) * 3 * (size_t)b->P);
    if (err) memcpy(b->err, err, sizeof(double) * 2 * (size_t)b->E);
    b->level = level; b->robust = robust; b->alevel = alevel;
    b->act = (uint8_t *)calloc((size_t)b->E + 1, 1);
    b->sidx = (int *)malloc(sizeof(int) * ((size_t)b->K + 1));
    b->pfree = (uint8_t *)calloc((size_t)b->P + 1, 1);
    ba_activate(b);
}

static void ba_free(ba_problem *b) {
    free(b->poses); free(b->points); free(b->err); free(b->act); free(b->sidx); free(b->pfree);
}

/* computeActiveErrors + activeRobustChi2 */
static double ba_active_chi2(ba_problem *b) {
    double chi = 0.0, rho[3];
    for (int e = 0; e < b->E; e++) {
        if (!b->act[e]) continue;
        ba_edge_error(b, e, b->err + 2 * e);
        double c2 = ba_edge_chi2_raw(b, e);
        if (!b->robust || b->robust[e]) { huber(b->d->huber_delta, c2, rho); chi += rho[0]; }
        else chi += c2;
    }
    return chi;
}

/* linearized system: Hpp [K*36], bp [K*6], Hll [P*9], bl [P*3], Hpl [E*18] (6x3 per edge, summed
   on the first edge of each (point, pose) pair: `lead`) */
typedef struct {
    double *Hpp, *bp, *Hll, *bl, *Hpl;
    int *lead;
} ba_system;

static void ba_system_alloc(const ba_problem *b, ba_system *s) {
    s->Hpp = (double *)calloc(36 * (size_t)b->K + 1, sizeof(double));
    s->bp = (double *)calloc(6 * (size_t)b->K + 1, sizeof(double));
    s->Hll = (double *)calloc(9 * (size_t)b->P + 1, sizeof(double));
    s->bl = (double *)calloc(3 * (size_t)b->P + 1, sizeof(double));
    s->Hpl = (double *)calloc(18 * (size_t)b->E + 1, sizeof(double));
    s->lead = (int *)malloc(sizeof(int) * ((size_t)b->E + 1));
    /* lead edge: first edge (caller order) of the same (point, pose) pair */
    const deftri_ba_desc *d = b->d;
    int *first = (int *)malloc(sizeof(int) * ((size_t)b->P * (size_t)(b->K > 0 ? b->K : 1) + 1));
    for (size_t i = 0; i < (size_t)b->P * (size_t)(b->K > 0 ? b->K : 1); i++) first[i] = -1;
    for (int e = 0; e < b->E; e++) {
        size_t key = (size_t)d->edge_point[e] * (size_t)b->K + (size_t)d->edge_pose[e];
        if (first[key] < 0) first[key] = e;
        s->lead[e] = first[key];
    }
    free(first);
}

static void ba_system_free(ba_system *s) { free(s->Hpp); free(s->bp); free(s->Hll); free(s->bl); free(s->Hpl); free(s->lead); }

/* EdgeSE3ProjectXYZ::linearizeOplus + constructQuadraticForm over active edges in edge order */
static void ba_build_system(ba_problem *b, ba_system *s) {
    const deftri_ba_desc *d = b->d;
    memset(s->Hpp, 0, sizeof(double) * 36 * (size_t)b->K);
    memset(s->bp, 0, sizeof(double) * 6 * (size_t)b->K);
    memset(s->Hll, 0, sizeof(double) * 9 * (size_t)b->P);
    memset(s->bl, 0, sizeof(double) * 3 * (size_t)b->P);
    memset(s->Hpl, 0, sizeof(double) * 18 * (size_t)b->E);
    for (int e = 0; e < b->E; e++) {
        if (!b->act[e]) continue;
        int k = d->edge_pose[e], l = d->edge_point[e];
        const se3q *T = &b->poses[k];
        double pc[3], R[9];
        se3_map(T, b->points + 3 * (size_t)l, pc);
        float pf[3] = {(float)pc[0], (float)pc[1], (float)pc[2]}, jf[6];
        kb8_project_jac(d->pose_kb8 + 8 * k, pf, jf);
        double A[6];
        for (int i = 0; i < 6; i++) A[i] = -(double)jf[i];          /* -pCamera->projectJac(xyz_trans) */
        q_to_mat(&T->r, R);
        double Jp[6], JT[12];
        for (int r = 0; r < 2; r++)
            for (int c = 0; c < 3; c++) Jp[3 * r + c] = A[3 * r] * R[c] + A[3 * r + 1] * R[3 + c] + A[3 * r + 2] * R[6 + c];
        double x = pc[0], y = pc[1], z = pc[2];
        double D[18] = {0.0, z, -y, 1.0, 0.0, 0.0, -z, 0.0, x, 0.0, 1.0, 0.0, y, -x, 0.0, 0.0, 0.0, 1.0};
        for (int r = 0; r < 2; r++)
            for (int c = 0; c < 6; c++) JT[6 * r + c] = A[3 * r] * D[c] + A[3 * r + 1] * D[6 + c] + A[3 * r + 2] * D[12 + c];
        /* constructQuadraticForm */
        double om = d->edge_info[e], e0 = b->err[2 * e], e1 = b->err[2 * e + 1];
        double rho[3] = {0, 1, 0};
        if (!b->robust || b->robust[e]) huber(d->huber_delta, ba_edge_chi2_raw(b, e), rho);
        double w = rho[1] * om;
        double or0 = (-(om * e0)) * rho[1], or1 = (-(om * e1)) * rho[1];
        int from_free = b->pfree[l], to_free = b->sidx[k] >= 0;
        if (from_free) {
            double *H = s->Hll + 9 * (size_t)l, *bb = s->bl + 3 * (size_t)l;
            for (int c = 0; c < 3; c++) {
                double a0 = Jp[c] * w, a1 = Jp[3 + c] * w;
                for (int dd = 0; dd < 3; dd++) H[3 * c + dd] += a0 * Jp[dd] + a1 * Jp[3 + dd];
                bb[c] += Jp[c] * or0 + Jp[3 + c] * or1;
            }
            if (to_free) {
                double *o = s->Hpl + 18 * (size_t)s->lead[e];
                for (int j = 0; j < 6; j++)
                    for (int c = 0; c < 3; c++) o[3 * j + c] += (Jp[c] * w) * JT[j] + (Jp[3 + c] * w) * JT[6 + j];
            }
        }
        if (to_free) {
            double *H = s->Hpp + 36 * (size_t)k, *bb = s->bp + 6 * (size_t)k;
            for (int i = 0; i < 6; i++) {
                double a0 = JT[i] * w, a1 = JT[6 + i] * w;
                for (int j = 0; j < 6; j++) H[6 * i + j] += a0 * JT[j] + a1 * JT[6 + j];
                bb[i] += JT[i] * or0 + JT[6 + i] * or1;
            }
        }
    }
}

/* Eigen compute_inverse_size3 (cofactor inverse) */
static void inv3(const double m[9], double Di[9]) {
#define M(i, j) m[3 * (i) + (j)]
#define COF(i, j) (M(((i) + 1) % 3, ((j) + 1) % 3) * M(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M(((i) + 1) % 3, ((j) + 2) % 3) * M(((i) + 2) % 3, ((j) + 1) % 3))
    double c00 = COF(0, 0), c10 = COF(1, 0), c20 = COF(2, 0);
    double det = (c00 * M(0, 0) + c10 * M(1, 0)) + c20 * M(2, 0);
    double invdet = 1.0 / det;
    Di[0] = c00 * invdet; Di[1] = c10 * invdet; Di[2] = c20 * invdet;
    Di[3] = COF(0, 1) * invdet; Di[4] = COF(1, 1) * invdet; Di[5] = COF(2, 1) * invdet;
    Di[6] = COF(0, 2) * invdet; Di[7] = COF(1, 2) * invdet; Di[8] = COF(2, 2) * invdet;
#undef COF
#undef M
}

/* dense LDL^T of the symmetric n x n (row-major, full) matrix in place; 0 on a zero (or, when
   positive is set, negative) pivot */
static int ldlt_dense(double *A, int n, int positive) {
    for (int k = 0; k < n; k++) {
        double dk = A[(size_t)k * n + k];
        for (int j = 0; j < k; j++) dk -= A[(size_t)k * n + j] * A[(size_t)k * n + j] * A[(size_t)j * n + j];
        A[(size_t)k * n + k] = dk;
        if (dk == 0.0 || (positive && dk < 0.0)) return 0;
        for (int i = k + 1; i < n; i++) {
            double s = A[(size_t)i * n + k];
            for (int j = 0; j < k; j++) s -= A[(size_t)i * n + j] * A[(size_t)k * n + j] * A[(size_t)j * n + j];
            A[(size_t)i * n + k] = s / dk;
        }
    }
    return 1;
}

static void ldlt_dense_solve(const double *A, int n, double *x) {
    for (int i = 0; i < n; i++)
        for (int j = 0; j < i; j++) x[i] -= A[(size_t)i * n + j] * x[j];
    for (int i = 0; i < n; i++) x[i] /= A[(size_t)i * n + i];
    for (int i = n - 1; i >= 0; i--)
        for (int j = i + 1; j < n; j++) x[i] -= A[(size_t)j * n + i] * x[j];
}

/* BlockSolver<6,3>::setLambda + solve.  Writes the damped Schur system (full, before factorization)
   into S/rhs if given, and the step into xp [6*nfree] / xl [3P].  Returns the solver's success. */
static int ba_schur_solve(const ba_problem *b, const ba_system *s, double lambda, double *S_out, double *rhs_out,
                          double *xp, double *xl) {
    const deftri_ba_desc *d = b->d;
    int ns = 6 * b->nfree;
    double *Hs = (double *)calloc((size_t)ns * ns + 1, sizeof(double));
    double *coef = (double *)calloc((size_t)ns + 1, sizeof(double));
    double *Dinv = (double *)calloc(9 * (size_t)b->P + 1, sizeof(double));
    /* Hschur = Hpp + lambda I (upper triangle in g2o; kept full here) */
    for (int k = 0; k < b->K; k++) {
        int a = b->sidx[k];
        if (a < 0) continue;
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < 6; j++)
                Hs[(size_t)(6 * a + i) * ns + 6 * a + j] = s->Hpp[36 * k + 6 * i + j] + (i == j ? lambda : 0.0);
    }
    /* landmark columns: (pose, lead edge) pairs of each free point, pose order */
    int *col_pose = (int *)malloc(sizeof(int) * ((size_t)b->K + 1));
    int *col_edge = (int *)malloc(sizeof(int) * ((size_t)b->K + 1));
    /* edges by point (caller order within a point) */
    int *pptr = (int *)calloc((size_t)b->P + 2, sizeof(int));
    int *pedges = (int *)malloc(sizeof(int) * ((size_t)b->E + 1));
    for (int e = 0; e < b->E; e++) pptr[d->edge_point[e] + 1]++;
    for (int l = 0; l < b->P; l++) pptr[l + 1] += pptr[l];
    {
        int *fill = (int *)malloc(sizeof(int) * ((size_t)b->P + 1));
        memcpy(fill, pptr, sizeof(int) * (size_t)b->P);
        for (int e = 0; e < b->E; e++) pedges[fill[d->edge_point[e]]++] = e;
        free(fill);
    }
    for (int l = 0; l < b->P; l++) {
        if (!b->pfree[l]) continue;
        double m[9];
        memcpy(m, s->Hll + 9 * (size_t)l, sizeof(m));
        m[0] += lambda; m[4] += lambda; m[8] += lambda;
        double *Di = Dinv + 9 * (size_t)l;
        inv3(m, Di);
        const double *bl = s->bl + 3 * (size_t)l;
        double db[3];
        for (int i = 0; i < 3; i++) db[i] = Di[3 * i] * bl[0] + Di[3 * i + 1] * bl[1] + Di[3 * i + 2] * bl[2];
        int nc = 0;
        for (int q = pptr[l]; q < pptr[l + 1]; q++) {
            int e = pedges[q];
            if (!b->act[e] || s->lead[e] != e) continue;
            /* a lead edge carries the pair's block only if some edge of the pair is active */
            int k = d->edge_pose[e];
            if (b->sidx[k] < 0) continue;
            int dup = 0;
            for (int c = 0; c < nc; c++) if (col_pose[c] == k) dup = 1;
            if (dup) continue;
            int pos = nc++;
            while (pos > 0 && col_pose[pos - 1] > k) { col_pose[pos] = col_pose[pos - 1]; col_edge[pos] = col_edge[pos - 1]; pos--; }
            col_pose[pos] = k; col_edge[pos] = e;
        }
        /* pairs whose lead edge is inactive but a duplicate is active */
        for (int q = pptr[l]; q < pptr[l + 1]; q++) {
            int e = pedges[q];
            if (!b->act[e] || s->lead[e] == e) continue;
            int k = d->edge_pose[e];
            if (b->sidx[k] < 0) continue;
            int dup = 0;
            for (int c = 0; c < nc; c++) if (col_pose[c] == k) dup = 1;
            if (dup) continue;
            int pos = nc++;
            while (pos > 0 && col_pose[pos - 1] > k) { col_pose[pos] = col_pose[pos - 1]; col_edge[pos] = col_edge[pos - 1]; pos--; }
            col_pose[pos] = k; col_edge[pos] = s->lead[e];
        }
        for (int c1 = 0; c1 < nc; c1++) {
            const double *Bi = s->Hpl + 18 * (size_t)col_edge[c1];
            int a = b->sidx[col_pose[c1]];
            double BDinv[18];
            for (int j = 0; j < 6; j++)
                for (int c = 0; c < 3; c++)
                    BDinv[3 * j + c] = Bi[3 * j] * Di[c] + Bi[3 * j + 1] * Di[3 + c] + Bi[3 * j + 2] * Di[6 + c];
            for (int j = 0; j < 6; j++) coef[6 * a + j] += Bi[3 * j] * db[0] + Bi[3 * j + 1] * db[1] + Bi[3 * j + 2] * db[2];
            for (int c2 = c1; c2 < nc; c2++) {
                const double *Bj = s->Hpl + 18 * (size_t)col_edge[c2];
                int bb = b->sidx[col_pose[c2]];
                for (int i = 0; i < 6; i++)
                    for (int j = 0; j < 6; j++) {
                        double v = BDinv[3 * i] * Bj[3 * j] + BDinv[3 * i + 1] * Bj[3 * j + 1] + BDinv[3 * i + 2] * Bj[3 * j + 2];
                        Hs[(size_t)(6 * a + i) * ns + 6 * bb + j] -= v;
                    }
            }
        }
    }
    /* symmetrize from the upper block triangle (g2o keeps the upper part) */
    for (int r = 0; r < ns; r++)
        for (int c = 0; c < ns; c++)
            if (r / 6 > c / 6) Hs[(size_t)r * ns + c] = Hs[(size_t)c * ns + r];
    double *bs = (double *)malloc(sizeof(double) * ((size_t)ns + 1));
    for (int k = 0; k < b->K; k++) {
        int a = b->sidx[k];
        if (a < 0) continue;
        for (int j = 0; j < 6; j++) bs[6 * a + j] = s->bp[6 * k + j] - coef[6 * a + j];
    }
    if (S_out) memcpy(S_out, Hs, sizeof(double) * (size_t)ns * ns);
    if (rhs_out) memcpy(rhs_out, bs, sizeof(double) * (size_t)ns);
    int ok = ldlt_dense(Hs, ns, b->nfree_pts == 0);
    if (ok) {
        memcpy(xp, bs, sizeof(double) * (size_t)ns);
        ldlt_dense_solve(Hs, ns, xp);
    } else {
        memset(xp, 0, sizeof(double) * (size_t)ns);
    }
    /* landmarks: cl = bl - Hpl^T xp ; xl = Dinv cl */
    memset(xl, 0, sizeof(double) * 3 * (size_t)b->P);
    for (int l = 0; l < b->P; l++) {
        if (!b->pfree[l]) continue;
        double cl[3] = {s->bl[3 * l], s->bl[3 * l + 1], s->bl[3 * l + 2]};
        for (int q = pptr[l]; q < pptr[l + 1]; q++) {
            int e = pedges[q];
            if (s->lead[e] != e) continue;
            int k = d->edge_pose[e];
            if (b->sidx[k] < 0) continue;
            /* pair present in the system iff some edge of the pair is active */
            int any = 0;
            for (int q2 = pptr[l]; q2 < pptr[l + 1]; q2++)
                if (s->lead[pedges[q2]] == e && b->act[pedges[q2]]) any = 1;
            if (!any) continue;
            const double *B = s->Hpl + 18 * (size_t)e;
            const double *xx = xp + 6 * b->sidx[k];
            for (int c = 0; c < 3; c++) {
                double acc = 0.0;
                for (int j = 0; j < 6; j++) acc += B[3 * j + c] * (-xx[j]);
                cl[c] += acc;
            }
        }
        const double *Di = Dinv + 9 * (size_t)l;
        for (int i = 0; i < 3; i++) xl[3 * l + i] = Di[3 * i] * cl[0] + Di[3 * i + 1] * cl[1] + Di[3 * i + 2] * cl[2];
    }
    free(Hs); free(coef); free(Dinv); free(col_pose); free(col_edge); free(pptr); free(pedges); free(bs);
    return ok;
}

static void ba_update(ba_problem *b, const double *xp, const double *xl) {
    for (int k = 0; k < b->K; k++)
        if (b->sidx[k] >= 0) se3_oplus(&b->poses[k], xp + 6 * b->sidx[k]);
    for (int l = 0; l < b->P; l++)
        if (b->pfree[l])
            for (int c = 0; c < 3; c++) b->points[3 * l + c] += xl[3 * l + c];
}

/* initializeOptimization(alevel); optimize(n).  poses/points/err in and out. */
int oracle_ba_solve(const deftri_ba_desc *d, const uint8_t *level, const uint8_t *robust, int32_t alevel,
                    const deftri_lm_params *prm, double *poses, double *points, double *err, deftri_report *rep) {
    double t_start = now_ms();
    ba_problem b;
    ba_init(&b, d, level, robust, alevel, poses, points, err);
    memset(rep, 0, sizeof(*rep));
    int ns = 6 * b.nfree;
    rep->n_unknowns = ns + 3 * (int64_t)b.nfree_pts;
    if (ns == 0 && b.nfree_pts == 0) {
        rep->status = DEFTRI_STATUS_TERMINATE;
        ba_free(&b);
        return 0;
    }
    ba_system s;
    ba_system_alloc(&b, &s);
    double *xp = (double *)calloc((size_t)ns + 1, sizeof(double));
    double *xl = (double *)calloc(3 * (size_t)b.P + 1, sizeof(double));
    se3q *pbak = (se3q *)malloc(sizeof(se3q) * ((size_t)b.K + 1));
    double *lbak = (double *)malloc(sizeof(double) * (3 * (size_t)b.P + 1));
    int max_trials = prm->max_trials > 0 ? prm->max_trials : 10;
    double tau = prm->tau > 0 ? prm->tau : 1e-5;
    double lambda = 0, ni = 2, currentChi = 0;
    int status = DEFTRI_STATUS_OK, it;
    for (it = 0; it < prm->n_iterations; it++) {
        currentChi = ba_active_chi2(&b);
        ba_build_system(&b, &s);
        if (it == 0) {
            rep->chi2_initial = currentChi;
            if (prm->user_lambda > 0) lambda = prm->user_lambda;
            else {
                double maxDiag = 0;
                for (int k = 0; k < b.K; k++)
                    if (b.sidx[k] >= 0)
                        for (int j = 0; j < 6; j++) maxDiag = fmax(maxDiag, fabs(s.Hpp[36 * k + 7 * j]));
                for (int l = 0; l < b.P; l++)
                    if (b.pfree[l])
                        for (int j = 0; j < 3; j++) maxDiag = fmax(maxDiag, fabs(s.Hll[9 * l + 4 * j]));
                lambda = tau * maxDiag;
            }
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            memcpy(pbak, b.poses, sizeof(se3q) * (size_t)b.K);
            memcpy(lbak, b.points, sizeof(double) * 3 * (size_t)b.P);
            int ok2 = ba_schur_solve(&b, &s, lambda, NULL, NULL, xp, xl);
            ba_update(&b, xp, xl);
            double tempChi = ba_active_chi2(&b);
            if (!ok2) tempChi = 1.79769313486231570815e+308;
            rho = currentChi - tempChi;
            double scale = 0;
            for (int k = 0; k < b.K; k++) {
                int a = b.sidx[k];
                if (a < 0) continue;
                for (int j = 0; j < 6; j++) scale += xp[6 * a + j] * (lambda * xp[6 * a + j] + s.bp[6 * k + j]);
            }
            for (int l = 0; l < b.P; l++)
                if (b.pfree[l])
                    for (int j = 0; j < 3; j++) scale += xl[3 * l + j] * (lambda * xl[3 * l + j] + s.bl[3 * l + j]);
            scale += 1e-3;
            rho /= scale;
            rep->trials_total++;
            if (rho > 0 && isfinite(tempChi) && ok2) {
                double alpha = 1. - pow((2 * rho - 1), 3);
                alpha = alpha < (2. / 3.) ? alpha : (2. / 3.);
                double scaleFactor = (1. / 3.) > alpha ? (1. / 3.) : alpha;
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                memcpy(b.poses, pbak, sizeof(se3q) * (size_t)b.K);
                memcpy(b.points, lbak, sizeof(double) * 3 * (size_t)b.P);
                rep->trials_rejected++;
            }
            qmax++;
            if (!isfinite(lambda)) break;
        } while (rho < 0 && qmax < max_trials);
        if (it < DEFTRI_MAX_REPORT_ITERS) { rep->chi2_iter[it] = currentChi; rep->trials_iter[it] = qmax; }
        if (prm->verbose)
            fprintf(stderr, "[oracle-ba] it %d chi2 %.9e lambda %.6e trials %d\n", it, currentChi, lambda, qmax);
        if (qmax == max_trials || rho == 0 || !isfinite(lambda)) { status = DEFTRI_STATUS_TERMINATE; it++; break; }
    }
    rep->status = status;
    rep->iterations = it;
    rep->chi2_final = currentChi;
    rep->lambda_final = lambda;
    rep->ms_total = now_ms() - t_start;
    for (int k = 0; k < b.K; k++) se3_to7(&b.poses[k], poses + 7 * k);
    memcpy(points, b.points, sizeof(double) * 3 * (size_t)b.P);
    if (err) memcpy(err, b.err, sizeof(double) * 2 * (size_t)b.E);
    free(xp); free(xl); free(pbak); free(lbak);
    ba_system_free(&s);
    ba_free(&b);
    return 0;
}

/* e->computeError() on every edge */
int oracle_ba_compute_errors(const deftri_ba_desc *d, const double *poses, const double *points, double *err) {
    ba_problem b;
    ba_init(&b, d, NULL, NULL, 0, poses, points, NULL);
    for (int e = 0; e < b.E; e++) ba_edge_error(&b, e, err + 2 * e);
    ba_free(&b);
    return 0;
}

/* e->chi2() of cached errors and e->isDepthPositive() at the given state */
int oracle_ba_edge_chi2(const deftri_ba_desc *d, const double *poses, const double *points, const double *err,
                        double *chi2, uint8_t *dpos) {
    ba_problem b;
    ba_init(&b, d, NULL, NULL, 0, poses, points, err);
    for (int e = 0; e < b.E; e++) {
        if (chi2) chi2[e] = ba_edge_chi2_raw(&b, e);
        if (dpos) {
            double pc[3];
            se3_map(&b.poses[d->edge_pose[e]], b.points + 3 * (size_t)d->edge_point[e], pc);
            dpos[e] = pc[2] > 0.0;
        }
    }
    ba_free(&b);
    return 0;
}

/* the damped Schur system at the given state: chi2, S [ns*ns], rhs [ns], dx [6K + 3P] (pose order,
   zeros for fixed / inactive vertices), b [6K + 3P]; *ns_out = 6 * free poses */
int oracle_ba_eval_system(const deftri_ba_desc *d, const uint8_t *level, const uint8_t *robust, int32_t alevel,
                          const double *poses, const double *points, double lambda, double *chi2, double *S,
                          double *rhs, double *dx, double *bvec, int32_t *ns_out) {
    ba_problem b;
    ba_init(&b, d, level, robust, alevel, poses, points, NULL);
    ba_system s;
    ba_system_alloc(&b, &s);
    double c = ba_active_chi2(&b);
    ba_build_system(&b, &s);
    int ns = 6 * b.nfree;
    double *xp = (double *)calloc((size_t)ns + 1, sizeof(double));
    double *xl = (double *)calloc(3 * (size_t)b.P + 1, sizeof(double));
    int ok = ba_schur_solve(&b, &s, lambda, S, rhs, xp, xl);
    if (chi2) *chi2 = c;
    if (ns_out) *ns_out = ns;
    if (dx) {
        for (int k = 0; k < b.K; k++)
            for (int j = 0; j < 6; j++) dx[6 * k + j] = b.sidx[k] >= 0 ? xp[6 * b.sidx[k] + j] : 0.0;
        memcpy(dx + 6 * (size_t)b.K, xl, sizeof(double) * 3 * (size_t)b.P);
    }
    if (bvec) {
        for (int k = 0; k < b.K; k++)
            for (int j = 0; j < 6; j++) bvec[6 * k + j] = b.sidx[k] >= 0 ? s.bp[6 * k + j] : 0.0;
        for (int l = 0; l < b.P; l++)
            for (int j = 0; j < 3; j++) bvec[6 * (size_t)b.K + 3 * l + j] = b.pfree[l] ? s.bl[3 * l + j] : 0.0;
    }
    free(xp); free(xl);
    ba_system_free(&s);
    ba_free(&b);
    return ok ? 0 : -4;
}
