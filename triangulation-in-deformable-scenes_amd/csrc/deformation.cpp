// deformation.cpp — deformationOptimization (reference Modules/Optimization/g2oBundleAdjustment.cc:
// 446-606) in native code behind the C-ABI: the outer rounds, NLopt's LN_NELDERMEAD weight search
// restated (nldrmd.c, the default initial step, elimdim, relstop — the same algorithm as
// deftri/nlopt_nm.py, which the tests hold it to), outerObjective (nloptOptimization.cc:4-37) on map
// clones, and Map::insertGlobalKeyFramesTransformation's table update (Map.cc:323-330).
//
// A Map clone (Map.cc:30-58) here is what arapOptimization can change: every keyframe's slot
// positions and depth scale; the keypoints, poses, calibration and observation tables are shared
// read-only.  Two properties of the reference's clone reach the solver and are kept:
//   - it does NOT copy mGTransformation_: a clone's global-transformation table is empty, so every
//     pair of a clone's graph starts T_g at the identity (:664-677);
//   - it inserts the KeyFrames in the source's unordered_map iteration order, so a clone iterates
//     them in the order libstdc++'s std::unordered_map gives that insertion sequence (reversed for
//     up to 13 keyframes).  The evaluation maps are clones of the round's clone (:499, then
//     nloptOptimization.cc:13), i.e. two such re-insertions.
// Every evaluation starts from the round's base map, so the context's graph memo answers its graph
// build and the iterative plan is reused (the evaluations differ only in the weights).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <functional>
#include <limits>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/deftri.h"

namespace {

// ---- NLopt LN_NELDERMEAD (nldrmd.c) restated; deftri/nlopt_nm.py is the same algorithm ----------
constexpr double kAlpha = 1.0, kBeta = 0.5, kGamma = 2.0, kDelta = 0.5;
enum { kSuccess = 1, kXtol = 4, kMaxeval = 5, kFailure = -1 };

void default_initial_step(int n, const double *x, const double *lb, const double *ub, double *dx) {
    for (int i = 0; i < n; i++) {
        double step = INFINITY;
        if (std::isfinite(ub[i]) && std::isfinite(lb[i]) && (ub[i] - lb[i]) * 0.25 < step && ub[i] > lb[i])
            step = (ub[i] - lb[i]) * 0.25;
        if (std::isfinite(ub[i]) && ub[i] - x[i] < step && ub[i] > x[i]) step = (ub[i] - x[i]) * 0.75;
        if (std::isfinite(lb[i]) && x[i] - lb[i] < step && x[i] > lb[i]) step = (x[i] - lb[i]) * 0.75;
        if (std::isinf(step)) {
            if (std::isfinite(ub[i]) && std::fabs(ub[i] - x[i]) < std::fabs(step)) step = (ub[i] - x[i]) * 1.1;
            if (std::isfinite(lb[i]) && std::fabs(x[i] - lb[i]) < std::fabs(step)) step = (x[i] - lb[i]) * 1.1;
        }
        if (std::isinf(step) || std::fabs(step) < 1e-300) step = x[i];
        if (std::isinf(step) || step == 0.0) step = 1.0;
        dx[i] = step;
    }
}

bool close_(double a, double b) { return std::fabs(a - b) <= 1e-13 * (std::fabs(a) + std::fabs(b)); }

bool relstop(double vold, double vnew, double reltol, double abstol) {
    if (std::isinf(vold)) return false;
    const double d = std::fabs(vnew - vold);
    return d < abstol || d < reltol * (std::fabs(vnew) + std::fabs(vold)) * 0.5 || (reltol > 0 && vnew == vold);
}

// xnew = c + scale (c - xold) pinned to the bounds; false when it coincides with c or xold
bool reflect(int n, const double *c, double scale, const double *xold, const double *lb, const double *ub, double *xnew) {
    bool eqc = true, eqold = true;
    for (int i = 0; i < n; i++) {
        double v = c[i] + scale * (c[i] - xold[i]);
        v = std::min(std::max(v, lb[i]), ub[i]);
        xnew[i] = v;
        eqc = eqc && close_(v, c[i]);
        eqold = eqold && close_(v, xold[i]);
    }
    return !(eqc || eqold);
}

void simplex_vertex(int n, const double *x, const double *xstep, const double *lo, const double *hi, int i, double *pt) {
    for (int k = 0; k < n; k++) pt[k] = x[k];
    pt[i] += xstep[i];
    if (pt[i] > hi[i]) pt[i] = hi[i] - x[i] > std::fabs(xstep[i]) * 0.1 ? hi[i] : x[i] - std::fabs(xstep[i]);
    if (pt[i] < lo[i]) {
        if (x[i] - lo[i] > std::fabs(xstep[i]) * 0.1) {
            pt[i] = lo[i];
        } else {
            pt[i] = x[i] + std::fabs(xstep[i]);
            if (pt[i] > hi[i]) pt[i] = 0.5 * ((hi[i] - x[i] > x[i] - lo[i] ? hi[i] : lo[i]) + x[i]);
        }
    }
}

struct Stop { int code; };

// opt.optimize(x, minf) of an LN_NELDERMEAD nlopt::opt over N = n0 dimensions (elimdim removes
// lb == ub); f(full x) -> value.  Returns the result code; x0 <- the best point.
int nelder_mead(const std::function<double(const double *)> &f, int n0, double *x0, const double *lb0, const double *ub0,
                double xtol_rel, double xtol_abs, int maxeval, double &minf, int &nevals) {
    std::vector<int> fr;
    for (int i = 0; i < n0; i++) if (lb0[i] != ub0[i]) fr.push_back(i);
    const int n = (int)fr.size();
    std::vector<double> xfull(x0, x0 + n0), xbest(x0, x0 + n0), tmp(n0);
    minf = INFINITY;
    nevals = 0;
    auto full = [&](const double *xr) {
        tmp = xfull;
        for (int k = 0; k < n; k++) tmp[fr[k]] = xr[k];
        return tmp.data();
    };
    auto feval = [&](const double *xr) { const double v = f(full(xr)); nevals++; return v; };
    auto check = [&](const double *xr, double fv) {        // CHECK_EVAL
        if (fv <= minf) {
            minf = fv;
            xbest = xfull;
            for (int k = 0; k < n; k++) xbest[fr[k]] = xr[k];
        }
        if (maxeval > 0 && nevals >= maxeval) throw Stop{kMaxeval};
    };
    int code = kSuccess;
    try {
        std::vector<double> x(n), lo(n), hi(n), xstep(n);
        for (int k = 0; k < n; k++) { x[k] = x0[fr[k]]; lo[k] = lb0[fr[k]]; hi[k] = ub0[fr[k]]; }
        if (n == 0) {
            check(x.data(), feval(x.data()));
            throw Stop{kSuccess};
        }
        default_initial_step(n, x.data(), lo.data(), hi.data(), xstep.data());
        const double fx = feval(x.data());                  // nldrmd_minimize: f(x0) first
        check(x.data(), fx);
        std::vector<double> pts((size_t)(n + 1) * n), fv(n + 1);
        auto P = [&](int k) { return &pts[(size_t)k * n]; };
        std::copy(x.begin(), x.end(), P(0));
        fv[0] = fx;
        for (int i = 0; i < n; i++) {
            simplex_vertex(n, x.data(), xstep.data(), lo.data(), hi.data(), i, P(i + 1));
            if (close_(P(i + 1)[i], x[i])) throw Stop{kFailure};
            fv[i + 1] = feval(P(i + 1));
            check(P(i + 1), fv[i + 1]);
        }
        std::vector<double> c(n), xcur(n), xr(n), xe(n), xc(n), xl(n), xh(n), xs(n);
        std::vector<int> order(n + 1);
        for (;;) {
            for (int k = 0; k <= n; k++) order[k] = k;
            std::sort(order.begin(), order.end(), [&](int a, int b) { return fv[a] != fv[b] ? fv[a] < fv[b] : a < b; });
            const int il = order[0], ih = order[n];
            const double fl = fv[il], fh = fv[ih];
            std::copy(P(il), P(il) + n, xl.begin());
            std::copy(P(ih), P(ih) + n, xh.begin());
            std::fill(c.begin(), c.end(), 0.0);
            for (int k = 0; k <= n; k++)
                if (k != ih)
                    for (int d = 0; d < n; d++) c[d] += P(k)[d];
            for (int d = 0; d < n; d++) c[d] *= 1.0 / n;
            bool stop = true;
            for (int d = 0; d < n; d++) {
                double m = 0.0;
                for (int k = 0; k <= n; k++) m = std::max(m, std::fabs(P(k)[d] - c[d]));
                xcur[d] = m + c[d];
                stop = stop && relstop(xcur[d], c[d], xtol_rel, xtol_abs);
            }
            if (stop) throw Stop{kXtol};
            if (!reflect(n, c.data(), kAlpha, xh.data(), lo.data(), hi.data(), xr.data())) throw Stop{kXtol};
            const double frv = feval(xr.data());
            check(xr.data(), frv);
            if (frv < fl) {                                   // new best: expand
                if (!reflect(n, c.data(), kGamma, xh.data(), lo.data(), hi.data(), xe.data())) throw Stop{kXtol};
                const double fe = feval(xe.data());
                check(xe.data(), fe);
                if (fe >= frv) { std::copy(xr.begin(), xr.end(), P(ih)); fv[ih] = frv; }
                else { std::copy(xe.begin(), xe.end(), P(ih)); fv[ih] = fe; }
            } else if (frv < fv[order[n - 1]]) {              // accept
                std::copy(xr.begin(), xr.end(), P(ih));
                fv[ih] = frv;
            } else {                                           // contract
                if (!reflect(n, c.data(), fh <= frv ? -kBeta : kBeta, xh.data(), lo.data(), hi.data(), xc.data()))
                    throw Stop{kXtol};
                const double fc = feval(xc.data());
                check(xc.data(), fc);
                if (fc < frv && fc < fh) {
                    std::copy(xc.begin(), xc.end(), P(ih));
                    fv[ih] = fc;
                } else {                                       // shrink towards the best
                    for (int k = 0; k <= n; k++) {
                        if (k == il) continue;
                        if (!reflect(n, xl.data(), -kDelta, P(k), lo.data(), hi.data(), xs.data())) throw Stop{kXtol};
                        std::copy(xs.begin(), xs.end(), P(k));
                        fv[k] = feval(P(k));
                        check(P(k), fv[k]);
                    }
                }
            }
        }
    } catch (const Stop &s) {
        code = s.code;
    }
    std::copy(xbest.begin(), xbest.end(), x0);
    return code;
}

// Iteration order of std::unordered_map<ID, KeyFrame_> (Map::mKeyFrames_, ID = long unsigned int)
// after inserting `ids` in the given order — the container the reference iterates, evaluated by the
// same standard library rather than restated.
void unordered_order(const int64_t *ids, int n, std::vector<int64_t> &out) {
    std::unordered_map<unsigned long, int> m;
    for (int k = 0; k < n; k++) m[(unsigned long)ids[k]] = k;
    out.clear();
    for (const auto &kv : m) out.push_back((int64_t)kv.first);
}

// ---- Map::insertGlobalKeyFramesTransformation (Map.cc:323-330): T and T.inverse() as Sophus
// SE3f, read back by getGlobalKeyFramesTransformation as g2o::SE3Quat (double) ----------------------
void se3f_as7(const float q[4], const float t[3], double out[7]) {
    // g2o::SE3Quat(T.unit_quaternion().cast<double>(), T.translation().cast<double>()), normalized
    // (SE3Quat::normalizeRotation: w >= 0)
    double d[4] = {q[0], q[1], q[2], q[3]};
    if (d[3] < 0) for (double &v : d) v = -v;
    const double nrm = std::sqrt(((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) + d[3] * d[3]);
    for (int k = 0; k < 4; k++) out[k] = d[k] / nrm;
    for (int k = 0; k < 3; k++) out[4 + k] = t[k];
}

}  // namespace

extern "C" int deftri_keyframe_order(const int64_t *insert_ids, int32_t n, int32_t clones, int64_t *out) {
    if (n < 0 || clones < 0 || (n > 0 && (!insert_ids || !out))) return DEFTRI_E_ARG;
    std::vector<int64_t> cur(insert_ids, insert_ids + n), next;
    for (int c = 0; c <= clones; c++) {
        unordered_order(cur.data(), n, next);
        cur.swap(next);
    }
    std::copy(cur.begin(), cur.end(), out);
    return 0;
}

extern "C" int deftri_global_insert(const double t7[7], double fwd7[7], double inv7[7]) {
    if (!t7 || !fwd7 || !inv7) return DEFTRI_E_ARG;
    // Sophus::SE3f(SE3Quat estimate cast to float): the unit quaternion normalized in float
    float q[4] = {(float)t7[0], (float)t7[1], (float)t7[2], (float)t7[3]};
    const float n2 = ((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3];
    const float inv_n = 1.0f / std::sqrt(n2);
    for (float &v : q) v *= inv_n;
    const float t[3] = {(float)t7[4], (float)t7[5], (float)t7[6]};
    se3f_as7(q, t, fwd7);
    // T.inverse(): the conjugate rotation, translation -(R^T t) by Eigen's quaternion-vector product
    // (uv = 2 (v_q x t); t' = t + w uv + v_q x uv with v_q the conjugate's vector part)
    const float qi[4] = {-q[0], -q[1], -q[2], q[3]};
    float uv[3] = {qi[1] * t[2] - qi[2] * t[1], qi[2] * t[0] - qi[0] * t[2], qi[0] * t[1] - qi[1] * t[0]};
    for (float &v : uv) v += v;
    const float cx[3] = {qi[1] * uv[2] - qi[2] * uv[1], qi[2] * uv[0] - qi[0] * uv[2], qi[0] * uv[1] - qi[1] * uv[0]};
    float ti[3];
    for (int k = 0; k < 3; k++) ti[k] = -((t[k] + qi[3] * uv[k]) + cx[k]);
    se3f_as7(qi, ti, inv7);
    return 0;
}

extern "C" int deftri_debug_nelder_mead(deftri_objective_fn f, void *user, int32_t n, double *x, const double *lb,
                                        const double *ub, double xtol_rel, double xtol_abs, int32_t maxeval,
                                        double *minf, int32_t *nevals, int32_t *result) {
    if (!f || !x || !lb || !ub || n < 0 || n > 8 || !minf || !nevals || !result) return DEFTRI_E_ARG;
    for (int i = 0; i < n; i++)
        if (x[i] < lb[i] || x[i] > ub[i]) return DEFTRI_E_ARG;            // NLOPT_INVALID_ARGS
    int ne = 0;
    double mf = 0.0;
    *result = nelder_mead([&](const double *xx) { return f(xx, n, user); }, n, x, lb, ub, xtol_rel, xtol_abs, maxeval,
                          mf, ne);
    *minf = mf;
    *nevals = ne;
    return 0;
}

namespace {

// the mutable part of a Map clone: every keyframe's slot positions and depth scale, in the clone's
// keyframe order; `view` is a deftri_map over them plus the source's read-only arrays, with an empty
// global table (Map::clone does not copy mGTransformation_) and T_g's start at the identity
struct MapClone {
    std::vector<deftri_keyframe> kfs;
    std::vector<std::vector<float>> pos;
    deftri_map view{};
    // Map::clone of `m`: keyframes re-inserted in m's iteration order
    void from(const deftri_map &m) {
        std::vector<int64_t> ids(m.n_keyframes), order;
        for (int k = 0; k < m.n_keyframes; k++) ids[k] = m.keyframes[k].id;
        unordered_order(ids.data(), m.n_keyframes, order);
        kfs.resize(m.n_keyframes);
        pos.resize(m.n_keyframes);
        for (int k = 0; k < m.n_keyframes; k++) {
            int src = 0;
            while (m.keyframes[src].id != order[k]) src++;
            kfs[k] = m.keyframes[src];
            pos[k].assign(m.keyframes[src].point_pos, m.keyframes[src].point_pos + 3 * (size_t)m.keyframes[src].n_slots);
            kfs[k].point_pos = pos[k].data();
        }
        view = m;
        view.keyframes = kfs.data();
        view.n_global = 0;
        view.globals = nullptr;
        const double identity[7] = {0, 0, 0, 1, 0, 0, 0};
        std::memcpy(view.global_t, identity, sizeof(identity));
    }
};

void table_insert(std::vector<deftri_global_entry> &g, int64_t a, int64_t b, const double t[7]) {
    for (auto &e : g)
        if (e.kf1 == a && e.kf2 == b) { std::memcpy(e.t, t, sizeof(e.t)); return; }
    deftri_global_entry e{};
    e.kf1 = a;
    e.kf2 = b;
    std::memcpy(e.t, t, sizeof(e.t));
    g.push_back(e);
}

}  // namespace

extern "C" int deftri_deformation_optimization(deftri_ctx *ctx, deftri_map *map, const deftri_deformation_params *prm,
                                               deftri_deformation_report *rep) {
    if (!ctx || !map || !prm || !rep || map->n_keyframes < 2 || !map->keyframes) return DEFTRI_E_ARG;
    if (prm->selection != 0 && prm->selection != 1) return DEFTRI_E_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    deftri_deformation_eval *evals = rep->evals;
    const int32_t max_evals = rep->max_evals;
    std::memset(rep, 0, sizeof(*rep));
    rep->evals = evals;
    rep->max_evals = max_evals;
    double w[3] = {prm->rep, prm->global, prm->arap};
    if (prm->selection == 1)
        for (int k = 0; k < 3; k++)
            if (w[k] < prm->lb[k] || w[k] > prm->ub[k]) return DEFTRI_E_ARG;   // NLOPT_INVALID_ARGS
    // the map's global table, which this loop owns from here on (the caller's array is read-only)
    std::vector<deftri_global_entry> table(map->globals, map->globals + std::max(map->n_global, 0));
    const deftri_global_entry *caller_globals = map->globals;
    const int32_t caller_n_global = map->n_global;
    MapClone base, eval;
    double update = 100.0;
    int rc = 0;
    int i = 1;
    for (; i <= prm->n_optimizations && update >= 0.0001 * prm->n_map_points; i++) {
        if (prm->selection == 1) {
            base.from(*map);                                   // optData.pMap = pMap->clone()
            int nev = 0, ev_round = 0;
            double minf = INFINITY;
            auto objective = [&](const double *x) -> double {  // outerObjective
                if (rc) return INFINITY;
                eval.from(base.view);                          // pData->pMap->clone()
                double upd = 0.0;
                int r = deftri_arap_optimization(ctx, &eval.view, x[0], x[1], x[2], prm->alpha, prm->beta, prm->depth_error,
                                                 prm->n_iterations, &upd, nullptr);
                deftri_pixels_error pe{};
                if (!r) r = deftri_pixels_stand_dev(ctx, &eval.view, &pe);
                if (r) { rc = r; return INFINITY; }
                rep->arap_calls++;
                // nloptOptimization.cc:31-33: pow(log(desvc), 2) — +inf at 0, NaN for a NaN deviation
                const double fv = std::pow(std::log(pe.desvc1), 2) + std::pow(std::log(pe.desvc2), 2);
                ev_round++;
                if (evals && rep->n_evals < max_evals) {
                    deftri_deformation_eval &e = evals[rep->n_evals];
                    e.round = i;
                    e.eval = ev_round;
                    std::memcpy(e.x, x, sizeof(e.x));
                    e.f = fv;
                }
                rep->n_evals++;
                return fv;
            };
            rep->nlopt_result = nelder_mead(objective, 3, w, prm->lb, prm->ub, prm->xtol_rel, prm->xtol_abs, prm->maxeval,
                                            minf, nev);
            if (rc) break;
            rep->minf = minf;
            // nlopt::opt::optimize throws on a failure code (the reference stops there, before :525)
            if (rep->nlopt_result < 0) {
                rc = DEFTRI_E_SEARCH;
                break;
            }
        }
        // arapOptimization on the map itself; positions and depth scales written back in place
        map->n_global = (int32_t)table.size();
        map->globals = table.data();
        rc = deftri_arap_optimization(ctx, map, w[0], w[1], w[2], prm->alpha, prm->beta, prm->depth_error,
                                      prm->n_iterations, &update, nullptr);
        map->globals = caller_globals;
        map->n_global = caller_n_global;
        if (rc) break;
        rep->arap_calls++;
        // pMap->insertGlobalKeyFramesTransformation(0, 1, T) (:1007: KF ids 0 and 1 whatever the map's)
        double fwd[7], inv[7];
        deftri_global_insert(map->global_t, fwd, inv);
        table_insert(table, 0, 1, fwd);
        table_insert(table, 1, 0, inv);
        if (i - 1 < 64) {
            rep->round_update[i - 1] = update;
            std::memcpy(rep->round_weights[i - 1], w, sizeof(w));
        }
    }
    rep->rounds = i - 1;
    std::memcpy(rep->weights, w, sizeof(w));
    rep->update = update;
    rep->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}
