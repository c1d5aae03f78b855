/* A compiled C consumer of include/deftri.h (no ctypes): what a reference-side adapter does around
   arapOptimization (g2oBundleAdjustment.cc:608-1008), on a deterministic two-keyframe scene.
     1. deftri_sim_two_view: the reference's simulated keypoints / depths / poses (SLAM.cc:223-338)
     2. fill two deftri_keyframe records slot by slot (MapPoint ids, positions, observation index,
        keypoints, octaves, depths, the Frame.cc:61-75 sigma table) and a deftri_map
     3. host-only context: deftri_arap_build_graph, deftri_problem_analyse, deftri_plan_stats
     4. with "gpu": deftri_arap_optimization (device LM + write-back), deftri_pixels_stand_dev
   Prints one "key value" per line for tests/test_c_consumer.py. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "deftri.h"

#define N 400

static int check(int rc, const char *what, deftri_ctx *ctx) {
    if (rc != 0) {
        fprintf(stderr, "%s failed: %d %s\n", what, rc, ctx ? deftri_last_error(ctx) : "");
        exit(1);
    }
    return rc;
}

int main(int argc, char **argv) {
    const int use_gpu = argc > 1 && strcmp(argv[1], "gpu") == 0;
    printf("abi %d\n", deftri_abi_version());
    /* a planar cloud like create_data.py's (deterministic grid + wobble), 20 cm in front */
    static float orig[3 * N], moved[3 * N];
    for (int i = 0; i < N; i++) {
        const float gx = (float)(i % 20) - 9.5f, gy = (float)(i / 20) - 9.5f;
        orig[3 * i] = 0.004f * gx + 0.0003f * sinf(1.7f * i);
        orig[3 * i + 1] = 0.004f * gy + 0.0003f * cosf(2.3f * i);
        orig[3 * i + 2] = 0.2f + 0.002f * sinf(0.3f * gx) * cosf(0.2f * gy);
        moved[3 * i] = orig[3 * i] + 0.0005f * sinf(0.9f * i);
        moved[3 * i + 1] = orig[3 * i + 1] + 0.0025f;
        moved[3 * i + 2] = orig[3 * i + 2] + 0.0005f * cosf(1.1f * i);
    }
    const float c1[3] = {-0.10f, 0.02f, 0.12f}, c2[3] = {0.14f, 0.01f, 0.06f};
    const float kb8[8] = {458.654f, 457.296f, 367.215f, 248.375f, 0, 0, 0, 0};
    static float uv1[2 * N], uv2[2 * N], d1[N], d2[N];
    float pose1[7], pose2[7];
    check(deftri_sim_two_view(N, orig, moved, c1, c2, kb8, kb8, 1.0f, 1, 3.0f, 0.4f, 1.7f, uv1, uv2, d1, d2,
                              pose1, pose2), "deftri_sim_two_view", NULL);
    printf("uv1_0 %.3f %.3f\n", uv1[0], uv1[1]);
    printf("d2_0 %.9g\n", d2[0]);

    /* Frame.cc:61-75: 8 octaves x 1.2 */
    float inv_sigma2[8], sf = 1.0f;
    for (int o = 0; o < 8; o++) { inv_sigma2[o] = 1.0f / (sf * sf); sf *= 1.2f; }
    /* the keyframes, as the adapter fills them from KeyFrame::getMapPoints() etc.  MapPoints are
       the perturbed ground truth (a triangulation stand-in); every slot is observed at its index */
    static int64_t ids[2][N];
    static float pos[2][3 * N];
    static int32_t obs[2][N], octv[2][N];
    deftri_keyframe kfs[2];
    const float *uv[2] = {uv1, uv2}, *dep[2] = {d1, d2}, *pose[2] = {pose1, pose2}, *src[2] = {orig, moved};
    for (int k = 0; k < 2; k++) {
        memset(&kfs[k], 0, sizeof(kfs[k]));
        kfs[k].id = k;
        for (int q = 0; q < 7; q++) kfs[k].pose[q] = pose[k][q];
        for (int q = 0; q < 8; q++) kfs[k].kb8[q] = kb8[q];
        kfs[k].n_scales = 8;
        kfs[k].inv_sigma2 = inv_sigma2;
        kfs[k].depth_scale = 1.0;
        kfs[k].n_slots = N;
        for (int i = 0; i < N; i++) {
            ids[k][i] = 2 * i + k;
            for (int c = 0; c < 3; c++) pos[k][3 * i + c] = src[k][3 * i + c] + 0.001f * sinf(3.1f * i + c + k);
            obs[k][i] = i;
            octv[k][i] = 0;
        }
        kfs[k].point_id = ids[k];
        kfs[k].point_pos = pos[k];
        kfs[k].obs_index = obs[k];
        kfs[k].kp_uv = uv[k];
        kfs[k].kp_octave = octv[k];
        kfs[k].depth = dep[k];
        kfs[k].n_obs = N;
    }
    /* the reference's unordered_map order: reverse insertion (KF 1, KF 0) */
    deftri_keyframe ordered[2] = {kfs[1], kfs[0]};
    deftri_map map;
    memset(&map, 0, sizeof(map));
    map.n_keyframes = 2;
    map.keyframes = ordered;
    map.global_t[3] = 1.0;
    map.n_global = 0;
    map.globals = NULL;

    deftri_ctx *host = NULL;
    check(deftri_ctx_create(-1, &host), "deftri_ctx_create(-1)", NULL);
    const deftri_problem_desc *desc = NULL;
    check(deftri_arap_build_graph(host, &map, 1.0, 2e5, 0.003f, &desc), "deftri_arap_build_graph", host);
    printf("graph %d %d %d %d %d %d\n", desc->n_points, desc->n_pairs, desc->n_scales, desc->n_rep, desc->n_depth,
           desc->n_arap);
    check(deftri_problem_analyse(host, desc), "deftri_problem_analyse", host);
    deftri_report st;
    check(deftri_plan_stats(host, &st), "deftri_plan_stats", host);
    printf("plan %lld %lld %.6f %d %d\n", (long long)st.n_unknowns, (long long)st.nnz_factor, st.factor_flops / 1e6,
           st.n_fronts, st.n_levels);
    if (use_gpu) {
        deftri_ctx *gpu = NULL;
        check(deftri_ctx_create(0, &gpu), "deftri_ctx_create(0)", NULL);
        deftri_pixels_error e0, e1;
        check(deftri_pixels_stand_dev(gpu, &map, &e0), "deftri_pixels_stand_dev", gpu);
        deftri_report rep;
        double upd = 0.0;
        check(deftri_arap_optimization(gpu, &map, 1.0, 50.0, 2e5, 0.0, 0.0, 0.003f, 10, &upd, &rep),
              "deftri_arap_optimization", gpu);
        check(deftri_pixels_stand_dev(gpu, &map, &e1), "deftri_pixels_stand_dev", gpu);
        printf("lm %d %d %.9e %.9e\n", rep.iterations, rep.trials_total, rep.chi2_initial, rep.chi2_final);
        printf("update %.9e\n", upd);
        printf("scales %.9e %.9e\n", ordered[0].depth_scale, ordered[1].depth_scale);
        printf("desv %.6f %.6f\n", e0.desv, e1.desv);
        printf("tg %.9e %.9e %.9e\n", map.global_t[4], map.global_t[5], map.global_t[6]);
        deftri_ctx_destroy(gpu);
    }
    deftri_ctx_destroy(host);
    printf("ok\n");
    return 0;
}
