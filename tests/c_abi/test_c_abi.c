/* test_c_abi.c — the C-ABI of include/dofs.h from plain C99 (gcc -std=c99 -Wall -Wextra -Werror -pedantic):
 * the header compiles as C, the library links, and the device-free entry points behave as the reference's
 * own tests expect (cpp/tests/test_liftig_3d.cpp:69-89 for get_intersect; get_mat / get_mat_upper literals
 * of :183-185). A device context is created only when argv[1] is "device" (the GPU box). */
#include <math.h>
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "dofs.h"

static int fails = 0;
#define CHECK(c)                                                      \
    do {                                                              \
        if (!(c)) {                                                   \
            fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                  \
        }                                                             \
    } while (0)

int main(int argc, char** argv) {
    dofs_params p;
    dofs_flow_params fp;
    float persp[9], inv[9], up[27], r[2];
    const float a1[2] = {1, 1}, a2[2] = {4, 4}, b1[2] = {1, 8}, b2[2] = {2, 4};
    const float c1[2] = {1, 1}, c2[2] = {1, 2}, d1[2] = {3, 3}, d2[2] = {3, 4};
    unsigned char bgr[6] = {10, 20, 30, 255, 255, 255}, gray[2] = {0, 0};

    CHECK(dofs_abi_version() == DOFS_ABI_VERSION);
    CHECK(sizeof(dofs_edge) == 16 && offsetof(dofs_edge, weight) == 8); /* graph.hpp:13-17 layout */

    dofs_default_params(&p);
    CHECK(p.blur_sigma == 3.0 && p.neighbor == 8 && p.min_size == 500);
    CHECK(p.score_threshold == 0.3 && p.overlay_min_score == 0.7);
    CHECK(p.obj_size[2][0] == 370 && p.obj_size[2][1] == 180);

    CHECK(dofs_calib(persp, inv, up) == DOFS_OK);
    CHECK(persp[8] == 1.0f && inv[8] == 1.0f && up[26] == 1.0f);
    CHECK(dofs_calib(NULL, inv, up) == DOFS_ERR_INVALID_ARG);

    dofs_intersect(a1, a2, b1, b2, r); /* test_liftig_3d.cpp:69-78 */
    CHECK(fabsf(r[0] - 2.4f) < 1e-2f && fabsf(r[1] - 2.4f) < 1e-2f);
    dofs_intersect(c1, c2, d1, d2, r); /* :80-89: parallel lines -> NaN */
    CHECK(isnan(r[0]) && isnan(r[1]));

    { /* get_upper_face_simple (lifting_3d.cpp:261-288): every corner lifted by min(lf[1].y, lf[2].y) - ymin */
        const int32_t box[4] = {10, 20, 60, 90};
        const float lf[8] = {12, 80, 15, 50, 55, 45, 58, 85};
        float uf[8];
        double os[2];
        dofs_upper_face_simple(box, lf, uf);
        CHECK(uf[0] == 12.0f && uf[1] == 80.0f - 25.0f && uf[5] == 45.0f - 25.0f);
        dofs_upper_face(box, lf, uf); /* get_upper_face (:290-348): E = (lf[2].x, ymin) */
        CHECK(uf[4] == 55.0f && uf[5] == 20.0f);
        CHECK(dofs_obj_size(0, os) == DOFS_OK && os[0] == 258.0 && os[1] == 84.0); /* :524-528 */
        CHECK(dofs_obj_size(3, os) == DOFS_ERR_INVALID_ARG);
    }

    dofs_default_flow_params(&fp);
    CHECK(fp.pyr_scale == 0.5 && fp.levels == 3 && fp.winsize == 15 && fp.iterations == 3);
    CHECK(fp.poly_n == 5 && fp.poly_sigma == 1.2 && fp.flags == 0);

    dofs_bgr_to_gray(bgr, 1, 2, 0, gray); /* cvtColor BGR2GRAY fixed point: white stays 255 */
    CHECK(gray[1] == 255);

    CHECK(dofs_segment(NULL, NULL, 1, 1, 0, persp, inv, up, &p, NULL) == DOFS_ERR_INVALID_ARG);
    CHECK(strlen(dofs_last_error(NULL)) > 0);

    if (argc > 1 && strcmp(argv[1], "device") == 0) {
        /* build_graph + segment_graph of a 4x3 field through the C-ABI on the device */
        float flow[12 * 2];
        dofs_edge edges[64];
        int64_t n = 0;
        int32_t labels[12], leaf[12];
        dofs_result res;
        dofs_ctx* ctx = dofs_create(0);
        int i;
        CHECK(ctx != NULL);
        if (ctx) {
            for (i = 0; i < 24; ++i) flow[i] = (float)((i * 7) % 5) * 0.25f;
            CHECK(dofs_build_graph(ctx, flow, 3, 4, 0, 1, edges, 64, &n) == DOFS_OK);
            CHECK(n == 4 * 12 - 3 * 4 - 3 * 3 + 2); /* E = 4WH - 3W - 3H + 2 */
            for (i = 1; i < (int)n; ++i) CHECK(edges[i - 1].weight <= edges[i].weight);
            memset(&res, 0, sizeof(res));
            res.labels = labels;
            res.leaf_order = leaf;
            CHECK(dofs_segment_graph(ctx, flow, 3, 4, 0, edges, n, persp, inv, up, &p, &res) == DOFS_OK);
            CHECK(res.stats.n_merges == 11 && res.stats.n_edges == n);
            { /* the Forest after the loop: one final root holding the whole 4x3 frame's box */
                int32_t rb[5];
                double sc[12];
                int64_t nr = 0;
                CHECK(dofs_final_roots(ctx, -1, 0, rb, 5, &nr) == DOFS_OK && nr == 1);
                CHECK(rb[1] == 0 && rb[2] == 0 && rb[3] == 3 && rb[4] == 2);
                CHECK(dofs_segment_scores(ctx, -1, 0, sc, 12) == DOFS_OK);
                CHECK(dofs_segment_scores(ctx, -1, 0, sc, 11) == DOFS_ERR_CAPACITY);
            }
            { /* per-merge events: refused on a batch issued without dofs_keep_events (the default), returned
               * for the batches issued after it */
                dofs_event ev[11];
                CHECK(dofs_events(ctx, 0, ev, 11) == DOFS_ERR_INVALID_ARG);
                CHECK(dofs_keep_events(ctx, 1) == DOFS_OK);
                CHECK(dofs_segment_graph(ctx, flow, 3, 4, 0, edges, n, persp, inv, up, &p, &res) == DOFS_OK);
                CHECK(dofs_events(ctx, 0, ev, 11) == DOFS_OK);
            }
            dofs_destroy(ctx);
        }
    }
    if (fails) return 1;
    printf("c_abi ok\n");
    return 0;
}
