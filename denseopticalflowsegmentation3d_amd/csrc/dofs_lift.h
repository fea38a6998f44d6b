// dofs_lift.h — 2D box → 3D box back-projection (get_bottom_variants) for one candidate event.
//
// Restates cpp/src/lifting_3d.cpp:63-439 and the class loop of get_score (cpp/src/graph.cpp:241-270)
// with the reference's exact float/double operation order (OpenCV Point2f operator semantics,
// no FMA: this file must be compiled with -ffp-contract=off). Transcendentals (atan2, sin, cos in
// double) use the device math library, which may differ from glibc by an ulp.
#pragma once
// DOFS_HDM: host+device qualifier for pure math (no atomics), defined by the including TU.

#include "dofs_common.h"

namespace dofs {

struct P2 {
    float x, y;
};

DOFS_HDM inline P2 mk(float x, float y) {
    P2 r;
    r.x = x;
    r.y = y;
    return r;
}
DOFS_HDM inline P2 p_add(P2 a, P2 b) { return mk(a.x + b.x, a.y + b.y); }
DOFS_HDM inline P2 p_sub(P2 a, P2 b) { return mk(a.x - b.x, a.y - b.y); }
DOFS_HDM inline P2 p_dmul(double a, P2 b) { return mk((float)((double)b.x * a), (float)((double)b.y * a)); }
DOFS_HDM inline P2 p_ddiv(P2 a, double b) { return mk((float)((double)a.x / b), (float)((double)a.y / b)); }
DOFS_HDM inline P2 p_idiv(P2 a, int b) { return mk(a.x / (float)b, a.y / (float)b); }
DOFS_HDM inline P2 p_imul(int a, P2 b) { return mk(b.x * (float)a, b.y * (float)a); }
DOFS_HDM inline double p_norm(P2 a) { return sqrt((double)a.x * (double)a.x + (double)a.y * (double)a.y); }
DOFS_HDM inline P2 p_iv(P2 a) { return mk(a.x, -a.y); }

// lifting_3d.cpp:63-89
DOFS_HDM inline P2 intersect(P2 A, P2 B, P2 C, P2 D) {
    float a1 = B.y - A.y;
    float b1 = A.x - B.x;
    float c1 = a1 * A.x + b1 * A.y;
    float a2 = D.y - C.y;
    float b2 = C.x - D.x;
    float c2 = a2 * C.x + b2 * C.y;
    float det = a1 * b2 - a2 * b1;
    if ((double)__builtin_fabsf(det) < 1e-9) return mk(__builtin_nanf(""), __builtin_nanf(""));
    return mk((b2 * c1 - b1 * c2) / det, (a1 * c2 - a2 * c1) / det);
}

// lifting_3d.cpp:112-121 (row-major Matx33f)
DOFS_HDM inline P2 warp(P2 p, const float* m) {
    float px = (m[0] * p.x + m[1] * p.y + m[2]) / (m[6] * p.x + m[7] * p.y + m[8]);
    float py = (m[3] * p.x + m[4] * p.y + m[5]) / (m[6] * p.x + m[7] * p.y + m[8]);
    return mk(px, py);
}

// lifting_3d.cpp:162-217; false <=> the reference returns an empty corner vector.
// co/si = cos(orient), sin(orient) (the reference evaluates them at every use; same values).
DOFS_HDM inline bool bottom(const P2 wc[4], double co, double si, double w, double h, double* err, P2 out[4]) {
    const float inf = __builtin_inff();
    P2 a0 = p_iv(wc[0]), a1 = p_iv(wc[1]), a2 = p_iv(wc[2]), a3 = p_iv(wc[3]);
    P2 k = intersect(a3, mk((float)(a3.x + co), (float)(a3.y + si)), a0, a1);
    if (k.x == inf || k.y == inf) return false;
    double l = p_norm(p_sub(a3, k));
    if (l == 0) return false;
    P2 c = p_ddiv(p_add(p_dmul(l - w, a0), p_dmul(w, a3)), l);
    P2 b = intersect(c, mk((float)(c.x + co), (float)(c.y + si)), a0, a1);
    if (b.x == inf) return false;
    double ew = p_norm(p_sub(c, b));
    double error_w = (ew < w) ? ew / w : w / ew;
    P2 d = intersect(c, mk((float)(c.x - si), (float)(c.y + co)), a3, a2);
    if (d.x == inf) return false;
    double el = p_norm(p_sub(c, d));
    double error_l = (el < h) ? el / h : h / el;
    P2 center = p_idiv(p_add(b, d), 2);
    P2 f = p_sub(p_imul(2, center), c);
    out[0] = p_iv(c);
    out[1] = p_iv(b);
    out[2] = p_iv(f);
    out[3] = p_iv(d);
    *err = error_w * error_l;
    return true;
}

// lifting_3d.cpp:219-253 (integer-division centre, unit direction, two warps, atan2)
DOFS_HDM inline double motion_direction(P2 dir, const int box[4], const float* persp) {
    int sum_x = box[0] + box[2];
    int sum_y = box[1] + box[3];
    P2 center = mk((float)(sum_x / 2), (float)(sum_y / 2));
    P2 nd = p_ddiv(dir, p_norm(dir));
    P2 t1 = warp(center, persp);
    P2 t2 = warp(p_add(center, nd), persp);
    double v_x = t2.x - t1.x;
    double v_y = t1.y - t2.y;
    return atan2(v_y, v_x);
}

// get_upper_face, lifting_3d.cpp:290-348 (the catch branch :325-338 is unreachable: get_intersect
// returns NaN for parallel lines instead of throwing, :77-82)
DOFS_HDM inline void upper_face(const int box[4], const P2 lf[4], P2 uf[4]) {
    uf[2] = p_sub(lf[2], mk(0.0f, lf[2].y - (float)box[1]));
    P2 right_van = intersect(lf[1], lf[2], lf[0], lf[3]);
    uf[1] = intersect(uf[2], right_van, mk((float)box[0], (float)box[1]), mk((float)box[0], (float)box[3]));
    P2 left_van = intersect(lf[2], lf[3], lf[0], lf[1]);
    uf[3] = intersect(uf[2], left_van, mk((float)box[2], (float)box[1]), mk((float)box[2], (float)box[3]));
    uf[0] = intersect(left_van, uf[1], right_van, uf[3]);
}

// get_upper_face_simple, lifting_3d.cpp:261-288 (not called by the path; public in lifting_3d.hpp:23-24).
// h_min = 0 - ymin + std::min(lf[1].y, lf[2].y) in double (xmin, ymin as double; h_max is unused), then
// every corner minus cv::Point2f(0, h_min): the double narrowed to float, the subtraction in float.
DOFS_HDM inline void upper_face_simple(const int box[4], const P2 lf[4], P2 uf[4]) {
    const double ymin = box[1];
    const float lo = lf[2].y < lf[1].y ? lf[2].y : lf[1].y;  // std::min(a, b) == (b < a) ? b : a
    const double h_min = 0 - ymin + (double)lo;
    const float h = (float)h_min;
    for (int k = 0; k < 4; ++k) uf[k] = p_sub(lf[k], mk(0.0f, h));
}

// getObjSize / get_obj_size (lifting_3d.cpp:255-259, :524-528): the class BEV sizes (length, width).
DOFS_HDM inline bool obj_size_of(int cls, int out[2]) {
    if (cls < 0 || cls > 2) return false;  // the reference indexes its 3-entry vector unchecked
    const int sz[3][2] = {{258, 84}, {349, 165}, {370, 180}};
    out[0] = sz[cls][0];
    out[1] = sz[cls][1];
    return true;
}

struct LiftMats {
    float persp[9];
    float inv[9];
    float inv_upper[27];
    int obj_size[3][2];
};

// Class-independent part of get_bottom_variants for one box: motion angle (:358, computed from the
// box and direction only), its cos/sin, and the BEV corners ps_bev (:373-378).
struct LiftPre {
    double ang, co, si;
    P2 ps_bev[4];
};

DOFS_HDM inline void lift_pre(P2 dir, const int box[4], const LiftMats& L, LiftPre* pre) {
    pre->ang = motion_direction(dir, box, L.persp);
    pre->co = cos(pre->ang);
    pre->si = sin(pre->ang);
    const P2 ps[4] = {mk((float)box[0], (float)box[3]), mk((float)box[0], (float)box[1]),
                      mk((float)box[2], (float)box[1]), mk((float)box[2], (float)box[3])};
    for (int i = 0; i < 4; ++i) pre->ps_bev[i] = warp(ps[i], L.persp);
}

// get_bottom_variants (lifting_3d.cpp:350-439) for one class. With s == NULL only the errors are
// produced (the scoring pass needs (w_error + h_error)/2 and validity only).
DOFS_HDM inline bool bottom_variant(const LiftPre& pre, const int box[4], const LiftMats& L, int cls,
                                    double* w_error, double* h_error, dofs_solution* s) {
    double err = 0.0;
    P2 corners[4];
    if (!bottom(pre.ps_bev, pre.co, pre.si, (double)L.obj_size[cls][0], (double)L.obj_size[cls][1], &err,
                corners)) {
        if (s) {
            s->cls = cls;
            s->valid = 0;
            s->w_error = 0.0;
            s->h_error = 0.0;
            s->orient = 0.0;
            for (int i = 0; i < 4; ++i) {
                s->ps_bev[i][0] = s->ps_bev[i][1] = 0.0f;
                s->lower_face[i][0] = s->lower_face[i][1] = 0.0f;
                s->upper_face[i][0] = s->upper_face[i][1] = 0.0f;
                s->rectangle[i][0] = s->rectangle[i][1] = 0.0f;
            }
        }
        return false;
    }
    P2 untop[4];
    for (int i = 0; i < 4; ++i) untop[i] = warp(corners[i], L.inv);
    P2 uf[4];
    upper_face(box, untop, uf);
    P2 expected_edge = warp(corners[0], L.inv_upper + 9 * cls);
    double expected_h = p_norm(p_sub(untop[0], expected_edge));
    double computed_h = p_norm(p_sub(uf[0], untop[0]));
    *w_error = err;
    *h_error = (computed_h < expected_h) ? (computed_h / expected_h) : (expected_h / computed_h);
    if (s) {
        s->cls = cls;
        s->valid = 1;
        for (int i = 0; i < 4; ++i) {
            s->ps_bev[i][0] = pre.ps_bev[i].x;
            s->ps_bev[i][1] = pre.ps_bev[i].y;
            s->lower_face[i][0] = untop[i].x;
            s->lower_face[i][1] = untop[i].y;
            s->upper_face[i][0] = uf[i].x;
            s->upper_face[i][1] = uf[i].y;
            s->rectangle[i][0] = corners[i].x;
            s->rectangle[i][1] = corners[i].y;
        }
        s->w_error = err;
        s->h_error = *h_error;
        s->orient = pre.ang;
    }
    return true;
}

DOFS_HDM inline void lift_one(P2 dir, const int box[4], const LiftMats& L, int cls, dofs_solution* s) {
    LiftPre pre;
    lift_pre(dir, box, L, &pre);
    if (__builtin_isinf(pre.ang)) {  // :360-364 (unreachable: atan2 is finite)
        s->cls = -1;
        s->valid = 0;
        s->w_error = -1.0;
        s->h_error = -1.0;
        s->orient = 0.0;
        return;
    }
    double we, he;
    bottom_variant(pre, box, L, cls, &we, &he, s);
}

// get_score (graph.cpp:241-270): best class by (w_error + h_error)/2, -1 when no rectangle.
// best may be NULL when only the score and class are needed.
DOFS_HDM inline double score_event(P2 dir, const int box[4], const LiftMats& L, int* best_cls, dofs_solution* best) {
    LiftPre pre;
    lift_pre(dir, box, L, &pre);
    double max_score = -1.0;
    *best_cls = -1;
    for (int cls = 0; cls < 3; ++cls) {
        double we, he;
        if (bottom_variant(pre, box, L, cls, &we, &he, nullptr) && max_score < (we + he) / 2) {
            max_score = (we + he) / 2;
            *best_cls = cls;
        }
    }
    if (best && *best_cls >= 0) {
        double we, he;
        bottom_variant(pre, box, L, *best_cls, &we, &he, best);
    }
    return max_score;
}

}  // namespace dofs
