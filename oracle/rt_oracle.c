/*
 * rt_oracle.c — CPU restatement of the reference trace path (checker / CPU baseline).
 *
 * TEST INFRASTRUCTURE ONLY — see rt_oracle.h.  PARITY UNPINNED (no buildable reference,
 * no reference fixtures); pinned by analytic known-answer tests.
 *
 * Every arithmetic expression keeps the reference's evaluation order so that a build with
 * -ffp-contract=off reproduces the reference's float semantics: e.g. Vec3::dot sums
 * 0.0f + x*x' + y*y' + z*z' left to right (include/Basic/Vec3.cuh:113-119), unitVector
 * multiplies by 1/length (Vec3.cuh:129-137).  Float libm overloads are used where the
 * reference calls cos/sin/tan/sqrt/pow on floats (CUDA / MSVC float overloads).
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define FZERO 1e-6f                       /* FLOAT_ZERO_VALUE, Global.cuh:147 */
#define ORACLE_PI ((float)M_PI)           /* PI, Global.cuh:149 */
#define BLAS_LEAF 4u                      /* BLAS.cuh:17 */
#define TLAS_LEAF 2u                      /* TLAS.cuh:22 */
#define TMIN 0.001f                       /* Kernel.cu:66 */

/* ------------------------------------------------------------------------------------
 * L1 value types: Vec3 / Point3 / Color3 (include/Basic/ *.cuh)
 * ---------------------------------------------------------------------------------- */
typedef struct { float x, y, z; } V3;

static inline V3 v3(float x, float y, float z) { V3 r = {x, y, z}; return r; }
static inline float vget(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline void vset(V3 *a, int i, float f) { if (i == 0) a->x = f; else if (i == 1) a->y = f; else a->z = f; }
static inline V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }    /* Vec3.cuh:59-66 */
static inline V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }    /* Vec3.cuh:67-74 */
static inline V3 vscale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }     /* Vec3.cuh:77-84 */
static inline V3 vdivs(V3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }      /* Vec3.cuh:85-92 */
static inline V3 vneg(V3 a) { return v3(-a.x, -a.y, -a.z); }                         /* Vec3.cuh:46-48 */
static inline V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }    /* Color3.cuh:57-64 */
static inline float vdot(V3 a, V3 b) {                                                /* Vec3.cuh:113-119 */
    float s = 0.0f; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s;
}
static inline float vlen2(V3 a) {                                                     /* Vec3.cuh:101-107 */
    float s = 0.0f; s += a.x * a.x; s += a.y * a.y; s += a.z * a.z; return s;
}
static inline V3 vcross(V3 a, V3 b) {                                                 /* Vec3.cuh:120-126 */
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline V3 vunit(V3 a) {                                                        /* Vec3.cuh:129-137 */
    const float f = 1.0f / sqrtf(vlen2(a));
    return v3(a.x * f, a.y * f, a.z * f);
}
static inline float pdist(V3 a, V3 b) {                                               /* Point3.cuh:75-84 */
    float s = 0.0f;
    s += (a.x - b.x) * (a.x - b.x); s += (a.y - b.y) * (a.y - b.y); s += (a.z - b.z) * (a.z - b.z);
    return sqrtf(s);
}
static inline V3 fromrt(rt_vec3 a) { return v3(a.x, a.y, a.z); }
static inline rt_vec3 tort(V3 a) { rt_vec3 r = {a.x, a.y, a.z}; return r; }

/* Range (include/Util/Range.cuh:20-77) */
typedef struct { float min, max; } Range;
static inline int near_zero(float v) { return fabsf(v) < FZERO; }                    /* Global.cuh:172-174 */
static inline int f_equals(float a, float b) { return fabsf(a - b) < FZERO; }        /* Global.cuh:180-182 */
static inline int in_range(Range r, float v) {                                        /* Range.cuh:33-43 */
    const int eqmin = f_equals(v, r.min);
    const int eqmax = f_equals(v, r.max);
    if (eqmin) return 1;     /* leftClose  */
    if (eqmax) return 1;     /* rightClose */
    return v > r.min && v < r.max;
}
static inline float range_length(Range r) {                                          /* Range.cuh:60-66 */
    if (r.min >= r.max || f_equals(r.min, r.max)) return 0.0f;
    return r.max - r.min;
}
static inline Range range_expand(Range r, float e) {                                  /* Range.cuh:50-58 */
    if (e > 0.0f) { r.min -= e; r.max += e; } else { r.min += e; r.max -= e; }
    return r;
}
static inline float clampf_ref(float v, float lo, float hi) {                         /* Range.cuh:68-76 */
    if (v > hi) return hi; else if (v < lo) return lo; return v;
}

/* ------------------------------------------------------------------------------------
 * Pinned RNG contract (replaces cuRAND XORWOW seeded with clock64(), Kernel.cu:114).
 * ---------------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
#define GOLDEN64 0x9E3779B97F4A7C15ull
#define SUBMUL64 0xD1B54A32D192ED03ull
uint64_t oracle_rng_init(uint64_t seed, uint64_t sub, uint64_t off) {
    return mix64((seed * GOLDEN64) ^ ((sub + 1ull) * SUBMUL64) ^ off);
}
/* state holds key + ctr*GOLDEN64; uniform = ((mix64(state += GOLDEN64) >> 40) + 1) * 2^-24 */
float oracle_rng_uniform(uint64_t *state) {
    *state += GOLDEN64;
    const uint64_t x = mix64(*state);
    return (float)((x >> 40) + 1ull) * 0x1p-24f;
}
static inline float rnd(uint64_t *st) { return oracle_rng_uniform(st); }                /* Global.cuh:198-200 */
static inline float rnd_range(uint64_t *st, float mn, float mx) {                      /* Global.cuh:209-211 */
    return mn + (mx - mn) * rnd(st);
}

/* Vec3::randomSpaceVector (src/Basic/Vec3.cu:54-65) */
static V3 random_space_vector(uint64_t *st, float length) {
    V3 r; float l2;
    do {
        r.x = rnd_range(st, -1.0f, 1.0f);
        r.y = rnd_range(st, -1.0f, 1.0f);
        r.z = rnd_range(st, -1.0f, 1.0f);
        l2 = vlen2(r);
    } while (l2 < FZERO * FZERO);
    r = vunit(r);
    return vscale(r, length);
}
/* Vec3::randomPlaneVector (src/Basic/Vec3.cu:29-36) */
static V3 random_plane_vector(uint64_t *st, float maxlen) {
    float x, y;
    do {
        x = rnd_range(st, -1.0f, 1.0f);
        y = rnd_range(st, -1.0f, 1.0f);
    } while (x * x + y * y > maxlen * maxlen);
    return v3(x, y, 0.0f);
}

/* ------------------------------------------------------------------------------------
 * Matrix (include/Util/Matrix.cuh, src/Util/Matrix.cu): 5x5 storage, 1-based 4x4.
 * ---------------------------------------------------------------------------------- */
typedef struct { float d[5][5]; int row, col; } Mat;

static Mat mat_mul(const Mat *a, const Mat *b) {                                       /* Matrix.cu:71-86 */
    Mat r; memset(&r, 0, sizeof r); r.row = a->row; r.col = b->col;
    for (int i = 1; i <= r.row; i++)
        for (int j = 1; j <= r.col; j++) {
            float sum = 0.0f;
            for (int n = 1; n <= a->col; n++) sum += a->d[i][n] * b->d[n][j];
            r.d[i][j] = sum;
        }
    return r;
}
static Mat mat_transpose(const Mat *a) {                                               /* Matrix.cu:89-98 */
    Mat r; memset(&r, 0, sizeof r); r.row = a->col; r.col = a->row;
    for (int i = 1; i <= a->row; i++)
        for (int j = 1; j <= a->col; j++) r.d[j][i] = a->d[i][j];
    return r;
}
static int elim_bottom(float m[5][9]) {                                                /* Matrix.cu:5-45 */
    for (int i = 1; i < 5; i++) {
        float mainv = fabsf(m[i][i]);
        int maxrow = i;
        for (int p = i + 1; p < 5; p++)
            if (fabsf(m[p][i]) > mainv) { mainv = fabsf(m[p][i]); maxrow = p; }
        if (near_zero(mainv)) return 1;
        if (maxrow != i) {
            float tmp[9] = {0};
            for (int j = 1; j < 9; j++) tmp[j] = m[maxrow][j];
            for (int j = 1; j < 9; j++) m[maxrow][j] = m[i][j];
            for (int j = 1; j < 9; j++) m[i][j] = tmp[j];
        }
        for (int j = i + 1; j < 5; j++) {
            const float factor = m[j][i] / m[i][i];
            for (int k = i; k < 9; k++) m[j][k] -= factor * m[i][k];
        }
    }
    return 0;
}
static int elim_top(float m[5][9]) {                                                   /* Matrix.cu:46-68 */
    for (int i = 4; i >= 1; i--) {
        if (near_zero(m[i][i])) return near_zero(m[i][8]) ? 2 : 1;
        float factor = 1.0f / m[i][i];
        for (int p = i; p < 9; p++) m[i][p] *= factor;
        for (int j = i - 1; j >= 1; j--) {
            factor = m[j][i];
            for (int k = j; k < 9; k++) m[j][k] -= factor * m[i][k];
        }
    }
    return 0;
}
static Mat mat_inverse(const Mat *a) {                                                 /* Matrix.cu:101-130 */
    float m[5][9]; memset(m, 0, sizeof m);
    for (int i = 1; i < 5; i++) {
        for (int j = 1; j < 5; j++) m[i][j] = a->d[i][j];
        m[i][4 + i] = 1.0f;
    }
    if (elim_bottom(m) != 0 || elim_top(m) != 0) return *a;
    Mat r; memset(&r, 0, sizeof r); r.row = 4; r.col = 4;
    for (int i = 1; i < 5; i++)
        for (int j = 1; j < 5; j++) r.d[i][j] = m[i][4 + j];
    return r;
}
static Mat mat_ident4(void) { Mat r; memset(&r, 0, sizeof r); r.row = r.col = 4; for (int i = 1; i < 5; i++) r.d[i][i] = 1.0f; return r; }
static Mat mat_shift(V3 s) {                                                           /* Matrix.cu:183-193 */
    Mat r = mat_ident4(); r.d[1][4] = s.x; r.d[2][4] = s.y; r.d[3][4] = s.z; return r;
}
static Mat mat_scale(V3 s) {                                                           /* Matrix.cu:195-205 */
    Mat r = mat_ident4(); r.d[1][1] = s.x; r.d[2][2] = s.y; r.d[3][3] = s.z; return r;
}
static Mat mat_rot_axis(float degree, int axis) {                                      /* Matrix.cu:207-242 */
    const float theta = degree * ORACLE_PI / 180.0f;                                   /* Global.cuh:154-156 */
    Mat r = mat_ident4();
    const float c = cosf(theta), s = sinf(theta);
    if (axis == 0) { r.d[2][2] = c; r.d[2][3] = -s; r.d[3][2] = s; r.d[3][3] = c; }
    else if (axis == 1) { r.d[1][1] = c; r.d[1][3] = s; r.d[3][1] = -s; r.d[3][3] = c; }
    else { r.d[1][1] = c; r.d[1][2] = -s; r.d[2][1] = s; r.d[2][2] = c; }
    return r;
}
static Mat mat_rot(V3 deg) {                                                           /* Matrix.cu:244-249 */
    const Mat mx = mat_rot_axis(deg.x, 0), my = mat_rot_axis(deg.y, 1), mz = mat_rot_axis(deg.z, 2);
    const Mat t = mat_mul(&mx, &my);
    return mat_mul(&t, &mz);
}
/* (M * toMatrix(Point3)).toPoint() — Matrix.cuh:41-59 with w = 1 */
static V3 mat_point(const Mat *m, V3 p) {
    V3 r;
    for (int i = 1; i <= 3; i++) {
        float sum = 0.0f;
        sum += m->d[i][1] * p.x; sum += m->d[i][2] * p.y; sum += m->d[i][3] * p.z; sum += m->d[i][4] * 1.0f;
        vset(&r, i - 1, sum);
    }
    return r;
}
/* (M * toMatrix(Vec3)).toVector() — Matrix.cuh:28-39 with w = 0 */
static V3 mat_vector(const Mat *m, V3 v) {
    V3 r;
    for (int i = 1; i <= 3; i++) {
        float sum = 0.0f;
        sum += m->d[i][1] * v.x; sum += m->d[i][2] * v.y; sum += m->d[i][3] * v.z; sum += m->d[i][4] * 0.0f;
        vset(&r, i - 1, sum);
    }
    return r;
}

/* ------------------------------------------------------------------------------------
 * BoundingBox (include/AS/BoundingBox.cuh, src/AS/BoundingBox.cu)
 * ---------------------------------------------------------------------------------- */
typedef struct { Range r[3]; } Box;

static Box box_ensure(Box b) {                                                         /* BoundingBox.cuh:24-28 */
    for (int i = 0; i < 3; i++)
        if (range_length(b.r[i]) < FZERO) b.r[i] = range_expand(b.r[i], FZERO);
    return b;
}
static Box box_points(V3 p1, V3 p2) {                                                  /* BoundingBox.cuh:41-47 */
    Box b;
    for (int i = 0; i < 3; i++) {
        const float a = vget(p1, i), c = vget(p2, i);
        if (a < c) { b.r[i].min = a; b.r[i].max = c; } else { b.r[i].min = c; b.r[i].max = a; }
    }
    return box_ensure(b);
}
static Box box_merge(Box a, Box b) {                                                   /* BoundingBox.cuh:50-55, Range.cuh:24-26 */
    Box r;
    for (int i = 0; i < 3; i++) {
        r.r[i].min = a.r[i].min < b.r[i].min ? a.r[i].min : b.r[i].min;
        r.r[i].max = a.r[i].max > b.r[i].max ? a.r[i].max : b.r[i].max;
    }
    return r;
}
static Box box_transform(Box b, const Mat *m) {                                        /* BoundingBox.cu:4-32 */
    V3 mn = v3(INFINITY, INFINITY, INFINITY), mx = v3(-INFINITY, -INFINITY, -INFINITY);
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                const float x = (float)i * b.r[0].max + (1.0f - (float)i) * b.r[0].min;
                const float y = (float)j * b.r[1].max + (1.0f - (float)j) * b.r[1].min;
                const float z = (float)k * b.r[2].max + (1.0f - (float)k) * b.r[2].min;
                const V3 p = mat_point(m, v3(x, y, z));
                for (int l = 0; l < 3; l++) {
                    const float pv = vget(p, l);
                    if (pv < vget(mn, l)) vset(&mn, l, pv);       /* std::min(min, p) keeps min on ties */
                    if (vget(mx, l) < pv) vset(&mx, l, pv);       /* std::max(max, p) keeps max on ties */
                }
            }
    return box_points(mn, mx);
}

typedef struct { V3 o, d; } Ray;

/* BoundingBox::hit (src/AS/BoundingBox.cu:34-72) */
static int box_hit(const Box *b, const Ray *ray, Range check, float *t) {
    Range cur = check;
    for (int axis = 0; axis < 3; axis++) {
        const Range ar = b->r[axis];
        const float q = vget(ray->o, axis);
        const float d = vget(ray->d, axis);
        if (fabsf(d) < FZERO) {
            if (q < ar.min || q > ar.max) return 0;
            continue;
        }
        const float t1 = (ar.min - q) / d;
        const float t2 = (ar.max - q) / d;
        if (t1 < t2) {
            if (t1 > cur.min) cur.min = t1;
            if (t2 < cur.max) cur.max = t2;
        } else {
            if (t2 > cur.min) cur.min = t2;
            if (t1 < cur.max) cur.max = t1;
        }
        if (cur.min >= cur.max) return 0;
    }
    *t = cur.min;
    return 1;
}

/* ------------------------------------------------------------------------------------
 * Primitives (include/Geometry, src/Geometry)
 * ---------------------------------------------------------------------------------- */
typedef struct { V3 center; float radius; uint32_t mtype, midx; } Sph;
typedef struct { V3 q, u, v; float area; V3 n; float d; uint32_t mtype, midx; } Quad;
typedef struct { V3 p[3]; V3 nrm[3]; V3 e1, e2; uint32_t mtype, midx; } Tri;

typedef struct {
    V3 point, normal;
    float t;
    int front;
    uint32_t mtype, midx;
    float u, v;
    /* bookkeeping for rt_hit */
    uint32_t inst, ptype, pidx;
} Hit;

static Quad make_quad(const rt_parallelogram *p) {                                     /* Parallelogram.cuh:26-39 */
    Quad g;
    g.q = fromrt(p->q); g.u = fromrt(p->u); g.v = fromrt(p->v);
    g.mtype = p->material_type; g.midx = p->material_index;
    g.n = vcross(g.u, g.v);
    g.area = sqrtf(vlen2(g.n));
    g.n = vunit(g.n);
    float sum = 0.0f;
    for (int i = 0; i < 3; i++) sum += vget(g.n, i) * vget(g.q, i);
    g.d = sum;
    return g;
}
static Tri make_tri(const rt_triangle *t) {                                            /* Triangle.cuh:26-46 */
    Tri r;
    for (int i = 0; i < 3; i++) r.p[i] = fromrt(t->vertex[i]);
    r.e1 = vsub(r.p[1], r.p[0]);
    r.e2 = vsub(r.p[2], r.p[0]);
    for (int i = 0; i < 3; i++)
        r.nrm[i] = t->has_normals ? fromrt(t->normal[i]) : vunit(vcross(r.e1, r.e2));
    r.mtype = t->material_type; r.midx = t->material_index;
    return r;
}

static int sphere_hit(const Sph *s, const Ray *ray, Range range, Hit *rec) {            /* Sphere.cu:4-49 */
    const V3 cq = vsub(s->center, ray->o);
    const V3 dir = ray->d;
    const float a = vdot(dir, dir);
    const float b = -2.0f * vdot(cq, dir);
    const float c = vdot(cq, cq) - s->radius * s->radius;
    float delta = b * b - 4.0f * a * c;
    if (delta < 0.0f) return 0;
    delta = sqrtf(delta);
    const float root1 = (-b - delta) / (a * 2.0f);
    const float root2 = (-b + delta) / (a * 2.0f);
    float root;
    if (in_range(range, root1)) root = root1;
    else if (in_range(range, root2)) root = root2;
    else return 0;
    rec->t = root;
    rec->point = vadd(ray->o, vscale(ray->d, root));                                   /* Ray.cuh:18-20 */
    rec->mtype = s->mtype; rec->midx = s->midx;
    const V3 outward = vunit(vsub(rec->point, s->center));
    rec->front = vdot(ray->d, outward) < 0.0f;
    rec->normal = rec->front ? outward : vneg(outward);
    rec->u = rec->v = 0.0f;     /* uvPair computed by the reference but unused by shading */
    return 1;
}
static int quad_hit(const Quad *g, const Ray *ray, Range range, Hit *rec) {            /* Parallelogram.cu:4-46 */
    const float ndd = vdot(g->n, ray->d);
    if (near_zero(ndd)) return 0;
    float ndp = 0.0f;
    for (int i = 0; i < 3; i++) ndp += vget(g->n, i) * vget(ray->o, i);
    const float t = (g->d - ndp) / ndd;
    if (!in_range(range, t)) return 0;
    const V3 inter = vadd(ray->o, vscale(ray->d, t));
    const V3 p = vsub(inter, g->q);
    const V3 normal = vcross(g->u, g->v);
    const float den = vlen2(normal);
    if (near_zero(den)) return 0;
    const float alpha = vdot(vcross(p, g->v), normal) / den;
    const float beta = vdot(vcross(g->u, p), normal) / den;
    const Range cr = {0.0f, 1.0f};
    if (!in_range(cr, alpha) || !in_range(cr, beta)) return 0;
    rec->t = t;
    rec->point = inter;
    rec->mtype = g->mtype; rec->midx = g->midx;
    rec->front = (double)vdot(ray->d, g->n) < 0.0;
    rec->normal = rec->front ? g->n : vneg(g->n);
    rec->u = alpha; rec->v = beta;
    return 1;
}
static int tri_hit(const Tri *tr, const Ray *ray, Range range, Hit *rec) {             /* Triangle.cu:4-44 */
    const V3 h = vcross(ray->d, tr->e2);
    const float det = vdot(tr->e1, h);
    if (near_zero(det)) return 0;
    const V3 s = vsub(ray->o, tr->p[0]);
    const Range cr = {0.0f, 1.0f};
    const float u = vdot(s, h) / det;
    if (!in_range(cr, u)) return 0;
    const V3 q = vcross(s, tr->e1);
    const float v = vdot(ray->d, q) / det;
    if (!in_range(cr, v) || u + v > 1.0f) return 0;
    const float t = vdot(tr->e2, q) / det;
    if (!in_range(range, t)) return 0;
    rec->t = t;
    rec->point = vadd(ray->o, vscale(ray->d, t));
    rec->mtype = tr->mtype; rec->midx = tr->midx;
    rec->u = u; rec->v = v;
    const V3 n = vunit(vadd(vadd(vscale(tr->nrm[0], (1.0f - u) - v), vscale(tr->nrm[1], u)), vscale(tr->nrm[2], v)));
    rec->front = vdot(ray->d, n) < 0.0f;
    rec->normal = rec->front ? n : vneg(n);
    return 1;
}

static Box sphere_box(const Sph *s) {                                                  /* Sphere.cu:51-55 */
    const V3 e = v3(s->radius, s->radius, s->radius);
    return box_points(vsub(s->center, e), vadd(s->center, e));
}
static Box quad_box(const Quad *g) {                                                   /* Parallelogram.cu:48-50 (q-centred, bug-compat) */
    const V3 h = vscale(vadd(g->u, g->v), 0.5f);
    return box_points(vadd(g->q, h), vsub(g->q, h));
}
static Box tri_box(const Tri *t) {                                                     /* Triangle.cu:46-62 */
    V3 mn, mx;
    for (int i = 0; i < 3; i++) {
        float a = vget(t->p[0], i), b = vget(t->p[1], i), c = vget(t->p[2], i);
        float lo = a; if (b < lo) lo = b; if (c < lo) lo = c;     /* std::min({..}) keeps first minimum */
        float hi = a; if (hi < b) hi = b; if (hi < c) hi = c;     /* std::max({..}) keeps first maximum */
        vset(&mn, i, lo); vset(&mx, i, hi);
    }
    return box_points(mn, mx);
}
static V3 sphere_centroid(const Sph *s) { return s->center; }                         /* Sphere.cuh:37-39 */
static V3 quad_centroid(const Quad *g) {                                               /* Parallelogram.cuh:45-47 */
    return vadd(vadd(g->q, vscale(g->u, 0.5f)), vscale(g->v, 0.5f));
}
static V3 tri_centroid(const Tri *t) {                                                 /* Triangle.cuh:53-61 */
    V3 r;
    for (int i = 0; i < 3; i++) {
        float f = vget(t->p[0], i) + vget(t->p[1], i) + vget(t->p[2], i);
        f /= 3.0f;
        vset(&r, i, f);
    }
    return r;
}

/* ------------------------------------------------------------------------------------
 * Acceleration structures (src/AS/BLAS.cu, src/AS/TLAS.cu, src/AS/Instance.cu)
 * ---------------------------------------------------------------------------------- */
typedef struct { Box box; uint32_t count; uint32_t index; } Node;   /* BLASNode / TLASNode */

typedef struct {
    Node *nodes; uint32_t n_nodes;
    uint32_t *refs; uint32_t n_refs;     /* primitive index (into the type's array) per slot */
    uint32_t type;
} Blas;

typedef struct {
    uint32_t ptype, pindex, pcount;
    uint32_t as_index;
    Mat fwd, inv, nrm;
    Box box; V3 centroid;
    Box tbox; V3 tcentroid;
    rt_xform x;
} Inst;

struct oracle_scene {
    Sph *sph; size_t n_sph;
    Quad *quad; size_t n_quad;
    Tri *tri; size_t n_tri;
    rt_rough *rough; size_t n_rough;
    rt_metal *metal; size_t n_metal;
    Inst *inst; size_t n_inst;
    Blas *blas; size_t n_blas;
    Node *tlas; uint32_t n_tlas;
    uint32_t *tlas_refs; uint32_t n_tlas_refs;
    rt_update_fn update; void *update_user;
    uint64_t build_seed;
    /* camera (RendererImpl.cuh:32-61) */
    int cam_ok;
    int W, H;
    V3 background, center, pixel_origin, pdx, pdy, cu, cv;
    float focus_radius, recip_sqrt;
    uint32_t sqrt_s, depth;
};

typedef struct { V3 c; uint32_t idx; Box box; } PrimInfo;  /* BLAS.cuh:74-83 (type implicit) */

static int g_sort_axis;
static int cmp_prim(const void *a, const void *b) {
    const PrimInfo *x = (const PrimInfo *)a, *y = (const PrimInfo *)b;
    const float fx = vget(x->c, g_sort_axis), fy = vget(y->c, g_sort_axis);
    if (fx < fy) return -1;
    if (fy < fx) return 1;
    return (x->idx < y->idx) ? -1 : (x->idx > y->idx);   /* pinned tie-break */
}
static pthread_mutex_t g_sort_lock = PTHREAD_MUTEX_INITIALIZER;

/* Pinned split-axis stream (replaces RandomGenerator::randomInteger(0,2), Global.cuh:360-365). */
static int axis_draw(uint64_t *st) {
    *st += GOLDEN64;
    return (int)((mix64(*st) >> 32) % 3ull);
}

/* Top-down median split shared by constructBLAS (BLAS.cu:4-117) and constructTLAS
 * (TLAS.cu:4-129).  prims[] is sorted in place; out refs receive prims[].idx in leaf order. */
static uint32_t build_tree(PrimInfo *prims, uint32_t n, uint32_t leaf_cap, uint64_t axis_state,
                           Node *nodes, uint32_t *refs) {
    typedef struct { uint32_t start, count, node; } Task;
    Task *stack = (Task *)malloc(sizeof(Task) * (64 + 2 * (size_t)n));
    uint32_t sp = 0, node_count = 0, nref = 0;
    stack[sp++] = (Task){0, n, 0};
    node_count++;
    while (sp > 0) {
        const Task task = stack[--sp];
        Node *node = &nodes[task.node];
        Box bb = prims[task.start].box;                     /* constructBoundingBoxForPrimitiveList */
        for (uint32_t i = task.start + 1; i < task.start + task.count; i++) bb = box_merge(bb, prims[i].box);
        if (task.count <= leaf_cap) {
            node->count = task.count;
            node->index = nref;
            node->box = bb;
            for (uint32_t i = 0; i < task.count; i++) refs[nref++] = prims[task.start + i].idx;
        } else {
            const uint32_t left = node_count++, right = node_count++;
            const int axis = axis_draw(&axis_state);
            pthread_mutex_lock(&g_sort_lock);
            g_sort_axis = axis;
            qsort(prims + task.start, task.count, sizeof(PrimInfo), cmp_prim);
            pthread_mutex_unlock(&g_sort_lock);
            node->box = bb;
            node->count = 0;
            node->index = left;
            const uint32_t mid = task.count / 2;
            stack[sp++] = (Task){task.start + mid, task.count - mid, right};
            stack[sp++] = (Task){task.start, mid, left};
        }
    }
    free(stack);
    return node_count;
}

static uint64_t blas_axis_seed(uint64_t seed, uint64_t blas_index) {
    return mix64(seed ^ ((blas_index + 1ull) * SUBMUL64));
}
static uint64_t tlas_axis_seed(uint64_t seed, uint64_t frame) {
    return mix64(seed ^ 0xA24BAED4963EE407ull ^ ((frame + 1ull) * GOLDEN64));
}

/* Instance::updateTransformArguments (src/AS/Instance.cu:4-17) */
static void inst_update(Inst *in, const rt_xform *x) {
    in->x = *x;
    const Mat sh = mat_shift(fromrt(x->shift));
    const Mat ro = mat_rot(fromrt(x->rotate_deg));
    const Mat sc = mat_scale(fromrt(x->scale));
    const Mat t = mat_mul(&sh, &ro);
    in->fwd = mat_mul(&t, &sc);
    in->inv = mat_inverse(&in->fwd);
    in->nrm = mat_transpose(&in->inv);
    in->tbox = box_transform(in->box, &in->fwd);
    in->tcentroid = mat_point(&in->fwd, in->centroid);
}

void oracle_instance_matrices(const rt_xform *x, float *out48) {
    Inst in; memset(&in, 0, sizeof in);
    in.box = box_points(v3(0, 0, 0), v3(0, 0, 0));
    inst_update(&in, x);
    const Mat *ms[3] = {&in.fwd, &in.inv, &in.nrm};
    for (int k = 0; k < 3; k++)
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) out48[k * 16 + i * 4 + j] = ms[k]->d[i + 1][j + 1];
}

/* Instance i after the last update (Instance.cu:4-17): rows 1-3 of the inverse, forward and inverse-
 * transpose matrices (12 floats each), the transformed box {xmin,xmax,...} (6) and centroid (3). */
int oracle_instance_state(const oracle_scene *s, uint32_t i, float *out45) {
    if (!s || i >= s->n_inst) return 1;
    const Inst *in = &s->inst[i];
    const Mat *ms[3] = {&in->inv, &in->fwd, &in->nrm};
    for (int k = 0; k < 3; k++)
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 4; c++) out45[k * 12 + r * 4 + c] = ms[k]->d[r + 1][c + 1];
    for (int a = 0; a < 3; a++) { out45[36 + 2 * a] = in->tbox.r[a].min; out45[37 + 2 * a] = in->tbox.r[a].max; }
    out45[42] = in->tcentroid.x; out45[43] = in->tcentroid.y; out45[44] = in->tcentroid.z;
    return 0;
}

static Box prim_box(const oracle_scene *s, uint32_t type, uint32_t idx) {
    if (type == RT_PRIM_SPHERE) return sphere_box(&s->sph[idx]);
    if (type == RT_PRIM_PARALLELOGRAM) return quad_box(&s->quad[idx]);
    return tri_box(&s->tri[idx]);
}
static V3 prim_centroid(const oracle_scene *s, uint32_t type, uint32_t idx) {
    if (type == RT_PRIM_SPHERE) return sphere_centroid(&s->sph[idx]);
    if (type == RT_PRIM_PARALLELOGRAM) return quad_centroid(&s->quad[idx]);
    return tri_centroid(&s->tri[idx]);
}
static size_t prim_array_len(const oracle_scene *s, uint32_t type) {
    return type == RT_PRIM_SPHERE ? s->n_sph : (type == RT_PRIM_PARALLELOGRAM ? s->n_quad : s->n_tri);
}

void oracle_scene_destroy(oracle_scene *s) {
    if (!s) return;
    for (size_t i = 0; i < s->n_blas; i++) { free(s->blas[i].nodes); free(s->blas[i].refs); }
    free(s->blas); free(s->sph); free(s->quad); free(s->tri); free(s->rough); free(s->metal);
    free(s->inst); free(s->tlas); free(s->tlas_refs);
    free(s);
}

static int build_tlas(oracle_scene *s, uint64_t frame) {                              /* TLAS.cu:4-129 */
    const uint32_t n = (uint32_t)s->n_inst;
    free(s->tlas); free(s->tlas_refs);
    s->tlas = (Node *)calloc(2 * (size_t)n, sizeof(Node));
    s->tlas_refs = (uint32_t *)calloc(n, sizeof(uint32_t));
    PrimInfo *pi = (PrimInfo *)malloc(sizeof(PrimInfo) * n);
    for (uint32_t i = 0; i < n; i++) { pi[i].c = s->inst[i].tcentroid; pi[i].idx = i; pi[i].box = s->inst[i].tbox; }
    s->n_tlas = build_tree(pi, n, TLAS_LEAF, tlas_axis_seed(s->build_seed, frame), s->tlas, s->tlas_refs);
    s->n_tlas_refs = n;
    free(pi);
    return 0;
}

oracle_scene *oracle_scene_create(const rt_scene_desc *d, uint64_t seed) {
    if (!d || d->instance_count == 0) return NULL;
    oracle_scene *s = (oracle_scene *)calloc(1, sizeof *s);
    s->build_seed = seed;
    s->update = d->update; s->update_user = d->update_user;
    s->n_sph = d->sphere_count; s->sph = (Sph *)calloc(s->n_sph + 1, sizeof(Sph));
    for (size_t i = 0; i < s->n_sph; i++) {
        s->sph[i].center = fromrt(d->spheres[i].center); s->sph[i].radius = d->spheres[i].radius;
        s->sph[i].mtype = d->spheres[i].material_type; s->sph[i].midx = d->spheres[i].material_index;
    }
    s->n_quad = d->parallelogram_count; s->quad = (Quad *)calloc(s->n_quad + 1, sizeof(Quad));
    for (size_t i = 0; i < s->n_quad; i++) s->quad[i] = make_quad(&d->parallelograms[i]);
    s->n_tri = d->triangle_count; s->tri = (Tri *)calloc(s->n_tri + 1, sizeof(Tri));
    for (size_t i = 0; i < s->n_tri; i++) s->tri[i] = make_tri(&d->triangles[i]);
    s->n_rough = d->rough_count; s->rough = (rt_rough *)calloc(s->n_rough + 1, sizeof(rt_rough));
    if (s->n_rough) memcpy(s->rough, d->roughs, s->n_rough * sizeof(rt_rough));
    s->n_metal = d->metal_count; s->metal = (rt_metal *)calloc(s->n_metal + 1, sizeof(rt_metal));
    if (s->n_metal) memcpy(s->metal, d->metals, s->n_metal * sizeof(rt_metal));

    s->n_inst = d->instance_count;
    s->inst = (Inst *)calloc(s->n_inst, sizeof(Inst));
    s->blas = (Blas *)calloc(s->n_inst, sizeof(Blas));
    /* buildBLASPinMem (src/Global/RenderPin.cu:99-201): complete instance info, dedup BLAS per
     * (type, primitiveIndex).  The reference's map stores the instance index i instead of the
     * BLAS index (RenderPin.cu:151); we store the BLAS index (identical for the demo order). */
    uint32_t *key_type = (uint32_t *)malloc(sizeof(uint32_t) * s->n_inst);
    uint32_t *key_idx = (uint32_t *)malloc(sizeof(uint32_t) * s->n_inst);
    for (size_t i = 0; i < s->n_inst; i++) {
        const rt_instance_desc *id = &d->instances[i];
        Inst *in = &s->inst[i];
        in->ptype = id->primitive_type; in->pindex = id->primitive_index; in->pcount = id->primitive_count;
        if (in->ptype > RT_PRIM_TRIANGLE) goto fail;
        const size_t len = prim_array_len(s, in->ptype);
        if (in->pcount == 0) {
            if (in->pindex >= len) goto fail;
            in->pcount = 1;
            in->box = prim_box(s, in->ptype, in->pindex);
            in->centroid = prim_centroid(s, in->ptype, in->pindex);
        } else {
            if ((size_t)in->pindex + in->pcount > len) goto fail;
            if (id->has_local_bounds) {                                                /* VTKReader.cu:208-209 */
                Box b;
                for (int k = 0; k < 3; k++) { b.r[k].min = id->local_bounds[2 * k]; b.r[k].max = id->local_bounds[2 * k + 1]; }
                in->box = box_ensure(b);
                in->centroid = fromrt(id->local_centroid);
            } else {
                Box b = prim_box(s, in->ptype, in->pindex);
                double cx = 0, cy = 0, cz = 0;
                for (uint32_t k = 0; k < in->pcount; k++) {
                    if (k) b = box_merge(b, prim_box(s, in->ptype, in->pindex + k));
                    const V3 c = prim_centroid(s, in->ptype, in->pindex + k);
                    cx += c.x; cy += c.y; cz += c.z;
                }
                in->box = b;
                in->centroid = v3((float)(cx / in->pcount), (float)(cy / in->pcount), (float)(cz / in->pcount));
            }
        }
        uint32_t found = UINT32_MAX;
        for (size_t b = 0; b < s->n_blas; b++)
            if (key_type[b] == in->ptype && key_idx[b] == in->pindex) { found = (uint32_t)b; break; }
        if (found != UINT32_MAX) { in->as_index = found; continue; }
        in->as_index = (uint32_t)s->n_blas;
        key_type[s->n_blas] = in->ptype; key_idx[s->n_blas] = in->pindex;
        /* BLAS::constructBLAS over this instance's primitives (BLAS.cu:4-117) */
        Blas *bl = &s->blas[s->n_blas];
        const uint32_t n = in->pcount;
        PrimInfo *pi = (PrimInfo *)malloc(sizeof(PrimInfo) * n);
        for (uint32_t k = 0; k < n; k++) {
            pi[k].idx = in->pindex + k;
            pi[k].box = prim_box(s, in->ptype, in->pindex + k);
            pi[k].c = prim_centroid(s, in->ptype, in->pindex + k);
        }
        bl->nodes = (Node *)calloc(2 * (size_t)n, sizeof(Node));
        bl->refs = (uint32_t *)calloc(n, sizeof(uint32_t));
        bl->type = in->ptype;
        bl->n_nodes = build_tree(pi, n, BLAS_LEAF, blas_axis_seed(seed, s->n_blas), bl->nodes, bl->refs);
        bl->n_refs = n;
        free(pi);
        s->n_blas++;
    }
    free(key_type); free(key_idx);
    for (size_t i = 0; i < s->n_inst; i++) inst_update(&s->inst[i], &d->instances[i].xform);
    if (oracle_scene_update(s, 0) != 0) { oracle_scene_destroy(s); return NULL; }
    return s;
fail:
    free(key_type); free(key_idx);
    oracle_scene_destroy(s);
    return NULL;
}

int oracle_scene_update(oracle_scene *s, uint64_t frame) {
    if (!s) return 1;
    if (s->update) {
        rt_xform *xs = (rt_xform *)malloc(sizeof(rt_xform) * s->n_inst);
        for (size_t i = 0; i < s->n_inst; i++) xs[i] = s->inst[i].x;
        s->update(s->update_user, xs, s->n_inst, frame);
        for (size_t i = 0; i < s->n_inst; i++) inst_update(&s->inst[i], &xs[i]);
        free(xs);
    }
    return build_tlas(s, frame);
}

uint32_t oracle_blas_count(const oracle_scene *s) { return s ? (uint32_t)s->n_blas : 0; }

static void export_nodes(const Node *nodes, uint32_t n, float *boxes, uint32_t *ci) {
    for (uint32_t i = 0; i < n; i++) {
        if (boxes) for (int k = 0; k < 3; k++) { boxes[6 * i + 2 * k] = nodes[i].box.r[k].min; boxes[6 * i + 2 * k + 1] = nodes[i].box.r[k].max; }
        if (ci) { ci[2 * i] = nodes[i].count; ci[2 * i + 1] = nodes[i].index; }
    }
}
int oracle_export_blas(const oracle_scene *s, uint32_t b, float *boxes, uint32_t *ci, uint32_t *refs,
                       uint32_t *n_nodes, uint32_t *n_prims) {
    if (!s || b >= s->n_blas) return 1;
    const Blas *bl = &s->blas[b];
    if (n_nodes) *n_nodes = bl->n_nodes;
    if (n_prims) *n_prims = bl->n_refs;
    export_nodes(bl->nodes, bl->n_nodes, boxes, ci);
    if (refs) memcpy(refs, bl->refs, sizeof(uint32_t) * bl->n_refs);
    return 0;
}
int oracle_export_tlas(const oracle_scene *s, float *boxes, uint32_t *ci, uint32_t *refs,
                       uint32_t *n_nodes, uint32_t *n_refs) {
    if (!s) return 1;
    if (n_nodes) *n_nodes = s->n_tlas;
    if (n_refs) *n_refs = s->n_tlas_refs;
    export_nodes(s->tlas, s->n_tlas, boxes, ci);
    if (refs) memcpy(refs, s->tlas_refs, sizeof(uint32_t) * s->n_tlas_refs);
    return 0;
}

/* ------------------------------------------------------------------------------------
 * Traversal: TLAS::hit -> Instance::hit -> BLAS::hit
 * ---------------------------------------------------------------------------------- */
typedef struct {
    const oracle_scene *s;
    oracle_counters *cnt;
    int brute;
} Ctx;

static int prim_hit(const Ctx *cx, uint32_t type, uint32_t idx, const Ray *ray, Range r, Hit *rec) {
    if (cx->cnt) { if (type == RT_PRIM_TRIANGLE) cx->cnt->triangle_tests++; else cx->cnt->sphere_quad_tests++; }
    if (type == RT_PRIM_SPHERE) return sphere_hit(&cx->s->sph[idx], ray, r, rec);
    if (type == RT_PRIM_PARALLELOGRAM) return quad_hit(&cx->s->quad[idx], ray, r, rec);
    return tri_hit(&cx->s->tri[idx], ray, r, rec);
}

static int blas_hit(const Ctx *cx, const Blas *bl, const Ray *ray, Range range, Hit *rec) {  /* BLAS.cu:119-206 */
    uint32_t stack[64]; uint32_t sp = 0;
    stack[sp++] = 0;
    Hit tmp; int is_hit = 0;
    Range cur = range;
    while (sp > 0) {
        const uint32_t index = stack[--sp];
        float t;
        if (cx->cnt) { cx->cnt->node_pops++; cx->cnt->aabb_tests++; }
        if (!box_hit(&bl->nodes[index].box, ray, cur, &t)) continue;
        const Node *node = &bl->nodes[index];
        if (node->count > 0) {
            for (uint32_t i = 0; i < node->count; i++) {
                const uint32_t pidx = bl->refs[node->index + i];
                if (prim_hit(cx, bl->type, pidx, ray, cur, &tmp)) {
                    is_hit = 1; cur.max = tmp.t; tmp.ptype = bl->type; tmp.pidx = pidx; *rec = tmp;
                }
            }
        } else {
            const uint32_t l = node->index, r = l + 1;
            float tl, tr;
            if (cx->cnt) cx->cnt->aabb_tests += 2;
            const int hl = box_hit(&bl->nodes[l].box, ray, cur, &tl);
            const int hr = box_hit(&bl->nodes[r].box, ray, cur, &tr);
            if (hl && hr) {
                if (tl > tr) { stack[sp++] = l; stack[sp++] = r; }
                else { stack[sp++] = r; stack[sp++] = l; }
            } else if (hl) stack[sp++] = l;
            else if (hr) stack[sp++] = r;
        }
    }
    return is_hit;
}

/* brute == 1: every primitive of the instance (NO_AS intent, Kernel.cu:10-62).
 * brute == 2: the same, gated by each primitive's own AABB (the box the BVH leaves are built
 * from), which reproduces the BVH path's clipping — e.g. of the q-centred parallelogram box
 * (Parallelogram.cu:48-50) — without any tree. */
static int blas_brute(const Ctx *cx, const Inst *in, const Ray *ray, Range range, Hit *rec) {
    Hit tmp; int is_hit = 0; Range cur = range;
    for (uint32_t k = 0; k < in->pcount; k++) {
        const uint32_t pidx = in->pindex + k;
        if (cx->brute == 2) {
            const Box pb = prim_box(cx->s, in->ptype, pidx);
            float te;
            if (!box_hit(&pb, ray, cur, &te)) continue;
        }
        if (prim_hit(cx, in->ptype, pidx, ray, cur, &tmp)) {
            is_hit = 1; cur.max = tmp.t; tmp.ptype = in->ptype; tmp.pidx = pidx; *rec = tmp;
        }
    }
    return is_hit;
}

static int instance_hit(const Ctx *cx, uint32_t ii, const Ray *ray, Range range, Hit *rec) { /* Instance.cu:19-50 */
    const Inst *in = &cx->s->inst[ii];
    if (cx->cnt) cx->cnt->instance_visits++;
    Ray lr;
    lr.o = mat_point(&in->inv, ray->o);
    lr.d = mat_vector(&in->inv, ray->d);
    const int h = cx->brute ? blas_brute(cx, in, &lr, range, rec)
                            : blas_hit(cx, &cx->s->blas[in->as_index], &lr, range, rec);
    if (!h) return 0;
    rec->point = mat_point(&in->fwd, rec->point);
    rec->normal = vunit(mat_vector(&in->nrm, rec->normal));
    rec->front = vdot(ray->d, rec->normal) < 0.0f;
    rec->inst = ii;
    return 1;
}

static int tlas_hit(const Ctx *cx, const Ray *ray, Range range, Hit *rec) {          /* TLAS.cu:131-201 */
    const oracle_scene *s = cx->s;
    if (cx->cnt) cx->cnt->rays++;
    Hit tmp; int is_hit = 0; Range cur = range;
    if (cx->brute) {
        for (uint32_t i = 0; i < s->n_inst; i++)
            if (instance_hit(cx, i, ray, cur, &tmp)) { is_hit = 1; cur.max = tmp.t; *rec = tmp; }
        return is_hit;
    }
    uint32_t stack[64]; uint32_t sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const uint32_t index = stack[--sp];
        float t;
        if (cx->cnt) { cx->cnt->node_pops++; cx->cnt->aabb_tests++; }
        if (!box_hit(&s->tlas[index].box, ray, cur, &t)) continue;
        const Node *node = &s->tlas[index];
        if (node->count > 0) {
            for (uint32_t i = 0; i < node->count; i++) {
                const uint32_t ii = s->tlas_refs[node->index + i];
                if (instance_hit(cx, ii, ray, cur, &tmp)) { is_hit = 1; cur.max = tmp.t; *rec = tmp; }
            }
        } else {
            const uint32_t l = node->index, r = l + 1;
            float tl, tr;
            if (cx->cnt) cx->cnt->aabb_tests += 2;
            const int hl = box_hit(&s->tlas[l].box, ray, cur, &tl);
            const int hr = box_hit(&s->tlas[r].box, ray, cur, &tr);
            if (hl && hr) {
                if (tl > tr) { stack[sp++] = l; stack[sp++] = r; }
                else { stack[sp++] = r; stack[sp++] = l; }
            } else if (hl) stack[sp++] = l;
            else if (hr) stack[sp++] = r;
        }
    }
    return is_hit;
}

/* ------------------------------------------------------------------------------------
 * Materials (include/Material/Rough.cuh, Metal.cuh) and rayColor / render (Kernel.cu)
 * ---------------------------------------------------------------------------------- */
static int rough_scatter(const rt_rough *m, uint64_t *st, const Hit *rec, V3 *att, Ray *out) {   /* Rough.cuh:14-29 */
    V3 dir = vadd(rec->normal, random_space_vector(st, 1.0f));
    if (f_equals(vlen2(dir), FZERO * FZERO)) dir = rec->normal;
    out->o = rec->point; out->d = dir;
    *att = fromrt(m->albedo);
    return 1;
}
static int metal_scatter(const rt_metal *m, uint64_t *st, const Ray *in, const Hit *rec, V3 *att, Ray *out) { /* Metal.cuh:15-32 */
    const V3 v = in->d, n = rec->normal;
    V3 r = vunit(vsub(v, vscale(n, 2.0f * vdot(v, n))));
    if (m->fuzz > 0.0f) r = vadd(r, vscale(random_space_vector(st, 1.0f), m->fuzz));
    out->o = rec->point; out->d = r;
    *att = fromrt(m->albedo);
    return vdot(out->d, rec->normal) > 0.0f;
}

static V3 ray_color(const Ctx *cx, const Ray *ray, uint64_t *st) {                    /* Kernel.cu:6-103 */
    const oracle_scene *s = cx->s;
    Hit rec; memset(&rec, 0, sizeof rec);
    Ray cur = *ray;
    V3 result = v3(1.0f, 1.0f, 1.0f);
    const Range range = {TMIN, INFINITY};
    for (uint32_t depth = 0; depth < s->depth; depth++) {
        if (tlas_hit(cx, &cur, range, &rec)) {
            Ray out; V3 att = v3(0, 0, 0);
            if (rec.mtype == RT_MAT_ROUGH) {
                rough_scatter(&s->rough[rec.midx], st, &rec, &att, &out);
            } else if (rec.mtype == RT_MAT_METAL) {
                if (!metal_scatter(&s->metal[rec.midx], st, &cur, &rec, &att, &out)) return result;
            } else {
                out = cur;   /* `default:;` leaves out/attenuation value-initialised in the reference */
            }
            cur = out;
            result = vmul(result, att);
        } else {
            result = vmul(result, s->background);
            break;
        }
    }
    return result;
}

int oracle_camera_set(oracle_scene *s, const rt_camera_input *c, uint32_t w, uint32_t h) { /* RenderPin.cu:73-95 */
    if (!s || !c || w == 0 || h == 0) return 1;
    const V3 center = fromrt(c->center), target = fromrt(c->target), up = fromrt(c->up);
    const float fd = pdist(center, target);
    const float theta = c->fov * ORACLE_PI / 180.0f;
    const float vw = 2.0f * tanf(theta / 2.0f) * fd;
    const float vh = vw / ((float)w * 1.0f / (float)h);
    const V3 W = vunit(vsub(target, center));
    const V3 U = vunit(vcross(W, up));
    const V3 V = vunit(vcross(U, W));
    const V3 vx = vscale(U, vw), vy = vscale(V, vh);
    const V3 pdx = vdivs(vx, (float)w), pdy = vdivs(vy, (float)h);
    const V3 vorg = vsub(vsub(vadd(center, vscale(W, fd)), vscale(vx, 0.5f)), vscale(vy, 0.5f));
    s->pixel_origin = vadd(vadd(vorg, vscale(pdx, 0.5f)), vscale(pdy, 0.5f));
    s->pdx = pdx; s->pdy = pdy; s->center = center; s->cu = U; s->cv = V;
    s->background = fromrt(c->background);
    s->focus_radius = c->focus_disk_radius;
    s->sqrt_s = (uint32_t)sqrt((double)c->sample_count);
    s->recip_sqrt = 1.0f / (float)s->sqrt_s;
    s->depth = c->ray_trace_depth;
    s->W = (int)w; s->H = (int)h;
    s->cam_ok = 1;
    return 0;
}

int oracle_camera_export(const oracle_scene *s, float *o) {
    if (!s || !s->cam_ok) return 1;
    const V3 vs[6] = {s->pixel_origin, s->pdx, s->pdy, s->center, s->cu, s->cv};
    for (int i = 0; i < 6; i++) { o[3 * i] = vs[i].x; o[3 * i + 1] = vs[i].y; o[3 * i + 2] = vs[i].z; }
    o[18] = s->recip_sqrt; o[19] = (float)s->sqrt_s;
    return 0;
}

/* One pixel of the render kernel (Kernel.cu:105-147). */
static void render_pixel(const Ctx *cx, uint64_t frame_seed, uint32_t x, uint32_t y, float *rgb, uint8_t *rgba) {
    const oracle_scene *s = cx->s;
    const uint32_t pitch = ((uint32_t)s->W + 15u) / 16u * 16u;       /* gridDim.x * blockDim.x (Kernel.cu:109) */
    const uint32_t pixel = pitch * y + x;
    uint64_t st = oracle_rng_init((uint64_t)pixel ^ frame_seed, pixel, 0);
    V3 result = v3(0.0f, 0.0f, 0.0f);
    for (uint32_t si = 0; si < s->sqrt_s; si++)
        for (uint32_t sj = 0; sj < s->sqrt_s; sj++) {
            const float ox = (((float)sj + rnd(&st)) * s->recip_sqrt) - 0.5f;
            const float oy = (((float)si + rnd(&st)) * s->recip_sqrt) - 0.5f;
            const V3 sp = vadd(vadd(s->pixel_origin, vscale(s->pdx, (float)x + ox)), vscale(s->pdy, (float)y + oy));
            V3 origin = s->center;
            if (s->focus_radius > 0.0f) {
                const V3 dv = random_plane_vector(&st, s->focus_radius);
                origin = vadd(vadd(s->center, vscale(s->cu, dv.x)), vscale(s->cv, dv.y));
            }
            Ray r; r.o = origin; r.d = vunit(vsub(sp, origin));
            result = vadd(result, ray_color(cx, &r, &st));
        }
    result = vscale(result, s->recip_sqrt * s->recip_sqrt);
    if (rgb) { rgb[0] = result.x; rgb[1] = result.y; rgb[2] = result.z; }
    if (rgba) {                                                                         /* Color3.cuh:99-114 */
        const float p = 1.0f / 2.0f;
        const float cr = powf(result.x, p), cg = powf(result.y, p), cb = powf(result.z, p);
        rgba[0] = (uint8_t)(256.0f * clampf_ref(cr, 0.0f, 0.999f));
        rgba[1] = (uint8_t)(256.0f * clampf_ref(cg, 0.0f, 0.999f));
        rgba[2] = (uint8_t)(256.0f * clampf_ref(cb, 0.0f, 0.999f));
        rgba[3] = 255;
    }
}

typedef struct {
    const oracle_scene *s; uint64_t seed;
    uint32_t x0, y0, w, h;
    float *rgb; uint8_t *rgba; int brute;
    uint32_t next_row; pthread_mutex_t lock;
    oracle_counters total;
} Job;

static void *render_worker(void *arg) {
    Job *job = (Job *)arg;
    oracle_counters local; memset(&local, 0, sizeof local);
    Ctx cx = {job->s, &local, job->brute};
    for (;;) {
        pthread_mutex_lock(&job->lock);
        const uint32_t row = job->next_row++;
        pthread_mutex_unlock(&job->lock);
        if (row >= job->h) break;
        for (uint32_t i = 0; i < job->w; i++) {
            const size_t o = (size_t)row * job->w + i;
            render_pixel(&cx, job->seed, job->x0 + i, job->y0 + row,
                         job->rgb ? job->rgb + 3 * o : NULL, job->rgba ? job->rgba + 4 * o : NULL);
        }
    }
    pthread_mutex_lock(&job->lock);
    job->total.rays += local.rays; job->total.aabb_tests += local.aabb_tests;
    job->total.triangle_tests += local.triangle_tests; job->total.sphere_quad_tests += local.sphere_quad_tests;
    job->total.instance_visits += local.instance_visits; job->total.node_pops += local.node_pops;
    pthread_mutex_unlock(&job->lock);
    return NULL;
}

int oracle_render(const oracle_scene *s, uint64_t frame_seed, uint32_t x0, uint32_t y0, uint32_t w, uint32_t h,
                  float *rgb, uint8_t *rgba, int threads, int brute, oracle_counters *counters) {
    if (!s || !s->cam_ok) return 1;
    if (x0 + w > (uint32_t)s->W || y0 + h > (uint32_t)s->H) return 2;
    Job job; memset(&job, 0, sizeof job);
    job.s = s; job.seed = frame_seed; job.x0 = x0; job.y0 = y0; job.w = w; job.h = h;
    job.rgb = rgb; job.rgba = rgba; job.brute = brute;
    pthread_mutex_init(&job.lock, NULL);
    if (threads <= 1) {
        render_worker(&job);
    } else {
        pthread_t *tids = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)threads);
        for (int i = 0; i < threads; i++) pthread_create(&tids[i], NULL, render_worker, &job);
        for (int i = 0; i < threads; i++) pthread_join(tids[i], NULL);
        free(tids);
    }
    pthread_mutex_destroy(&job.lock);
    if (counters) *counters = job.total;
    return 0;
}

int oracle_trace(const oracle_scene *s, const float *rays, size_t n, rt_hit *hits, int brute, oracle_counters *counters) {
    if (!s) return 1;
    oracle_counters local; memset(&local, 0, sizeof local);
    Ctx cx = {s, &local, brute};
    const Range range = {TMIN, INFINITY};
    for (size_t i = 0; i < n; i++) {
        Ray r; r.o = v3(rays[6 * i], rays[6 * i + 1], rays[6 * i + 2]); r.d = v3(rays[6 * i + 3], rays[6 * i + 4], rays[6 * i + 5]);
        Hit rec; memset(&rec, 0, sizeof rec);
        rt_hit *o = &hits[i];
        memset(o, 0, sizeof *o);
        if (tlas_hit(&cx, &r, range, &rec)) {
            o->t = rec.t; o->instance = rec.inst; o->primitive_type = rec.ptype; o->primitive_index = rec.pidx;
            o->point = tort(rec.point); o->normal = tort(rec.normal);
            o->material_type = rec.mtype; o->material_index = rec.midx;
        } else {
            o->t = INFINITY; o->instance = 0xFFFFFFFFu;
        }
    }
    if (counters) *counters = local;
    return 0;
}

/* ------------------------------------------------------------------------------------
 * Single-primitive KAT entry points
 * ---------------------------------------------------------------------------------- */
static void hit_out(const Hit *h, float *out) {
    out[0] = h->t; out[1] = h->point.x; out[2] = h->point.y; out[3] = h->point.z;
    out[4] = h->normal.x; out[5] = h->normal.y; out[6] = h->normal.z; out[7] = h->u; out[8] = h->v;
}
static Ray ray_in(const float *r) { Ray x; x.o = v3(r[0], r[1], r[2]); x.d = v3(r[3], r[4], r[5]); return x; }
int oracle_hit_sphere(const rt_sphere *sp, const float *ray, const float *range, float *out) {
    Sph s; s.center = fromrt(sp->center); s.radius = sp->radius; s.mtype = sp->material_type; s.midx = sp->material_index;
    const Ray r = ray_in(ray); const Range rg = {range[0], range[1]}; Hit h;
    if (!sphere_hit(&s, &r, rg, &h)) return 0;
    hit_out(&h, out); return 1;
}
int oracle_hit_parallelogram(const rt_parallelogram *pg, const float *ray, const float *range, float *out) {
    const Quad q = make_quad(pg); const Ray r = ray_in(ray); const Range rg = {range[0], range[1]}; Hit h;
    if (!quad_hit(&q, &r, rg, &h)) return 0;
    hit_out(&h, out); return 1;
}
int oracle_hit_triangle(const rt_triangle *tr, const float *ray, const float *range, float *out) {
    const Tri t = make_tri(tr); const Ray r = ray_in(ray); const Range rg = {range[0], range[1]}; Hit h;
    if (!tri_hit(&t, &r, rg, &h)) return 0;
    hit_out(&h, out); return 1;
}
int oracle_hit_aabb(const float *box, const float *ray, const float *range, float *t_entry) {
    Box b;
    for (int k = 0; k < 3; k++) { b.r[k].min = box[2 * k]; b.r[k].max = box[2 * k + 1]; }
    const Ray r = ray_in(ray); const Range rg = {range[0], range[1]};
    float t = 0.0f;
    const int h = box_hit(&b, &r, rg, &t);
    if (h && t_entry) *t_entry = t;
    return h;
}
void oracle_prim_bounds(uint32_t type, const void *prim, float *box6) {
    Box b;
    if (type == RT_PRIM_SPHERE) {
        const rt_sphere *sp = (const rt_sphere *)prim;
        Sph s; s.center = fromrt(sp->center); s.radius = sp->radius;
        b = sphere_box(&s);
    } else if (type == RT_PRIM_PARALLELOGRAM) {
        const Quad q = make_quad((const rt_parallelogram *)prim);
        b = quad_box(&q);
    } else {
        const Tri t = make_tri((const rt_triangle *)prim);
        b = tri_box(&t);
    }
    for (int k = 0; k < 3; k++) { box6[2 * k] = b.r[k].min; box6[2 * k + 1] = b.r[k].max; }
}

/* updateInstance (src/Global/Main.cu:6-42): the demo animation, oracle's own copy. */
void oracle_demo_update(void *user, rt_xform *x, size_t n, uint64_t frame) {
    (void)user;
    const V3 init = v3(0.0f, 2.0f, 0.0f);
    const float radius = 2.0f, speed = 0.02f;
    const float angle = (float)frame * speed;
    const V3 c1 = v3(init.x + radius * cosf(angle) * 1.5f,
                     init.y + radius * sinf(angle) * cosf(angle),
                     init.z + radius * sinf(angle) * 1.5f);
    const V3 c2 = v3(-c1.x, c1.y, -c1.z);
    const V3 c3 = v3(-c1.x, c1.y + 5.0f, c1.z);
    const float rot = (float)frame * 0.4f;
    const rt_xform t[5] = {
        {{0.0f, -1000.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
        {{c1.x, c1.y, c1.z}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
        {{-5.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
        {{c2.x, c2.y, c2.z}, {rot, rot, rot}, {3.0f, 3.0f, 3.0f}},
        {{c3.x, c3.y, c3.z}, {0.0f, 0.0f, 0.0f}, {1.0f, 1.0f, 1.0f}},
    };
    for (size_t i = 0; i < n && i < 5; i++) x[i] = t[i];
}
