// host_math.hpp — host-side scene math of the product (builders, instance matrices, camera).
//
// Restates the reference's host arithmetic so that everything the kernels consume (trees,
// matrices, camera vectors) is bit-identical to what the reference computes on its host:
// Vec3 / Point3 ops (include/Basic/Vec3.cuh, Point3.cuh), Range (include/Util/Range.cuh),
// BoundingBox construction (include/AS/BoundingBox.cuh, src/AS/BoundingBox.cu:4-32),
// Matrix (src/Util/Matrix.cu) and primitive boxes / centroids (src/Geometry/*.cu).
// Compiled with -ffp-contract=off: the evaluation order below is the reference's.  The instance math
// (matrices, inverse, transformed boxes) is __host__ __device__: the GPU frame chain (instances.hip)
// computes the same bits from host-computed sines and cosines.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/rt.h"

#if defined(__HIPCC__)
#define HM_HD __host__ __device__
#else
#define HM_HD
#endif

namespace rtamd {
namespace hm {

constexpr float FZERO = 1e-6f;                        // Global.cuh:147
constexpr float PI = (float)M_PI;                     // Global.cuh:149

struct V3 {
    float x, y, z;
    HM_HD float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    HM_HD float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
HM_HD inline V3 v3(float x, float y, float z) { return V3{x, y, z}; }
HM_HD inline V3 of(const rt_vec3 &a) { return V3{a.x, a.y, a.z}; }
HM_HD inline V3 operator+(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
HM_HD inline V3 operator-(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
HM_HD inline V3 operator*(V3 a, float s) { return V3{a.x * s, a.y * s, a.z * s}; }
HM_HD inline V3 operator/(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
HM_HD inline float dot(V3 a, V3 b) { float s = 0.0f; s += a.x * b.x; s += a.y * b.y; s += a.z * b.z; return s; }
HM_HD inline V3 cross(V3 a, V3 b) { return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
HM_HD inline float length(V3 a) { return std::sqrt(dot(a, a)); }
HM_HD inline V3 unit(V3 a) { const float f = 1.0f / length(a); return V3{a.x * f, a.y * f, a.z * f}; }
HM_HD inline float distance(V3 a, V3 b) {                   // Point3.cuh:75-84
    float s = 0.0f;
    for (int i = 0; i < 3; i++) s += (a[i] - b[i]) * (a[i] - b[i]);
    return std::sqrt(s);
}

struct Range { float min, max; };
HM_HD inline bool feq(float a, float b) { return std::fabs(a - b) < FZERO; }
HM_HD inline float rlength(Range r) { return (r.min >= r.max || feq(r.min, r.max)) ? 0.0f : r.max - r.min; }

struct Box {
    Range r[3];
    HM_HD void ensure_volume() {                            // BoundingBox.cuh:24-28
        for (auto &x : r)
            if (rlength(x) < FZERO) { x.min -= FZERO; x.max += FZERO; }
    }
    HM_HD static Box from_ranges(Range x, Range y, Range z) { Box b{{x, y, z}}; b.ensure_volume(); return b; }
    HM_HD static Box from_points(V3 p1, V3 p2) {            // BoundingBox.cuh:41-47
        Box b;
        for (int i = 0; i < 3; i++) b.r[i] = p1[i] < p2[i] ? Range{p1[i], p2[i]} : Range{p2[i], p1[i]};
        b.ensure_volume();
        return b;
    }
    HM_HD static Box merge(const Box &a, const Box &b) {    // BoundingBox.cuh:50-55
        Box m;
        for (int i = 0; i < 3; i++)
            m.r[i] = Range{a.r[i].min < b.r[i].min ? a.r[i].min : b.r[i].min,
                           a.r[i].max > b.r[i].max ? a.r[i].max : b.r[i].max};
        return m;
    }
    HM_HD void store(float *o) const { for (int i = 0; i < 3; i++) { o[2 * i] = r[i].min; o[2 * i + 1] = r[i].max; } }
};

// 4x4 matrix in the reference's 1-based 5x5 storage (include/Util/Matrix.cuh:22-25).
struct Mat {
    float d[5][5];
    int row, col;
    HM_HD static Mat zero(int r, int c) {
        Mat m;
        for (int i = 0; i < 5; i++)
            for (int j = 0; j < 5; j++) m.d[i][j] = 0.0f;
        m.row = r; m.col = c;
        return m;
    }
    HM_HD static Mat identity() { Mat m = zero(4, 4); for (int i = 1; i < 5; i++) m.d[i][i] = 1.0f; return m; }
};
HM_HD inline Mat operator*(const Mat &a, const Mat &b) {    // Matrix.cu:71-86
    Mat r = Mat::zero(a.row, b.col);
    for (int i = 1; i <= r.row; i++)
        for (int j = 1; j <= r.col; j++) {
            float sum = 0.0f;
            for (int n = 1; n <= a.col; n++) sum += a.d[i][n] * b.d[n][j];
            r.d[i][j] = sum;
        }
    return r;
}
HM_HD inline Mat transpose(const Mat &a) {                  // Matrix.cu:89-98
    Mat r = Mat::zero(a.col, a.row);
    for (int i = 1; i <= a.row; i++)
        for (int j = 1; j <= a.col; j++) r.d[j][i] = a.d[i][j];
    return r;
}
HM_HD inline Mat inverse(const Mat &a) {                    // Matrix.cu:5-68, 101-130 (Gauss-Jordan, partial pivot)
    float m[5][9];
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 9; j++) m[i][j] = 0.0f;
    for (int i = 1; i < 5; i++) {
        for (int j = 1; j < 5; j++) m[i][j] = a.d[i][j];
        m[i][4 + i] = 1.0f;
    }
    for (int i = 1; i < 5; i++) {                     // forward elimination
        float best = std::fabs(m[i][i]);
        int prow = i;
        for (int p = i + 1; p < 5; p++)
            if (std::fabs(m[p][i]) > best) { best = std::fabs(m[p][i]); prow = p; }
        if (std::fabs(best) < FZERO) return a;        // singular: the reference returns *this
        if (prow != i)
            for (int j = 1; j < 9; j++) { const float t = m[prow][j]; m[prow][j] = m[i][j]; m[i][j] = t; }
        for (int j = i + 1; j < 5; j++) {
            const float f = m[j][i] / m[i][i];
            for (int k = i; k < 9; k++) m[j][k] -= f * m[i][k];
        }
    }
    for (int i = 4; i >= 1; i--) {                    // back substitution
        if (std::fabs(m[i][i]) < FZERO) return a;
        float f = 1.0f / m[i][i];
        for (int p = i; p < 9; p++) m[i][p] *= f;
        for (int j = i - 1; j >= 1; j--) {
            f = m[j][i];
            for (int k = j; k < 9; k++) m[j][k] -= f * m[i][k];
        }
    }
    Mat r = Mat::zero(4, 4);
    for (int i = 1; i < 5; i++)
        for (int j = 1; j < 5; j++) r.d[i][j] = m[i][4 + j];
    return r;
}
HM_HD inline Mat shift_matrix(V3 s) { Mat m = Mat::identity(); m.d[1][4] = s.x; m.d[2][4] = s.y; m.d[3][4] = s.z; return m; }
HM_HD inline Mat scale_matrix(V3 s) { Mat m = Mat::identity(); m.d[1][1] = s.x; m.d[2][2] = s.y; m.d[3][3] = s.z; return m; }
// rotation about one axis from its cosine and sine (Matrix.cu:207-242); the host takes them from the
// degrees (rotate_cos_sin) so host and device matrices share one cos / sin evaluation
HM_HD inline Mat rotate_matrix_cs(float c, float s, int axis) {
    Mat m = Mat::identity();
    switch (axis) {
        case 0: m.d[2][2] = c; m.d[2][3] = -s; m.d[3][2] = s; m.d[3][3] = c; break;
        case 1: m.d[1][1] = c; m.d[1][3] = s; m.d[3][1] = -s; m.d[3][3] = c; break;
        default: m.d[1][1] = c; m.d[1][2] = -s; m.d[2][1] = s; m.d[2][2] = c; break;
    }
    return m;
}
inline void rotate_cos_sin(float degree, float &c, float &s) {   // Matrix.cu:207-212 (host libm)
    const float theta = degree * PI / 180.0f;
    c = std::cos(theta);
    s = std::sin(theta);
}
inline Mat rotate_matrix(float degree, int axis) {
    float c, s;
    rotate_cos_sin(degree, c, s);
    return rotate_matrix_cs(c, s, axis);
}
inline Mat rotate_matrix(V3 deg) {                    // Matrix.cu:244-249
    return rotate_matrix(deg.x, 0) * rotate_matrix(deg.y, 1) * rotate_matrix(deg.z, 2);
}
// Instance::updateTransformArguments (Instance.cu:4-17) from (shift, cos, sin, scale): the product order
// of the host path (shift * ((Rx * Ry) * Rz)) * scale
HM_HD inline Mat instance_matrix(V3 shift, V3 c, V3 s, V3 scale) {
    return shift_matrix(shift) * ((rotate_matrix_cs(c.x, s.x, 0) * rotate_matrix_cs(c.y, s.y, 1)) * rotate_matrix_cs(c.z, s.z, 2)) *
           scale_matrix(scale);
}
HM_HD inline V3 apply_point(const Mat &m, V3 p) {           // (M * toMatrix(Point3)).toPoint()
    V3 r;
    for (int i = 1; i <= 3; i++) {
        float s = 0.0f;
        s += m.d[i][1] * p.x; s += m.d[i][2] * p.y; s += m.d[i][3] * p.z; s += m.d[i][4] * 1.0f;
        r[i - 1] = s;
    }
    return r;
}
HM_HD inline Box transform_box(const Box &b, const Mat &m) {   // BoundingBox.cu:4-32
    V3 mn{INFINITY, INFINITY, INFINITY}, mx{-INFINITY, -INFINITY, -INFINITY};
    for (int i = 0; i < 2; i++)
        for (int j = 0; j < 2; j++)
            for (int k = 0; k < 2; k++) {
                const float x = (float)i * b.r[0].max + (1.0f - (float)i) * b.r[0].min;
                const float y = (float)j * b.r[1].max + (1.0f - (float)j) * b.r[1].min;
                const float z = (float)k * b.r[2].max + (1.0f - (float)k) * b.r[2].min;
                const V3 p = apply_point(m, V3{x, y, z});
                for (int l = 0; l < 3; l++) {
                    if (p[l] < mn[l]) mn[l] = p[l];
                    if (mx[l] < p[l]) mx[l] = p[l];
                }
            }
    return Box::from_points(mn, mx);
}

// ---- primitives (src/Geometry/*.cu, include/Geometry/*.cuh) --------------------------
HM_HD inline Box sphere_box(const rt_sphere &s) {           // Sphere.cu:51-55
    const V3 c = of(s.center), e{s.radius, s.radius, s.radius};
    return Box::from_points(c - e, c + e);
}
HM_HD inline V3 sphere_centroid(const rt_sphere &s) { return of(s.center); }

struct QuadDerived { V3 n; float area; float d; V3 nx; float den; };
HM_HD inline QuadDerived quad_derive(const rt_parallelogram &p) {   // Parallelogram.cuh:26-39, .cu:23-24
    QuadDerived q;
    q.nx = cross(of(p.u), of(p.v));
    q.area = length(q.nx);
    q.n = unit(q.nx);
    float sum = 0.0f;
    for (int i = 0; i < 3; i++) sum += q.n[i] * of(p.q)[i];
    q.d = sum;
    q.den = dot(q.nx, q.nx);
    return q;
}
HM_HD inline Box quad_box(const rt_parallelogram &p) {      // Parallelogram.cu:48-50 — q-centred (bug-compat)
    const V3 h = (of(p.u) + of(p.v)) * 0.5f;
    return Box::from_points(of(p.q) + h, of(p.q) - h);
}
HM_HD inline V3 quad_centroid(const rt_parallelogram &p) {  // Parallelogram.cuh:45-47
    return of(p.q) + of(p.u) * 0.5f + of(p.v) * 0.5f;
}

struct TriDerived { V3 e1, e2; V3 n[3]; };
HM_HD inline TriDerived tri_derive(const rt_triangle &t) {  // Triangle.cuh:26-46
    TriDerived d;
    d.e1 = of(t.vertex[1]) - of(t.vertex[0]);
    d.e2 = of(t.vertex[2]) - of(t.vertex[0]);
    for (int i = 0; i < 3; i++) d.n[i] = t.has_normals ? of(t.normal[i]) : unit(cross(d.e1, d.e2));
    return d;
}
HM_HD inline Box tri_box(const rt_triangle &t) {            // Triangle.cu:46-62 (std::min/max of 3)
    V3 mn, mx;
    for (int i = 0; i < 3; i++) {
        const float a = of(t.vertex[0])[i], b = of(t.vertex[1])[i], c = of(t.vertex[2])[i];
        float lo = a, hi = a;
        if (b < lo) lo = b;
        if (c < lo) lo = c;
        if (hi < b) hi = b;
        if (hi < c) hi = c;
        mn[i] = lo; mx[i] = hi;
    }
    return Box::from_points(mn, mx);
}
HM_HD inline V3 tri_centroid(const rt_triangle &t) {        // Triangle.cuh:53-61
    V3 r;
    for (int i = 0; i < 3; i++) {
        r[i] = of(t.vertex[0])[i] + of(t.vertex[1])[i] + of(t.vertex[2])[i];
        r[i] /= 3.0f;
    }
    return r;
}

// ---- pinned pseudo-random split axis (replaces std::mt19937 in BLAS.cu:84 / TLAS.cu:68) --
constexpr uint64_t GOLDEN64 = 0x9E3779B97F4A7C15ull;
constexpr uint64_t SUBMUL64 = 0xD1B54A32D192ED03ull;
HM_HD inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
HM_HD inline uint64_t blas_axis_state(uint64_t seed, uint64_t blas) { return mix64(seed ^ ((blas + 1ull) * SUBMUL64)); }
HM_HD inline uint64_t tlas_axis_state(uint64_t seed, uint64_t frame) {
    return mix64(seed ^ 0xA24BAED4963EE407ull ^ ((frame + 1ull) * GOLDEN64));
}
HM_HD inline int draw_axis(uint64_t &st) { st += GOLDEN64; return (int)((mix64(st) >> 32) % 3ull); }

}  // namespace hm
}  // namespace rtamd
