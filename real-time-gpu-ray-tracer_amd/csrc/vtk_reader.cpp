// vtk_reader.cpp — scene ingestion for the trace path: legacy VTK polydata
// particle files and their .vtk.series index, converted to the C ABI's triangles and instances.
//
// Restates VTKReader::readVTKFile (src/Global/VTKReader.cu:16-164), VTKReader::convertToRendererData
// (VTKReader.cu:166-220) and Renderer::configureVTKFiles (src/Global/Renderer.cu:394-443) without
// the VTK 9.5 library (Windows binaries in the reference) or nlohmann::json:
//   * the legacy format is parsed directly: header, ASCII|BINARY (big-endian), DATASET POLYDATA,
//     POINTS float|double, TRIANGLE_STRIPS (any other cell type is rejected, as VTKReader.cu:80-84
//     does), CELL_DATA arrays "id" and "vel" given as SCALARS / VECTORS / FIELD arrays; POINT_DATA
//     arrays are skipped;
//   * per particle (= one strip cell): id, velocity, bounds (cell->GetBounds, doubles cast to float),
//     centroid (mean of the cell's points in double, cast to float), the strip's vertices;
//   * vertex normals: the reference runs vtkPolyDataNormals (VTKReader.cu:60-70: point normals,
//     no splitting, consistency, auto-orient).  That third-party filter is restated from its
//     documented behaviour — strips decomposed into triangles with alternating orientation,
//     degenerate triangles dropped, windings made consistent across shared edges, each triangle's
//     unit normal (Newell's method) summed into its points, sums normalised; per strip, the
//     orientation is flipped when the normal at the point of largest x points to -x (auto-orient
//     outward).  PARITY UNPINNED at this boundary
//     (SURVEY §8c): the build and the oracle consume the same normals, so image parity is checked
//     downstream of them.
//   * conversion: strip of N points -> N-2 triangles, odd triangles swap their 2nd/3rd vertex and
//     normal (VTKReader.cu:182-197), material METAL 0; one instance per particle with the particle's
//     bounds / centroid and the transform shift (0,4,0), rotate (90,0,0), scale 3 (VTKReader.cu:204-214).
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/rt.h"

void rtamd_set_error(const std::string &msg);

namespace {

rt_status vfail(rt_status s, const std::string &m) {
    rtamd_set_error(m);                        // rt_last_error() (rt_api.cpp)
    return s;
}

struct Cursor {
    const std::vector<uint8_t> &d;
    size_t p = 0;
    explicit Cursor(const std::vector<uint8_t> &data) : d(data) {}
    std::string line() {                       // rest of the current line, terminator consumed
        std::string s;
        while (p < d.size() && d[p] != '\n') s.push_back((char)d[p++]);
        if (p < d.size()) p++;
        if (!s.empty() && s.back() == '\r') s.pop_back();
        return s;
    }
    std::string token() {                      // next whitespace-separated token
        while (p < d.size() && std::isspace(d[p])) p++;
        std::string s;
        while (p < d.size() && !std::isspace(d[p])) s.push_back((char)d[p++]);
        return s;
    }
    void end_of_line() {                       // skip to just after the current line's '\n'
        while (p < d.size() && d[p] != '\n') p++;
        if (p < d.size()) p++;
    }
};

uint64_t be(const uint8_t *b, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | b[i];
    return v;
}

int type_size(const std::string &t) {
    if (t == "double" || t == "long" || t == "unsigned_long" || t == "vtkIdType") return 8;
    if (t == "float" || t == "int" || t == "unsigned_int") return 4;
    if (t == "short" || t == "unsigned_short") return 2;
    if (t == "char" || t == "unsigned_char") return 1;
    return 0;
}

// a * b without wrap-around (counts read from the file are untrusted)
bool mul_ok(size_t a, size_t b, size_t &r) {
    if (a != 0 && b > SIZE_MAX / a) return false;
    r = a * b;
    return true;
}

// Reads n values of VTK type `t` as doubles (binary: a big-endian block; the next keyword is found by
// skipping whitespace, as vtkDataReader does — some writers put no newline after a block).  n is bounded
// by the bytes left in the file before anything is allocated: sz bytes per binary value, at least one
// byte per ASCII token.
bool read_values(Cursor &c, bool binary, const std::string &t, size_t n, std::vector<double> &out) {
    const size_t left = c.d.size() - c.p;
    if (!binary && n > left) return false;
    if (binary) {
        const int sz = type_size(t);
        if (sz == 0 || n > left / (size_t)sz) return false;
    }
    out.resize(n);
    if (!binary) {
        for (size_t i = 0; i < n; i++) {
            const std::string tok = c.token();
            if (tok.empty()) return false;
            char *e = nullptr;
            out[i] = std::strtod(tok.c_str(), &e);
            if (e == tok.c_str()) return false;
        }
        return true;
    }
    const int sz = type_size(t);
    const uint8_t *b = c.d.data() + c.p;
    for (size_t i = 0; i < n; i++, b += sz) {
        const uint64_t u = be(b, sz);
        if (t == "double") { double v; std::memcpy(&v, &u, 8); out[i] = v; }
        else if (t == "float") { const uint32_t w = (uint32_t)u; float v; std::memcpy(&v, &w, 4); out[i] = v; }
        else if (t == "int") out[i] = (double)(int32_t)(uint32_t)u;
        else if (t == "unsigned_int") out[i] = (double)(uint32_t)u;
        else if (t == "long" || t == "vtkIdType") out[i] = (double)(int64_t)u;
        else if (t == "unsigned_long") out[i] = (double)u;
        else if (t == "short") out[i] = (double)(int16_t)(uint16_t)u;
        else if (t == "unsigned_short") out[i] = (double)(uint16_t)u;
        else if (t == "char") out[i] = (double)(int8_t)(uint8_t)u;
        else out[i] = (double)(uint8_t)u;
    }
    c.p += (size_t)sz * n;      // no line skip: writers may start the next keyword right after the block
    return true;
}

struct V3d { double x, y, z; };

// Newell's method (vtkPolygon::ComputeNormal) for a triangle; zero for degenerate triangles.
V3d newell(V3d a, V3d b, V3d c) {
    const V3d p[3] = {a, b, c};
    V3d n{0, 0, 0};
    for (int i = 0; i < 3; i++) {
        const V3d &u = p[i], &v = p[(i + 1) % 3];
        n.x += (u.y - v.y) * (u.z + v.z);
        n.y += (u.z - v.z) * (u.x + v.x);
        n.z += (u.x - v.x) * (u.y + v.y);
    }
    const double l = std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
    if (l == 0.0) return {0, 0, 0};
    return {n.x / l, n.y / l, n.z / l};
}

}  // namespace

struct rt_vtk_file {
    std::vector<V3d> points;
    std::vector<uint32_t> strip_offsets;     // cells + 1
    std::vector<uint32_t> strip_points;      // point ids of all strips
    std::vector<V3d> normals;                // per point
    std::vector<double> ids;                 // per cell
    std::vector<double> vel;                 // 3 per cell
};

struct rt_vtk_series {
    std::vector<std::string> paths;
    std::vector<float> times;
};

namespace {

void take_cell_array(rt_vtk_file &f, const std::string &name, size_t comps, size_t tuples, const std::vector<double> &v) {
    size_t need = 0;
    if (comps == 0 || !mul_ok(comps, tuples, need) || v.size() < need) return;   // read_values read exactly `need`
    if (name == "id") {
        f.ids.resize(tuples);
        for (size_t i = 0; i < tuples; i++) f.ids[i] = v[i * comps];
    } else if (name == "vel" && comps >= 3) {
        f.vel.resize(3 * tuples);
        for (size_t i = 0; i < tuples; i++)
            for (int a = 0; a < 3; a++) f.vel[3 * i + a] = v[i * comps + a];
    }
}


// One strip = one connected region: decompose into triangles (alternating orientation), drop
// degenerate ones, make the windings consistent across shared edges (breadth-first from the first
// triangle, flipping a neighbour that runs a shared edge in the same direction — SetConsistency),
// sum unit face normals into the points and normalise, then orient the region outward: if the
// normal at the point of largest x points to -x, every normal of the region flips
// (SetAutoOrientNormals).
void orient_and_accumulate(rt_vtk_file &f, size_t s) {
    const uint32_t *p = f.strip_points.data() + f.strip_offsets[s];
    const uint32_t m = f.strip_offsets[s + 1] - f.strip_offsets[s];
    struct Tri { uint32_t v[3]; };
    std::vector<Tri> tris;
    for (uint32_t j = 0; j + 2 < m; j++) {
        Tri t{{p[j], (j & 1) ? p[j + 2] : p[j + 1], (j & 1) ? p[j + 1] : p[j + 2]}};
        if (t.v[0] == t.v[1] || t.v[1] == t.v[2] || t.v[0] == t.v[2]) continue;
        tris.push_back(t);
    }
    if (tris.empty()) return;
    std::vector<std::pair<uint64_t, uint32_t>> edges;            // (undirected edge key, triangle)
    for (uint32_t t = 0; t < tris.size(); t++)
        for (int e = 0; e < 3; e++) {
            const uint32_t a = tris[t].v[e], b = tris[t].v[(e + 1) % 3];
            edges.push_back({((uint64_t)std::min(a, b) << 32) | std::max(a, b), t});
        }
    std::sort(edges.begin(), edges.end());
    auto has_directed = [](const Tri &t, uint32_t a, uint32_t b) {
        for (int e = 0; e < 3; e++)
            if (t.v[e] == a && t.v[(e + 1) % 3] == b) return true;
        return false;
    };
    std::vector<uint8_t> seen(tris.size(), 0);
    std::vector<uint32_t> queue;
    for (uint32_t seed = 0; seed < tris.size(); seed++) {
        if (seen[seed]) continue;
        seen[seed] = 1;
        queue.assign(1, seed);
        for (size_t qi = 0; qi < queue.size(); qi++) {
            const Tri cur = tris[queue[qi]];
            for (int e = 0; e < 3; e++) {
                const uint32_t a = cur.v[e], b = cur.v[(e + 1) % 3];
                const uint64_t key = ((uint64_t)std::min(a, b) << 32) | std::max(a, b);
                auto it = std::lower_bound(edges.begin(), edges.end(), std::make_pair(key, 0u));
                for (; it != edges.end() && it->first == key; ++it) {
                    const uint32_t nb = it->second;
                    if (seen[nb]) continue;
                    seen[nb] = 1;
                    if (has_directed(tris[nb], a, b)) std::swap(tris[nb].v[1], tris[nb].v[2]);
                    queue.push_back(nb);
                }
            }
        }
    }
    std::vector<uint32_t> pts;
    for (const Tri &t : tris) {
        const V3d n = newell(f.points[t.v[0]], f.points[t.v[1]], f.points[t.v[2]]);
        for (uint32_t q : t.v) {
            f.normals[q].x += n.x; f.normals[q].y += n.y; f.normals[q].z += n.z;
            pts.push_back(q);
        }
    }
    std::sort(pts.begin(), pts.end());
    pts.erase(std::unique(pts.begin(), pts.end()), pts.end());
    uint32_t best = pts[0];
    for (uint32_t q : pts) {
        V3d &n = f.normals[q];
        const double l = std::sqrt(n.x * n.x + n.y * n.y + n.z * n.z);
        n = l > 0 ? V3d{n.x / l, n.y / l, n.z / l} : V3d{0, 0, 0};
        if (f.points[q].x > f.points[best].x) best = q;
    }
    if (f.normals[best].x < 0.0)
        for (uint32_t q : pts) f.normals[q] = V3d{-f.normals[q].x, -f.normals[q].y, -f.normals[q].z};
}

rt_status parse_vtk(const std::vector<uint8_t> &data, rt_vtk_file &f) {
    Cursor c(data);
    const std::string head = c.line();
    if (head.find("# vtk DataFile Version") == std::string::npos)           // VTKReader.cu:27-30
        return vfail(RT_ERR_INVALID_ARGUMENT, "illegal vtk file header: " + head);
    c.line();                                                                 // title
    const std::string fmt = c.token();
    c.end_of_line();
    const bool binary = fmt == "BINARY";
    if (!binary && fmt != "ASCII") return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: format must be ASCII or BINARY");
    if (c.token() != "DATASET" || c.token() != "POLYDATA")
        return vfail(RT_ERR_UNSUPPORTED, "vtk: only DATASET POLYDATA is supported");
    c.end_of_line();
    std::vector<double> vals;
    size_t n_cell_tuples = 0, n_point_tuples = 0;
    bool in_cell_data = false;
    while (true) {
        const std::string kw = c.token();
        if (kw.empty()) break;
        if (kw == "POINTS") {
            const size_t n = std::strtoull(c.token().c_str(), nullptr, 10);
            const std::string t = c.token();
            c.end_of_line();
            size_t n3 = 0;
            if (!mul_ok(3, n, n3) || n > 0xFFFFFFFFull) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: POINTS count out of range");
            if (!read_values(c, binary, t, n3, vals)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: truncated POINTS");
            f.points.resize(n);
            for (size_t i = 0; i < n; i++) f.points[i] = {vals[3 * i], vals[3 * i + 1], vals[3 * i + 2]};
        } else if (kw == "TRIANGLE_STRIPS") {
            const size_t n = std::strtoull(c.token().c_str(), nullptr, 10);
            const size_t size = std::strtoull(c.token().c_str(), nullptr, 10);
            c.end_of_line();
            if (!read_values(c, binary, "int", size, vals)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: truncated TRIANGLE_STRIPS");
            size_t k = 0;
            f.strip_offsets.assign(1, 0);
            for (size_t s = 0; s < n; s++) {
                if (k >= size) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: strip list shorter than its cell count");
                const double mv = vals[k++];
                if (!(mv >= 0.0) || mv > (double)(size - k)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: strip runs past its list");
                const size_t m = (size_t)mv;
                if (k + m > size) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: strip runs past its list");
                for (size_t j = 0; j < m; j++) {
                    const double id = vals[k++];
                    if (id < 0 || id >= (double)f.points.size()) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: strip point id out of range");
                    f.strip_points.push_back((uint32_t)id);
                }
                f.strip_offsets.push_back((uint32_t)f.strip_points.size());
            }
        } else if (kw == "VERTICES" || kw == "LINES" || kw == "POLYGONS") {      // VTKReader.cu:80-84
            return vfail(RT_ERR_UNSUPPORTED, "vtk: found illegal cell type " + kw + " (only triangle strips)");
        } else if (kw == "CELL_DATA" || kw == "POINT_DATA") {
            const size_t n = std::strtoull(c.token().c_str(), nullptr, 10);
            c.end_of_line();
            in_cell_data = kw == "CELL_DATA";
            (in_cell_data ? n_cell_tuples : n_point_tuples) = n;
        } else if (kw == "SCALARS" || kw == "VECTORS" || kw == "NORMALS") {
            const std::string name = c.token(), t = c.token();
            size_t comps = kw == "SCALARS" ? 1 : 3;
            const std::string rest = c.line();                                 // SCALARS: optional numComp
            if (kw == "SCALARS") {
                const size_t nc = std::strtoull(rest.c_str(), nullptr, 10);
                if (nc > 0) comps = nc;
                const size_t save = c.p;
                if (c.token() == "LOOKUP_TABLE") c.end_of_line();
                else c.p = save;
            }
            const size_t tuples = in_cell_data ? n_cell_tuples : n_point_tuples;
            size_t nv = 0;
            if (!mul_ok(comps, tuples, nv)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: " + kw + " " + name + " size out of range");
            if (!read_values(c, binary, t, nv, vals)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: truncated " + kw + " " + name);
            if (in_cell_data) take_cell_array(f, name, comps, tuples, vals);
        } else if (kw == "FIELD") {
            c.token();                                                          // field name
            const size_t arrays = std::strtoull(c.token().c_str(), nullptr, 10);
            c.end_of_line();
            for (size_t a = 0; a < arrays; a++) {
                const std::string name = c.token();
                const size_t comps = std::strtoull(c.token().c_str(), nullptr, 10);
                const size_t tuples = std::strtoull(c.token().c_str(), nullptr, 10);
                const std::string t = c.token();
                c.end_of_line();
                size_t nv = 0;
                if (!mul_ok(comps, tuples, nv)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: FIELD array " + name + " size out of range");
                if (!read_values(c, binary, t, nv, vals)) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: truncated FIELD array " + name);
                if (in_cell_data) take_cell_array(f, name, comps, tuples, vals);
            }
        } else {
            return vfail(RT_ERR_UNSUPPORTED, "vtk: unsupported keyword " + kw);
        }
    }
    if (f.points.empty()) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: no points in this file");     // VTKReader.cu:38-41
    const size_t cells = f.strip_offsets.empty() ? 0 : f.strip_offsets.size() - 1;
    if (cells == 0) return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: no triangle strips in this file");
    if (f.ids.size() != cells || f.vel.size() != 3 * cells)                                           // VTKReader.cu:51-57
        return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: failed to read cell data (id / vel)");
    for (size_t s = 0; s < cells; s++)
        if (f.strip_offsets[s + 1] - f.strip_offsets[s] < 3)
            return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: triangle strip with fewer than 3 points");

    // vertex normals (restatement of vtkPolyDataNormals, see the header: parity unpinned)
    f.normals.assign(f.points.size(), V3d{0, 0, 0});
    for (size_t s = 0; s < cells; s++) orient_and_accumulate(f, s);
    return RT_OK;
}

bool read_file(const char *path, std::vector<uint8_t> &data) {
    FILE *fp = std::fopen(path, "rb");
    if (!fp) return false;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) data.insert(data.end(), buf, buf + n);
    std::fclose(fp);
    return true;
}

// ---- minimal JSON for .vtk.series: {"file-series-version": s, "files": [{"name": s, "time": x}, ...]} ----
struct Json {
    enum Kind { NUL, NUM, STR, ARR, OBJ, BOOL } kind = NUL;
    double num = 0;
    std::string str;
    std::vector<Json> items;
    std::vector<std::pair<std::string, Json>> members;
    const Json *get(const std::string &k) const {
        for (const auto &m : members)
            if (m.first == k) return &m.second;
        return nullptr;
    }
};

struct JsonParser {
    const std::string &s;
    size_t p = 0;
    bool ok = true;
    void ws() { while (p < s.size() && std::isspace((unsigned char)s[p])) p++; }
    bool str(std::string &out) {
        if (p >= s.size() || s[p] != '"') return false;
        p++;
        while (p < s.size() && s[p] != '"') {
            if (s[p] == '\\' && p + 1 < s.size()) {
                const char e = s[++p];
                out.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e);
                p++;
            } else {
                out.push_back(s[p++]);
            }
        }
        if (p >= s.size()) return false;
        p++;
        return true;
    }
    Json value(int depth = 0) {
        Json v;
        ws();
        if (p >= s.size() || depth > 64) { ok = false; return v; }
        const char ch = s[p];
        if (ch == '{') {
            v.kind = Json::OBJ;
            p++;
            ws();
            if (p < s.size() && s[p] == '}') { p++; return v; }
            while (ok) {
                ws();
                std::string k;
                if (!str(k)) { ok = false; break; }
                ws();
                if (p >= s.size() || s[p] != ':') { ok = false; break; }
                p++;
                v.members.push_back({k, value(depth + 1)});
                ws();
                if (p < s.size() && s[p] == ',') { p++; continue; }
                if (p < s.size() && s[p] == '}') { p++; break; }
                ok = false;
            }
        } else if (ch == '[') {
            v.kind = Json::ARR;
            p++;
            ws();
            if (p < s.size() && s[p] == ']') { p++; return v; }
            while (ok) {
                v.items.push_back(value(depth + 1));
                ws();
                if (p < s.size() && s[p] == ',') { p++; continue; }
                if (p < s.size() && s[p] == ']') { p++; break; }
                ok = false;
            }
        } else if (ch == '"') {
            v.kind = Json::STR;
            if (!str(v.str)) ok = false;
        } else if (s.compare(p, 4, "true") == 0) { v.kind = Json::BOOL; v.num = 1; p += 4; }
        else if (s.compare(p, 5, "false") == 0) { v.kind = Json::BOOL; p += 5; }
        else if (s.compare(p, 4, "null") == 0) { p += 4; }
        else {
            char *e = nullptr;
            v.kind = Json::NUM;
            v.num = std::strtod(s.c_str() + p, &e);
            if (e == s.c_str() + p) ok = false;
            p = (size_t)(e - s.c_str());
        }
        return v;
    }
};

}  // namespace

extern "C" {

// No C++ exception may cross the C ABI (std::terminate would end the caller's process): allocation
// failures become RT_ERR_OUT_OF_MEMORY, anything else RT_ERR_INVALID_ARGUMENT.
#define VTK_GUARD_BEGIN try {
#define VTK_GUARD_END                                                                          \
    }                                                                                          \
    catch (const std::bad_alloc &) { return vfail(RT_ERR_OUT_OF_MEMORY, "vtk: host allocation failed"); } \
    catch (const std::exception &e) { return vfail(RT_ERR_INVALID_ARGUMENT, std::string("vtk: ") + e.what()); } \
    catch (...) { return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: malformed input"); }

rt_status rt_vtk_read(const char *path, rt_vtk_file **out) {
    if (!path || !out) return vfail(RT_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    rt_vtk_file *f = nullptr;
    VTK_GUARD_BEGIN
    std::vector<uint8_t> data;
    if (!read_file(path, data)) return vfail(RT_ERR_INVALID_ARGUMENT, std::string("failed to open vtk file: ") + path);
    f = new rt_vtk_file();
    const rt_status st = parse_vtk(data, *f);
    if (st != RT_OK) { delete f; return st; }
    *out = f;
    return RT_OK;
    }
    catch (const std::bad_alloc &) { delete f; return vfail(RT_ERR_OUT_OF_MEMORY, "vtk: host allocation failed"); }
    catch (const std::exception &e) { delete f; return vfail(RT_ERR_INVALID_ARGUMENT, std::string("vtk: ") + e.what()); }
    catch (...) { delete f; return vfail(RT_ERR_INVALID_ARGUMENT, "vtk: malformed input"); }
}

void rt_vtk_free(rt_vtk_file *f) { delete f; }

rt_status rt_vtk_get_info(const rt_vtk_file *f, rt_vtk_info *info) {
    if (!f || !info) return vfail(RT_ERR_INVALID_ARGUMENT, "null argument");
    info->point_count = f->points.size();
    info->particle_count = f->strip_offsets.size() - 1;
    info->strip_vertex_count = f->strip_points.size();
    info->triangle_count = f->strip_points.size() - 2 * info->particle_count;
    return RT_OK;
}

rt_status rt_vtk_particles(const rt_vtk_file *f, rt_vtk_particle *out) {
    if (!f || !out) return vfail(RT_ERR_INVALID_ARGUMENT, "null argument");
    const size_t cells = f->strip_offsets.size() - 1;
    for (size_t s = 0; s < cells; s++) {
        rt_vtk_particle &P = out[s];
        P.id = (uint64_t)f->ids[s];                                             // VTKReader.cu:87
        P.velocity = rt_vec3{(float)f->vel[3 * s], (float)f->vel[3 * s + 1], (float)f->vel[3 * s + 2]};
        const uint32_t b = f->strip_offsets[s], e = f->strip_offsets[s + 1];
        double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY}, c[3] = {0, 0, 0};
        for (uint32_t j = b; j < e; j++) {
            const V3d &q = f->points[f->strip_points[j]];
            const double v[3] = {q.x, q.y, q.z};
            for (int a = 0; a < 3; a++) {
                lo[a] = v[a] < lo[a] ? v[a] : lo[a];
                hi[a] = v[a] > hi[a] ? v[a] : hi[a];
                c[a] += v[a];                                                   // VTKReader.cu:108-119
            }
        }
        for (int a = 0; a < 3; a++) {
            P.bounds[2 * a] = (float)lo[a];
            P.bounds[2 * a + 1] = (float)hi[a];
        }
        const double n = (double)(e - b);
        P.centroid = rt_vec3{(float)(c[0] / n), (float)(c[1] / n), (float)(c[2] / n)};
        P.first_vertex = b;
        P.vertex_count = e - b;
    }
    return RT_OK;
}

rt_status rt_vtk_vertices(const rt_vtk_file *f, rt_vec3 *positions, rt_vec3 *normals) {
    if (!f) return vfail(RT_ERR_INVALID_ARGUMENT, "null argument");
    for (size_t j = 0; j < f->strip_points.size(); j++) {
        const uint32_t q = f->strip_points[j];
        if (positions) positions[j] = rt_vec3{(float)f->points[q].x, (float)f->points[q].y, (float)f->points[q].z};
        if (normals) normals[j] = rt_vec3{(float)f->normals[q].x, (float)f->normals[q].y, (float)f->normals[q].z};
    }
    return RT_OK;
}

rt_status rt_vtk_convert(const rt_vtk_file *f, uint32_t triangle_index_base, rt_triangle *triangles,
                         rt_instance_desc *instances) {
    if (!f || !triangles || !instances) return vfail(RT_ERR_INVALID_ARGUMENT, "null argument");
    const size_t cells = f->strip_offsets.size() - 1;
    VTK_GUARD_BEGIN
    std::vector<rt_vtk_particle> parts(cells);
    const rt_status st = rt_vtk_particles(f, parts.data());
    if (st != RT_OK) return st;
    auto P3 = [&](uint32_t q) { return rt_vec3{(float)f->points[q].x, (float)f->points[q].y, (float)f->points[q].z}; };
    auto N3 = [&](uint32_t q) { return rt_vec3{(float)f->normals[q].x, (float)f->normals[q].y, (float)f->normals[q].z}; };
    size_t t = 0;
    for (size_t s = 0; s < cells; s++) {
        const uint32_t *p = f->strip_points.data() + f->strip_offsets[s];
        const uint32_t m = f->strip_offsets[s + 1] - f->strip_offsets[s];
        const uint32_t first = (uint32_t)t;
        for (uint32_t j = 0; j + 2 < m; j++, t++) {                            // VTKReader.cu:177-201
            const uint32_t a = p[j], b = (j & 1) ? p[j + 2] : p[j + 1], c = (j & 1) ? p[j + 1] : p[j + 2];
            rt_triangle &T = triangles[t];
            std::memset(&T, 0, sizeof T);
            T.vertex[0] = P3(a); T.vertex[1] = P3(b); T.vertex[2] = P3(c);
            T.normal[0] = N3(a); T.normal[1] = N3(b); T.normal[2] = N3(c);
            T.material_type = RT_MAT_METAL;
            T.material_index = 0;
            T.has_normals = 1;
        }
        rt_instance_desc &I = instances[s];                                     // VTKReader.cu:203-215
        std::memset(&I, 0, sizeof I);
        I.primitive_type = RT_PRIM_TRIANGLE;
        I.primitive_index = triangle_index_base + first;
        I.primitive_count = m - 2;
        I.has_local_bounds = 1;
        std::memcpy(I.local_bounds, parts[s].bounds, sizeof I.local_bounds);
        I.local_centroid = parts[s].centroid;
        I.xform.shift = rt_vec3{0.0f, 4.0f, 0.0f};
        I.xform.rotate_deg = rt_vec3{90.0f, 0.0f, 0.0f};
        I.xform.scale = rt_vec3{3.0f, 3.0f, 3.0f};
    }
    return RT_OK;
    VTK_GUARD_END
}

rt_status rt_vtk_series_read(const char *path, rt_vtk_series **out) {
    if (!path || !out) return vfail(RT_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    VTK_GUARD_BEGIN
    std::vector<uint8_t> data;
    if (!read_file(path, data)) return vfail(RT_ERR_INVALID_ARGUMENT, std::string("could not open the series file: ") + path);
    const std::string text(data.begin(), data.end());
    JsonParser jp{text};
    const Json root = jp.value();
    if (!jp.ok || root.kind != Json::OBJ) return vfail(RT_ERR_INVALID_ARGUMENT, "JSON parsing error in series file");
    const Json *files = root.get("files");
    if (!files || files->kind != Json::ARR) return vfail(RT_ERR_INVALID_ARGUMENT, "failed to parse files array in series file");
    std::unique_ptr<rt_vtk_series> s(new rt_vtk_series());
    // names are relative to the series file's directory (Renderer.cu:440 strips the file name)
    std::string dir(path);
    const size_t slash = dir.find_last_of('/');
    dir = slash == std::string::npos ? std::string() : dir.substr(0, slash + 1);
    for (const Json &it : files->items) {
        const Json *name = it.get("name"), *time = it.get("time");
        if (!name || name->kind != Json::STR || !time || time->kind != Json::NUM) {
            return vfail(RT_ERR_INVALID_ARGUMENT, "series entry without name / time");
        }
        s->paths.push_back(!name->str.empty() && name->str[0] == '/' ? name->str : dir + name->str);
        s->times.push_back((float)time->num);
    }
    *out = s.release();
    return RT_OK;
    VTK_GUARD_END
}

size_t rt_vtk_series_count(const rt_vtk_series *s) { return s ? s->paths.size() : 0; }

rt_status rt_vtk_series_entry(const rt_vtk_series *s, size_t i, const char **path, float *time) {
    if (!s || i >= s->paths.size()) return vfail(RT_ERR_INVALID_ARGUMENT, "no such series entry");
    if (path) *path = s->paths[i].c_str();
    if (time) *time = s->times[i];
    return RT_OK;
}

void rt_vtk_series_free(rt_vtk_series *s) { delete s; }

}  // extern "C"
