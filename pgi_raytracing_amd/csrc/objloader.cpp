// objloader.cpp -- Wavefront OBJ/MTL ingest with the reference loader's semantics
// (APP/objloader.cpp:53-507, APP/surface.cpp:4-22, APP/material.cpp:9-26).
//
// Output is the de-indexed layout Raytracer::LoadScene uploads to Embree
// (APP/raytracer.cpp:96-120): 3 vertices per triangle, per-vertex normal and UV, one material
// per surface (group), surfaces in file order.  Reproduced quirks:
//  * lines are strtok("\n") tokens, so empty lines vanish; three passes (mtllib, v/vn/vt, g/u/f)
//  * sscanf("%*s %f %f %f") partial parses keep defaults ("Ks 1.0. 1.0 1.0" sets only Ks.x)
//  * vn is normalised with Vector3::Normalize in float
//  * 'f' lines are classified by their number of ' ' characters after trimming: 3 -> triangle,
//    4 -> quad split into (0,1,2)+(0,2,3), anything else re-uses the previous face's tokens;
//    "%[0-9]/%[0-9]/%[0-9]" conversions that fail keep the previous buffer contents
//  * a surface's material is the LAST usemtl seen when the next 'g' (or EOF) closes it; an
//    unknown name leaves it NULL in the reference (a crash in trace) -- here it maps to a
//    trailing default Material() (type 0 -> Phong)
// Texture files (map_Kd) are returned as paths; decoding is left to the caller.
#include <cctype>
#include <cstdlib>
#include <stdexcept>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "pgrt.h"

namespace {

struct Mtl {
    std::string name = "default";
    float ambient[3] = {0.1f, 0.1f, 0.1f};
    float diffuse[3] = {0.4f, 0.4f, 0.4f};
    float specular[3] = {0.8f, 0.8f, 0.8f};
    float emission[3] = {0.0f, 0.0f, 0.0f};
    float shininess = 1.0f;
    float ior = 1.5f;
    int type = 0;
    int tex = -1;
};

std::string g_error;

std::vector<std::string> split_lines(const std::string& text) {
    std::vector<std::string> out;
    size_t a = 0;
    while (a < text.size()) {
        size_t b = text.find('\n', a);
        if (b == std::string::npos) b = text.size();
        if (b > a) out.emplace_back(text, a, b - a);
        a = b + 1;
    }
    return out;
}

bool read_file(const char* path, std::string& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    out.resize(n > 0 ? (size_t)n : 0);
    size_t got = n > 0 ? std::fread(&out[0], 1, (size_t)n, f) : 0;
    std::fclose(f);
    out.resize(got);
    return true;
}

std::string trim(const std::string& s) {  // Trim = RTrim(LTrim(s)) (APP/utils.cpp:177-200)
    size_t a = 0, b = s.size();
    while (a < b && (std::isspace((unsigned char)s[a]) || s[a] == 0)) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

// sscanf(line, "%*s %f %f %f", ...): read up to n floats after the first token
void scan_floats(const std::string& line, int n, float* dst) {
    const char* p = line.c_str();
    while (*p && std::isspace((unsigned char)*p)) ++p;
    while (*p && !std::isspace((unsigned char)*p)) ++p;
    for (int i = 0; i < n; ++i) {
        char* end = nullptr;
        float v = std::strtof(p, &end);
        if (end == p) return;
        dst[i] = v;
        p = end;
    }
}

bool scan_word(const std::string& line, std::string& w) {  // sscanf(line, "%*s %s", w)
    size_t a = line.find_first_not_of(" \t\r\n\v\f");
    if (a == std::string::npos) return false;
    size_t b = line.find_first_of(" \t\r\n\v\f", a);
    if (b == std::string::npos) return false;
    size_t c = line.find_first_not_of(" \t\r\n\v\f", b);
    if (c == std::string::npos) return false;
    size_t d = line.find_first_of(" \t\r\n\v\f", c);
    w = line.substr(c, d == std::string::npos ? std::string::npos : d - c);
    return true;
}

void normalize3(float* v) {  // Vector3::Normalize (APP/vector3.cpp:155-167)
    const float norm = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    if (norm != 0) {
        const float rn = 1 / std::sqrt(norm);
        v[0] *= rn;
        v[1] *= rn;
        v[2] *= rn;
    }
}

}  // namespace

struct pgrt_obj {
    std::vector<float> pos, nrm, uv;
    std::vector<int> mat;
    std::vector<pgrt_material> mats;
    std::vector<std::string> mat_names;
    std::vector<std::string> tex_paths;
    std::vector<std::string> surf_names;
    std::vector<int> surf_first, surf_count;
};

namespace {

// LoadMTL (APP/objloader.cpp:53-208)
bool load_mtl(const std::string& file, const std::string& path, std::vector<Mtl>& mats,
              std::map<std::string, int>& tex_index, std::vector<std::string>& tex_paths) {
    std::string text;
    if (!read_file(file.c_str(), text)) {
        g_error = "File " + file + " not found.";
        return false;
    }
    std::unique_ptr<Mtl> m;
    std::string material_name;
    for (const std::string& line : split_lines(text)) {
        if (line[0] == '#') continue;
        if (line.compare(0, 6, "newmtl") == 0) {
            if (m) {
                m->name = material_name;
                bool exists = false;
                for (auto& x : mats) exists |= x.name == material_name;
                if (!exists) mats.push_back(*m);
            }
            std::string w;
            if (scan_word(line, w)) material_name = w;
            m.reset(new Mtl());
            continue;
        }
        if (!m) continue;
        const std::string tmp = trim(line);
        auto starts = [&](const char* k) { return tmp.compare(0, std::strlen(k), k) == 0; };
        if (starts("Ka")) scan_floats(tmp, 3, m->ambient);
        if (starts("shader")) {
            const char* p = tmp.c_str() + 6;
            char* end = nullptr;
            long v = std::strtol(p, &end, 10);
            if (end != p) m->type = (int)v;
        }
        if (starts("Ni")) scan_floats(tmp, 1, &m->ior);
        if (starts("Kd")) scan_floats(tmp, 3, m->diffuse);
        if (starts("Ks")) scan_floats(tmp, 3, m->specular);
        if (starts("Ke")) scan_floats(tmp, 3, m->emission);
        if (starts("Ns")) scan_floats(tmp, 1, &m->shininess);
        if (starts("map_Kd")) {
            std::string w;
            if (scan_word(tmp, w)) {
                const std::string full = path + w;  // TextureProxy caches by full name
                auto it = tex_index.find(full);
                if (it == tex_index.end()) {
                    tex_index[full] = (int)tex_paths.size();
                    m->tex = (int)tex_paths.size();
                    tex_paths.push_back(full);
                } else {
                    m->tex = it->second;
                }
            }
        }
    }
    if (m) {
        m->name = material_name;
        mats.push_back(*m);
    }
    return true;
}

struct FaceVertex {
    int v, t, n;
};

// sscanf(tok, "%[0-9]/%[0-9]/%[0-9]", b0, b1, b2) with persistent buffers
void parse_indices(const std::string& tok, std::string buf[3]) {
    size_t p = 0;
    for (int k = 0; k < 3; ++k) {
        size_t q = p;
        while (q < tok.size() && std::isdigit((unsigned char)tok[q])) ++q;
        if (q == p) return;
        buf[k] = tok.substr(p, q - p);
        p = q;
        if (k < 2) {
            if (p < tok.size() && tok[p] == '/') ++p;
            else return;
        }
    }
}

}  // namespace

extern "C" {

const char* pgrt_obj_error(void) { return g_error.c_str(); }

// LoadOBJ (APP/objloader.cpp:210-507)
int pgrt_obj_load(const char* obj_path, int flip_yz, pgrt_obj** out) {
    if (!obj_path || !out) return PGRT_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    try {
        std::string text;
        if (!read_file(obj_path, text)) {
            g_error = std::string("File ") + obj_path + " not found.";
            return PGRT_ERR_IO;
        }
        const std::string file(obj_path);
        const size_t slash = file.rfind('/');
        const std::string path = slash == std::string::npos ? "" : file.substr(0, slash + 1);
        const std::vector<std::string> lines = split_lines(text);
        std::vector<Mtl> mats;
        std::map<std::string, int> tex_index;
        std::unique_ptr<pgrt_obj> o(new pgrt_obj());
        for (const auto& line : lines) {  // pass 1: material libraries
            if (line[0] == 'm') {
                std::string w;
                if (scan_word(line, w) && !load_mtl(path + w, path, mats, tex_index, o->tex_paths)) {
                    // the reference prints and continues without the library
                }
            }
        }
        std::vector<float> v, vn, vt;  // pass 2: coordinates
        for (const auto& line : lines) {
            if (line[0] != 'v' || line.size() < 2) continue;
            float a[3] = {0, 0, 0};
            if (line[1] == ' ') {
                scan_floats(line, 3, a);
                if (flip_yz) {
                    v.push_back(a[0]);
                    v.push_back(-a[2]);
                    v.push_back(a[1]);
                } else {
                    v.insert(v.end(), a, a + 3);
                }
            } else if (line[1] == 'n') {
                scan_floats(line, 3, a);
                float nn[3] = {a[0], a[1], a[2]};
                if (flip_yz) {
                    nn[1] = -a[2];
                    nn[2] = a[1];
                }
                normalize3(nn);
                vn.insert(vn.end(), nn, nn + 3);
            } else if (line[1] == 't') {
                scan_floats(line, 3, a);
                vt.push_back(a[0]);
                vt.push_back(a[1]);
            }
        }
        const int nv = (int)v.size() / 3, nn = (int)vn.size() / 3, nt = (int)vt.size() / 2;
        std::vector<FaceVertex> face;
        std::string group_name, material_name;
        std::string tokens[4];
        std::string buf[3];
        const int default_mat = (int)mats.size();
        bool used_default = false;
        auto close_group = [&]() {
            int mi = -1;
            for (size_t i = 0; i < mats.size(); ++i)
                if (mats[i].name == material_name) {
                    mi = (int)i;
                    break;
                }
            if (mi < 0) {
                mi = default_mat;
                used_default = true;
            }
            const int first = (int)o->mat.size();
            for (size_t k = 0; k < face.size(); ++k) {
                const FaceVertex& fv = face[k];
                o->pos.insert(o->pos.end(), &v[3 * (size_t)fv.v], &v[3 * (size_t)fv.v] + 3);
                o->nrm.insert(o->nrm.end(), &vn[3 * (size_t)fv.n], &vn[3 * (size_t)fv.n] + 3);
                o->uv.insert(o->uv.end(), &vt[2 * (size_t)fv.t], &vt[2 * (size_t)fv.t] + 2);
                if (k % 3 == 2) o->mat.push_back(mi);
            }
            o->surf_names.push_back(group_name);
            o->surf_first.push_back(first);
            o->surf_count.push_back((int)face.size() / 3);
            face.clear();
        };
        auto vertex = [&](const std::string& tok) -> FaceVertex {
            parse_indices(tok, buf);
            // atoi(b) - 1 in the reference (objloader.cpp:443-452), range-checked here in 64 bits:
            // an index past INT_MAX (atoi's overflow, then INT_MIN - 1) is undefined there
            // (make asan: UBSan caught it).  The raw 1-based value is checked against [1, n] BEFORE
            // the subtraction, so no value strtoll can return (LLONG_MIN / LLONG_MAX when it
            // saturates, 0 for an empty field) reaches an overflowing expression
            auto index = [&](const std::string& b, long long n) -> int {
                const long long raw = std::strtoll(b.c_str(), nullptr, 10);
                if (raw < 1 || raw > n) throw std::runtime_error("face index out of range in '" + tok + "'");
                return (int)(raw - 1);
            };
            const int iv = index(buf[0], nv), it = index(buf[1], nt), in = index(buf[2], nn);
            return FaceVertex{iv, it, in};
        };
        for (const auto& line : lines) {  // pass 3: groups, materials, faces
            const char c = line[0];
            if (c == 'g') {
                if (!face.empty()) close_group();
                std::string w;
                if (scan_word(line, w)) group_name = w;
            } else if (c == 'u') {
                std::string w;
                if (scan_word(line, w)) material_name = w;
            } else if (c == 'f') {
                std::string t = line;
                while (!t.empty() && std::isspace((unsigned char)t.back())) t.pop_back();
                int spaces = 0;
                for (char ch : t) spaces += ch == ' ';
                std::vector<std::string> parts;
                size_t a = 0;
                while (true) {
                    a = t.find_first_not_of(" \t\r\n\v\f", a);
                    if (a == std::string::npos) break;
                    size_t b = t.find_first_of(" \t\r\n\v\f", a);
                    parts.push_back(t.substr(a, b == std::string::npos ? std::string::npos : b - a));
                    if (b == std::string::npos) break;
                    a = b;
                }
                if (spaces == 3 && parts.size() >= 4)
                    for (int k = 0; k < 3; ++k) tokens[k] = parts[1 + k];
                else if (spaces == 4 && parts.size() >= 5)
                    for (int k = 0; k < 4; ++k) tokens[k] = parts[1 + k];
                for (int k = 0; k < 3; ++k) face.push_back(vertex(tokens[k]));
                if (spaces == 4) {
                    const int idx[3] = {0, 2, 3};
                    for (int k = 0; k < 3; ++k) face.push_back(vertex(tokens[idx[k]]));
                }
            }
        }
        if (!face.empty()) close_group();
        for (const Mtl& m : mats) {
            pgrt_material pm{};
            for (int k = 0; k < 3; ++k) {
                pm.diffuse[k] = m.diffuse[k];
                pm.specular[k] = m.specular[k];
            }
            pm.shininess = m.shininess;
            pm.ior = m.ior;
            pm.type = m.type;
            pm.diffuse_tex = m.tex;
            o->mats.push_back(pm);
            o->mat_names.push_back(m.name);
        }
        {  // trailing default Material() (APP/material.cpp:9-26) for unmatched surfaces
            Mtl d;
            pgrt_material pm{};
            for (int k = 0; k < 3; ++k) {
                pm.diffuse[k] = d.diffuse[k];
                pm.specular[k] = d.specular[k];
            }
            pm.shininess = d.shininess;
            pm.ior = d.ior;
            pm.type = d.type;
            pm.diffuse_tex = -1;
            o->mats.push_back(pm);
            o->mat_names.push_back("default");
        }
        (void)used_default;
        *out = o.release();
        return PGRT_OK;
    } catch (const std::exception& e) {
        g_error = e.what();
        return PGRT_ERR_IO;
    }
}

void pgrt_obj_free(pgrt_obj* obj) { delete obj; }

int pgrt_obj_scene(const pgrt_obj* o, pgrt_scene_desc* d) {
    if (!o || !d) return PGRT_ERR_INVALID_ARGUMENT;
    std::memset(d, 0, sizeof(*d));
    d->num_triangles = (int)o->mat.size();
    d->positions = o->pos.data();
    d->normals = o->nrm.data();
    d->uvs = o->uv.data();
    d->material_ids = o->mat.data();
    d->num_materials = (int)o->mats.size();
    d->materials = o->mats.data();
    d->num_textures = 0;
    d->textures = nullptr;
    d->env_texture = -1;
    d->num_lights = 0;
    d->lights = nullptr;
    return PGRT_OK;
}

int pgrt_obj_counts(const pgrt_obj* o, int* ns, int* nm, int* nt) {
    if (!o) return PGRT_ERR_INVALID_ARGUMENT;
    if (ns) *ns = (int)o->surf_names.size();
    if (nm) *nm = (int)o->mats.size();
    if (nt) *nt = (int)o->tex_paths.size();
    return PGRT_OK;
}

const char* pgrt_obj_texture_path(const pgrt_obj* o, int i) {
    if (!o || i < 0 || i >= (int)o->tex_paths.size()) return nullptr;
    return o->tex_paths[i].c_str();
}

const char* pgrt_obj_material_name(const pgrt_obj* o, int i) {
    if (!o || i < 0 || i >= (int)o->mat_names.size()) return nullptr;
    return o->mat_names[i].c_str();
}

int pgrt_obj_surface_range(const pgrt_obj* o, int i, int* first, int* count) {
    if (!o || i < 0 || i >= (int)o->surf_names.size()) return PGRT_ERR_INVALID_ARGUMENT;
    if (first) *first = o->surf_first[i];
    if (count) *count = o->surf_count[i];
    return PGRT_OK;
}

}  // extern "C"
