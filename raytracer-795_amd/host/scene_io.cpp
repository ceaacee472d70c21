// scene_io.cpp — native host side of the drop-in: the reference's Parser (src/Parser.h),
// Image::saveImage (src/Image.cpp:26-107, src/Helper.cpp:361-412) and renderScene's camera
// loop (src/Scene.cpp:294-363), in C++ above the C ABI of include/rtg.h.
//
// The parse follows src/Parser.h function by function (file:line cited per block) with the
// same numeric conversions (sscanf "%f" / tinyxml2 Query*Text for attributes and vectors,
// atof for VertexData / TexCoordData / happly doubles for PLY) and the same quirks as the
// Python mirror rtg/scene.py (tests/test_host_native.py checks the two descriptors are
// identical): texture-map state carried from one <TextureMap> to the next, only the first
// <Transformations> token may be a composite, PLY quads split (0,1,2),(2,3,0), texture offsets
// relative to the mesh's vertex offset, the last replace_background texture wins.
// hw7 additions (no reference code): <Renderer>/<RendererParams>, <LightSphere>, <LightMesh>.
#include "../../include/rtg_host.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cstdint>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#ifdef RTGH_HAVE_PNG
#include <png.h>
#endif
#ifdef RTGH_HAVE_JPEG
#include <dlfcn.h>
#include <jpeglib.h>
#endif

#include "exr_read.hpp"
#include "xml.hpp"

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& m) { g_err = m; return code; }

struct TexData {
    rtg_texture_desc d{};
    std::vector<float> texels;     // h * w * 3
    int image_id = 0;
};
struct ObjData {
    rtg_object_desc d{};
    std::vector<rtg_xform_ref> xf;
    std::vector<int32_t> faces;    // triples
};
struct InstData {
    rtg_instance_desc d{};
    std::vector<rtg_xform_ref> xf;
};
struct CamData {
    rtg_camera_desc d{};
    std::string image_name;
    bool has_tonemap = false;
    rtg_tonemap_desc tm{};
};

// ------------------------------------------------------------------ text helpers (tinyxml2 / libc)
const char* text_of(const rtgh::XmlElement* e) { return (e && e->has_text) ? e->text.c_str() : (e ? "" : nullptr); }
const char* child_text(const rtgh::XmlElement* e, const char* tag) { return e ? text_of(e->child(tag)) : nullptr; }

bool query_int(const char* s, int& out) {          // XMLElement::QueryIntText: sscanf "%d"
    if (!s) return false;
    int v;
    if (sscanf(s, "%d", &v) != 1) return false;
    out = v;
    return true;
}
bool query_float(const char* s, float& out) {      // XMLElement::QueryFloatText: sscanf "%f"
    if (!s) return false;
    float v;
    if (sscanf(s, "%f", &v) != 1) return false;
    out = v;
    return true;
}
void scan3(const char* s, float* v) {               // sscanf(str, "%f %f %f", ...) into zeroed storage
    v[0] = v[1] = v[2] = 0.0f;
    if (s) sscanf(s, "%f %f %f", &v[0], &v[1], &v[2]);
}
// attribute scan with strncmp semantics (Parser.h: shadingMode / handedness / degamma / type ...)
bool attr_prefix(const rtgh::XmlElement* e, const char* name, const char* value) {
    for (const auto& a : e->attrs)
        if (strncmp(a.first.c_str(), name, strlen(name)) == 0) return strncmp(a.second.c_str(), value, strlen(value)) == 0;
    return false;
}
bool attr_int(const rtgh::XmlElement* e, const char* name, int& out) {   // QueryIntAttribute
    const std::string* v = e->attr(name);
    return v && sscanf(v->c_str(), "%d", &out) == 1;
}

// Parser::ParseObjectTransformations (src/Parser.h:769-796)
void parse_object_transformations(const char* str, std::vector<rtg_xform_ref>& out) {
    size_t cur = 0, n = strlen(str);
    while (cur < n) {
        const char ch = str[cur];
        int type = ch == 't' ? RTG_XF_TRANSLATION : ch == 's' ? RTG_XF_SCALING : ch == 'r' ? RTG_XF_ROTATION
                 : ch == 'c' ? RTG_XF_COMPOSITE : 0;
        if (type) out.push_back({type, atoi(str + cur + 1)});
        cur++;
        while (cur < n && str[cur] != 's' && str[cur] != 't' && str[cur] != 'r') cur++;
    }
}

// object <Textures> (src/Parser.h:830-853): two ids iff the text holds a space
std::vector<int> parse_textures_list(const char* str) {
    std::vector<int> v;
    const char* p = str;
    while (*p) {
        char* e;
        long x = strtol(p, &e, 10);
        if (e == p) { p++; continue; }
        v.push_back((int)x);
        p = e;
    }
    const bool two = strchr(str, ' ') != nullptr;
    if (v.size() > (two ? 2u : 1u)) v.resize(two ? 2 : 1);
    return v;
}

// whitespace-separated numbers, what the reference's atof cursor loops read
// (ParseVertices Parser.h:684-727, ParseTextureCoordinates Parser.h:729-767, mesh faces Parser.h:1117-1141)
std::vector<double> numbers(const char* s) {
    std::vector<double> v;
    if (!s) return v;
    const char* p = s;
    while (*p) {
        while (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r') p++;
        if (!*p) break;
        char* e;
        double x = strtod(p, &e);
        if (e == p) { while (*p && !(*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; continue; }
        v.push_back(x);
        p = e;
    }
    return v;
}

bool read_file(const std::string& path, std::string& out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::ostringstream ss;
    ss << f.rdbuf();
    out = ss.str();
    return true;
}

// ------------------------------------------------------------------ PLY (what happly gives Parser.h Parser.h:1020-1106)
// Vertex x,y,z (+u,v) as doubles and face index lists (flat: fcount[k] indices each), for
// ascii, binary_little_endian and binary_big_endian files.  Property types are resolved once
// per header so the 1 M-triangle meshes load at memory speed.
struct Ply {
    std::vector<double> xyz, uv;                 // per vertex
    std::vector<int64_t> fidx;                   // all face indices, in order
    std::vector<int> fcount;                     // indices per face
};
enum PlyType { PT_NONE, PT_I8, PT_U8, PT_I16, PT_U16, PT_I32, PT_U32, PT_F32, PT_F64 };
PlyType ply_type(const std::string& t) {
    if (t == "char" || t == "int8") return PT_I8;
    if (t == "uchar" || t == "uint8") return PT_U8;
    if (t == "short" || t == "int16") return PT_I16;
    if (t == "ushort" || t == "uint16") return PT_U16;
    if (t == "int" || t == "int32") return PT_I32;
    if (t == "uint" || t == "uint32") return PT_U32;
    if (t == "float" || t == "float32") return PT_F32;
    if (t == "double" || t == "float64") return PT_F64;
    return PT_NONE;
}
const int kPlySize[] = {0, 1, 1, 2, 2, 4, 4, 4, 8};

int read_ply(const std::string& path, Ply& out) {
    std::string data;
    if (!read_file(path, data)) return fail(RTG_ERR_INVALID, "cannot read PLY " + path);
    size_t he = data.find("end_header");
    if (he == std::string::npos) return fail(RTG_ERR_INVALID, "PLY without end_header: " + path);
    size_t body = data.find('\n', he);
    if (body == std::string::npos) return fail(RTG_ERR_INVALID, "truncated PLY header");
    body++;
    struct Prop { bool list; PlyType type, count_type; std::string name; };
    struct Elem { std::string name; long count; std::vector<Prop> props; };
    std::vector<Elem> elems;
    std::string fmt;
    std::istringstream hs(data.substr(0, body));
    std::string line;
    while (std::getline(hs, line)) {
        std::istringstream ls(line);
        std::string k;
        ls >> k;
        if (k == "format") ls >> fmt;
        else if (k == "element") { Elem e; ls >> e.name >> e.count; elems.push_back(e); }
        else if (k == "property" && !elems.empty()) {
            Prop p;
            std::string t, ct, it;
            ls >> t;
            if (t == "list") { p.list = true; ls >> ct >> it >> p.name; p.count_type = ply_type(ct); p.type = ply_type(it); }
            else { p.list = false; p.type = ply_type(t); p.count_type = PT_NONE; ls >> p.name; }
            if (p.type == PT_NONE || (p.list && p.count_type == PT_NONE))
                return fail(RTG_ERR_INVALID, "PLY property type in " + path);
            elems.back().props.push_back(p);
        }
    }
    const bool ascii = fmt == "ascii", be = fmt == "binary_big_endian";
    if (!ascii && fmt != "binary_little_endian" && !be) return fail(RTG_ERR_INVALID, "unsupported PLY format " + fmt);
    const unsigned char* b = (const unsigned char*)data.data() + body;
    const size_t nb = data.size() - body;
    size_t off = 0;
    bool ok = true;
    auto bin = [&](PlyType t) -> double {
        const int s = kPlySize[t];
        if (off + s > nb) { ok = false; return 0.0; }
        unsigned char tmp[8];
        if (be) for (int i = 0; i < s; i++) tmp[i] = b[off + s - 1 - i];
        else memcpy(tmp, b + off, s);
        off += s;
        switch (t) {
        case PT_I8: return (double)(int8_t)tmp[0];
        case PT_U8: return (double)tmp[0];
        case PT_I16: { int16_t x; memcpy(&x, tmp, 2); return x; }
        case PT_U16: { uint16_t x; memcpy(&x, tmp, 2); return x; }
        case PT_I32: { int32_t x; memcpy(&x, tmp, 4); return x; }
        case PT_U32: { uint32_t x; memcpy(&x, tmp, 4); return x; }
        case PT_F32: { float x; memcpy(&x, tmp, 4); return x; }
        default: { double x; memcpy(&x, tmp, 8); return x; }
        }
    };
    const char* ap = data.c_str() + body;
    auto asc = [&]() -> double {
        char* e;
        const double v = strtod(ap, &e);
        if (e == ap) ok = false;
        ap = e;
        return v;
    };
    auto next = [&](PlyType t) { return ascii ? asc() : bin(t); };
    for (const Elem& e : elems) {
        int ix = -1, iy = -1, iz = -1, iu = -1, iv = -1;
        for (size_t k = 0; k < e.props.size(); k++) {
            const std::string& n = e.props[k].name;
            if (n == "x") ix = (int)k; else if (n == "y") iy = (int)k; else if (n == "z") iz = (int)k;
            else if (n == "u") iu = (int)k; else if (n == "v") iv = (int)k;
        }
        const bool isv = e.name == "vertex", isf = e.name == "face";
        if (isv && (ix < 0 || iy < 0 || iz < 0)) return fail(RTG_ERR_INVALID, "PLY vertex without x/y/z");
        if (isv) {
            out.xyz.reserve(out.xyz.size() + 3 * (size_t)e.count);
            if (iu >= 0 && iv >= 0) out.uv.reserve(out.uv.size() + 2 * (size_t)e.count);
        }
        if (isf) out.fcount.reserve(out.fcount.size() + (size_t)e.count);
        double vals[64];
        if (e.props.size() > 64) return fail(RTG_ERR_UNSUPPORTED, "PLY element with > 64 properties");
        for (long r = 0; r < e.count && ok; r++) {
            for (size_t k = 0; k < e.props.size(); k++) {
                const Prop& p = e.props[k];
                if (p.list) {
                    const long cnt = (long)next(p.count_type);
                    if (isf) out.fcount.push_back((int)cnt);
                    for (long q = 0; q < cnt; q++) {
                        const double x = next(p.type);
                        if (isf) out.fidx.push_back((int64_t)x);
                    }
                } else {
                    vals[k] = next(p.type);
                }
            }
            if (isv) {
                out.xyz.push_back(vals[ix]); out.xyz.push_back(vals[iy]); out.xyz.push_back(vals[iz]);
                if (iu >= 0 && iv >= 0) { out.uv.push_back(vals[iu]); out.uv.push_back(vals[iv]); }
            }
        }
        if (!ok) return fail(RTG_ERR_INVALID, "truncated PLY element " + e.name + " in " + path);
    }
    return RTG_OK;
}

// ------------------------------------------------------------------ images (src/Texture.cpp:133-300)
// Decoded as the texture code sees them: 8-bit RGB raw values 0..255 as floats, row 0 first.
int read_ppm(const std::string& path, std::vector<float>& px, int& w, int& h) {
    std::string d;
    if (!read_file(path, d)) return fail(RTG_ERR_INVALID, "cannot read image " + path);
    size_t p = 0;
    auto tok = [&]() {
        while (p < d.size()) {
            if (d[p] == '#') { while (p < d.size() && d[p] != '\n') p++; continue; }
            if (isspace((unsigned char)d[p])) { p++; continue; }
            break;
        }
        size_t b = p;
        while (p < d.size() && !isspace((unsigned char)d[p])) p++;
        return d.substr(b, p - b);
    };
    std::string magic = tok();
    w = atoi(tok().c_str()); h = atoi(tok().c_str());
    int mx = atoi(tok().c_str());
    if (w <= 0 || h <= 0 || mx <= 0) return fail(RTG_ERR_INVALID, "bad PPM header " + path);
    px.assign((size_t)w * h * 3, 0.0f);
    if (magic == "P6") {
        p++;
        if (p + (size_t)w * h * 3 > d.size()) return fail(RTG_ERR_INVALID, "truncated PPM " + path);
        const float s = mx != 255 ? 255.0f / mx : 1.0f;
        for (size_t i = 0; i < px.size(); i++) px[i] = mx != 255 ? (float)(unsigned char)d[p + i] * s : (float)(unsigned char)d[p + i];
    } else if (magic == "P3") {
        for (size_t i = 0; i < px.size(); i++) px[i] = (float)atoi(tok().c_str());
    } else {
        return fail(RTG_ERR_UNSUPPORTED, "PPM flavour " + magic);
    }
    return RTG_OK;
}

#ifdef RTGH_HAVE_PNG
int read_png(const std::string& path, std::vector<float>& px, int& w, int& h) {
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return fail(RTG_ERR_INVALID, "cannot read image " + path);
    png_structp ps = png_create_read_struct(PNG_LIBPNG_VER_STRING, nullptr, nullptr, nullptr);
    png_infop pi = png_create_info_struct(ps);
    if (setjmp(png_jmpbuf(ps))) { png_destroy_read_struct(&ps, &pi, nullptr); fclose(f); return fail(RTG_ERR_INVALID, "PNG decode " + path); }
    png_init_io(ps, f);
    png_read_info(ps, pi);
    const int ct = png_get_color_type(ps, pi), bd = png_get_bit_depth(ps, pi);
    if (bd == 16) png_set_strip_16(ps);
    if (ct == PNG_COLOR_TYPE_PALETTE) png_set_palette_to_rgb(ps);
    if ((ct == PNG_COLOR_TYPE_GRAY || ct == PNG_COLOR_TYPE_GRAY_ALPHA) && bd < 8) png_set_expand_gray_1_2_4_to_8(ps);
    if (ct == PNG_COLOR_TYPE_GRAY || ct == PNG_COLOR_TYPE_GRAY_ALPHA) png_set_gray_to_rgb(ps);
    if (ct & PNG_COLOR_MASK_ALPHA) png_set_strip_alpha(ps);
    png_set_strip_alpha(ps);
    png_read_update_info(ps, pi);
    w = (int)png_get_image_width(ps, pi); h = (int)png_get_image_height(ps, pi);
    const size_t rb = png_get_rowbytes(ps, pi);
    std::vector<unsigned char> buf(rb * h);
    std::vector<png_bytep> rows(h);
    for (int y = 0; y < h; y++) rows[y] = buf.data() + rb * y;
    png_read_image(ps, rows.data());
    png_destroy_read_struct(&ps, &pi, nullptr);
    fclose(f);
    px.resize((size_t)w * h * 3);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w * 3; x++) px[(size_t)y * w * 3 + x] = (float)buf[rb * y + x];
    return RTG_OK;
}
#endif
#ifdef RTGH_HAVE_JPEG
// libjpeg 9 is resolved at run time (env RTGH_LIBJPEG or the build's path) so that linking the
// library's directory never shadows the system C++ runtime.
struct JpegApi {
    jpeg_error_mgr* (*std_error)(jpeg_error_mgr*);
    void (*create)(j_decompress_ptr, int, size_t);
    void (*stdio_src)(j_decompress_ptr, FILE*);
    int (*read_header)(j_decompress_ptr, boolean);
    boolean (*start)(j_decompress_ptr);
    JDIMENSION (*read_scanlines)(j_decompress_ptr, JSAMPARRAY, JDIMENSION);
    boolean (*finish)(j_decompress_ptr);
    void (*destroy)(j_decompress_ptr);
    bool ok = false;
};
const JpegApi& jpeg_api() {
    static JpegApi a = [] {
        JpegApi x{};
        const char* path = getenv("RTGH_LIBJPEG");
        void* h = dlopen(path ? path : RTGH_LIBJPEG, RTLD_NOW | RTLD_LOCAL);
        if (!h) return x;
        x.std_error = (jpeg_error_mgr * (*)(jpeg_error_mgr*)) dlsym(h, "jpeg_std_error");
        x.create = (void (*)(j_decompress_ptr, int, size_t))dlsym(h, "jpeg_CreateDecompress");
        x.stdio_src = (void (*)(j_decompress_ptr, FILE*))dlsym(h, "jpeg_stdio_src");
        x.read_header = (int (*)(j_decompress_ptr, boolean))dlsym(h, "jpeg_read_header");
        x.start = (boolean(*)(j_decompress_ptr))dlsym(h, "jpeg_start_decompress");
        x.read_scanlines = (JDIMENSION(*)(j_decompress_ptr, JSAMPARRAY, JDIMENSION))dlsym(h, "jpeg_read_scanlines");
        x.finish = (boolean(*)(j_decompress_ptr))dlsym(h, "jpeg_finish_decompress");
        x.destroy = (void (*)(j_decompress_ptr))dlsym(h, "jpeg_destroy_decompress");
        x.ok = x.std_error && x.create && x.stdio_src && x.read_header && x.start && x.read_scanlines && x.finish &&
               x.destroy;
        return x;
    }();
    return a;
}
int read_jpeg(const std::string& path, std::vector<float>& px, int& w, int& h) {
    const JpegApi& J = jpeg_api();
    if (!J.ok) return fail(RTG_ERR_UNSUPPORTED, "libjpeg 9 not loadable (set RTGH_LIBJPEG): " + path);
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return fail(RTG_ERR_INVALID, "cannot read image " + path);
    jpeg_decompress_struct cinfo;
    jpeg_error_mgr jerr;
    cinfo.err = J.std_error(&jerr);
    J.create(&cinfo, JPEG_LIB_VERSION, sizeof(cinfo));
    J.stdio_src(&cinfo, f);
    J.read_header(&cinfo, TRUE);
    cinfo.out_color_space = JCS_RGB;
    J.start(&cinfo);
    w = (int)cinfo.output_width; h = (int)cinfo.output_height;
    std::vector<unsigned char> row((size_t)w * 3);
    px.resize((size_t)w * h * 3);
    for (int y = 0; y < h; y++) {
        unsigned char* r = row.data();
        J.read_scanlines(&cinfo, &r, 1);
        for (int x = 0; x < w * 3; x++) px[(size_t)y * w * 3 + x] = (float)row[x];
    }
    J.finish(&cinfo);
    J.destroy(&cinfo);
    fclose(f);
    return RTG_OK;
}
#endif

std::string lower(std::string s) { for (char& c : s) c = (char)tolower((unsigned char)c); return s; }
bool ends_with(const std::string& s, const char* t) { size_t k = strlen(t); return s.size() >= k && s.compare(s.size() - k, k, t) == 0; }

int load_image(const std::string& path, std::vector<float>& px, int& w, int& h) {
    const std::string l = lower(path);
    if (ends_with(l, ".ppm") || ends_with(l, ".pnm")) return read_ppm(path, px, w, h);
    if (ends_with(l, ".exr")) {             // Texture::ReadExr (src/Texture.cpp:185-189): linear floats
        std::vector<float> rgba;
        std::string e;
        if (!rtgh::read_exr_rgba(path, rgba, w, h, e)) return fail(RTG_ERR_INVALID, e);
        px.resize((size_t)w * h * 3);
        for (size_t i = 0; i < (size_t)w * h; i++)
            for (int c = 0; c < 3; c++) px[3 * i + c] = rgba[4 * i + c];
        return RTG_OK;
    }
#ifdef RTGH_HAVE_PNG
    if (ends_with(l, ".png")) return read_png(path, px, w, h);
#endif
#ifdef RTGH_HAVE_JPEG
    if (ends_with(l, ".jpg") || ends_with(l, ".jpeg")) return read_jpeg(path, px, w, h);
#endif
    return fail(RTG_ERR_UNSUPPORTED, "image format not supported by this build: " + path);
}

}  // namespace

// ------------------------------------------------------------------ the parsed scene
struct rtgh_scene {
    int max_depth = 1;
    float shadow_eps = 0.002f, int_eps = 0.001f;
    float background[3] = {0, 0, 0}, ambient[3] = {0, 0, 0};
    int background_texture = -1, environment_light = -1;
    std::vector<CamData> cameras;
    std::vector<rtg_material_desc> materials;
    std::vector<TexData> textures;
    std::vector<std::string> images;
    std::vector<float> translations, scalings, rotations, composites;
    std::vector<float> vertices, texcoords;
    std::vector<ObjData> objects;
    std::vector<InstData> instances;
    std::vector<rtg_light_desc> lights;
    // flattened descriptor storage
    std::vector<rtg_xform_ref> xrefs;
    std::vector<int32_t> faces;
    std::vector<rtg_object_desc> objs;
    std::vector<rtg_instance_desc> insts;
    std::vector<rtg_texture_desc> texs;
    rtg_scene_desc desc{};
};

namespace {

int parse(const std::string& xml_path, rtgh_scene& sc) {
    std::string src;
    if (!read_file(xml_path, src)) return fail(RTG_ERR_INVALID, "cannot read " + xml_path);
    std::string err;
    rtgh::XmlParser xp;
    auto root = xp.parse(src, err);
    if (!root) return fail(RTG_ERR_INVALID, err);
    const size_t slash = xml_path.rfind('/');
    const std::string base = slash == std::string::npos ? "" : xml_path.substr(0, slash + 1);

    // ParseSceneAttributes (src/Parser.h:17-50)
    query_int(child_text(root.get(), "MaxRecursionDepth"), sc.max_depth);
    scan3(child_text(root.get(), "BackgroundColor"), sc.background);
    query_float(child_text(root.get(), "ShadowRayEpsilon"), sc.shadow_eps);
    query_float(child_text(root.get(), "IntersectionTestEpsilon"), sc.int_eps);

    // ParseCameras (Parser.h:52-164)
    if (const rtgh::XmlElement* ce0 = root->child("Cameras")) {
        for (const rtgh::XmlElement* ce : ce0->all("Camera")) {
            CamData c;
            rtg_camera_desc& d = c.d;
            d.left = -1; d.right = 1; d.bottom = -1; d.top = 1;
            d.near_distance = 1.0f; d.num_samples = 1;
            d.gaze[2] = -1; d.up[1] = 1;
            d.left_handed = attr_prefix(ce, "handedness", "left");
            if (ce->child("FocusDistance")) { query_float(child_text(ce, "FocusDistance"), d.focus_distance); d.is_dof = 1; }
            if (ce->child("ApertureSize")) query_float(child_text(ce, "ApertureSize"), d.aperture_size);
            query_int(child_text(ce, "NumSamples"), d.num_samples);
            scan3(child_text(ce, "Position"), d.position);
            if (ce->child("Gaze")) scan3(child_text(ce, "Gaze"), d.gaze);
            if (ce->child("GazePoint")) {                                  // Parser.h:116-123
                float gp[3];
                scan3(child_text(ce, "GazePoint"), gp);
                for (int k = 0; k < 3; k++) d.gaze[k] = gp[k] - d.position[k];
            }
            scan3(child_text(ce, "Up"), d.up);
            query_float(child_text(ce, "NearDistance"), d.near_distance);
            if (const char* r = child_text(ce, "ImageResolution")) sscanf(r, "%d %d", &d.nx, &d.ny);
            if (const char* n = child_text(ce, "ImageName")) {
                std::string s = n;
                size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
                c.image_name = a == std::string::npos ? "" : s.substr(a, b - a + 1);
            }
            if (const char* np = child_text(ce, "NearPlane")) sscanf(np, "%f %f %f %f", &d.left, &d.right, &d.bottom, &d.top);
            if (ce->child("FovY")) {                                       // Parser.h:144-158
                float fov = 0.0f;
                query_float(child_text(ce, "FovY"), fov);
                const float fovr = (float)((double)(fov * 0.5f) * (3.14159265358979323846 / (double)180.0f));
                const float aspect = (float)d.nx / (float)d.ny;
                const float y = (float)tan((double)fovr) * d.near_distance;
                const float x = aspect * y;
                d.left = -x; d.right = x; d.bottom = -y; d.top = y;
            }
            // hw5 <Tonemap> (pages/Page5.md:47-53; no parser code in src/): Photographic TMO
            if (const rtgh::XmlElement* tm = ce->child("Tonemap")) {
                const char* tmo = child_text(tm, "TMO");
                std::string t = lower(tmo ? tmo : "photographic");
                size_t a = t.find_first_not_of(" \t\r\n");
                if (a != std::string::npos && t.compare(a, 12, "photographic") == 0) {
                    c.has_tonemap = true;
                    c.tm.tmo = RTG_TMO_PHOTOGRAPHIC;
                    c.tm.key = 0.18f; c.tm.burn_percent = 1.0f;
                    if (const char* o = child_text(tm, "TMOOptions")) {
                        c.tm.key = c.tm.burn_percent = 0.0f;
                        sscanf(o, "%f %f", &c.tm.key, &c.tm.burn_percent);
                    }
                    c.tm.saturation = 1.0f; c.tm.gamma = 2.2f;
                    query_float(child_text(tm, "Saturation"), c.tm.saturation);
                    query_float(child_text(tm, "Gamma"), c.tm.gamma);
                }
            }
            // hw7 (pages/Page7.md): <Renderer>PathTracing</Renderer>, <RendererParams>
            if (const char* r = child_text(ce, "Renderer")) {
                std::string s = lower(r);
                size_t a = s.find_first_not_of(" \t\r\n");
                if (a != std::string::npos && s.compare(a, 11, "pathtracing") == 0) d.integrator = RTG_INTEGRATOR_PATH;
            }
            if (const char* r = child_text(ce, "RendererParams")) {
                std::istringstream ss(lower(r));
                std::string t;
                while (ss >> t) {
                    if (t == "importancesampling") d.pt_flags |= RTG_PT_IMPORTANCE;
                    else if (t == "nexteventestimation") d.pt_flags |= RTG_PT_NEE;
                    else if (t == "russianroulette") d.pt_flags |= RTG_PT_RUSSIAN_ROULETTE;
                }
            }
            sc.cameras.push_back(c);
        }
    }

    // ParseBRDF (Parser.h:166-302): (type, id, exponent)
    struct Brdf { int type, id, exp; };
    std::vector<Brdf> brdfs;
    if (const rtgh::XmlElement* be = root->child("BRDFs")) {
        for (const char* tag : {"ModifiedBlinnPhong", "OriginalBlinnPhong", "ModifiedPhong", "OriginalPhong", "TorranceSparrow"}) {
            for (const rtgh::XmlElement* b : be->all(tag)) {
                Brdf x{0, 0, 0};
                attr_int(b, "id", x.id);
                query_int(child_text(b, "Exponent"), x.exp);
                const std::string t = tag;
                if (t == "ModifiedBlinnPhong") x.type = attr_prefix(b, "normalized", "true") ? RTG_BRDF_MBPN : RTG_BRDF_MBP;
                else if (t == "OriginalBlinnPhong") x.type = RTG_BRDF_OBP;
                else if (t == "ModifiedPhong") x.type = attr_prefix(b, "normalized", "true") ? RTG_BRDF_MPN : RTG_BRDF_MP;
                else if (t == "OriginalPhong") x.type = RTG_BRDF_OP;
                else x.type = attr_prefix(b, "kdfresnel", "true") ? RTG_BRDF_TSF : RTG_BRDF_TS;
                brdfs.push_back(x);
            }
        }
    }

    // ParseMaterials (Parser.h:304-474)
    if (const rtgh::XmlElement* me0 = root->child("Materials")) {
        for (const rtgh::XmlElement* me : me0->all("Material")) {
            rtg_material_desc m{};
            const bool degamma = attr_prefix(me, "degamma", "true");
            int bidx = -1;
            attr_int(me, "BRDF", bidx);
            if (bidx != -1)
                for (const Brdf& b : brdfs)
                    if (b.id == bidx) { m.phong_exp = b.exp; m.brdf = b.type; }
            scan3(child_text(me, "AmbientReflectance"), m.ambient);
            scan3(child_text(me, "DiffuseReflectance"), m.diffuse);
            scan3(child_text(me, "SpecularReflectance"), m.specular);
            if (degamma)
                for (float* v : {m.ambient, m.diffuse, m.specular})
                    for (int k = 0; k < 3; k++) v[k] = (float)pow((double)v[k], (double)2.2f);
            if (me->child("Roughness")) { query_float(child_text(me, "Roughness"), m.roughness); m.is_rough = 1; }
            scan3(child_text(me, "MirrorReflectance"), m.mirror);
            if (me->child("PhongExponent")) query_int(child_text(me, "PhongExponent"), m.phong_exp);
            m.type = RTG_MAT_NORMAL;
            for (const auto& a : me->attrs) {
                if (strncmp(a.first.c_str(), "type", 4) != 0) continue;
                const char* v = a.second.c_str();
                if (strncmp(v, "dielectric", 10) == 0) m.type = RTG_MAT_DIELECTRIC;
                else if (strncmp(v, "conductor", 9) == 0) m.type = RTG_MAT_CONDUCTOR;
                else if (strncmp(v, "mirror", 6) == 0) m.type = RTG_MAT_MIRROR;
                break;
            }
            query_float(child_text(me, "RefractionIndex"), m.refraction_index);
            query_float(child_text(me, "AbsorptionIndex"), m.absorption_index);
            scan3(child_text(me, "AbsorptionCoefficient"), m.absorption_coeff);
            sc.materials.push_back(m);
        }
    }

    // ParseTextures (Parser.h:476-605): fields carry over between TextureMaps
    std::map<std::string, std::pair<std::vector<float>, std::pair<int, int>>> cache;
    auto image = [&](const std::string& path, TexData& t) -> int {
        auto it = cache.find(path);
        if (it == cache.end()) {
            std::vector<float> px;
            int w = 0, h = 0;
            int rc = load_image(path, px, w, h);
            if (rc) return rc;
            it = cache.emplace(path, std::make_pair(std::move(px), std::make_pair(w, h))).first;
        }
        t.texels = it->second.first;
        t.d.width = it->second.second.first;
        t.d.height = it->second.second.second;
        return RTG_OK;
    };
    if (const rtgh::XmlElement* te = root->child("Textures")) {
        if (const rtgh::XmlElement* ie = te->child("Images"))
            for (const rtgh::XmlElement* im : ie->all("Image")) {
                std::string s = text_of(im);
                size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
                sc.images.push_back(base + (a == std::string::npos ? "" : s.substr(a, b - a + 1)));
            }
        bool is_image = false;
        int image_id = 0, normalizer = 255, dm = RTG_DECAL_NONE, nc = RTG_NC_LINEAR, interp = RTG_INTERP_NN;
        float noise_scale = 1.0f, bump = 1.0f;
        for (const rtgh::XmlElement* tm : te->all("TextureMap")) {
            for (const auto& a : tm->attrs)
                if (strncmp(a.first.c_str(), "type", 4) == 0) { is_image = strncmp(a.second.c_str(), "image", 5) == 0; break; }
            if (tm->child("ImageId")) query_int(child_text(tm, "ImageId"), image_id);
            if (const char* s = child_text(tm, "DecalMode")) {
                static const std::pair<const char*, int> modes[] = {
                    {"blend_kd", RTG_DECAL_BLEND_KD}, {"replace_kd", RTG_DECAL_REPLACE_KD},
                    {"replace_all", RTG_DECAL_REPLACE_ALL}, {"bump_normal", RTG_DECAL_BUMP_NORMAL},
                    {"replace_normal", RTG_DECAL_REPLACE_NORMAL}, {"replace_background", RTG_DECAL_REPLACE_BACKGROUND}};
                for (const auto& md : modes)
                    if (strncmp(s, md.first, strlen(md.first)) == 0) { dm = md.second; break; }
            }
            if (const char* s = child_text(tm, "NoiseConversion")) nc = strncmp(s, "absval", 6) == 0 ? RTG_NC_ABSVAL : RTG_NC_LINEAR;
            if (const char* s = child_text(tm, "Interpolation")) {
                if (strncmp(s, "nearest", 7) == 0) interp = RTG_INTERP_NN;
                else if (strncmp(s, "bilinear", 8) == 0) interp = RTG_INTERP_BILINEAR;
            }
            if (tm->child("Normalizer")) query_int(child_text(tm, "Normalizer"), normalizer);
            if (tm->child("NoiseScale")) query_float(child_text(tm, "NoiseScale"), noise_scale);
            if (tm->child("BumpFactor")) query_float(child_text(tm, "BumpFactor"), bump);
            TexData t;
            t.d.decal = dm; t.d.interp = interp; t.d.normalizer = normalizer; t.d.bump_factor = bump;
            t.d.noise_conv = nc; t.d.noise_scale = noise_scale;
            if (is_image) {
                t.d.kind = RTG_TEX_IMAGE;
                t.image_id = image_id;
                if (image_id < 1 || image_id > (int)sc.images.size()) return fail(RTG_ERR_INVALID, "TextureMap ImageId out of range");
                int rc = image(sc.images[image_id - 1], t);
                if (rc) return rc;
            } else {
                t.d.kind = RTG_TEX_PERLIN;
            }
            sc.textures.push_back(std::move(t));
        }
    }

    // ParseTransformations (Parser.h:607-682)
    if (const rtgh::XmlElement* tr = root->child("Transformations")) {
        for (const rtgh::XmlElement* t : tr->all("Translation")) { float v[3]; scan3(text_of(t), v); sc.translations.insert(sc.translations.end(), v, v + 3); }
        for (const rtgh::XmlElement* t : tr->all("Scaling")) { float v[3]; scan3(text_of(t), v); sc.scalings.insert(sc.scalings.end(), v, v + 3); }
        for (const rtgh::XmlElement* t : tr->all("Rotation")) {
            float v[4] = {0, 0, 0, 0};
            sscanf(text_of(t), "%f %f %f %f", &v[0], &v[1], &v[2], &v[3]);
            sc.rotations.insert(sc.rotations.end(), v, v + 4);
        }
        for (const rtgh::XmlElement* t : tr->all("Composite")) {
            float v[16] = {0};
            const char* p = text_of(t);
            for (int k = 0; k < 16; k++) {                                  // XML row-major -> [col][row]
                char* e;
                float x = strtof(p, &e);
                if (e == p) break;
                v[k] = x;
                p = e;
            }
            float cm[16];
            for (int k = 0; k < 16; k++) cm[(k % 4) * 4 + k / 4] = v[k];
            sc.composites.insert(sc.composites.end(), cm, cm + 16);
        }
    }

    // ParseVertices / ParseTextureCoordinates (Parser.h:684-767): atof -> double -> float
    {
        std::vector<double> v = numbers(child_text(root.get(), "VertexData"));
        for (size_t k = 0; k + 2 < v.size(); k += 3)
            sc.vertices.insert(sc.vertices.end(), {(float)v[k], (float)v[k + 1], (float)v[k + 2]});
        std::vector<double> t = numbers(child_text(root.get(), "TexCoordData"));
        for (size_t k = 0; k + 1 < t.size(); k += 2) sc.texcoords.insert(sc.texcoords.end(), {(float)t[k], (float)t[k + 1]});
    }

    // ParseObjects (Parser.h:798-1195); hw7: <LightSphere> after the spheres, <LightMesh> after the meshes
    const rtgh::XmlElement* oe = root->child("Objects");
    if (!oe) return fail(RTG_ERR_INVALID, "no <Objects>");
    auto common = [&](const rtgh::XmlElement* el, ObjData& o) {
        o.d.center = 1; o.d.radius = 1.0f; o.d.v[0] = 1; o.d.v[1] = 2; o.d.v[2] = 3;   // rtg/scene.py defaults
        attr_int(el, "id", o.d.id);
        o.d.material = 1;
        query_int(child_text(el, "Material"), o.d.material);
        if (const char* x = child_text(el, "Transformations")) parse_object_transformations(x, o.xf);
        if (const char* x = child_text(el, "Textures")) {
            std::vector<int> t = parse_textures_list(x);
            o.d.num_textures = (int)t.size();
            for (size_t k = 0; k < t.size(); k++) o.d.textures[k] = t[k];
        }
        if (el->child("MotionBlur")) scan3(child_text(el, "MotionBlur"), o.d.blur);
    };
    auto light = [&](const rtgh::XmlElement* el, ObjData& o) {
        o.d.is_light = 1;
        scan3(child_text(el, "Radiance"), o.d.radiance);
    };
    for (const char* tag : {"Sphere", "LightSphere"})
        for (const rtgh::XmlElement* el : oe->all(tag)) {
            ObjData o;
            o.d.type = RTG_OBJ_SPHERE;
            common(el, o);
            o.d.center = 1; o.d.radius = 1.0f;
            query_int(child_text(el, "Center"), o.d.center);
            query_float(child_text(el, "Radius"), o.d.radius);
            if (strcmp(tag, "LightSphere") == 0) light(el, o);
            sc.objects.push_back(std::move(o));
        }
    for (const rtgh::XmlElement* el : oe->all("Triangle")) {
        ObjData o;
        o.d.type = RTG_OBJ_TRIANGLE;
        common(el, o);
        if (const char* s = child_text(el, "Indices")) sscanf(s, "%d %d %d", &o.d.v[0], &o.d.v[1], &o.d.v[2]);
        sc.objects.push_back(std::move(o));
    }
    const int mesh_start = (int)sc.objects.size();
    std::vector<const rtgh::XmlElement*> meshes = oe->all("Mesh");
    for (const rtgh::XmlElement* el : oe->all("LightMesh")) meshes.push_back(el);
    for (const rtgh::XmlElement* el : meshes) {
        ObjData o;
        o.d.type = RTG_OBJ_MESH;
        common(el, o);
        if (el->name == "LightMesh") light(el, o);
        o.d.smooth = attr_prefix(el, "shadingMode", "smooth");
        const rtgh::XmlElement* fe = el->child("Faces");
        if (!fe) return fail(RTG_ERR_INVALID, "mesh without <Faces>");
        const std::string* ply = nullptr;
        for (const auto& a : fe->attrs)
            if (strncmp(a.first.c_str(), "plyFile", 7) == 0) { ply = &a.second; break; }
        if (ply) {                                                          // Parser.h:1020-1106
            Ply P;
            int rc = read_ply(base + *ply, P);
            if (rc) return rc;
            const int texture_offset = (int)(sc.texcoords.size() / 2) + 1;
            for (double x : P.uv) sc.texcoords.push_back((float)x);
            const int vertex_count = (int)(sc.vertices.size() / 3) + 1;
            o.faces.reserve(6 * P.fcount.size());
            size_t q = 0;
            for (int cnt : P.fcount) {
                const int64_t* f = P.fidx.data() + q;
                q += (size_t)cnt;
                if (cnt == 4) {
                    o.faces.insert(o.faces.end(), {(int)(f[0] + vertex_count), (int)(f[1] + vertex_count), (int)(f[2] + vertex_count)});
                    o.faces.insert(o.faces.end(), {(int)(f[2] + vertex_count), (int)(f[3] + vertex_count), (int)(f[0] + vertex_count)});
                } else if (cnt >= 3) {
                    o.faces.insert(o.faces.end(), {(int)(f[0] + vertex_count), (int)(f[1] + vertex_count), (int)(f[2] + vertex_count)});
                }
            }
            for (double x : P.xyz) sc.vertices.push_back((float)x);
            o.d.texture_offset = texture_offset - vertex_count;
        } else {                                                            // Parser.h:1109-1149
            int vo = 0, to = 0;
            attr_int(fe, "vertexOffset", vo);
            attr_int(fe, "textureOffset", to);
            std::vector<double> v = numbers(text_of(fe));
            for (size_t k = 0; k + 2 < v.size(); k += 3)
                o.faces.insert(o.faces.end(), {(int)v[k] + vo, (int)v[k + 1] + vo, (int)v[k + 2] + vo});
            o.d.texture_offset = to - vo;
        }
        sc.objects.push_back(std::move(o));
    }
    for (const rtgh::XmlElement* el : oe->all("MeshInstance")) {           // Parser.h:1151-1195
        InstData it;
        attr_int(el, "id", it.d.id);
        int base_id = 0;
        attr_int(el, "baseMeshId", base_id);
        if (const std::string* rt = el->attr("resetTransform")) {
            std::string v = lower(*rt);
            size_t a = v.find_first_not_of(" \t\r\n"), b = v.find_last_not_of(" \t\r\n");
            v = a == std::string::npos ? "" : v.substr(a, b - a + 1);
            it.d.reset_transform = v == "true" || v == "1";
        }
        it.d.material = 1;
        query_int(child_text(el, "Material"), it.d.material);
        if (const char* x = child_text(el, "Transformations")) parse_object_transformations(x, it.xf);
        if (el->child("MotionBlur")) scan3(child_text(el, "MotionBlur"), it.d.blur);
        int found = -1;
        for (int i = mesh_start; i < (int)sc.objects.size(); i++)
            if (sc.objects[i].d.id == base_id) found = i;
        if (found < 0) return fail(RTG_ERR_INVALID, "MeshInstance " + std::to_string(it.d.id) + ": base mesh not found");
        it.d.base_object = found;
        sc.instances.push_back(it);
    }

    // ParseLights (Parser.h:1197-1315): Point, Directional, Spot, Area, SphericalDirectional
    if (const rtgh::XmlElement* le = root->child("Lights")) {
        scan3(child_text(le, "AmbientLight"), sc.ambient);
        for (const rtgh::XmlElement* l : le->all("PointLight")) {
            rtg_light_desc d{};
            d.type = RTG_LIGHT_POINT; d.texture = -1; d.direction[1] = -1;
            scan3(child_text(l, "Position"), d.position);
            scan3(child_text(l, "Intensity"), d.intensity);
            sc.lights.push_back(d);
        }
        for (const rtgh::XmlElement* l : le->all("DirectionalLight")) {
            rtg_light_desc d{};
            d.type = RTG_LIGHT_DIRECTIONAL; d.texture = -1;
            scan3(child_text(l, "Direction"), d.direction);
            scan3(child_text(l, "Radiance"), d.intensity);
            sc.lights.push_back(d);
        }
        for (const rtgh::XmlElement* l : le->all("SpotLight")) {
            rtg_light_desc d{};
            d.type = RTG_LIGHT_SPOT; d.texture = -1;
            scan3(child_text(l, "Position"), d.position);
            scan3(child_text(l, "Direction"), d.direction);
            scan3(child_text(l, "Intensity"), d.intensity);
            query_float(child_text(l, "CoverageAngle"), d.coverage_deg);
            query_float(child_text(l, "FalloffAngle"), d.falloff_deg);
            sc.lights.push_back(d);
        }
        for (const rtgh::XmlElement* l : le->all("AreaLight")) {
            rtg_light_desc d{};
            d.type = RTG_LIGHT_AREA; d.texture = -1;
            scan3(child_text(l, "Position"), d.position);
            scan3(child_text(l, "Normal"), d.direction);
            scan3(child_text(l, l->child("Radiance") ? "Radiance" : "Intensity"), d.intensity);
            query_float(child_text(l, "Size"), d.size);
            sc.lights.push_back(d);
        }
        for (const rtgh::XmlElement* l : le->all("SphericalDirectionalLight")) {
            sc.environment_light = (int)sc.lights.size();
            int iid = 1;
            query_int(child_text(l, "ImageId"), iid);
            if (iid < 1 || iid > (int)sc.images.size()) return fail(RTG_ERR_INVALID, "SphericalDirectionalLight ImageId out of range");
            TexData t;
            t.d.kind = RTG_TEX_IMAGE; t.d.decal = RTG_DECAL_NONE; t.d.interp = RTG_INTERP_BILINEAR; t.d.normalizer = 1;
            t.d.bump_factor = 1.0f; t.d.noise_conv = RTG_NC_LINEAR; t.d.noise_scale = 1.0f;
            t.image_id = iid;
            int rc = image(sc.images[iid - 1], t);
            if (rc) return rc;
            sc.textures.push_back(std::move(t));
            rtg_light_desc d{};
            d.type = RTG_LIGHT_ENVIRONMENT; d.texture = (int)sc.textures.size() - 1; d.direction[1] = -1;
            sc.lights.push_back(d);
        }
    }
    // Scene ctor: the last replace_background texture (src/Scene.cpp:494-500)
    for (size_t i = 0; i < sc.textures.size(); i++)
        if (sc.textures[i].d.decal == RTG_DECAL_REPLACE_BACKGROUND) sc.background_texture = (int)i;
    return RTG_OK;
}

void flatten(rtgh_scene& sc) {
    sc.xrefs.clear(); sc.faces.clear(); sc.objs.clear(); sc.insts.clear(); sc.texs.clear();
    for (ObjData& o : sc.objects) {
        rtg_object_desc d = o.d;
        d.xform_first = (int)sc.xrefs.size(); d.xform_count = (int)o.xf.size();
        sc.xrefs.insert(sc.xrefs.end(), o.xf.begin(), o.xf.end());
        if (d.type == RTG_OBJ_MESH) {
            d.face_first = (int)(sc.faces.size() / 3); d.face_count = (int)(o.faces.size() / 3);
            sc.faces.insert(sc.faces.end(), o.faces.begin(), o.faces.end());
        }
        sc.objs.push_back(d);
    }
    for (InstData& it : sc.instances) {
        rtg_instance_desc d = it.d;
        d.xform_first = (int)sc.xrefs.size(); d.xform_count = (int)it.xf.size();
        sc.xrefs.insert(sc.xrefs.end(), it.xf.begin(), it.xf.end());
        sc.insts.push_back(d);
    }
    for (TexData& t : sc.textures) {
        rtg_texture_desc d = t.d;
        d.texels = t.texels.empty() ? nullptr : t.texels.data();
        sc.texs.push_back(d);
    }
    rtg_scene_desc& d = sc.desc;
    memset(&d, 0, sizeof d);
    d.abi_version = RTG_ABI_VERSION;
    d.max_recursion_depth = sc.max_depth;
    d.shadow_ray_eps = sc.shadow_eps;
    d.intersection_test_eps = sc.int_eps;
    memcpy(d.background, sc.background, 12);
    memcpy(d.ambient_light, sc.ambient, 12);
    d.background_texture = sc.background_texture;
    d.environment_light = sc.environment_light;
    auto P = [](auto& v) { return v.empty() ? nullptr : v.data(); };
    d.vertices = P(sc.vertices); d.num_vertices = (int)(sc.vertices.size() / 3);
    d.texcoords = P(sc.texcoords); d.num_texcoords = (int)(sc.texcoords.size() / 2);
    d.faces = P(sc.faces); d.num_faces = (int)(sc.faces.size() / 3);
    d.translations = P(sc.translations); d.num_translations = (int)(sc.translations.size() / 3);
    d.scalings = P(sc.scalings); d.num_scalings = (int)(sc.scalings.size() / 3);
    d.rotations = P(sc.rotations); d.num_rotations = (int)(sc.rotations.size() / 4);
    d.composites = P(sc.composites); d.num_composites = (int)(sc.composites.size() / 16);
    d.xform_refs = P(sc.xrefs); d.num_xform_refs = (int)sc.xrefs.size();
    d.objects = P(sc.objs); d.num_objects = (int)sc.objs.size();
    d.instances = P(sc.insts); d.num_instances = (int)sc.insts.size();
    d.materials = P(sc.materials); d.num_materials = (int)sc.materials.size();
    d.textures = P(sc.texs); d.num_textures = (int)sc.texs.size();
    d.lights = P(sc.lights); d.num_lights = (int)sc.lights.size();
}

// Image::IsPNG (src/Image.cpp:36-60): ".png" anywhere in the name
bool is_png(const char* name) {
    int c = 0;
    for (const char* p = name; *p; p++) {
        if (*p == '.') c = 1;
        else if (*p == 'p' && c == 1) c = 2;
        else if (*p == 'n' && c == 2) c = 3;
        else if (*p == 'g' && c == 3) return true;
        else c = 0;
    }
    return false;
}

uint16_t half_of(float f) {            // IEEE binary16, round to nearest even
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ax = x & 0x7FFFFFFFu;
    if (ax >= 0x7F800000u) return (uint16_t)(sign | 0x7C00u | (ax > 0x7F800000u ? 0x200u : 0u));
    if (ax >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u);           // rounds to inf
    if (ax < 0x38800000u) {                                              // subnormal half
        if (ax < 0x33000000u) return (uint16_t)sign;
        const uint32_t m = (ax & 0x7FFFFFu) | 0x800000u;
        const int shift = 126 - (int)(ax >> 23);                          // value / 2^-24 = m * 2^(e - 126)
        uint32_t r = m >> shift;
        const uint32_t rem = m & ((1u << shift) - 1), halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (r & 1u))) r++;
        return (uint16_t)(sign | r);
    }
    uint32_t r = ((ax >> 13) - (112u << 10));
    const uint32_t rem = ax & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) r++;
    return (uint16_t)(sign | r);
}

}  // namespace

// Exceptions (std::bad_alloc from host containers, ...) never cross the C ABI.
template <class F>
static int32_t guarded(F&& f) {
    try {
        return f();
    } catch (const std::bad_alloc&) {
        return fail(RTG_ERR_OOM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(RTG_ERR_INVALID, std::string("internal error: ") + e.what());
    }
}

extern "C" {

const char* rtgh_last_error(void) { return g_err.c_str(); }

int32_t rtgh_parse_xml(const char* path, rtgh_scene** out) {
    return guarded([&]() -> int32_t {
        if (!path || !out) return fail(RTG_ERR_INVALID, "null argument");
        *out = nullptr;
        rtgh_scene* sc = new (std::nothrow) rtgh_scene();
        if (!sc) return fail(RTG_ERR_OOM, "host allocation");
        int rc = parse(path, *sc);
        if (rc) { delete sc; return rc; }
        flatten(*sc);
        *out = sc;
        return RTG_OK;
    });
}

const rtg_scene_desc* rtgh_scene_desc(const rtgh_scene* s) { return s ? &s->desc : nullptr; }
int32_t rtgh_num_cameras(const rtgh_scene* s) { return s ? (int32_t)s->cameras.size() : 0; }

int32_t rtgh_camera(const rtgh_scene* s, int32_t i, rtg_camera_desc* out, char* image_name, int32_t cap) {
    if (!s || !out || i < 0 || i >= (int32_t)s->cameras.size()) return fail(RTG_ERR_INVALID, "camera index");
    *out = s->cameras[i].d;
    if (image_name && cap > 0) {
        strncpy(image_name, s->cameras[i].image_name.c_str(), (size_t)cap - 1);
        image_name[cap - 1] = '\0';
    }
    return RTG_OK;
}

int32_t rtgh_camera_tonemap(const rtgh_scene* s, int32_t i, rtg_tonemap_desc* out) {
    if (!s || !out || i < 0 || i >= (int32_t)s->cameras.size()) return fail(RTG_ERR_INVALID, "camera index");
    if (!s->cameras[i].has_tonemap) return 0;
    *out = s->cameras[i].tm;
    return 1;
}

void rtgh_free(rtgh_scene* s) { delete s; }

int32_t rtgh_read_image(const char* path, float** rgb, int32_t* nx, int32_t* ny) {
    return guarded([&]() -> int32_t {
        if (!path || !rgb || !nx || !ny) return fail(RTG_ERR_INVALID, "null argument");
        *rgb = nullptr;
        std::vector<float> px;
        int w = 0, h = 0;
        int rc = load_image(path, px, w, h);
        if (rc) return rc;
        float* out = (float*)malloc(sizeof(float) * (px.empty() ? 1 : px.size()));
        if (!out) return fail(RTG_ERR_OOM, "host allocation");
        memcpy(out, px.data(), sizeof(float) * px.size());
        *rgb = out;
        *nx = w;
        *ny = h;
        return RTG_OK;
    });
}

void rtgh_free_image(float* rgb) { free(rgb); }

int32_t rtgh_save_image(const char* name, const float* rgb, int32_t nx, int32_t ny) {
    return guarded([&]() -> int32_t {
        if (!name || !rgb || nx < 1 || ny < 1) return fail(RTG_ERR_INVALID, "bad image");
        FILE* f = fopen(name, "wb");
        if (!f) return fail(RTG_ERR_INVALID, std::string("cannot write ") + name);
        if (is_png(name)) {                      // Image::SavePng (src/Image.cpp:62-103): P3 text
            fprintf(f, "P3\n%d %d\n255\n", nx, ny);
            std::string row;
            for (int y = 0; y < ny; y++) {
                row.clear();
                for (int x = 0; x < nx * 3; x++) {
                    float v = rgb[(size_t)y * nx * 3 + x];
                    if (v > 255) v = 255;        // src/Image.cpp:64-68
                    // (unsigned char)_data[i] (src/Image.cpp:96) as x86-64 gcc compiles it: cvttss2si to a
                    // 32-bit int, low byte kept (-1 -> 255, -300 -> 212); NaN / out-of-range -> 0x80000000 -> 0
                    const int u = (v >= -2147483648.0f) ? ((int)v & 0xFF) : 0;
                    row += std::to_string(u);
                    row += (x + 1 < nx * 3) ? " " : " \n";
                }
                fputs(row.c_str(), f);
            }
        } else {                                 // ExrLibrary::SaveExr (src/Helper.cpp:361-412): HALF B,G,R
            std::string h;
            auto i32 = [&](int32_t v) { h.append((const char*)&v, 4); };
            auto attr = [&](const char* n, const char* t, const std::string& data) {
                h += n; h += '\0'; h += t; h += '\0'; i32((int32_t)data.size()); h += data;
            };
            h.append("\x76\x2f\x31\x01", 4);
            i32(2);
            std::string chl;
            for (const char* ch : {"B", "G", "R"}) {
                chl += ch; chl += '\0';
                int32_t pt = 1; chl.append((const char*)&pt, 4);
                chl += '\0'; chl.append(3, '\0');
                int32_t one = 1; chl.append((const char*)&one, 4); chl.append((const char*)&one, 4);
            }
            chl += '\0';
            attr("channels", "chlist", chl);
            attr("compression", "compression", std::string(1, '\0'));
            int32_t box[4] = {0, 0, nx - 1, ny - 1};
            attr("dataWindow", "box2i", std::string((const char*)box, 16));
            attr("displayWindow", "box2i", std::string((const char*)box, 16));
            attr("lineOrder", "lineOrder", std::string(1, '\0'));
            float par = 1.0f, swc[2] = {0, 0}, sww = 1.0f;
            attr("pixelAspectRatio", "float", std::string((const char*)&par, 4));
            attr("screenWindowCenter", "v2f", std::string((const char*)swc, 8));
            attr("screenWindowWidth", "float", std::string((const char*)&sww, 4));
            h += '\0';
            const int64_t line_bytes = (int64_t)nx * 2 * 3;
            const int64_t first = (int64_t)h.size() + 8 * (int64_t)ny;
            for (int y = 0; y < ny; y++) { int64_t o = first + y * (8 + line_bytes); h.append((const char*)&o, 8); }
            fwrite(h.data(), 1, h.size(), f);
            std::vector<uint16_t> line((size_t)nx * 3);
            for (int y = 0; y < ny; y++) {
                int32_t hdr[2] = {y, (int32_t)line_bytes};
                fwrite(hdr, 4, 2, f);
                for (int c = 2, k = 0; c >= 0; c--, k++)
                    for (int x = 0; x < nx; x++) line[(size_t)k * nx + x] = half_of(rgb[((size_t)y * nx + x) * 3 + c]);
                fwrite(line.data(), 2, line.size(), f);
            }
        }
        fclose(f);
        return RTG_OK;
    });
}

// Scene::renderScene (src/Scene.cpp:294-363): precompute once, render and save every camera.
int32_t rtgh_render_scene(const char* xml_path, int32_t device, uint64_t seed, const char* out_dir) {
    return rtgh_render_scene_multi(xml_path, device, 0, seed, out_dir);
}

int32_t rtgh_render_scene_multi(const char* xml_path, int32_t device, int32_t num_devices, uint64_t seed,
                                const char* out_dir) {
    return guarded([&]() -> int32_t {
        if (num_devices < 0 || num_devices > 64) return fail(RTG_ERR_INVALID, "num_devices");
        // num_devices >= 1: the multi-GPU path (rtg_render_opts.devices = device, device+1, ...),
        // even for one GPU (one RCCL rank); 0: the single-device render
        const int visible = rtg_device_count();
        if (num_devices > visible) return fail(RTG_ERR_NO_DEVICE, "more devices requested than visible");
        std::vector<int32_t> devs(num_devices);
        for (int r = 0; r < num_devices; r++) devs[r] = (device + r) % std::max(visible, 1);
        rtgh_scene* sc = nullptr;
        int rc = rtgh_parse_xml(xml_path, &sc);
        if (rc) return rc;
        rtg_scene* gpu = nullptr;
        rtg_build_opts bo{};
        bo.bvh_builder = RTG_BVH_AUTO;   // tlas / traversal_tree: automatic (0)
        rc = rtg_scene_create_ex(&sc->desc, device, &bo, &gpu);
        if (rc) { g_err = rtg_last_error(); rtgh_free(sc); return rc; }
        printf("BVH construction complete.\n");
        for (const CamData& c : sc->cameras) {
            std::vector<float> rgb((size_t)c.d.nx * c.d.ny * 3);
            rtg_render_opts o{};
            o.seed = seed;
            o.num_devices = num_devices;   // row-block shards, one host thread per GPU, RCCL gather
            o.devices = num_devices > 0 ? devs.data() : nullptr;
            rc = rtg_render(gpu, &c.d, &o, rgb.data());
            if (rc) { g_err = rtg_last_error(); break; }
            std::string name = c.image_name;
            if (out_dir && *out_dir) {
                const size_t s = name.rfind('/');
                name = std::string(out_dir) + "/" + (s == std::string::npos ? name : name.substr(s + 1));
            }
            // hw5 <Tonemap>: the tone-mapped image goes to the name with a .png extension (a .png
            // ImageName is written tone-mapped instead of clamped), the HDR one to ImageName
            const bool png = is_png(name.c_str());
            if (!c.has_tonemap || !png) {
                rc = rtgh_save_image(name.c_str(), rgb.data(), c.d.nx, c.d.ny);
                if (rc) break;
            }
            if (c.has_tonemap) {
                std::vector<float> ldr(rgb.size());
                rc = rtg_tonemap(device, rgb.data(), c.d.nx, c.d.ny, &c.tm, ldr.data());
                if (rc) { g_err = rtg_last_error(); break; }
                const size_t dot = name.rfind('.'), sl = name.rfind('/');
                const std::string tname = (dot == std::string::npos || (sl != std::string::npos && dot < sl) ? name : name.substr(0, dot)) + ".png";
                rc = rtgh_save_image(tname.c_str(), ldr.data(), c.d.nx, c.d.ny);
                if (rc) break;
            }
            rtg_render_stats st{};
            rtg_last_render_stats(gpu, &st);
            printf("%s: %.1f ms, %.1f Mray/s, %d GPU%s\n", name.c_str(), st.render_ms, st.total_rays / (st.render_ms * 1e3),
                   st.devices, st.devices == 1 ? "" : "s");
        }
        rtg_scene_destroy(gpu);
        rtgh_free(sc);
        return rc;
    });
}

}  // extern "C"
