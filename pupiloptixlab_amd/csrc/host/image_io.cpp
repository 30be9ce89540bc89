// image_io.cpp — output side of the path: headless
// writers for the float4 "final result" buffer, replacing util::BitmapTexture::Save
// (framework/util/texture.cpp:12-85,152-160; tinyexr / stb_image_write are not
// available, so the files are written directly):
//   EXR: scanline, uncompressed, FLOAT channels stored B, G, R (texture.cpp:57-63),
//        rows flipped so the file's first line is the image top (texture.cpp:36-43)
//   HDR: Radiance RGBE, flat scanlines, flipped the same way
//        (stbi_flip_vertically_on_write(true), texture.cpp:13-14)
//   PFM: little-endian float RGB, bottom row first (the buffer's own order)
#include <cctype>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/pupil_pt.h"

namespace Pupil {
void set_last_error(const std::string &m);  // engine.hip
}

namespace {

int ierr(const std::string &m) {
    Pupil::set_last_error(m);
    return PUPIL_ERR_IO;
}

struct Bytes {
    std::vector<unsigned char> b;
    void raw(const void *p, size_t n) {
        const auto *c = static_cast<const unsigned char *>(p);
        b.insert(b.end(), c, c + n);
    }
    void str(const char *s) { raw(s, std::strlen(s) + 1); }
    void i32(int32_t v) { raw(&v, 4); }
    void u64(uint64_t v) { raw(&v, 8); }
    void f32(float v) { raw(&v, 4); }
    void u8(uint8_t v) { raw(&v, 1); }
    void attr(const char *name, const char *type, int32_t size) {
        str(name);
        str(type);
        i32(size);
    }
};

bool write_file(const char *path, const std::vector<unsigned char> &b) {
    FILE *f = std::fopen(path, "wb");
    if (!f) return false;
    const bool ok = std::fwrite(b.data(), 1, b.size(), f) == b.size();
    return std::fclose(f) == 0 && ok;
}

int save_exr(const char *path, uint32_t w, uint32_t h, const float *rgba) {
    Bytes o;
    const unsigned char magic[4] = {0x76, 0x2f, 0x31, 0x01};
    o.raw(magic, 4);
    o.i32(2);  // version 2, single-part scanline
    const char *chans[3] = {"B", "G", "R"};
    o.attr("channels", "chlist", 3 * (2 + 16) + 1);
    for (const char *c : chans) {
        o.str(c);
        o.i32(2);  // FLOAT
        o.u8(0);   // pLinear
        o.u8(0), o.u8(0), o.u8(0);
        o.i32(1), o.i32(1);  // x/y sampling
    }
    o.u8(0);
    o.attr("compression", "compression", 1);
    o.u8(0);  // NO_COMPRESSION
    o.attr("dataWindow", "box2i", 16);
    o.i32(0), o.i32(0), o.i32((int32_t)w - 1), o.i32((int32_t)h - 1);
    o.attr("displayWindow", "box2i", 16);
    o.i32(0), o.i32(0), o.i32((int32_t)w - 1), o.i32((int32_t)h - 1);
    o.attr("lineOrder", "lineOrder", 1);
    o.u8(0);  // INCREASING_Y
    o.attr("pixelAspectRatio", "float", 4);
    o.f32(1.f);
    o.attr("screenWindowCenter", "v2f", 8);
    o.f32(0.f), o.f32(0.f);
    o.attr("screenWindowWidth", "float", 4);
    o.f32(1.f);
    o.u8(0);  // end of header
    const uint64_t line_bytes = 8ull + 3ull * 4ull * w;
    const uint64_t table = o.b.size();
    for (uint32_t r = 0; r < h; r++) o.u64(table + 8ull * h + r * line_bytes);
    for (uint32_t r = 0; r < h; r++) {
        const uint32_t y = h - 1 - r;  // first line = image top
        o.i32((int32_t)r);
        o.i32((int32_t)(3 * 4 * w));
        for (int c : {2, 1, 0})  // B, G, R
            for (uint32_t x = 0; x < w; x++) o.f32(rgba[4 * ((size_t)y * w + x) + c]);
    }
    return write_file(path, o.b) ? PUPIL_OK : ierr(std::string("cannot write ") + path);
}

int save_hdr(const char *path, uint32_t w, uint32_t h, const float *rgba) {
    Bytes o;
    const std::string head = "#?RADIANCE\nFORMAT=32-bit_rle_rgbe\n\n-Y " + std::to_string(h) + " +X " +
                             std::to_string(w) + "\n";
    o.raw(head.data(), head.size());
    for (uint32_t r = 0; r < h; r++) {
        const uint32_t y = h - 1 - r;
        for (uint32_t x = 0; x < w; x++) {
            const float *p = rgba + 4 * ((size_t)y * w + x);
            const float m = std::fmax(p[0], std::fmax(p[1], p[2]));
            unsigned char e[4] = {0, 0, 0, 0};
            if (m >= 1e-32f) {
                int ex;
                const float s = std::frexp(m, &ex) * 256.f / m;
                e[0] = (unsigned char)(p[0] * s);
                e[1] = (unsigned char)(p[1] * s);
                e[2] = (unsigned char)(p[2] * s);
                e[3] = (unsigned char)(ex + 128);
            }
            o.raw(e, 4);
        }
    }
    return write_file(path, o.b) ? PUPIL_OK : ierr(std::string("cannot write ") + path);
}

int save_pfm(const char *path, uint32_t w, uint32_t h, const float *rgba) {
    Bytes o;
    const std::string head = "PF\n" + std::to_string(w) + " " + std::to_string(h) + "\n-1.0\n";
    o.raw(head.data(), head.size());
    for (size_t i = 0; i < (size_t)w * h; i++) o.raw(rgba + 4 * i, 12);
    return write_file(path, o.b) ? PUPIL_OK : ierr(std::string("cannot write ") + path);
}

bool ends_with(const std::string &s, const char *suf) {
    const size_t n = std::strlen(suf);
    if (s.size() < n) return false;
    for (size_t i = 0; i < n; i++)
        if (std::tolower((unsigned char)s[s.size() - n + i]) != suf[i]) return false;
    return true;
}

}  // namespace

extern "C" int pupil_image_save(const char *path, uint32_t width, uint32_t height, const float *rgba,
                                uint32_t format) {
    if (!path || !rgba || !width || !height) {
        Pupil::set_last_error("invalid image");
        return PUPIL_ERR_INVALID;
    }
    const std::string p(path);
    if (format == PUPIL_IMAGE_AUTO)
        format = ends_with(p, ".exr") ? PUPIL_IMAGE_EXR
                 : ends_with(p, ".hdr") ? PUPIL_IMAGE_HDR
                 : ends_with(p, ".pfm") ? PUPIL_IMAGE_PFM
                                        : 0u;
    switch (format) {
    case PUPIL_IMAGE_EXR: return save_exr(path, width, height, rgba);
    case PUPIL_IMAGE_HDR: return save_hdr(path, width, height, rgba);
    case PUPIL_IMAGE_PFM: return save_pfm(path, width, height, rgba);
    default: Pupil::set_last_error("unknown image format (use .exr, .hdr or .pfm)"); return PUPIL_ERR_UNSUPPORTED;
    }
}
