// image_load.cpp — input side of the bitmap path: the
// decoders behind util::BitmapTexture::Load (framework/util/texture.cpp:87-174),
// which the reference takes from tinyexr and stb_image (empty submodules here,
// so both are restated from their published behaviour):
//   * extension ".exr" (exact, case-sensitive, texture.cpp:166-170) -> LoadEXR:
//     single-part scanline files, NONE / RLE / ZIPS / ZIP compression, HALF /
//     FLOAT / UINT channels; output R, G, B and A (1 when absent), a single
//     channel replicated into all four (tinyexr LoadEXR);
//   * otherwise stb_image: Radiance HDR by signature (stbi_is_hdr) through
//     stbi_loadf (RGBE -> float with ldexp(1, e - 136)), else 8-bit PNG / JPEG
//     through stbi_load with the file's own channel count, mapped as the
//     reference does: rgb = pow(v / 255, 2.2), a = v / 255 when 4 channels, else 1
//     (texture.cpp:107-117; for 1- and 2-channel files that loop reads the next
//     pixels' bytes as G and B, reproduced here, with bytes past the end as 0);
//   * ".pfm" (this repo's own test format; not an stb format).
// Rows come out top first (stb and tinyexr order).  PNG: every colour type and
// bit depth, tRNS, Adam7; 16-bit samples keep their high byte (stbi_load).
// JPEG: baseline / extended sequential Huffman (SOF0/SOF1), 1 or 3 components,
// any sampling factors, restart markers; stb's integer IDCT, its YCbCr
// fixed-point conversion and its "fancy" triangle upsampling.  Progressive JPEG,
// PIZ/PXR24/B44 EXR and tiled / deep / multipart EXR are rejected with an error
// (the caller then renders the texture black, like TextureManager::GetTexture
// on a failed load, resource/texture.cpp:53-60).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include <zlib.h>

#include "../../../include/pupil_pt.h"

namespace Pupil {
void set_last_error(const std::string &m);  // engine.hip
}

namespace Pupil::image {

namespace {

bool read_file(const std::string &path, std::vector<uint8_t> &out) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    f.seekg(0, std::ios::end);
    const std::streamoff n = f.tellg();
    if (n < 0) return false;
    f.seekg(0, std::ios::beg);
    out.resize((size_t)n);
    if (n) f.read(reinterpret_cast<char *>(out.data()), n);
    return (bool)f;
}

bool inflate_all(const uint8_t *src, size_t n, std::vector<uint8_t> &out, size_t expect, bool raw_deflate = false) {
    z_stream z{};
    if (inflateInit2(&z, raw_deflate ? -15 : 15) != Z_OK) return false;
    out.resize(expect ? expect : std::max<size_t>(n * 4, 1024));
    z.next_in = const_cast<Bytef *>(src);
    z.avail_in = (uInt)n;
    size_t have = 0;
    int rc = Z_OK;
    while (rc == Z_OK) {
        if (have == out.size()) {
            if (expect) break;
            out.resize(out.size() * 2);
        }
        z.next_out = out.data() + have;
        z.avail_out = (uInt)(out.size() - have);
        rc = inflate(&z, Z_NO_FLUSH);
        have = out.size() - z.avail_out;
        if (rc == Z_BUF_ERROR && z.avail_in == 0) break;
    }
    inflateEnd(&z);
    out.resize(have);
    return rc == Z_STREAM_END || (expect && have == expect);
}

// ------------------------------------------------------------------ EXR (tinyexr LoadEXR)
float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1Fu, m = h & 0x3FFu;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) {
            bits = s;
        } else {  // subnormal half -> normal float
            int ee = -1;
            uint32_t mm = m;
            do {
                ee++;
                mm <<= 1;
            } while ((mm & 0x400u) == 0);
            bits = s | ((uint32_t)(127 - 15 - ee) << 23) | ((mm & 0x3FFu) << 13);
        }
    } else if (e == 31) {
        bits = s | 0x7F800000u | (m << 13);
    } else {
        bits = s | ((e - 15 + 127) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

struct ExrChannel {
    std::string name;
    int type;  // 0 UINT, 1 HALF, 2 FLOAT
    int xs, ys;
};

// OpenEXR's ZIP / RLE byte layout: predictor over the interleaved halves
void exr_unpredict_deinterleave(std::vector<uint8_t> &buf) {
    for (size_t i = 1; i < buf.size(); i++) buf[i] = (uint8_t)(buf[i - 1] + buf[i] - 128);
    std::vector<uint8_t> out(buf.size());
    const size_t half = (buf.size() + 1) / 2;
    for (size_t i = 0, a = 0, b = half; i < buf.size(); i++) out[i] = (i & 1) ? buf[b++] : buf[a++];
    buf.swap(out);
}

bool exr_rle(const uint8_t *p, size_t n, std::vector<uint8_t> &out, size_t expect) {
    out.clear();
    size_t i = 0;
    while (i < n) {
        const int c = (int8_t)p[i++];
        if (c < 0) {
            const size_t k = (size_t)(-c);
            if (i + k > n) return false;
            out.insert(out.end(), p + i, p + i + k);
            i += k;
        } else {
            if (i >= n) return false;
            out.insert(out.end(), (size_t)c + 1, p[i++]);
        }
        if (out.size() > expect) return false;
    }
    return out.size() == expect;
}

// NUL-terminated string at f[at] that must end before `limit` (untrusted input: no
// read past the buffer when the terminator is missing)
bool read_cstr(const std::vector<uint8_t> &f, size_t at, size_t limit, std::string &out) {
    limit = std::min(limit, f.size());
    if (at >= limit) return false;
    const void *z = std::memchr(f.data() + at, 0, limit - at);
    if (!z) return false;
    out.assign(reinterpret_cast<const char *>(f.data() + at), static_cast<const uint8_t *>(z) - (f.data() + at));
    return true;
}

bool load_exr(const std::vector<uint8_t> &f, std::vector<float> &rgba, int &w, int &h, std::string &err) {
    size_t pos = 0;
    auto need = [&](size_t k) { return pos + k <= f.size(); };
    auto rd32 = [&](size_t at) {
        int32_t v;
        std::memcpy(&v, f.data() + at, 4);
        return v;
    };
    if (!need(8) || !(f[0] == 0x76 && f[1] == 0x2f && f[2] == 0x31 && f[3] == 0x01)) return err = "not an EXR file", false;
    const uint32_t flags = (uint32_t)rd32(4);
    if ((flags & 0xFFu) != 2u) return err = "unsupported EXR version", false;
    if (flags & (0x200u | 0x800u | 0x1000u)) return err = "tiled, deep or multipart EXR not supported", false;
    pos = 8;
    std::vector<ExrChannel> ch;
    int comp = -1, line_order = 0;
    int32_t dw[4] = {0, 0, -1, -1};
    bool have_dw = false;
    for (;;) {
        if (!need(1)) return err = "truncated EXR header", false;
        if (f[pos] == 0) {
            pos++;
            break;
        }
        std::string name, type;
        if (!read_cstr(f, pos, f.size(), name)) return err = "truncated EXR header", false;
        pos += name.size() + 1;
        if (!read_cstr(f, pos, f.size(), type)) return err = "truncated EXR header", false;
        pos += type.size() + 1;
        if (!need(4)) return err = "truncated EXR header", false;
        const int32_t size = rd32(pos);
        pos += 4;
        if (size < 0 || !need((size_t)size)) return err = "truncated EXR attribute", false;
        const size_t end = pos + (size_t)size;
        if (name == "channels" && type == "chlist") {
            size_t q = pos;
            while (q < end && f[q] != 0) {
                ExrChannel c;
                if (!read_cstr(f, q, end, c.name)) return err = "bad EXR channel list", false;
                q += c.name.size() + 1;
                if (q + 16 > end) return err = "bad EXR channel list", false;
                c.type = rd32(q);
                c.xs = rd32(q + 8);
                c.ys = rd32(q + 12);
                q += 16;
                ch.push_back(c);
            }
        } else if (name == "compression" && size >= 1) {
            comp = f[pos];
        } else if (name == "dataWindow" && size >= 16) {
            for (int k = 0; k < 4; k++) dw[k] = rd32(pos + 4 * k);
            have_dw = true;
        } else if (name == "lineOrder" && size >= 1) {
            line_order = f[pos];
        }
        pos = end;
    }
    (void)line_order;  // chunks carry their own first line number
    if (!have_dw || ch.empty() || comp < 0) return err = "EXR header lacks channels / compression / dataWindow", false;
    const int64_t w64 = (int64_t)dw[2] - dw[0] + 1, h64 = (int64_t)dw[3] - dw[1] + 1;
    if (w64 <= 0 || h64 <= 0 || w64 * h64 > (1ll << 28)) return err = "bad EXR data window", false;
    w = (int)w64;
    h = (int)h64;
    for (const auto &c : ch)
        if (c.xs != 1 || c.ys != 1 || c.type < 0 || c.type > 2) return err = "EXR channel sampling / type not supported", false;
    int lines;
    switch (comp) {
    case 0: case 1: case 2: lines = 1; break;  // NONE, RLE, ZIPS
    case 3: lines = 16; break;                 // ZIP
    default: return err = "EXR compression " + std::to_string(comp) + " not supported (NONE, RLE, ZIPS, ZIP)", false;
    }
    size_t bpl = 0;  // bytes per scanline
    for (const auto &c : ch) bpl += (size_t)w * (c.type == 1 ? 2 : 4);
    const int chunks = (h + lines - 1) / lines;
    if (!need((size_t)chunks * 8)) return err = "truncated EXR offset table", false;
    std::vector<std::vector<float>> planes(ch.size(), std::vector<float>((size_t)w * h, 0.f));
    std::vector<uint8_t> buf;
    for (int k = 0; k < chunks; k++) {
        uint64_t off;
        std::memcpy(&off, f.data() + pos + 8 * (size_t)k, 8);
        // offsets come from the file: compare without forming off + k (no wrap-around)
        if (off > f.size() || f.size() - off < 8) return err = "bad EXR chunk offset", false;
        const int32_t y0 = rd32((size_t)off), size = rd32((size_t)off + 4);
        if (size < 0 || (uint64_t)size > f.size() - off - 8) return err = "truncated EXR chunk", false;
        const uint8_t *src = f.data() + off + 8;
        const int64_t first64 = (int64_t)y0 - dw[1];
        if (first64 < 0 || first64 >= h) return err = "EXR chunk outside the data window", false;
        const int first = (int)first64;
        const int nl = std::min(lines, h - first);
        const size_t expect = bpl * (size_t)nl;
        if ((size_t)size == expect || comp == 0) {  // stored uncompressed
            if ((size_t)size < expect) return err = "short EXR chunk", false;
            buf.assign(src, src + expect);
        } else if (comp == 1) {
            if (!exr_rle(src, (size_t)size, buf, expect)) return err = "bad EXR RLE chunk", false;
            exr_unpredict_deinterleave(buf);
        } else {
            if (!inflate_all(src, (size_t)size, buf, expect) || buf.size() != expect) return err = "bad EXR ZIP chunk", false;
            exr_unpredict_deinterleave(buf);
        }
        size_t q = 0;
        for (int l = 0; l < nl; l++)
            for (size_t c = 0; c < ch.size(); c++) {
                float *dst = planes[c].data() + (size_t)(first + l) * w;
                for (int x = 0; x < w; x++) {
                    if (ch[c].type == 1) {
                        uint16_t v;
                        std::memcpy(&v, buf.data() + q, 2);
                        dst[x] = half_to_float(v);
                        q += 2;
                    } else if (ch[c].type == 2) {
                        std::memcpy(&dst[x], buf.data() + q, 4);
                        q += 4;
                    } else {
                        uint32_t v;
                        std::memcpy(&v, buf.data() + q, 4);
                        dst[x] = (float)v;
                        q += 4;
                    }
                }
            }
    }
    rgba.assign((size_t)w * h * 4, 0.f);
    if (ch.size() == 1) {  // tinyexr: a single channel fills R, G, B and A
        for (size_t i = 0; i < (size_t)w * h; i++)
            rgba[4 * i] = rgba[4 * i + 1] = rgba[4 * i + 2] = rgba[4 * i + 3] = planes[0][i];
        return true;
    }
    int ir = -1, ig = -1, ib = -1, ia = -1;
    for (size_t c = 0; c < ch.size(); c++) {
        if (ch[c].name == "R") ir = (int)c;
        if (ch[c].name == "G") ig = (int)c;
        if (ch[c].name == "B") ib = (int)c;
        if (ch[c].name == "A") ia = (int)c;
    }
    if (ir < 0 || ig < 0 || ib < 0) return err = "EXR R, G or B channel not found", false;
    for (size_t i = 0; i < (size_t)w * h; i++) {
        rgba[4 * i + 0] = planes[ir][i];
        rgba[4 * i + 1] = planes[ig][i];
        rgba[4 * i + 2] = planes[ib][i];
        rgba[4 * i + 3] = ia >= 0 ? planes[ia][i] : 1.f;
    }
    return true;
}

// ------------------------------------------------------------------ Radiance HDR (stbi__hdr_load)
bool is_hdr(const std::vector<uint8_t> &f) {
    auto starts = [&](const char *s) {
        const size_t n = std::strlen(s);
        return f.size() >= n && std::memcmp(f.data(), s, n) == 0;
    };
    return starts("#?RADIANCE\n") || starts("#?RGBE\n");
}

bool load_hdr(const std::vector<uint8_t> &f, std::vector<float> &rgb, int &w, int &h, std::string &err) {
    size_t pos = 0;
    auto line = [&]() {
        std::string s;
        while (pos < f.size() && f[pos] != '\n') s += (char)f[pos++];
        if (pos < f.size()) pos++;
        return s;
    };
    line();  // signature
    bool valid = false;
    for (;;) {
        if (pos >= f.size()) return err = "truncated HDR header", false;
        const std::string s = line();
        if (s.empty()) break;
        if (s == "FORMAT=32-bit_rle_rgbe") valid = true;
    }
    if (!valid) return err = "unsupported HDR format", false;
    const std::string res = line();
    if (res.compare(0, 3, "-Y ") != 0) return err = "unsupported HDR data layout", false;
    const char *c = res.c_str() + 3;
    char *e = nullptr;
    h = (int)std::strtol(c, &e, 10);
    while (*e == ' ') e++;
    if (std::strncmp(e, "+X ", 3) != 0) return err = "unsupported HDR data layout", false;
    w = (int)std::strtol(e + 3, nullptr, 10);
    if (w <= 0 || h <= 0 || (int64_t)w * h > (1ll << 28)) return err = "bad HDR size", false;
    std::vector<uint8_t> rgbe((size_t)w * h * 4);
    auto flat = [&](size_t from) {  // remaining pixels as plain RGBE quadruples
        const size_t n = rgbe.size() - from;
        if (pos + n > f.size()) return false;
        std::memcpy(rgbe.data() + from, f.data() + pos, n);
        pos += n;
        return true;
    };
    bool ok = true;
    if (w < 8 || w >= 32768) {
        ok = flat(0);
    } else {
        std::vector<uint8_t> sl((size_t)w * 4);
        for (int y = 0; y < h && ok; y++) {
            if (pos + 4 > f.size()) return err = "truncated HDR data", false;
            const uint8_t c1 = f[pos], c2 = f[pos + 1], len = f[pos + 2];
            if (c1 != 2 || c2 != 2 || (len & 0x80)) {  // not run-length encoded: the rest is flat
                ok = flat((size_t)y * w * 4);
                break;
            }
            const int n = (f[pos + 2] << 8) | f[pos + 3];
            pos += 4;
            if (n != w) return err = "invalid HDR scanline", false;
            for (int k = 0; k < 4 && ok; k++) {
                int i = 0;
                while (i < w) {
                    if (pos >= f.size()) return err = "truncated HDR data", false;
                    int count = f[pos++];
                    if (count > 128) {
                        count -= 128;
                        if (count > w - i || pos >= f.size()) return err = "bad HDR run", false;
                        const uint8_t v = f[pos++];
                        for (int z = 0; z < count; z++) sl[(size_t)(i++) * 4 + k] = v;
                    } else {
                        if (count == 0 || count > w - i || pos + count > f.size()) return err = "bad HDR dump", false;
                        for (int z = 0; z < count; z++) sl[(size_t)(i++) * 4 + k] = f[pos++];
                    }
                }
            }
            std::memcpy(rgbe.data() + (size_t)y * w * 4, sl.data(), sl.size());
        }
    }
    if (!ok) return err = "truncated HDR data", false;
    rgb.assign((size_t)w * h * 3, 0.f);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        const uint8_t *q = rgbe.data() + 4 * i;
        if (q[3] != 0) {  // stbi__hdr_convert
            const float f1 = (float)std::ldexp(1.0f, q[3] - (int)(128 + 8));
            rgb[3 * i + 0] = q[0] * f1;
            rgb[3 * i + 1] = q[1] * f1;
            rgb[3 * i + 2] = q[2] * f1;
        }
    }
    return true;
}

// ------------------------------------------------------------------ PNG (stbi__png_load, req_comp 0)
uint32_t be32(const uint8_t *p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }

int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    if (pb <= pc) return b;
    return c;
}

bool load_png(const std::vector<uint8_t> &f, std::vector<uint8_t> &out, int &w, int &h, int &comp, std::string &err) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) return err = "not a PNG file", false;
    size_t pos = 8;
    int depth = 0, color = -1, interlace = 0;
    std::vector<uint8_t> idat, pal;
    std::vector<uint8_t> trns;
    bool have_trns = false;
    while (pos + 8 <= f.size()) {
        const uint32_t len = be32(f.data() + pos);
        const uint32_t type = be32(f.data() + pos + 4);
        const uint8_t *d = f.data() + pos + 8;
        if (pos + 12 + (size_t)len > f.size()) return err = "truncated PNG chunk", false;
        if (type == 0x49484452u) {  // IHDR
            if (len < 13) return err = "bad IHDR", false;
            w = (int)be32(d);
            h = (int)be32(d + 4);
            depth = d[8];
            color = d[9];
            interlace = d[12];
            if (d[10] != 0 || d[11] != 0) return err = "bad PNG compression / filter method", false;
        } else if (type == 0x504C5445u) {  // PLTE
            pal.assign(d, d + len);
        } else if (type == 0x74524E53u) {  // tRNS
            trns.assign(d, d + len);
            have_trns = true;
        } else if (type == 0x49444154u) {  // IDAT
            idat.insert(idat.end(), d, d + len);
        } else if (type == 0x49454E44u) {  // IEND
            break;
        }
        pos += 12 + (size_t)len;
    }
    if (w <= 0 || h <= 0 || (int64_t)w * h > (1ll << 28)) return err = "bad PNG size", false;
    int img_n;
    switch (color) {
    case 0: img_n = 1; break;
    case 2: img_n = 3; break;
    case 3: img_n = 1; break;
    case 4: img_n = 2; break;
    case 6: img_n = 4; break;
    default: return err = "bad PNG color type", false;
    }
    if (!(depth == 1 || depth == 2 || depth == 4 || depth == 8 || depth == 16) || (color == 3 && depth == 16) ||
        ((color == 2 || color == 4 || color == 6) && depth < 8))
        return err = "bad PNG bit depth", false;
    if (color == 3 && (pal.empty() || pal.size() % 3)) return err = "PNG palette missing", false;
    std::vector<uint8_t> raw;
    if (!inflate_all(idat.data(), idat.size(), raw, 0)) return err = "corrupt PNG data", false;
    // stb output channels: palette -> 3 (4 with tRNS); grey / rgb with tRNS gain an alpha channel
    const int out_n = color == 3 ? (have_trns ? 4 : 3) : img_n + ((have_trns && (color == 0 || color == 2)) ? 1 : 0);
    const int bytes = depth == 16 ? 2 : 1;
    std::vector<uint16_t> samples((size_t)w * h * img_n);  // unfiltered samples at full precision
    size_t rp = 0;
    auto decode_pass = [&](int pw, int ph, auto &&place) -> bool {
        if (pw == 0 || ph == 0) return true;
        const size_t stride = ((size_t)pw * img_n * depth + 7) / 8;
        const int filt_bpp = std::max(1, img_n * depth / 8);
        std::vector<uint8_t> prev(stride, 0), cur(stride);
        for (int y = 0; y < ph; y++) {
            if (rp + 1 + stride > raw.size()) return false;
            const int ft = raw[rp++];
            for (size_t i = 0; i < stride; i++) {
                const int x = raw[rp + i];
                const int a = i >= (size_t)filt_bpp ? cur[i - filt_bpp] : 0;
                const int b = prev[i];
                const int c = i >= (size_t)filt_bpp ? prev[i - filt_bpp] : 0;
                int v;
                switch (ft) {
                case 0: v = x; break;
                case 1: v = x + a; break;
                case 2: v = x + b; break;
                case 3: v = x + ((a + b) >> 1); break;
                case 4: v = x + paeth(a, b, c); break;
                default: return false;
                }
                cur[i] = (uint8_t)v;
            }
            rp += stride;
            for (int x = 0; x < pw; x++)
                for (int k = 0; k < img_n; k++) {
                    const size_t s = (size_t)x * img_n + k;
                    uint16_t v;
                    if (depth == 16) v = (uint16_t)((cur[2 * s] << 8) | cur[2 * s + 1]);
                    else if (depth == 8) v = cur[s];
                    else v = (uint16_t)((cur[(s * depth) >> 3] >> (8 - depth - (int)((s * depth) & 7))) & ((1 << depth) - 1));
                    place(x, y, k, v);
                }
            prev.swap(cur);
        }
        return true;
    };
    bool ok = true;
    if (interlace == 0) {
        ok = decode_pass(w, h, [&](int x, int y, int k, uint16_t v) { samples[((size_t)y * w + x) * img_n + k] = v; });
    } else {  // Adam7
        static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
        static const int xs[7] = {8, 8, 4, 4, 2, 2, 1}, ys[7] = {8, 8, 8, 4, 4, 2, 2};
        for (int p = 0; p < 7 && ok; p++) {
            const int pw = (w - xo[p] + xs[p] - 1) / xs[p], ph = (h - yo[p] + ys[p] - 1) / ys[p];
            if (w <= xo[p] || h <= yo[p]) continue;
            ok = decode_pass(pw, ph, [&](int x, int y, int k, uint16_t v) {
                samples[((size_t)(yo[p] + y * ys[p]) * w + xo[p] + x * xs[p]) * img_n + k] = v;
            });
        }
    }
    if (!ok) return err = "corrupt PNG scanlines", false;
    (void)bytes;
    static const int scale[9] = {0, 0xff, 0x55, 0, 0x11, 0, 0, 0, 0x01};  // stbi__depth_scale_table
    comp = out_n;
    out.assign((size_t)w * h * out_n, 0);
    for (size_t i = 0; i < (size_t)w * h; i++) {
        const uint16_t *s = samples.data() + i * img_n;
        uint8_t *o = out.data() + i * out_n;
        if (color == 3) {
            const size_t ix = s[0];
            for (int k = 0; k < 3; k++) o[k] = 3 * ix + k < pal.size() ? pal[3 * ix + k] : 0;
            if (out_n == 4) o[3] = ix < trns.size() ? trns[ix] : 255;
            continue;
        }
        for (int k = 0; k < img_n; k++) {
            const uint16_t v = s[k];
            o[k] = depth == 16 ? (uint8_t)(v >> 8) : (uint8_t)(depth < 8 ? v * scale[depth] : v);
        }
        if (out_n == img_n + 1) {  // tRNS key colour of a grey / rgb image
            bool match = true;
            for (int k = 0; k < img_n; k++) {
                const size_t at = 2 * (size_t)k;
                const uint16_t key = at + 1 < trns.size() ? (uint16_t)((trns[at] << 8) | trns[at + 1]) : 0;
                const uint16_t kv = depth == 16 ? key : (uint16_t)(depth < 8 ? (key & ((1 << depth) - 1)) : (key & 0xFF));
                if (s[k] != kv) match = false;
            }
            o[img_n] = match ? 0 : 255;
        }
    }
    return true;
}

// ------------------------------------------------------------------ JPEG (stb_image baseline path)
constexpr uint8_t kZigzag[64 + 15] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                      12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                      35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                      58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
                                      63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

uint8_t clamp8(int x) { return (unsigned)x > 255 ? (x < 0 ? 0 : 255) : (uint8_t)x; }
constexpr int f2f(float x) { return (int)((x)*4096 + 0.5); }
constexpr int fsh(int x) { return x * 4096; }

// stbi__idct_block: integer IDCT (jidctint-style constants scaled by 4096), with
// the same all-zero column shortcut and rounding; stb's SSE2 / NEON versions are
// documented as bit-identical to it.
void idct_block(uint8_t *out, int stride, const short *data) {
    int val[64];
    int *v = val;
    const short *d = data;
#define IDCT_1D(s0, s1, s2, s3, s4, s5, s6, s7)                                                                       \
    int t0, t1, t2, t3, p1, p2, p3, p4, p5, x0, x1, x2, x3;                                                          \
    p2 = s2;                                                                                                          \
    p3 = s6;                                                                                                          \
    p1 = (p2 + p3) * f2f(0.5411961f);                                                                                 \
    t2 = p1 + p3 * f2f(-1.847759065f);                                                                                \
    t3 = p1 + p2 * f2f(0.765366865f);                                                                                 \
    p2 = s0;                                                                                                          \
    p3 = s4;                                                                                                          \
    t0 = fsh(p2 + p3);                                                                                                \
    t1 = fsh(p2 - p3);                                                                                                \
    x0 = t0 + t3;                                                                                                     \
    x3 = t0 - t3;                                                                                                     \
    x1 = t1 + t2;                                                                                                     \
    x2 = t1 - t2;                                                                                                     \
    t0 = s7;                                                                                                          \
    t1 = s5;                                                                                                          \
    t2 = s3;                                                                                                          \
    t3 = s1;                                                                                                          \
    p3 = t0 + t2;                                                                                                     \
    p4 = t1 + t3;                                                                                                     \
    p1 = t0 + t3;                                                                                                     \
    p2 = t1 + t2;                                                                                                     \
    p5 = (p3 + p4) * f2f(1.175875602f);                                                                               \
    t0 = t0 * f2f(0.298631336f);                                                                                      \
    t1 = t1 * f2f(2.053119869f);                                                                                      \
    t2 = t2 * f2f(3.072711026f);                                                                                      \
    t3 = t3 * f2f(1.501321110f);                                                                                      \
    p1 = p5 + p1 * f2f(-0.899976223f);                                                                                \
    p2 = p5 + p2 * f2f(-2.562915447f);                                                                                \
    p3 = p3 * f2f(-1.961570560f);                                                                                     \
    p4 = p4 * f2f(-0.390180644f);                                                                                     \
    t3 += p1 + p4;                                                                                                    \
    t2 += p2 + p3;                                                                                                    \
    t1 += p2 + p4;                                                                                                    \
    t0 += p1 + p3;
    for (int i = 0; i < 8; ++i, ++d, ++v) {
        if (d[8] == 0 && d[16] == 0 && d[24] == 0 && d[32] == 0 && d[40] == 0 && d[48] == 0 && d[56] == 0) {
            const int dc = d[0] * 4;
            v[0] = v[8] = v[16] = v[24] = v[32] = v[40] = v[48] = v[56] = dc;
        } else {
            IDCT_1D(d[0], d[8], d[16], d[24], d[32], d[40], d[48], d[56])
            x0 += 512;
            x1 += 512;
            x2 += 512;
            x3 += 512;
            v[0] = (x0 + t3) >> 10;
            v[56] = (x0 - t3) >> 10;
            v[8] = (x1 + t2) >> 10;
            v[48] = (x1 - t2) >> 10;
            v[16] = (x2 + t1) >> 10;
            v[40] = (x2 - t1) >> 10;
            v[24] = (x3 + t0) >> 10;
            v[32] = (x3 - t0) >> 10;
        }
    }
    v = val;
    uint8_t *o = out;
    for (int i = 0; i < 8; ++i, v += 8, o += stride) {
        IDCT_1D(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7])
        x0 += 65536 + (128 << 17);
        x1 += 65536 + (128 << 17);
        x2 += 65536 + (128 << 17);
        x3 += 65536 + (128 << 17);
        o[0] = clamp8((x0 + t3) >> 17);
        o[7] = clamp8((x0 - t3) >> 17);
        o[1] = clamp8((x1 + t2) >> 17);
        o[6] = clamp8((x1 - t2) >> 17);
        o[2] = clamp8((x2 + t1) >> 17);
        o[5] = clamp8((x2 - t1) >> 17);
        o[3] = clamp8((x3 + t0) >> 17);
        o[4] = clamp8((x3 - t0) >> 17);
    }
#undef IDCT_1D
}

struct Huffman {
    // canonical decode tables: code lengths 1..16
    uint16_t code[256];
    uint8_t size[256], values[256];
    int maxcode[18], delta[17];
    int count = 0;
    bool build(const uint8_t *counts, const uint8_t *vals) {
        int k = 0;
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < counts[i]; j++) {
                if (k >= 256) return false;
                size[k++] = (uint8_t)(i + 1);
            }
        count = k;
        std::memcpy(values, vals, (size_t)k);
        int c = 0;
        k = 0;
        for (int j = 1; j <= 16; j++) {
            delta[j] = k - c;
            if (k < count && size[k] == j) {
                while (k < count && size[k] == j) code[k++] = (uint16_t)(c++);
                if (c - 1 >= (1 << j)) return false;
            }
            maxcode[j] = c << (16 - j);
            c <<= 1;
        }
        maxcode[17] = 0x7fffffff;
        return true;
    }
};

struct JpegComponent {
    int id, h, v, tq, hd, ha, dc_pred;
    int x, y, w2, h2;
    std::vector<uint8_t> data;
};

struct Jpeg {
    const std::vector<uint8_t> &f;
    size_t pos = 0;
    uint32_t bits = 0;
    int nbits = 0;
    bool marker_hit = false;
    uint16_t dq[4][64];
    Huffman hdc[4], hac[4];
    std::vector<JpegComponent> comp;
    int w = 0, h = 0, hmax = 1, vmax = 1, restart = 0, app14_transform = -1;
    bool jfif = false;
    std::string err;
    explicit Jpeg(const std::vector<uint8_t> &file) : f(file) {}

    int byte() { return pos < f.size() ? f[pos++] : 0; }
    int u16() {
        const int a = byte();
        return (a << 8) | byte();
    }
    void fill() {  // stbi__grow_buffer_unsafe: 0xFF00 stuffing, stop at a marker
        while (nbits <= 24) {
            int c = marker_hit ? 0 : byte();
            if (c == 0xFF && !marker_hit) {
                int c2 = pos < f.size() ? f[pos] : 0;
                while (c2 == 0xFF) {
                    pos++;
                    c2 = pos < f.size() ? f[pos] : 0;
                }
                if (c2 != 0) {  // a marker: leave pos on its 0xFF for the marker scan
                    marker_hit = true;
                    c = 0;
                    pos--;
                } else {
                    pos++;
                }
            }
            bits |= (uint32_t)c << (24 - nbits);
            nbits += 8;
        }
    }
    int decode(const Huffman &hf) {
        if (nbits < 16) fill();
        const uint32_t t = bits >> 16;
        int k = 1;
        while (k <= 16 && (int)t >= hf.maxcode[k]) k++;
        if (k > 16) {
            nbits = 0;
            return -1;
        }
        if (k > nbits) return -1;
        const int c = (int)(((bits >> (32 - k)) & ((1u << k) - 1)) + hf.delta[k]);
        bits <<= k;
        nbits -= k;
        return c >= 0 && c < hf.count ? hf.values[c] : -1;
    }
    int extend_receive(int n) {  // stbi__extend_receive
        if (n == 0) return 0;
        if (nbits < n) fill();
        const int sgn = (int32_t)bits >> 31;
        uint32_t k = (bits << n) | (bits >> (32 - n));
        const uint32_t mask = (1u << n) - 1;
        bits = k & ~mask;
        k &= mask;
        nbits -= n;
        static const int bias[17] = {0, -1, -3, -7, -15, -31, -63, -127, -255, -511, -1023, -2047, -4095, -8191, -16383, -32767, -65535};
        return (int)k + (bias[n] & ~sgn);
    }
    bool decode_block(short data[64], JpegComponent &c) {
        std::memset(data, 0, 64 * sizeof(short));
        const int t = decode(hdc[c.hd]);
        if (t < 0 || t > 15) return err = "bad JPEG huffman code", false;
        const int diff = t ? extend_receive(t) : 0;
        c.dc_pred += diff;
        data[0] = (short)(c.dc_pred * dq[c.tq][0]);
        int k = 1;
        do {
            const int rs = decode(hac[c.ha]);
            if (rs < 0) return err = "bad JPEG huffman code", false;
            const int s = rs & 15, r = rs >> 4;
            if (s == 0) {
                if (rs != 0xf0) break;  // end of block
                k += 16;
            } else {
                k += r;
                if (k > 63) return err = "bad JPEG run length", false;
                const int zig = kZigzag[k++];
                data[zig] = (short)(extend_receive(s) * dq[c.tq][zig]);
            }
        } while (k < 64);
        return true;
    }
    void reset_bits() {
        bits = 0;
        nbits = 0;
        marker_hit = false;
        for (auto &c : comp) c.dc_pred = 0;
    }
    bool skip_restart() {  // RSTn after every `restart` MCUs
        // the bit reader stopped at the marker; find and consume it
        while (pos + 1 < f.size() && !(f[pos] == 0xFF && f[pos + 1] >= 0xD0 && f[pos + 1] <= 0xD7)) pos++;
        if (pos + 1 >= f.size()) return err = "missing JPEG restart marker", false;
        pos += 2;
        reset_bits();
        return true;
    }
    bool scan(const std::vector<int> &order) {
        reset_bits();
        short data[64];
        int todo = restart ? restart : 0x7fffffff;
        if (order.size() == 1) {  // non-interleaved: the component's own block raster
            JpegComponent &c = comp[order[0]];
            const int bw = (c.x + 7) >> 3, bh = (c.y + 7) >> 3;
            for (int j = 0; j < bh; j++)
                for (int i = 0; i < bw; i++) {
                    if (!decode_block(data, c)) return false;
                    idct_block(c.data.data() + (size_t)c.w2 * j * 8 + i * 8, c.w2, data);
                    if (--todo <= 0 && !(j == bh - 1 && i == bw - 1)) {
                        if (!skip_restart()) return false;
                        todo = restart;
                    }
                }
            return true;
        }
        const int mx = (w + 8 * hmax - 1) / (8 * hmax), my = (h + 8 * vmax - 1) / (8 * vmax);
        for (int j = 0; j < my; j++)
            for (int i = 0; i < mx; i++) {
                for (int k : order) {
                    JpegComponent &c = comp[k];
                    for (int y = 0; y < c.v; y++)
                        for (int x = 0; x < c.h; x++) {
                            const int x2 = (i * c.h + x) * 8, y2 = (j * c.v + y) * 8;
                            if (!decode_block(data, c)) return false;
                            idct_block(c.data.data() + (size_t)c.w2 * y2 + x2, c.w2, data);
                        }
                }
                if (--todo <= 0 && !(j == my - 1 && i == mx - 1)) {
                    if (!skip_restart()) return false;
                    todo = restart;
                }
            }
        return true;
    }
    bool run() {
        if (f.size() < 4 || f[0] != 0xFF || f[1] != 0xD8) return err = "not a JPEG file", false;
        pos = 2;
        bool frame = false, scanned = false;
        for (;;) {
            while (pos < f.size() && f[pos] != 0xFF) pos++;  // stray bytes after entropy data
            while (pos < f.size() && f[pos] == 0xFF) pos++;
            if (pos >= f.size()) break;
            const int m = f[pos++];
            if (m == 0xD9) break;  // EOI
            if (m >= 0xD0 && m <= 0xD7) continue;
            const size_t seg = pos;
            const int len = u16();
            if (len < 2 || seg + (size_t)len > f.size()) return err = "truncated JPEG segment", false;
            const size_t end = seg + (size_t)len;
            if (m == 0xDB) {  // DQT
                while (pos < end) {
                    const int pq = byte(), t = pq & 15, p = pq >> 4;
                    if (t > 3 || p > 1) return err = "bad JPEG DQT", false;
                    for (int i = 0; i < 64; i++) dq[t][kZigzag[i]] = (uint16_t)(p ? u16() : byte());
                }
            } else if (m == 0xC4) {  // DHT
                while (pos < end) {
                    const int q = byte(), tc = q >> 4, th = q & 15;
                    uint8_t counts[16], vals[256];
                    int n = 0;
                    for (int i = 0; i < 16; i++) n += counts[i] = (uint8_t)byte();
                    if (tc > 1 || th > 3 || n > 256) return err = "bad JPEG DHT", false;
                    for (int i = 0; i < n; i++) vals[i] = (uint8_t)byte();
                    if (!(tc ? hac[th] : hdc[th]).build(counts, vals)) return err = "bad JPEG huffman table", false;
                }
            } else if (m == 0xC0 || m == 0xC1) {  // baseline / extended sequential Huffman
                if (byte() != 8) return err = "only 8-bit JPEG supported", false;
                h = u16();
                w = u16();
                const int n = byte();
                if (w <= 0 || h <= 0 || (n != 1 && n != 3)) return err = "unsupported JPEG frame", false;
                comp.resize((size_t)n);
                for (auto &c : comp) {
                    c.id = byte();
                    const int hv = byte();
                    c.h = hv >> 4;
                    c.v = hv & 15;
                    c.tq = byte();
                    if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) return err = "bad JPEG component", false;
                    hmax = std::max(hmax, c.h);
                    vmax = std::max(vmax, c.v);
                }
                // stb_image rejects sampling factors that do not divide the maxima ("bad H" /
                // "bad V"): the resampler reads hmax / h samples per component sample, so a
                // non-divisor would read past the end of the component's rows
                for (const auto &c : comp)
                    if (hmax % c.h != 0 || vmax % c.v != 0) return err = "bad JPEG sampling factors", false;
                const int mx = (w + 8 * hmax - 1) / (8 * hmax), my = (h + 8 * vmax - 1) / (8 * vmax);
                for (auto &c : comp) {
                    c.x = (w * c.h + hmax - 1) / hmax;
                    c.y = (h * c.v + vmax - 1) / vmax;
                    c.w2 = mx * c.h * 8;
                    c.h2 = my * c.v * 8;
                    c.data.assign((size_t)c.w2 * c.h2, 0);
                }
                frame = true;
            } else if (m >= 0xC2 && m <= 0xCF && m != 0xC4 && m != 0xC8 && m != 0xCC) {
                return err = "progressive / lossless / arithmetic JPEG not supported", false;
            } else if (m == 0xDD) {  // DRI
                restart = u16();
            } else if (m == 0xDA) {  // SOS
                if (!frame) return err = "JPEG scan before frame", false;
                const int ns = byte();
                std::vector<int> order;
                for (int i = 0; i < ns; i++) {
                    const int id = byte(), t = byte();
                    int k = -1;
                    for (size_t c = 0; c < comp.size(); c++)
                        if (comp[c].id == id) k = (int)c;
                    if (k < 0) return err = "bad JPEG scan component", false;
                    comp[k].hd = t >> 4;
                    comp[k].ha = t & 15;
                    if (comp[k].hd > 3 || comp[k].ha > 3) return err = "bad JPEG scan tables", false;
                    order.push_back(k);
                }
                pos = end;
                if (!scan(order)) return false;
                scanned = true;
                continue;  // the marker search resumes after the entropy-coded data
            } else if (m == 0xE0) {
                if (len >= 7 && std::memcmp(f.data() + seg + 2, "JFIF\0", 5) == 0) jfif = true;
            } else if (m == 0xEE) {  // Adobe APP14: transform flag
                if (len >= 14 && std::memcmp(f.data() + seg + 2, "Adobe", 5) == 0) app14_transform = f[seg + 13];
            }
            pos = end;
        }
        if (!scanned) return err = "JPEG has no scan", false;
        return true;
    }
};

uint8_t div4(int x) { return (uint8_t)(x >> 2); }
uint8_t div16(int x) { return (uint8_t)(x >> 4); }

// stbi__resample_row_*: output row of one component at full horizontal resolution
const uint8_t *resample(uint8_t *out, const uint8_t *in_near, const uint8_t *in_far, int w, int hs, int vs) {
    if (hs == 1 && vs == 1) return in_near;
    if (hs == 1 && vs == 2) {
        for (int i = 0; i < w; i++) out[i] = div4(3 * in_near[i] + in_far[i] + 2);
        return out;
    }
    if (hs == 2 && vs == 1) {
        const uint8_t *in = in_near;
        if (w == 1) {
            out[0] = out[1] = in[0];
            return out;
        }
        out[0] = in[0];
        out[1] = div4(in[0] * 3 + in[1] + 2);
        int i;
        for (i = 1; i < w - 1; ++i) {
            const int n = 3 * in[i] + 2;
            out[i * 2 + 0] = div4(n + in[i - 1]);
            out[i * 2 + 1] = div4(n + in[i + 1]);
        }
        out[i * 2 + 0] = div4(in[w - 2] * 3 + in[w - 1] + 2);
        out[i * 2 + 1] = in[w - 1];
        return out;
    }
    if (hs == 2 && vs == 2) {
        if (w == 1) {
            out[0] = out[1] = div4(3 * in_near[0] + in_far[0] + 2);
            return out;
        }
        int t1 = 3 * in_near[0] + in_far[0], t0;
        out[0] = div4(t1 + 2);
        for (int i = 1; i < w; ++i) {
            t0 = t1;
            t1 = 3 * in_near[i] + in_far[i];
            out[i * 2 - 1] = div16(3 * t0 + t1 + 8);
            out[i * 2] = div16(3 * t1 + t0 + 8);
        }
        out[w * 2 - 1] = div4(t1 + 2);
        return out;
    }
    for (int i = 0; i < w; ++i)  // stbi__resample_row_generic
        for (int j = 0; j < hs; ++j) out[i * hs + j] = in_near[i];
    return out;
}

constexpr int float2fixed(float x) { return ((int)((x)*4096.0f + 0.5f)) << 8; }

bool load_jpeg(const std::vector<uint8_t> &file, std::vector<uint8_t> &out, int &w, int &h, int &comp,
               std::string &err) {
    Jpeg j(file);
    if (!j.run()) return err = j.err, false;
    w = j.w;
    h = j.h;
    const int n = (int)j.comp.size();
    comp = n;
    out.assign((size_t)w * h * n, 0);
    struct Res {
        int hs, vs, ystep, ypos, wl;
        const uint8_t *line0, *line1;
        std::vector<uint8_t> buf;
    };
    std::vector<Res> rs((size_t)n);
    for (int k = 0; k < n; k++) {
        auto &c = j.comp[k];
        Res &r = rs[k];
        r.hs = j.hmax / c.h;
        r.vs = j.vmax / c.v;
        r.ystep = r.vs >> 1;
        r.wl = (w + r.hs - 1) / r.hs;
        r.ypos = 0;
        r.line0 = r.line1 = c.data.data();
        r.buf.assign((size_t)w + 3, 0);
    }
    // 3 components: YCbCr unless the Adobe marker says RGB or the ids spell R, G, B (stb's rgb detection)
    const bool rgb_ids = n == 3 && j.comp[0].id == 'R' && j.comp[1].id == 'G' && j.comp[2].id == 'B';
    const bool ycc = n == 3 && !rgb_ids && !(j.app14_transform == 0 && !j.jfif);
    std::vector<const uint8_t *> row((size_t)n);
    for (int y = 0; y < h; y++) {
        for (int k = 0; k < n; k++) {
            Res &r = rs[k];
            const bool bot = r.ystep >= (r.vs >> 1);
            row[k] = resample(r.buf.data(), bot ? r.line1 : r.line0, bot ? r.line0 : r.line1, r.wl, r.hs, r.vs);
            if (++r.ystep >= r.vs) {
                r.ystep = 0;
                r.line0 = r.line1;
                if (++r.ypos < j.comp[k].y) r.line1 += j.comp[k].w2;
            }
        }
        uint8_t *o = out.data() + (size_t)y * w * n;
        if (n == 1) {
            std::memcpy(o, row[0], (size_t)w);
        } else if (!ycc) {
            for (int x = 0; x < w; x++)
                for (int k = 0; k < 3; k++) o[3 * x + k] = row[k][x];
        } else {  // stbi__YCbCr_to_RGB_row
            for (int x = 0; x < w; x++) {
                const int yf = (row[0][x] << 20) + (1 << 19);
                const int cr = row[2][x] - 128, cb = row[1][x] - 128;
                int r = yf + cr * float2fixed(1.40200f);
                int g = yf + (cr * -float2fixed(0.71414f)) + ((cb * -float2fixed(0.34414f)) & (int)0xffff0000);
                int b = yf + cb * float2fixed(1.77200f);
                o[3 * x + 0] = clamp8(r >> 20);
                o[3 * x + 1] = clamp8(g >> 20);
                o[3 * x + 2] = clamp8(b >> 20);
            }
        }
    }
    return true;
}

bool load_pfm(const std::vector<uint8_t> &f, std::vector<float> &rgba, int &w, int &h, std::string &err) {
    std::string head;
    size_t pos = 0;
    int fields = 0;
    std::string tok[4];
    while (pos < f.size() && fields < 4) {  // "PF"/"Pf", width, height, scale, then one whitespace byte
        while (pos < f.size() && std::isspace(f[pos])) pos++;
        while (pos < f.size() && !std::isspace(f[pos])) tok[fields] += (char)f[pos++];
        fields++;
    }
    pos++;
    if (fields < 4 || (tok[0] != "PF" && tok[0] != "Pf")) return err = "not a PFM file", false;
    w = std::atoi(tok[1].c_str());
    h = std::atoi(tok[2].c_str());
    const int ch = tok[0] == "PF" ? 3 : 1;
    if (w <= 0 || h <= 0 || pos + (size_t)w * h * ch * 4 > f.size()) return err = "truncated PFM file", false;
    rgba.assign((size_t)w * h * 4, 1.f);
    for (int y = 0; y < h; y++)  // PFM rows are stored bottom-to-top; row 0 = top like stb/tinyexr
        for (int x = 0; x < w; x++) {
            const size_t src = pos + (((size_t)(h - 1 - y) * w + x) * ch) * 4;
            for (int k = 0; k < 3; k++) std::memcpy(&rgba[((size_t)y * w + x) * 4 + k], f.data() + src + 4 * (ch == 3 ? k : 0), 4);
        }
    return true;
}

}  // namespace

// BitmapTexture::Load (texture.cpp:162-174): RGBA float, w * h * 4, row 0 = top.
bool LoadBitmap(const std::string &path, std::vector<float> &rgba, int &w, int &h, std::string &err) {
    std::vector<uint8_t> f;
    if (!read_file(path, f)) return err = "cannot open " + path, false;
    const size_t dot = path.find_last_of('.');
    const std::string ext = dot == std::string::npos ? "" : path.substr(dot);
    if (ext == ".exr") return load_exr(f, rgba, w, h, err);
    if (ext == ".pfm") return load_pfm(f, rgba, w, h, err);
    if (is_hdr(f)) {  // StbImageLoad, is_hdr branch (texture.cpp:93-104): stbi_loadf, 3 channels
        std::vector<float> rgb;
        if (!load_hdr(f, rgb, w, h, err)) return false;
        rgba.assign((size_t)w * h * 4, 1.f);
        for (size_t i = 0; i < (size_t)w * h; i++)
            for (int k = 0; k < 3; k++) rgba[4 * i + k] = rgb[3 * i + k];
        return true;
    }
    std::vector<uint8_t> px;
    int c = 0;
    bool ok;
    if (f.size() >= 8 && f[0] == 137 && f[1] == 'P' && f[2] == 'N' && f[3] == 'G') ok = load_png(f, px, w, h, c, err);
    else if (f.size() >= 2 && f[0] == 0xFF && f[1] == 0xD8) ok = load_jpeg(f, px, w, h, c, err);
    else return err = "unsupported image format (EXR, HDR, PNG, JPEG, PFM)", false;
    if (!ok) return false;
    // texture.cpp:107-117, including its reads of the following pixels' bytes as G / B
    // when the file has fewer than 3 channels (bytes past the end read as 0 here)
    const size_t n = px.size();
    auto at = [&](size_t i) -> float { return i < n ? (float)px[i] : 0.f; };
    rgba.assign((size_t)w * h * 4, 0.f);
    for (size_t i = 0, j = 0; i < n; i += (size_t)c) {
        rgba[j++] = std::pow(at(i + 0) * 1.f / 255.f, 2.2f);
        rgba[j++] = std::pow(at(i + 1) * 1.f / 255.f, 2.2f);
        rgba[j++] = std::pow(at(i + 2) * 1.f / 255.f, 2.2f);
        rgba[j++] = c == 4 ? at(i + 3) * 1.f / 255.f : 1.f;
    }
    return true;
}

}  // namespace Pupil::image

extern "C" int pupil_image_load(const char *path, uint32_t *width, uint32_t *height, float *rgba) {
    if (!path || !width || !height) {
        Pupil::set_last_error("null argument");
        return PUPIL_ERR_INVALID;
    }
    std::vector<float> px;
    int w = 0, h = 0;
    std::string err;
    if (!Pupil::image::LoadBitmap(path, px, w, h, err)) {
        Pupil::set_last_error(err);
        return PUPIL_ERR_IO;
    }
    *width = (uint32_t)w;
    *height = (uint32_t)h;
    if (rgba) std::memcpy(rgba, px.data(), px.size() * sizeof(float));
    return PUPIL_OK;
}
