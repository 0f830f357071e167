// tiff.cpp -- baseline TIFF reader/writer for the measurement frames.
//
// The reference loads frames with cv::imread(path, -1*CV_LOAD_IMAGE_ANYDEPTH)
// (fpmMain.cpp:118-119), i.e. unchanged depth, and then reads them as uint16
// (fpmMain.cpp:380).  This reader accepts what that path can use:
// uncompressed, single-sample, 8- or 16-bit unsigned grayscale, strip or
// single-strip layout, either byte order.  8-bit frames are widened to uint16.
#include "tiff.hpp"

#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>

namespace fpmhost {

namespace {

struct Rd {
    const std::vector<uint8_t> &b;
    bool be;
    bool ok = true;
    uint16_t u16(size_t o) {
        if (o + 2 > b.size()) { ok = false; return 0; }
        return be ? (uint16_t)(b[o] << 8 | b[o + 1]) : (uint16_t)(b[o] | b[o + 1] << 8);
    }
    uint32_t u32(size_t o) {
        if (o + 4 > b.size()) { ok = false; return 0; }
        return be ? ((uint32_t)b[o] << 24 | (uint32_t)b[o + 1] << 16 | (uint32_t)b[o + 2] << 8 | b[o + 3])
                  : ((uint32_t)b[o] | (uint32_t)b[o + 1] << 8 | (uint32_t)b[o + 2] << 16 | (uint32_t)b[o + 3] << 24);
    }
};

}  // namespace

bool read_tiff(const std::string &path, Frame *out, std::string *err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { *err = "cannot open " + path; return false; }
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (b.size() < 8 || !((b[0] == 'I' && b[1] == 'I') || (b[0] == 'M' && b[1] == 'M'))) {
        *err = path + ": not a TIFF file";
        return false;
    }
    Rd r{b, b[0] == 'M'};
    if (r.u16(2) != 42) { *err = path + ": bad TIFF magic"; return false; }
    size_t ifd = r.u32(4);
    const uint16_t nent = r.u16(ifd);
    uint32_t width = 0, height = 0, bps = 1, comp = 1, spp = 1, rps = 0xFFFFFFFF, fmt = 1, planar = 1;
    std::vector<uint32_t> offs, cnts;
    auto values = [&](size_t e, std::vector<uint32_t> *v) {
        const uint16_t type = r.u16(e + 2);
        const uint32_t n = r.u32(e + 4);
        const size_t sz = (type == 3) ? 2 : 4;
        size_t p = (n * sz <= 4) ? e + 8 : r.u32(e + 8);
        for (uint32_t i = 0; i < n; ++i) v->push_back(type == 3 ? r.u16(p + i * sz) : r.u32(p + i * sz));
    };
    for (uint16_t i = 0; i < nent; ++i) {
        const size_t e = ifd + 2 + (size_t)i * 12;
        const uint16_t tag = r.u16(e);
        std::vector<uint32_t> v;
        values(e, &v);
        if (v.empty()) continue;
        switch (tag) {
            case 256: width = v[0]; break;
            case 257: height = v[0]; break;
            case 258: bps = v[0]; break;
            case 259: comp = v[0]; break;
            case 273: offs = v; break;
            case 277: spp = v[0]; break;
            case 278: rps = v[0]; break;
            case 279: cnts = v; break;
            case 284: planar = v[0]; break;
            case 339: fmt = v[0]; break;
            default: break;
        }
    }
    if (!r.ok || width == 0 || height == 0 || offs.empty()) { *err = path + ": malformed TIFF"; return false; }
    if (comp != 1) { *err = path + ": compressed TIFF not supported"; return false; }
    if (spp != 1 || planar != 1 || fmt != 1 || (bps != 8 && bps != 16)) {
        *err = path + ": only single-channel unsigned 8/16-bit TIFF is supported";
        return false;
    }
    (void)rps;
    out->width = (int)width;
    out->height = (int)height;
    out->px.assign((size_t)width * height, 0);
    const size_t bpp = bps / 8, total = (size_t)width * height;
    size_t k = 0;
    for (size_t s = 0; s < offs.size() && k < total; ++s) {
        size_t o = offs[s];
        size_t n = (s < cnts.size()) ? cnts[s] / bpp : total - k;
        for (size_t i = 0; i < n && k < total; ++i, ++k) out->px[k] = (bps == 16) ? r.u16(o + 2 * i) : b.at(o + i);
    }
    if (!r.ok || k != total) { *err = path + ": truncated TIFF"; return false; }
    return true;
}

bool write_tiff16(const std::string &path, int width, int height, const uint16_t *px, std::string *err) {
    FILE *f = fopen(path.c_str(), "wb");
    if (!f) { *err = "cannot create " + path; return false; }
    auto w16 = [&](uint16_t v) { fwrite(&v, 2, 1, f); };
    auto w32 = [&](uint32_t v) { fwrite(&v, 4, 1, f); };
    const uint32_t data_off = 8, nbytes = (uint32_t)width * height * 2;
    fputc('I', f); fputc('I', f); w16(42); w32(data_off + nbytes);
    fwrite(px, 2, (size_t)width * height, f);
    const uint16_t tags[][2] = {{256, 4}, {257, 4}, {258, 3}, {259, 3}, {262, 3}, {273, 4}, {277, 3}, {278, 4}, {279, 4}};
    const uint32_t vals[] = {(uint32_t)width, (uint32_t)height, 16, 1, 1, data_off, 1, (uint32_t)height, nbytes};
    w16(9);
    for (int i = 0; i < 9; ++i) {
        w16(tags[i][0]); w16(tags[i][1]); w32(1);
        if (tags[i][1] == 3) { w16((uint16_t)vals[i]); w16(0); } else w32(vals[i]);
    }
    w32(0);
    fclose(f);
    return true;
}

}  // namespace fpmhost
