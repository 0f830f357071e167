// api_host.cpp -- extern "C" boundary of libfpm_host.so (include/fpm_host.h).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/fpm_host.h"
#include "dataset.hpp"
#include "tiff.hpp"

using namespace fpmhost;

namespace {
thread_local std::string g_herr;
int herr(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_herr = buf;
    return code;
}
}  // namespace

struct fpm_host {
    JsonParseResult parsed;
    Config cfg;
    bool has_table = false;
    LedTable table;
    std::vector<int> present;
    std::vector<std::string> names;   // file names when scanned from disk
    std::vector<LedGeom> geoms;
    std::vector<int16_t> order;       // sortedIndicies (LED numbers)
    std::vector<uint16_t> stack;      // [used][Np][Np] in order
    std::vector<int16_t> bg;          // per stack entry
    bool geometry_done = false;
};

extern "C" {

const char *fpm_host_last_error(void) { return g_herr.c_str(); }

int fpm_host_open_text(const char *text, fpm_host **out) {
    if (!out) return herr(-22, "null out");
    fpm_host *h = new fpm_host();
    std::string t = text ? text : "";
    if (!t.empty()) h->parsed = parse_json(t);
    else {
        h->parsed.ok = false;
        h->parsed.error = "empty document";
    }
    try {
        h->cfg = config_from_json(h->parsed);
    } catch (const std::exception &e) {
        delete h;
        return herr(-22, "config: %s", e.what());
    }
    *out = h;
    return 0;
}

int fpm_host_open(const char *path, fpm_host **out) {
    std::string text;
    if (!path || !read_file(path, &text)) text.clear();  // reference ignores a failed ifstream
    return fpm_host_open_text(text.c_str(), out);
}

void fpm_host_close(fpm_host *h) { delete h; }

int fpm_host_get_config(const fpm_host *h, fpm_host_config *o) {
    if (!h || !o) return herr(-22, "null argument");
    const Config &c = h->cfg;
    std::memset(o, 0, sizeof *o);
    o->np = c.np;
    o->nlarge = c.nlarge;
    o->res_improvement_factor = c.res_improvement_factor;
    o->na_radius = c.na_radius;
    o->led_count = c.led_count;
    o->crop_x = c.crop_x;
    o->crop_y = c.crop_y;
    o->bk1_crop_x = c.bk1_crop_x;
    o->bk1_crop_y = c.bk1_crop_y;
    o->bk2_crop_x = c.bk2_crop_x;
    o->bk2_crop_y = c.bk2_crop_y;
    o->center_led = c.center_led;
    o->darkfield_exp_multiplier = c.darkfield_exp_multiplier;
    o->color = c.color;
    o->flip_x = c.flip_x;
    o->flip_y = c.flip_y;
    o->debug = c.debug;
    o->hole_coordinates_present = c.hole_coordinates_array;
    o->hole_coordinates_count = (int)c.hole_coordinates.size();
    o->json_ok = c.json_ok;
    o->pixel_size = c.pixel_size;
    o->objective_mag = c.objective_mag;
    o->objective_na = c.objective_na;
    o->max_illumination_na = c.max_illumination_na;
    o->lambda = c.lambda;
    o->ps_eff = c.ps_eff;
    o->du = c.du;
    o->ps = c.ps;
    o->bg_threshold = c.bg_threshold;
    o->delta1 = c.delta1;
    o->delta2 = c.delta2;
    o->array_rotation = c.array_rotation;
    snprintf(o->dataset_root, sizeof o->dataset_root, "%s", c.dataset_root.c_str());
    snprintf(o->file_prefix, sizeof o->file_prefix, "%s", c.file_prefix.c_str());
    snprintf(o->file_extension, sizeof o->file_extension, "%s", c.file_extension.c_str());
    return 0;
}

int fpm_host_override(fpm_host *h, const char *key, double value) {
    if (!h || !key) return herr(-22, "null argument");
    try {
        const double iv = (double)(long long)value;
        h->parsed.root.set(key, iv == value ? Json::make_int((long long)value) : Json::make_real(value));
        h->cfg = config_from_json(h->parsed);
    } catch (const std::exception &e) {
        return herr(-22, "override %s: %s", key, e.what());
    }
    h->geometry_done = false;
    return 0;
}

int fpm_host_set_led_table(fpm_host *h, const float *xyz, int n) {
    if (!h || (!xyz && n > 0) || n < 0) return herr(-22, "bad LED table");
    h->table.xyz.assign(xyz, xyz + (size_t)3 * n);
    h->has_table = true;
    h->geometry_done = false;
    return 0;
}

int fpm_host_set_present(fpm_host *h, const int32_t *leds, int n) {
    if (!h || (!leds && n > 0) || n < 0) return herr(-22, "bad LED list");
    h->present.assign(leds, leds + n);
    h->names.clear();
    h->geometry_done = false;
    return 0;
}

int fpm_host_scan(fpm_host *h) {
    if (!h) return herr(-22, "null argument");
    h->present.clear();
    h->names.clear();
    std::string err;
    if (scan_dataset(h->cfg, &h->present, &h->names, &err)) return herr(-2, "%s", err.c_str());
    h->geometry_done = false;
    return (int)h->present.size();
}

int fpm_host_geometry(fpm_host *h) {
    if (!h) return herr(-22, "null argument");
    try {
        const LedTable *t = nullptr;
        if (h->has_table) t = &h->table;
        else if (!h->cfg.hole_coordinates_array && !h->cfg.hole_coordinates.is_null())
            return herr(-22, "dataset JSON has no holeCoordinates array (the reference aborts with "
                             "Json::LogicError here); supply an LED table, e.g. the 508-LED dome");
        h->geoms = compute_geometry(h->cfg, h->present, t);
        h->order = sorted_indices(h->cfg, h->geoms);
    } catch (const std::exception &e) {
        return herr(-22, "geometry: %s", e.what());
    }
    int used = 0;
    for (auto &g : h->geoms) used += g.used;
    if (used <= 0) return herr(-2, "ERROR - No images found in given directory.");
    h->geometry_done = true;
    return used;
}

int fpm_host_n_present(const fpm_host *h) { return h ? (int)h->present.size() : -22; }

int fpm_host_n_used(const fpm_host *h) { return (h && h->geometry_done) ? (int)h->order.size() : 0; }

int fpm_host_get_leds(const fpm_host *h, fpm_host_led *out, int n) {
    if (!h || !out) return herr(-22, "null argument");
    if (!h->geometry_done) return herr(-71, "geometry not computed");
    int k = 0;
    for (size_t i = 0; i < h->geoms.size() && k < n; ++i, ++k) {
        const LedGeom &g = h->geoms[i];
        fpm_host_led &o = out[k];
        std::memset(&o, 0, sizeof o);
        o.led = g.led;
        o.used = g.used;
        for (int j = 0; j < 3; ++j) o.pos[j] = g.pos[j];
        o.sin_theta_x = g.sin_x;
        o.sin_theta_y = g.sin_y;
        o.illumination_na = g.na;
        o.uled = g.uled;
        o.vled = g.vled;
        o.idx_u = g.idx_u;
        o.idx_v = g.idx_v;
        o.crop_x0 = g.crop_x0;
        o.crop_y0 = g.crop_y0;
        o.crop_x1 = g.crop_x1;
        o.crop_y1 = g.crop_y1;
        o.bg_val = 0;
        for (size_t s = 0; s < h->order.size() && s < h->bg.size(); ++s)
            if (h->order[s] == g.led) o.bg_val = h->bg[s];
    }
    return k;
}

int fpm_host_get_order(const fpm_host *h, int32_t *leds, int n) {
    if (!h || !leds) return herr(-22, "null argument");
    if (!h->geometry_done) return herr(-71, "geometry not computed");
    int k = 0;
    for (; k < (int)h->order.size() && k < n; ++k) leds[k] = h->order[k];
    return k;
}

static const LedGeom *find_led(const fpm_host *h, int led) {
    for (auto &g : h->geoms)
        if (g.led == led && g.used) return &g;
    return nullptr;
}

int fpm_host_get_crops(const fpm_host *h, int32_t *x0, int32_t *y0, int n) {
    if (!h || !x0 || !y0) return herr(-22, "null argument");
    if (!h->geometry_done) return herr(-71, "geometry not computed");
    int k = 0;
    for (; k < (int)h->order.size() && k < n; ++k) {
        const LedGeom *g = find_led(h, h->order[k]);
        if (!g) return herr(-22, "LED %d in order has no geometry", h->order[k]);
        x0[k] = g->crop_x0;
        y0[k] = g->crop_y0;
    }
    return k;
}

int fpm_host_load_images(fpm_host *h) {
    if (!h) return herr(-22, "null argument");
    if (!h->geometry_done) return herr(-71, "geometry not computed");
    if (h->cfg.color) return herr(-22, "colour datasets (isColor) are not supported by this build");
    const int np = h->cfg.np;
    h->stack.assign(h->order.size() * (size_t)np * np, 0);
    h->bg.assign(h->order.size(), 0);
    for (size_t s = 0; s < h->order.size(); ++s) {
        const int led = h->order[s];
        std::string name;
        for (size_t i = 0; i < h->present.size() && i < h->names.size(); ++i)
            if (h->present[i] == led) name = h->names[i];
        if (name.empty()) return herr(-2, "no file for LED %d (scan the dataset first)", led);
        Frame f;
        std::string err;
        if (!read_tiff(h->cfg.dataset_root + name, &f, &err)) return herr(-5, "%s", err.c_str());
        const LedGeom *g = find_led(h, led);
        std::vector<uint16_t> img;
        int16_t bg = 0;
        if (!preprocess_frame(h->cfg, f, g->na, &img, &bg, &err)) return herr(-22, "%s: %s", name.c_str(), err.c_str());
        std::memcpy(h->stack.data() + s * (size_t)np * np, img.data(), img.size() * sizeof(uint16_t));
        h->bg[s] = bg;
    }
    return (int)h->order.size();
}

int fpm_host_load_frames(const fpm_host *h, uint16_t *out, size_t n, int32_t *width, int32_t *height) {
    if (!h) return herr(-22, "null argument");
    if (!h->geometry_done) return herr(-71, "geometry not computed");
    if (h->cfg.color) return herr(-22, "colour datasets (isColor) are not supported by this build");
    int W = -1, H = -1;
    for (size_t s = 0; s < h->order.size(); ++s) {  // fpmMain.cpp:109-121, stack order
        const int led = h->order[s];
        std::string name;
        for (size_t i = 0; i < h->present.size() && i < h->names.size(); ++i)
            if (h->present[i] == led) name = h->names[i];
        if (name.empty()) return herr(-2, "no file for LED %d (scan the dataset first)", led);
        Frame f;
        std::string err;
        if (!read_tiff(h->cfg.dataset_root + name, &f, &err)) return herr(-5, "%s", err.c_str());
        if (s == 0) {
            W = f.width;
            H = f.height;
            if (width) *width = W;
            if (height) *height = H;
            if (!out) return 0;
            if (n < h->order.size() * (size_t)W * H)
                return herr(-22, "buffer too small: %zu < %zu", n, h->order.size() * (size_t)W * H);
        } else if (f.width != W || f.height != H) {
            return herr(-22, "%s: frame %dx%d differs from %dx%d", name.c_str(), f.width, f.height, W, H);
        }
        std::memcpy(out + s * (size_t)W * H, f.px.data(), (size_t)W * H * sizeof(uint16_t));
    }
    return (int)h->order.size();
}

int fpm_host_get_stack(const fpm_host *h, uint16_t *out, size_t n) {
    if (!h || !out) return herr(-22, "null argument");
    if (h->stack.empty()) return herr(-71, "images not loaded");
    if (n < h->stack.size()) return herr(-22, "buffer too small: %zu < %zu", n, h->stack.size());
    std::memcpy(out, h->stack.data(), h->stack.size() * sizeof(uint16_t));
    return 0;
}

int fpm_host_read_tiff(const char *path, uint16_t *out, size_t cap, int32_t *w, int32_t *hgt) {
    Frame f;
    std::string err;
    if (!path || !read_tiff(path, &f, &err)) return herr(-5, "%s", err.c_str());
    if (w) *w = f.width;
    if (hgt) *hgt = f.height;
    if (out) {
        if (cap < f.px.size()) return herr(-22, "buffer too small");
        std::memcpy(out, f.px.data(), f.px.size() * sizeof(uint16_t));
    }
    return 0;
}

int fpm_host_write_tiff16(const char *path, const uint16_t *px, int32_t w, int32_t hgt) {
    std::string err;
    if (!path || !px || !write_tiff16(path, w, hgt, px, &err)) return herr(-5, "%s", err.c_str());
    return 0;
}

}  // extern "C"
